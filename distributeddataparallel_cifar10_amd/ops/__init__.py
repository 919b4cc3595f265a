"""ops: general-purpose MI355X layer kernels (HIP, gfx950) as autograd functions, and model forwards on them.

The NetResDeep fast path is the fused engine (``runtime/engine.py``); this layer is what any other model (and
NetResDeep outside the engine) trains on: MFMA GEMM (bf16 / fp8 e4m3), im2col convolution, BatchNorm with
fused ReLU / residual, pooling, cross-entropy, flat SGD, fp8 quantisation -- see ``functional.py``.
"""
from .functional import (batch_norm_act, conv2d, conv_bn_act, cross_entropy, fp8_alpha, gemm, global_avg_pool, linear,  # noqa: F401
                         max_pool2d, quantize_fp8, sgd_step_)
from .models import OpsModel  # noqa: F401
