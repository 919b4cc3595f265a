"""Native library: builds for gfx950 on the CPU host, exports the C ABI, and its layout matches the Python side."""
import ctypes
import os
import re

import numpy as np
import torch

import __graft_entry__
from distributeddataparallel_cifar10_amd import build as nbuild
from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
from distributeddataparallel_cifar10_amd.runtime import engine as E

COMMON_H = os.path.join(nbuild.CSRC, "common.h")


def _consts():
    out = {}
    for m in re.finditer(r"constexpr int (\w+) = (\d+);", open(COMMON_H).read()):
        out[m.group(1)] = int(m.group(2))
    return out


def test_layout_matches_common_h():
    c = _consts()
    names = {"fc1.weight": "OFF_FC1W", "fc2.weight": "OFF_FC2W", "fc1.bias": "OFF_FC1B", "fc2.bias": "OFF_FC2B",
             "resblocks.0.conv.weight": "OFF_CONVW", "resblocks.0.batch_norm.weight": "OFF_BNW",
             "resblocks.0.batch_norm.bias": "OFF_BNB", "conv1.weight": "OFF_C1W", "conv1.bias": "OFF_C1B"}
    for pname, cname in names.items():
        assert E.LAYOUT[pname][0] == c[cname], pname
    assert (E.FLAT_N, E.FLAT_ALLOC, E.OFF_RS, E.BUCKET_A_END) == (c["FLAT_N"], c["FLAT_ALLOC"], c["OFF_RS"],
                                                                   c["BUCKET_A_END"])
    # segments do not overlap and are 16-byte aligned where the kernels use vector loads
    spans = sorted((off, off + int(np.prod(shape))) for off, shape in E.LAYOUT.values())
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
    assert spans[-1][1] <= E.OFF_RS
    assert all(E.LAYOUT[k][0] % 4 == 0 for k in ("fc1.weight", "fc2.weight", "resblocks.0.conv.weight"))


def test_bind_flat_parameters_views():
    m = NetResDeep()
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    flat, grads = E.bind_flat_parameters(m, "cpu")
    for n, p in m.named_parameters():
        off, shape = E.LAYOUT[n]
        assert p.data_ptr() == flat[off:].data_ptr()
        assert p.grad.data_ptr() == grads[off:].data_ptr()
        assert torch.equal(p.detach(), before[n])
    assert m.resblocks[4].conv.weight.data_ptr() == flat[E.LAYOUT["resblocks.0.conv.weight"][0]:].data_ptr()


def test_tile_layout_conversion():
    # element (row, col = 4q + i, ch = 16h + c) at row*512 + h*256 + (16q + c)*4 + i  (persistent kernel tl())
    count, batch = 2, 3
    nhwc = torch.randn(count, batch, 16, 16, 32)
    raw = torch.empty(count, batch, 8192)
    for row in range(16):
        for col in range(16):
            q, i = divmod(col, 4)
            for ch in range(32):
                h, c = divmod(ch, 16)
                raw[:, :, row * 512 + h * 256 + (16 * q + c) * 4 + i] = nhwc[:, :, row, col, ch]
    assert torch.equal(E.tile_to_nhwc(raw.reshape(-1), count, batch), nhwc)


def test_graft_build_and_abi():
    __graft_entry__.build()  # hipcc --offload-arch=gfx950 (cross-compiles without a GPU)
    path = nbuild.lib_path()
    assert os.path.exists(path)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    lib.dca_abi_version.restype = ctypes.c_int
    assert lib.dca_abi_version() > 0
    for sym in ("dca_engine_create", "dca_engine_run", "dca_engine_destroy", "dca_engine_errors",
                "dca_nccl_unique_id", "dca_engine_precapture", "dca_engine_comm_time"):
        assert hasattr(lib, sym), sym


def test_code_object_targets_gfx950():
    # the fat binary embeds the offload bundle id "hipv4-amdgcn-amd-amdhsa--gfx950"
    blob = open(nbuild.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_ops_library_builds_and_exports():
    """The ops layer's library (csrc/ops_api.hip) cross-compiles for gfx950 and exports its C ABI."""
    path = nbuild.build(variant="ops")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    lib.dca_ops_abi_version.restype = ctypes.c_int
    from distributeddataparallel_cifar10_amd.ops import _native
    assert lib.dca_ops_abi_version() == _native.ABI_VERSION
    for sym in ("dca_ops_gemm", "dca_ops_im2col", "dca_ops_col2im", "dca_ops_bn_fwd", "dca_ops_bn_bwd",
                "dca_ops_maxpool_fwd", "dca_ops_maxpool_bwd", "dca_ops_avgpool_fwd", "dca_ops_avgpool_bwd",
                "dca_ops_cross_entropy", "dca_ops_sgd", "dca_ops_quant_fp8", "dca_ops_fp8_alpha"):
        assert hasattr(lib, sym), sym
    assert b"amdgcn-amd-amdhsa--gfx950" in open(path, "rb").read()


def test_ops_gemm_args_mirror_matches_header():
    """ops/_native.py GemmArgs lists the fields of csrc/ops_gemm.hip GemmArgs in the same order."""
    src = open(os.path.join(nbuild.CSRC, "ops_gemm.hip")).read()
    body = src[src.index("struct GemmArgs {"):src.index("};", src.index("struct GemmArgs {"))]
    names = []
    for line in body.splitlines()[1:]:
        decl = line.split("//")[0].strip().rstrip(";")
        if decl:
            names += [n.strip() for n in re.sub(r"^(const\s+)?\w+\s*\**\s*", "", decl).split(",")]
    from distributeddataparallel_cifar10_amd.ops._native import GemmArgs
    assert [f[0] for f in GemmArgs._fields_] == [n.strip() for n in names]


def test_ops_reject_cpu_tensors():
    import pytest
    from distributeddataparallel_cifar10_amd import ops
    with pytest.raises(ValueError):
        ops.gemm(torch.zeros(4, 8, dtype=torch.bfloat16), torch.zeros(4, 8, dtype=torch.bfloat16))
