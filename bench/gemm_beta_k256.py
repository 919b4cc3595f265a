"""Layer-3 conv1 dgrad with the residual join (M 50176, N 1024, K 256, beta 1, bf16 out): the default dispatch
(glds with C_old) against the stream kernel forced (DCA_OPS_STREAM=1) with C_old and with the masked source.
Run once per DCA_OPS_STREAM setting; prints median us over 50 launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from distributeddataparallel_cifar10_amd.ops.functional import gemm
    dev = torch.device("cuda", 0)
    M, N, K = 50176, 1024, 256
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = torch.randn(N, K, device=dev).to(torch.bfloat16)
    c = torch.randn(M, N, device=dev).to(torch.bfloat16)
    src = torch.randn(M, N, device=dev).to(torch.bfloat16)
    mask = torch.randint(0, 256, (M * N // 8,), device=dev, dtype=torch.int32).to(torch.uint8)

    def t(f):
        for _ in range(5):
            f()
        ts = []
        for _ in range(50):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return sorted(ts)[len(ts) // 2]

    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    tag = os.environ.get("DCA_OPS_STREAM", "default")
    print(f"stream={tag} beta C_old: {t(lambda: gemm(a, b, out_dtype=torch.bfloat16, out=c, beta=1.0)):.1f} us")
    print(f"stream={tag} masked src: "
          f"{t(lambda: gemm(a, b, out_dtype=torch.bfloat16, out=out, beta=1.0, beta_src=src, beta_mask=mask)):.1f} us")


if __name__ == "__main__":
    main()
