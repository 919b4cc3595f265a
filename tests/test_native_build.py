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


def test_wgrad_split_rules_for_the_row_kernels(monkeypatch):
    """ops/functional.py _wgrad_splits: the row-ring weight gradients (csrc/ops_wgrad.hip) get one split slab per
    workgroup -- 512 for the 64-channel 3x3 on rows <= 64 pixels, 128 for the 128-channel one on rows <= 32, 768 for
    the s2d stem on rows <= 128 -- and every other shape, or the knob off, keeps the k_wgrad rule."""
    from distributeddataparallel_cifar10_amd.ops import functional as F
    monkeypatch.setattr(F, "WGRAD_ROWS", True)
    k1, k2 = 256 * 56 * 56, 256 * 28 * 28
    assert F._wgrad_splits(64, 576, k1, True, row_w=56) == 512
    assert F._wgrad_splits(64, 576, 1000, True, row_w=10) == 3  # K // 256
    assert F._wgrad_splits(128, 1152, k2, True, row_w=28) == 128
    assert F._wgrad_splits(64, 256, 256 * 112 * 112, True, row_w=115) == 768  # the s2d stem
    assert F._wgrad_splits(64, 256, 256 * 112 * 112, True, row_w=134) == F._wgrad_splits(64, 256, 256 * 112 * 112, True)
    old1, old2 = F._wgrad_splits(64, 576, k1, True), F._wgrad_splits(128, 1152, k2, True)
    assert (old1, old2) == (205, 57)
    assert F._wgrad_splits(64, 576, k1, True, row_w=70) == old1
    assert F._wgrad_splits(128, 1152, k2, True, row_w=40) == old2
    monkeypatch.setattr(F, "WGRAD_ROWS", False)
    assert F._wgrad_splits(64, 576, k1, True, row_w=56) == old1


def test_row_kernel_lds_maps_are_conflict_free():
    """The LDS layouts of the row-ring kernels, mirrored here from csrc/ops_gemm.hip / ops_wgrad.hip (the test also
    checks the C++ still spells them this way): every ds_read_b128 lane group (4 x 16 lanes, bank = byte / 4 mod 64)
    of the forward kernels and every 32-lane half of the ds_read_b64_tr_b16 reads of the weight gradients touches each
    bank at most once, for every tap / pixel shift."""
    src = "".join(open(os.path.join(nbuild.CSRC, f)).read() for f in ("ops_gemm.hip", "ops_wgrad.hip"))
    for spelled in ("return px * (2 * C) + ((chunk ^ (px & (C / 8 - 1))) << 4);",
                    "return C == 64 ? j : (j < 8 ? j ^ 4 : j);",
                    "return C == 64 ? 4 * h + q : 8 * (q & 1) + 4 * (q >> 1) + h;",
                    "return px * 128 + ((chunk ^ ((((px >> 1) & 3) << 1) ^ (((px >> 3) & 1) << 2))) << 4);",
                    "else return px * 256 + ((chunk ^ (((px & 3) | (((px >> 3) & 1) << 2)) << 1)) << 4);",
                    "return px * 128 + ((chunk ^ (((px >> 1) & 3) << 1)) << 4);"):
        assert spelled in src, spelled

    def crc(C, px, c):
        return px * 2 * C + ((c ^ (px & (C // 8 - 1))) << 4)

    def pix(C, j):
        return j if C == 64 else (j ^ 4 if j < 8 else j)

    def chunk(C, h, q):
        return 4 * h + q if C == 64 else 8 * (q & 1) + 4 * (q >> 1) + h

    def wr(px, c):
        return px * 128 + ((c ^ ((((px >> 1) & 3) << 1) ^ (((px >> 3) & 1) << 2))) << 4)

    def wx128(px, c):
        return px * 256 + ((c ^ (((px & 3) | (((px >> 3) & 1) << 2)) << 1)) << 4)

    def ws2(px, c):
        return px * 128 + ((c ^ (((px >> 1) & 3) << 1)) << 4)

    def worst(addrs, width):
        banks = {}
        for a in addrs:
            for b in range(width // 4):
                k = (a // 4 + b) % 64
                banks[k] = banks.get(k, 0) + 1
        return max(banks.values())

    g16 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
           list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
    g16 += [[lane + 32 for lane in g] for g in g16]
    for C in (64, 128):  # forward: A fragment reads, lane (q, j) = pixel pix(j) + shift, chunk(h, q)
        for o in range(40):
            for h in range(C // 32):
                for g in g16:
                    assert worst([crc(C, pix(C, lane & 15) + o, chunk(C, h, lane >> 4)) for lane in g], 16) == 1
    # weight gradients: one 32-lane half = lane groups q, q + 1; lane 4 a + p of a group reads row a of its block
    # (pixel base + 8 q + 4 r + a, k_wgrad3x3_rows; base + 4 q + 16 r + a, k_wgrad_s2d_rows), 8 B at column 4 p
    for o in range(40):
        for cb in range(8):
            for r in range(2):
                for C, off in ((64, wr), (128, wx128)):
                    if C == 64 and cb >= 4:
                        continue
                    ad = [off(o + 8 * q + 4 * r + a, 2 * cb + (p >> 1)) + 8 * (p & 1)
                          for q in (0, 1) for a in range(4) for p in range(4)]
                    assert worst(ad, 8) == 1, (C, o, cb, r)
                if cb < 4:
                    ad = [ws2(o + 4 * q + 16 * r + a, 2 * cb + (p >> 1)) + 8 * (p & 1)
                          for q in (0, 1) for a in range(4) for p in range(4)]
                    assert worst(ad, 8) == 1, ("s2d dY", o, cb, r)
                    ad = [(o + 4 * q + 16 * r + a) * 32 + 8 * p for q in (0, 1) for a in range(4) for p in range(4)]
                    assert worst(ad, 8) == 1, ("s2d X", o, r)
