"""The co-residency rule of the sliced engine (csrc/engine.hip coresident_budget, mirrored in runtime/engine.py): one
rule for a device of its own and a device shared by n ranks.  CPU-only (pure arithmetic); the GPU tier checks that
the native rule refuses the same configurations (tests/test_engine_gpu.py::test_shared_device_budget_refuses_exact_fill).
"""
import os
import re

from distributeddataparallel_cifar10_amd.runtime.engine import coresident_budget, max_sliced_batch

MI355X_CUS = 256  # one step workgroup per CU (512 threads x 256 VGPRs)


def test_dedicated_device_keeps_one_cu():
    assert coresident_budget(1, MI355X_CUS) == 255
    assert max_sliced_batch(1, MI355X_CUS) == 63  # batch 64 (256 live workgroups) -> multi-kernel engine
    assert coresident_budget(1, MI355X_CUS, full_device=True) == 256  # explicit persistent=True may use every CU
    assert max_sliced_batch(1, MI355X_CUS, full_device=True) == 64


def test_shared_device_same_margin():
    # round 4's rule gave 8 ranks 256 / 8 = 32 CUs each: batch 8 (32 live workgroups) filled every CU and a BN
    # exchange once timed out; with the margin batch 8 is refused and batch 4 (16 per rank) runs
    assert coresident_budget(1, MI355X_CUS, 8) == 31
    assert max_sliced_batch(1, MI355X_CUS, 8) == 7
    assert 8 * 4 > coresident_budget(1, MI355X_CUS, 8) >= 4 * 4
    assert coresident_budget(1, MI355X_CUS, 2) == 127
    assert max_sliced_batch(1, MI355X_CUS, 2) == 31
    # the fc workers (65) fit beside 2 ranks x batch 8 (32 live each), not beside 2 ranks x batch 16
    assert 8 * 4 + 65 <= coresident_budget(1, MI355X_CUS, 2) < 16 * 4 + 65
    # the full-device request never applies to a shared device
    assert coresident_budget(1, MI355X_CUS, 8, full_device=True) == 31


def test_several_blocks_per_cu_keep_one_per_cu():
    assert coresident_budget(2, MI355X_CUS) == 256
    assert coresident_budget(2, MI355X_CUS, 4) == 64


def test_native_rule_is_the_same_formula():
    """The C++ function must keep the same margin expression (a drift would let the two disagree silently)."""
    src = open(os.path.join(os.path.dirname(__file__), "..", "distributeddataparallel_cifar10_amd", "csrc",
                            "engine.hip")).read()
    body = re.search(r"static int coresident_budget\(.*?\n}", src, re.S).group(0)
    assert "per_cu > 1 ? ncu : (full_device && n_share <= 1 ? 0 : 1)" in body
    assert "(slots - margin) / std::max(n_share, 1)" in body
