"""CU masks of CU-limited streams (runtime.hip cain_cu_mask): n of the device's CUs, whole groups of 8 consecutive
mask bits, balanced over the 8 XCDs whether the mask numbering interleaves the XCDs (CU i on XCD i % 8) or runs
through them in turn (32 CUs per XCD)."""
import pytest

from cain_amd import ops

if not ops.available():  # pragma: no cover
    pytest.skip("kernel library not built", allow_module_level=True)


def bits(mask):
    return [32 * w + i for w, m in enumerate(mask) for i in range(32) if m >> i & 1]


@pytest.mark.parametrize("n", [64, 128, 192, 256])
def test_mask_balanced_over_xcds(n):
    on = bits(ops.cu_mask(n, 256))
    assert len(on) == n
    interleaved = [sum(1 for i in on if i % 8 == x) for x in range(8)]
    blocked = [sum(1 for i in on if i // 32 == x) for x in range(8)]
    assert interleaved == [n // 8] * 8
    assert blocked == [n // 8] * 8


@pytest.mark.parametrize("n", [8, 40, 96, 248])
def test_mask_counts_and_groups(n):
    on = bits(ops.cu_mask(n, 256))
    assert len(on) == n and len(set(on)) == n
    assert all(i % 8 == 0 and all(i + b in on for b in range(8)) for i in on if i % 8 == 0)


@pytest.mark.parametrize("n", [0, 7, 260])
def test_mask_rejects(n):
    with pytest.raises(ValueError):
        ops.cu_mask(n, 256)


def test_budget_defaults_to_device():
    ops.set_cu_budget(64)
    try:
        assert ops.cu_budget() == 64
    finally:
        ops.set_cu_budget(0)
    assert ops.cu_budget() >= 64
