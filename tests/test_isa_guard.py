"""The few-row MXFP4 stream kernels keep their counted load waits in the BUILT library (CPU-only check).

Round 5 compiled a runtime split-K branch into every w4_stream_kernel instance; hipcc then drained the weight ring
(``s_waitcnt vmcnt(0)``) at every item and batch-1 MXFP4 decode fell 5-13 % on all seven models while every
numerics test passed.  This reads the gfx950 code objects out of libcain_kernels.so
(tools/isa_guard.py) and bounds the vmcnt(0) waits inside each unsplit stream kernel's loop at what the counted-wait
code has: one per unrolled ring item at most (the epilogue's residual / bias loads at a tile edge, EPI_BF16 /
EPI_RESID), <= 2 for the fp32 / activation epilogues, and the fused QKV epilogue's 17 (RoPE tables and cache
stores at the tile edge).  The round-5 binary measured 15 / 10 / 25 on the same counter."""
import re
import shutil
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))

import isa_guard  # noqa: E402

# EPI -> the most vmcnt(0) an unsplit stream kernel's loop may hold (gemm_epi.h: BF16 0, RESID 1, F32 2, SILU 3,
# GELU 4, QKV_ROPE 5)
LIMIT = {0: 5, 1: 5, 2: 2, 3: 2, 4: 2, 5: 17}


@pytest.fixture(scope="module")
def stream_kernels():
    if not (isa_guard.LLVM / "llvm-objdump").exists() or shutil.which("hipcc") is None and not Path("/opt/rocm/bin/hipcc").exists():
        pytest.skip("ROCm llvm tools not available")
    from cain_amd import build

    lib = build.build_kernels()
    found = {}
    for co in isa_guard.code_objects(lib):
        found.update(isa_guard.kernel_loop_waits(isa_guard.disassemble(co), "w4_stream_kernel"))
    assert found, "no w4_stream_kernel in the library"
    return found


def _params(name):
    # _Z16w4_stream_kernelILi<WAVES>ELi<U>ELi<EPI>ELb<NORM>ELb<SPLIT>E...
    m = re.search(r"w4_stream_kernelILi(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELb(\d)E", name)
    assert m, name
    return tuple(int(g) for g in m.groups())


def test_unsplit_stream_kernels_keep_counted_waits(stream_kernels):
    checked = 0
    for name, (n_loop, waits) in stream_kernels.items():
        waves, u, epi, norm, split = _params(name)
        if split:
            continue
        assert n_loop > 0, f"{name}: no loop found"
        assert waits <= LIMIT[epi], f"{name}: {waits} vmcnt(0) in the loop (limit {LIMIT[epi]})"
        checked += 1
    assert checked >= 20  # 2 shapes x 5 epilogues x 2 norms, + the 4-wave QKV pair


def test_no_split_or_eight_wave_qkv_instance(stream_kernels):
    """The split path is compiled only where a launch can take it (not the fused QKV epilogue), and the 8-wave QKV
    stream kernel (FOLD, never chosen by the shape rule) is gone from the shipped library."""
    for name in stream_kernels:
        waves, u, epi, norm, split = _params(name)
        assert not (epi == 5 and (split or waves == 8)), name


# gemm_q4.hip's stream kernels: the same loop, plus the activation-staging loop's gain loads (4 waits)
Q4_LIMIT = {0: 9, 1: 9, 2: 5, 3: 5, 4: 5, 5: 21}


def test_q4_stream_kernels_keep_counted_waits():
    from cain_amd import build

    lib = build.build_kernels()
    found = {}
    for co in isa_guard.code_objects(lib):
        found.update(isa_guard.kernel_loop_waits(isa_guard.disassemble(co), "q4_stream_kernel"))
    assert len(found) >= 20
    for name, (n_loop, waits) in found.items():
        m = re.search(r"q4_stream_kernelILi(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELi(\d)E", name)
        waves, u, epi, norm, fmt = (int(x) for x in m.groups())
        assert n_loop > 0 and waits <= Q4_LIMIT[epi], f"{name}: {waits} vmcnt(0) in its loops"
        assert not (epi == 5 and waves == 8), name
