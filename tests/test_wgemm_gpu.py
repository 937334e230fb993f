"""Wide-batch GEMM (csrc/wgemm.hip, 64 < M <= 256) against a PyTorch fp32 reference, every epilogue, fused
RMSNorm on and off, split-K (narrow N) and unsplit (wide N) plans, N not a multiple of the 128-column block."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.models.weights import fold_gain, interleave_tiles, pack_mfma_a  # noqa: E402

DEV = torch.device("cuda")


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _normed(x, norm, eps=1e-6):
    xr = x.float()
    return xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + eps) if norm else xr


@pytest.fixture(autouse=True)
def _wide_on():
    ops.set_wide_gemm_min_m(64)
    yield
    ops.set_wide_gemm_min_m(64)


@pytest.mark.parametrize("M", [65, 128, 129, 200, 256])
@pytest.mark.parametrize("N,K,norm", [(4096, 4096, True), (6144, 4096, False), (32064, 3072, True),
                                      (1920, 8960, False), (16384, 2048, True), (4096, 14336, False)])
def test_wide_f32_matches_reference(M, N, K, norm):
    torch.manual_seed(M + N)
    assert ops.wide_gemm_eligible(N, K, M)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    wp = pack_mfma_a(W)
    ys = [ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=norm, eps=1e-6) for _ in range(2)]
    ref = _normed(x, norm) @ W.float().t()
    assert rel_err(ys[0], ref) < 2e-3
    assert torch.equal(ys[0], ys[1])  # deterministic (fixed split order)


@pytest.mark.parametrize("M", [100, 256])
def test_wide_bias_and_residual(M):
    torch.manual_seed(5)
    N, K = 4096, 4096
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV)
    y = ops.skinny_gemm(pack_mfma_a(W), x, N, ops.EPI_BF16, bias=bias)
    assert rel_err(y, x.float() @ W.float().t() + bias) < 1e-2
    r = torch.randn(M, N, device=DEV).bfloat16()
    ref = x.float() @ W.float().t() + r.float()
    ops.skinny_gemm(pack_mfma_a(W), x, N, ops.EPI_RESID, out=r)
    assert rel_err(r, ref) < 1e-2


@pytest.mark.parametrize("act", ["silu", "gelu"])
@pytest.mark.parametrize("M,F,K", [(256, 14336, 4096), (130, 2048, 1024), (256, 1024, 3072)])
def test_wide_gateup_fused_norm(act, M, F, K):
    torch.manual_seed(9)
    Wg = (torch.randn(F, K, device=DEV) * 0.02).bfloat16()
    Wu = (torch.randn(F, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.3 * torch.randn(K, device=DEV)).bfloat16()
    epi = ops.EPI_SILU if act == "silu" else ops.EPI_GELU
    y = ops.skinny_gemm(pack_mfma_a(interleave_tiles(fold_gain(Wg, g), fold_gain(Wu, g), tile=8)), x, 2 * F, epi,
                        norm=True, eps=1e-5)
    xn = _normed(x, True, 1e-5) * g.float()
    a = xn @ Wg.float().t()
    a = torch.nn.functional.silu(a) if act == "silu" else torch.nn.functional.gelu(a, approximate="tanh")
    assert rel_err(y, a * (xn @ Wu.float().t())) < 2e-2


def test_wide_matches_previous_batched_kernel():
    torch.manual_seed(3)
    N, K, M = 6144, 4096, 256
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    wp = pack_mfma_a(W)
    y_new = ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=True)
    ops.set_wide_gemm_min_m(0)
    y_old = ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=True)
    assert rel_err(y_new, y_old) < 1e-3


@pytest.mark.parametrize("N,K,norm,epi", [(4096, 4096, False, "resid"), (6144, 4096, True, "f32"),
                                          (4096, 14336, False, "f32"), (1920, 8960, True, "f32")])
def test_wide_splitk_repeatable_after_batched_path(N, K, norm, epi):
    """Split-K plans (narrow N) right after a batched-path (M <= 64) GEMM on the same workspace: the two paths'
    counter regions must not overlap (their slabs do), and repeated launches give identical results."""
    torch.manual_seed(N + K)
    M = 256
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    wp = pack_mfma_a(W)
    ops.skinny_gemm(wp, x[:48], N, ops.EPI_F32, norm=norm)  # the batched path's split-K slabs + tickets
    ref = _normed(x, norm) @ W.float().t()
    if epi == "resid":
        r0 = torch.randn(M, N, device=DEV).bfloat16()
        outs = []
        for _ in range(3):
            r = r0.clone()
            ops.skinny_gemm(wp, x, N, ops.EPI_RESID, out=r, norm=norm)
            outs.append(r)
        assert rel_err(outs[0], ref + r0.float()) < 1e-2
    else:
        outs = [ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=norm, eps=1e-6) for _ in range(3)]
        assert rel_err(outs[0], ref) < 2e-3
    assert all(torch.equal(o, outs[0]) for o in outs)


@pytest.mark.parametrize("ks,variant", [(3, 4), (6, 0), (16, 4), (1, 0)])
def test_shape_plan_override(ks, variant):
    """A per-shape plan (split count, ring variant) changes the launch, not the result (up to the fp16 rounding of the
    split-K slabs, which differs with the split count: ~1e-4 relative, 8x below the bf16 output rounding)."""
    torch.manual_seed(ks)
    N, K, M = 4096, 4096, 256
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    wp = pack_mfma_a(W)
    ref = ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=True)
    try:
        ops.set_wide_gemm_plan(N, K, 256, ks, variant)
        assert ops.wide_gemm_plan(N, K, M) == (ks, variant)
        y = ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=True)
    finally:
        ops.clear_wide_gemm_plans()
    assert rel_err(y, ref) < 1e-3


@pytest.mark.parametrize("norm", [True, False])
@pytest.mark.parametrize("scale", [1e3, 1e5])
def test_fp16_slabs_scale_outlier_rows(norm, scale):
    """the default fp16 split-K slabs on rows of outliers (values ~1e3-1e5, as a residual stream can carry)
    for a NORM shape (the QKV split, partials taken before the RMSNorm scale) and a RESID-sized one: every 16 x 16
    slab unit is stored scaled by a power of two, so the result equals the fp32-slab variant (4) to fp16's relative
    precision instead of saturating at 65504."""
    torch.manual_seed(int(scale) % 97 + norm)
    N, K, M = 4096, 4096, 256
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV)
    x[::7] *= scale  # every 7th row an outlier row
    x = x.bfloat16()
    wp = pack_mfma_a(W)
    assert ops.wide_gemm_plan(N, K, M)[0] > 1  # a split plan: the slabs are used
    y16 = ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=norm, eps=1e-6)
    try:
        ops.set_wide_gemm_plan(N, K, 256, 0, 4)  # the default split count, fp32 slabs
        y32 = ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=norm, eps=1e-6)
    finally:
        ops.clear_wide_gemm_plans()
    ref = _normed(x, norm) @ W.float().t()
    assert bool(torch.isfinite(y16).all())
    for rows in (slice(0, None, 7), slice(1, None, 7)):  # outlier rows and ordinary rows, each against fp32
        assert rel_err(y16[rows], y32[rows]) < 2e-3, (rows, rel_err(y16[rows], y32[rows]))
        assert rel_err(y16[rows], ref[rows]) < 3e-3


@pytest.mark.parametrize("N,K,norm,epi,variant", [(4096, 4096, False, "resid", 0), (6144, 4096, True, "f32", 0),
                                                  (4096, 14336, False, "f32", 0), (4096, 4096, True, "f32", 4),
                                                  (2048, 8192, True, "f32", 0)])
def test_inline_combine_matches_the_reduce_launch(N, K, norm, epi, variant):
    """the split-K combine inside the GEMM launch (wg_inline_combine) gives the same outputs as
    the separate wgemm_reduce_kernel launch -- also on the give-up path, where no partner waits and the last arriver
    combines every piece -- and leaves the block counters at zero for the next launch."""
    torch.manual_seed(N ^ K)
    M = 256
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    x[7] *= 300.0  # an outlier row (fp16 slab scaling)
    wp = pack_mfma_a(W)
    r0 = torch.randn(M, N, device=DEV).bfloat16()
    outs = {}
    mode0 = ops.wide_gemm_inline_mode()
    try:
        ops.set_wide_gemm_variant(variant)
        for mode in (0, 1, 2, 1):
            ops.set_wide_gemm_inline(mode)
            assert ops.wide_gemm_inline(N, K, M) == (mode > 0 and ops.wide_gemm_plan(N, K, M)[0] > 1)
            if epi == "resid":
                r = r0.clone()
                ops.skinny_gemm(wp, x, N, ops.EPI_RESID, out=r, norm=norm)
                outs.setdefault(mode, []).append(r)
            else:
                outs.setdefault(mode, []).append(ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=norm, eps=1e-6))
            torch.cuda.synchronize()
            ws = ops._ws_cache[x.device]
            assert int(ws[16384:16384 + 4096].count_nonzero()) == 0  # the wide path's counter words, reset
    finally:
        ops.set_wide_gemm_inline(mode0)
        ops.set_wide_gemm_variant(0)
    assert ops.wide_gemm_plan(N, K, M)[0] > 1  # a split plan: the combine ran
    ref = _normed(x, norm) @ W.float().t() + (r0.float() if epi == "resid" else 0)
    assert rel_err(outs[0][0], ref) < (1e-2 if epi == "resid" else 2e-3)
    for mode in (1, 2):
        for y in outs[mode]:
            assert bool((y == outs[0][0]).all()), mode  # same pieces summed in the same order


def test_inline_combine_falls_back_when_the_grid_exceeds_the_cus():
    """A split plan whose grid is larger than the CU count cannot have every partner resident: it runs the separate
    reduce launch (the plan override asks for 16 splits of 32 column blocks = 512 workgroups)."""
    N, K, M = 4096, 4096, 256
    mode0 = ops.wide_gemm_inline_mode()
    try:
        ops.set_wide_gemm_inline(1)
        ops.set_wide_gemm_plan(N, K, 256, 16, 0)
        assert not ops.wide_gemm_inline(N, K, M)
        ops.set_wide_gemm_plan(N, K, 256, 4, 0)
        assert ops.wide_gemm_inline(N, K, M)
    finally:
        ops.clear_wide_gemm_plans()
        ops.set_wide_gemm_inline(mode0)
