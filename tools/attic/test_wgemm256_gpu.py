"""The 256-column wide GEMM (csrc/wgemm256.hip: 256 x 256 workgroup tiles, 32x32x16 MFMAs, no loader waves) against a
PyTorch fp32 reference: every epilogue, fused RMSNorm on and off, unsplit (its own LDS-staged epilogue, incl. the LM
head's chunk maxima) and split-K plans (fp16 slabs through wgemm.hip's reducer), rows below the 256-row tile."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.models.weights import fold_gain, interleave_tiles, pack_mfma_a, rope_pair_order  # noqa: E402

DEV = torch.device("cuda")
V256 = 5  # csrc/wgemm.hip ring variant of the 256-column kernel (10: 4 loading waves, 11: loader waves)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _normed(x, norm, eps=1e-6):
    xr = x.float()
    return xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + eps) if norm else xr


@pytest.fixture(autouse=True, params=[5, 10, 11])
def _v256(request):
    global V256
    V256 = request.param
    ops.set_wide_gemm_min_m(64)
    ops.set_wide_gemm_variant(V256)
    yield
    ops.set_wide_gemm_variant(0)
    ops.clear_wide_gemm_plans()
    V256 = 5


def _plan(N, K, ks):
    ops.clear_wide_gemm_plans()
    if ks:
        ops.set_wide_gemm_plan(N, K, 256, ks, V256)


@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("N,K,norm,ks", [(4096, 4096, True, 0), (4096, 4096, False, 1), (6144, 4096, True, 0),
                                         (4096, 14336, False, 0), (28672, 4096, True, 0), (2048, 1536, True, 2),
                                         (4096, 4096, True, 3), (1024, 8960, False, 0)])
def test_v256_f32_matches_reference(M, N, K, norm, ks):
    torch.manual_seed(M + N + ks)
    _plan(N, K, ks)
    plan = ops.wide_gemm_plan(N, K, M)
    assert plan[1] == V256 and (not ks or plan[0] == ks), plan
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    wp = pack_mfma_a(W)
    ys = [ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=norm, eps=1e-6) for _ in range(2)]
    ref = _normed(x, norm) @ W.float().t()
    assert rel_err(ys[0], ref) < 2e-3, (plan, rel_err(ys[0], ref))
    assert torch.equal(ys[0], ys[1])  # deterministic


def test_v256_ineligible_shape_falls_back():
    """N not a multiple of 256 (e.g. 1920): the default 128-column ring runs instead (variant 0)."""
    assert ops.wide_gemm_plan(1920, 8960, 256)[1] == 0
    torch.manual_seed(1)
    W = (torch.randn(1920, 8960, device=DEV) * 0.02).bfloat16()
    x = torch.randn(256, 8960, device=DEV).bfloat16()
    y = ops.skinny_gemm(pack_mfma_a(W), x, 1920, ops.EPI_F32)
    assert rel_err(y, x.float() @ W.float().t()) < 2e-3


@pytest.mark.parametrize("ks", [0, 1])
@pytest.mark.parametrize("M", [160, 256])
def test_v256_bias_and_residual(ks, M):
    torch.manual_seed(5 + ks)
    N, K = 4096, 4096
    _plan(N, K, ks)
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
@pytest.mark.parametrize("ks", [0, 1])
@pytest.mark.parametrize("M,F,K", [(256, 14336, 4096), (130, 2048, 1024)])
def test_v256_gateup_fused_norm(act, ks, M, F, K):
    torch.manual_seed(9 + ks)
    _plan(2 * F, K, ks)
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


def test_v256_lm_head_chunk_maxima():
    """Unsplit LM head (N = 32000: 125 column blocks, one split forced): fp32 logits and the sampler's 16-column
    chunk maxima."""
    torch.manual_seed(2)
    N, K, M = 32000, 4096, 256
    _plan(N, K, 1)
    assert ops.wide_gemm_plan(N, K, M) == (1, V256)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    cmax = torch.full((M, N // 16), -1e30, device=DEV)
    lib = ops.load()
    lib.cain_gemm_set_cmax(ops._p(cmax))
    y = ops.skinny_gemm(pack_mfma_a(W), x, N, ops.EPI_F32, norm=True, eps=1e-6)
    ref = _normed(x, True) @ W.float().t()
    assert rel_err(y, ref) < 2e-3
    assert torch.equal(cmax, y.view(M, N // 16, 16).amax(-1))


@pytest.mark.parametrize("norm", [True, False])
@pytest.mark.parametrize("scale", [1e3, 1e5])
def test_v256_fp16_slabs_scale_outlier_rows(norm, scale):
    """Rows of outliers through the 256-column kernel's scaled fp16 split-K slabs (as wgemm.hip's)."""
    torch.manual_seed(int(scale) % 97 + norm)
    N, K, M = 4096, 4096, 256
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV)
    x[::7] *= scale
    x = x.bfloat16()
    assert ops.wide_gemm_plan(N, K, M)[0] > 1
    y = ops.skinny_gemm(pack_mfma_a(W), x, N, ops.EPI_F32, norm=norm, eps=1e-6)
    ref = _normed(x, norm) @ W.float().t()
    assert bool(torch.isfinite(y).all())
    for rows in (slice(0, None, 7), slice(1, None, 7)):
        assert rel_err(y[rows], ref[rows]) < 3e-3


def _rope_tables(hd, T_max, theta=10000.0):
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(T_max, dtype=torch.float64)[:, None] * inv[None]
    return ang.cos().float().to(DEV), ang.sin().float().to(DEV)


def _rot(x, c, s_):
    half = x.shape[-1] // 2
    return torch.cat([x[..., :half] * c - x[..., half:] * s_, x[..., half:] * c + x[..., :half] * s_], -1)


@pytest.mark.parametrize("ks", [0, 1])
def test_v256_qkv_rope_kv_append(ks):
    """llama3.1:8b's fused QKV (norm, RoPE, KV-cache append) at 256 rows on the 256-column kernel."""
    torch.manual_seed(8 + ks)
    H, Hkv, hd, M, K, T_max = 32, 8, 128, 256, 4096, 256
    qkv_dim = (H + 2 * Hkv) * hd
    _plan(qkv_dim, K, ks)
    W = (torch.randn(qkv_dim, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    per = rope_pair_order(hd).to(DEV)
    perm = torch.cat([h * hd + per for h in range(H + Hkv)] + [torch.arange((H + Hkv) * hd, qkv_dim, device=DEV)])
    kc = torch.zeros(M, Hkv, T_max, hd, device=DEV).bfloat16()
    vt = torch.zeros(M, Hkv, hd, T_max, device=DEV).bfloat16()
    q = torch.zeros(M, H * hd, device=DEV).bfloat16()
    slot = torch.randperm(M, device=DEV).int()
    pos = torch.randint(0, T_max, (M,), device=DEV).int()
    cos_t, sin_t = _rope_tables(hd, T_max)
    g = (1 + 0.2 * torch.randn(K, device=DEV)).bfloat16()
    ops.qkv_rope(pack_mfma_a(fold_gain(W[perm], g)), x, qkv_dim, q, kc, vt, slot, pos, cos_t, sin_t, H, Hkv, hd,
                 norm=True, eps=1e-6)
    xr = x.float()
    xr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * g.float()
    ref = (xr @ W.float().t()).bfloat16().float()
    kn, vn = ops.unpack_kcache(kc), ops.unpack_vcache(vt)
    for m in range(0, M, 17):
        p, sl = int(pos[m]), int(slot[m])
        c, s_ = cos_t[p], sin_t[p]
        assert rel_err(q[m].view(H, hd), _rot(ref[m, : H * hd].view(H, hd), c, s_)) < 1e-2
        assert rel_err(kn[sl, :, p], _rot(ref[m, H * hd:(H + Hkv) * hd].view(Hkv, hd), c, s_)) < 1e-2
        assert rel_err(vn[sl, :, p], ref[m, (H + Hkv) * hd:].view(Hkv, hd)) < 1e-2
