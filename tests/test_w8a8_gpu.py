"""W8A8 wide-batch GEMM (csrc/wgemm8.hip: e4m3 weights x per-row-quantised e4m3 activations on the block-scaled
fp8 MFMA) against plain PyTorch fp32 references on the dequantised operands, every epilogue, split and
unsplit plans; the activation quantiser; and the fp8 engine at 256 rows against the fp32 oracle (VERDICT r1
'what to do next' #8)."""
import dataclasses

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.engine import DecodeEngine  # noqa: E402
from cain_amd.models.config import get_config  # noqa: E402
from cain_amd.models.reference import ReferenceModel, fp8_kv_roundtrip  # noqa: E402
from cain_amd.models.weights import (dequantize_fp8_rows, fold_gain, fp8_roundtrip_weights,  # noqa: E402
                                     interleave_tiles, pack_mfma_a_fp8_k128, quantize_fp8_rows, rope_pair_order)

DEV = torch.device("cuda")


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def q8(w):
    q, s = quantize_fp8_rows(w)
    return pack_mfma_a_fp8_k128(q), s, dequantize_fp8_rows(q, s)


def deq_x(x, norm=False, eps=1e-6):
    """The activations exactly as the kernel multiplies them: e4m3(x8) * xs."""
    x8, xs = ops.quant_rows(x, norm, eps)
    return x8.view(torch.float8_e4m3fn).float() * xs[:, None]


@pytest.mark.parametrize("norm", [False, True])
@pytest.mark.parametrize("K", [512, 4096, 14336])
def test_quant_rows(norm, K):
    torch.manual_seed(K)
    M = 37
    x = (3 * torch.randn(M, K, device=DEV)).bfloat16()
    x[3] = 0  # an all-zero row keeps a finite scale
    x8, xs = ops.quant_rows(x, norm, 1e-6)
    xf = x.float()
    amax = xf.abs().amax(-1)
    scale = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    nf = torch.rsqrt(xf.pow(2).mean(-1) + 1e-6) if norm else torch.ones_like(amax)
    assert torch.allclose(xs, scale * nf, rtol=1e-5)
    deq = x8.view(torch.float8_e4m3fn).float() * scale[:, None]
    assert rel_err(deq, xf) < 3e-2
    assert float(x8.view(torch.float8_e4m3fn).float().abs().amax()) <= 448.0


@pytest.mark.parametrize("M", [17, 64, 128, 129, 256])
@pytest.mark.parametrize("N,K,norm", [(4096, 4096, True), (6144, 4096, False), (32064, 3072, True),
                                      (1920, 8960, False), (4096, 14336, False), (28672, 4096, True)])
def test_w8a8_f32_matches_dequantised_reference(M, N, K, norm):
    torch.manual_seed(M + N)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    wq, s, Wd = q8(W)
    ys = [ops.gemm_w8a8(wq, s, x, N, ops.EPI_F32, norm=norm, eps=1e-6) for _ in range(2)]
    ref = deq_x(x, norm) @ Wd.t()
    assert rel_err(ys[0], ref) < 1e-3
    assert torch.equal(ys[0], ys[1])
    # and the whole W8A8 approximation stays near the bf16 GEMM
    xr = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-6) if norm else x.float()
    assert rel_err(ys[0], xr @ W.float().t()) < 6e-2


@pytest.mark.parametrize("M", [100, 256])
def test_w8a8_bias_and_residual(M):
    torch.manual_seed(5)
    N, K = 4096, 4096
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, s, Wd = q8(W)
    bias = torch.randn(N, device=DEV)
    y = ops.gemm_w8a8(wq, s, x, N, ops.EPI_BF16, bias=bias)
    assert rel_err(y, deq_x(x) @ Wd.t() + bias) < 1e-2
    r = torch.randn(M, N, device=DEV).bfloat16()
    ref = deq_x(x) @ Wd.t() + r.float()
    ops.gemm_w8a8(wq, s, x, N, ops.EPI_RESID, out=r)
    assert rel_err(r, ref) < 1e-2


@pytest.mark.parametrize("act", ["silu", "gelu"])
@pytest.mark.parametrize("M,F,K", [(256, 14336, 4096), (130, 2048, 1024), (40, 1024, 3072)])
def test_w8a8_gateup_norm(act, M, F, K):
    torch.manual_seed(9)
    Wg = (torch.randn(F, K, device=DEV) * 0.02).bfloat16()
    Wu = (torch.randn(F, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.3 * torch.randn(K, device=DEV)).bfloat16()
    wq, s, Wd = q8(interleave_tiles(fold_gain(Wg, g), fold_gain(Wu, g), tile=8))
    epi = ops.EPI_SILU if act == "silu" else ops.EPI_GELU
    y = ops.gemm_w8a8(wq, s, x, 2 * F, epi, norm=True, eps=1e-5)
    gu = (deq_x(x, True, 1e-5) @ Wd.t()).view(M, F // 8, 2, 8)
    gg, u = gu[:, :, 0].reshape(M, F), gu[:, :, 1].reshape(M, F)
    a = torch.nn.functional.silu(gg) if act == "silu" else torch.nn.functional.gelu(gg, approximate="tanh")
    assert rel_err(y, a * u) < 1.5e-2


def _rot(x, c, s_):
    half = x.shape[-1] // 2
    return torch.cat([x[..., :half] * c - x[..., half:] * s_, x[..., half:] * c + x[..., :half] * s_], -1)


@pytest.mark.parametrize("H,Hkv,hd", [(32, 8, 128), (8, 1, 256)])
@pytest.mark.parametrize("kv", ["bf16", "fp8"])
def test_w8a8_qkv_rope_kv_append(H, Hkv, hd, kv):
    torch.manual_seed(8)
    M, K, T_max, S = 200, 1024, 256, 256
    qkv_dim = (H + 2 * Hkv) * hd
    W = (torch.randn(qkv_dim, K, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(qkv_dim, device=DEV)
    x = torch.randn(M, K, device=DEV).bfloat16()
    per = rope_pair_order(hd).to(DEV)
    perm = torch.cat([h * hd + per for h in range(H + Hkv)] + [torch.arange((H + Hkv) * hd, qkv_dim, device=DEV)])
    kt = torch.uint8 if kv == "fp8" else torch.bfloat16
    kc = torch.zeros(S, Hkv, T_max, hd, device=DEV, dtype=kt)
    vt = torch.zeros(S, Hkv, hd, T_max, device=DEV, dtype=kt)
    q = torch.zeros(M, H * hd, device=DEV).bfloat16()
    slot = torch.randperm(S, device=DEV)[:M].int()
    pos = torch.randint(0, T_max, (M,), device=DEV).int()
    inv = 1.0 / (10000.0 ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(T_max, dtype=torch.float64)[:, None] * inv[None]
    cos_t, sin_t = ang.cos().float().to(DEV), ang.sin().float().to(DEV)
    qw, s = quantize_fp8_rows(W)
    Wd = dequantize_fp8_rows(qw, s)
    ops.gemm_w8a8(pack_mfma_a_fp8_k128(qw[perm]), s[perm].contiguous(), x, qkv_dim, ops.EPI_QKV_ROPE,
                  bias=bias[perm], out=q,
                  rope=dict(kc=kc, vtc=vt, slot=slot, pos=pos, cos_t=cos_t, sin_t=sin_t, H=H, Hkv=Hkv, hd=hd))
    ref = (deq_x(x) @ Wd.t() + bias).bfloat16().float()
    kn, vn = ops.unpack_kcache(kc), ops.unpack_vcache(vt)
    rt = (lambda t: t)  # noqa: E731
    if kv == "fp8":  # the cache holds e4m3: compare with the oracle's values rounded the same way
        kn, vn = kn.view(torch.float8_e4m3fn).float(), vn.view(torch.float8_e4m3fn).float()
        rt = fp8_kv_roundtrip
    tol = 2e-2 if kv == "fp8" else 1e-2
    for m in range(0, M, 7):
        p, sl = int(pos[m]), int(slot[m])
        c, s_ = cos_t[p], sin_t[p]
        assert rel_err(q[m].view(H, hd), _rot(ref[m, : H * hd].view(H, hd), c, s_)) < 1e-2
        assert rel_err(kn[sl, :, p], rt(_rot(ref[m, H * hd:(H + Hkv) * hd].view(Hkv, hd), c, s_))) < tol
        assert rel_err(vn[sl, :, p], rt(ref[m, (H + Hkv) * hd:].view(Hkv, hd))) < tol


def _prompts(n):
    topics = ["India", "World War II", "Elizabeth II", "The Beatles", "Lady Gaga", "Barack Obama"]
    return [f"In {100 * (1 + i % 3)} words, please give me information about {topics[i % len(topics)]}"
            + " and more" * (i % 4) for i in range(n)]


@pytest.mark.parametrize("name", ["llama3.1:8b", "gemma:2b", "qwen2:1.5b"])
def test_w8a8_engine_logits_near_oracle(name):
    """The fp8 engine at 1 (W8A16), 64 and 256 rows (W8A8) against the fp32 oracle on the dequantised weights
    with the same per-row e4m3 rounding of every GEMM input, on the real layer dimensions cut to 3 layers:
    random-init stacks amplify rounding noise with depth (the full 32-layer llama lands at cos ~0.92 from fp8
    activation noise alone: kernel and oracle round slightly different fp32 sums into different e4m3 bins),
    so depth would test the weights' chaos, not the kernels, which tests above pin exactly."""
    cfg = dataclasses.replace(get_config(name), n_layers=3)
    eng = DecodeEngine(cfg, device="cuda", max_batch=256, max_context=128, keep_natural=True, seed=29,
                       weight_dtype="fp8")
    assert eng.w8a8 and eng.max_batch == 256
    wq = fp8_roundtrip_weights(eng.weights)
    ref = {"bf16": ReferenceModel(wq, memo_weights=True), "fp8": ReferenceModel(wq, memo_weights=True,
                                                                                act_dtype="fp8")}
    for m, rows in ((1, [0]), (64, [0, 63]), (256, [0, 255])):
        prompts = _prompts(m)
        got = eng.last_logits(prompts)
        # one short prompt prefills in <= 16 rows: W8A16 (bf16 activations); wider forwards W8A8
        oracle = ref["bf16" if m == 1 else "fp8"]
        for i in rows:
            want = oracle.forward(torch.tensor([eng.encode(prompts[i])], device="cuda"), last_only=True)[0, -1]
            cos = float(torch.nn.functional.cosine_similarity(got[i].float(), want, dim=0))
            assert cos > 0.98, (name, m, i, cos)
    eng.close()
    del ref
    torch.cuda.empty_cache()


def test_w8a8_full_depth_tracks_bf16_engine():
    """Full 32-layer llama3.1:8b at 256 rows through the W8A8 kernels, against the fp32 oracle on the same
    fp8-rounded weights with the same per-row e4m3 rounding of every GEMM input: the engine's relative logit error
    stays within 1.25x that of the torch fp8-emulated bf16 path (bf16 compute, e4m3 activations) on the same
    weights -- a relative criterion (tests/numerics.py) instead of an absolute cosine, which at this depth would
    measure the random weights' chaos rather than the kernels."""
    from numerics import assert_within_eager, rel

    prompts = _prompts(256)
    rows = [0, 99, 255]
    e8 = DecodeEngine("llama3.1:8b", device="cuda", max_batch=256, max_context=128, keep_natural=True, seed=31,
                      weight_dtype="fp8")
    assert e8.w8a8
    got = e8.last_logits(prompts)[rows].float()
    wq = fp8_roundtrip_weights(e8.weights)
    e8.close()
    oracle = ReferenceModel(wq, memo_weights=True, act_dtype="fp8")
    eager = ReferenceModel(wq, compute_dtype=torch.bfloat16, memo_weights=True, act_dtype="fp8")
    e_eng, e_eager = [], []
    for j, i in enumerate(rows):
        toks = torch.tensor([e8.encode(prompts[i])], device="cuda")
        want = oracle.forward(toks, last_only=True)[0, -1]
        e_eng.append(rel(got[j], want))
        e_eager.append(rel(eager.forward(toks, last_only=True)[0, -1], want))
    assert_within_eager(e_eng, e_eager, "llama3.1:8b W8A8 full depth")
    del oracle, eager, wq
    torch.cuda.empty_cache()
