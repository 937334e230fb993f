"""W4A8 wide-batch GEMM (csrc/wgemm8.hip FP4: MXFP4 weights in the few-row kernel's packing x per-row-quantised e4m3
activations on the block-scaled fp4 x fp8 MFMA, the e8m0 block scales as the MFMA's per-lane A scales) against
plain PyTorch fp32 references on the dequantised operands, every epilogue, split and unsplit plans, and the fp4
engine above 64 rows against the fp32 oracle with the same per-row e4m3 rounding of every GEMM input."""
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
from cain_amd.models.weights import (dequantize_mxfp4, fold_gain, interleave_tiles,  # noqa: E402
                                     mxfp4_roundtrip_weights, pack_mxfp4, quantize_mxfp4, rope_pair_order)

DEV = torch.device("cuda")


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def q4(w):
    c, s = quantize_mxfp4(w)
    wq, ws = pack_mxfp4(c, s)
    return wq, ws, dequantize_mxfp4(c, s)


def deq_x(x, norm=False, eps=1e-6):
    """The activations exactly as the kernel multiplies them: e4m3(x8) * xs."""
    x8, xs = ops.quant_rows(x, norm, eps)
    return x8.view(torch.float8_e4m3fn).float() * xs[:, None]


def test_w4a8_operand_layout_exact():
    """Exact integer data: one-hot activation rows pick weight columns (Y[m][n] = W[n][m], e2m1 codes at unit scale,
    e4m3 1.0 exact), so a k permutation between the fp4 A and fp8 B operands shows up element by element."""
    torch.manual_seed(1)
    N, K, M = 256, 512, 48
    vals = torch.tensor([0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0], device=DEV)
    W = vals[torch.randint(0, 8, (N, K), device=DEV)] * (1 - 2 * torch.randint(0, 2, (N, K), device=DEV)).float()
    W[:, ::32] = 6.0  # every block's amax 6: unit scale
    cols = torch.randperm(K, device=DEV)[:M]
    x = torch.zeros(M, K, device=DEV)
    x[torch.arange(M, device=DEV), cols] = 1.0
    wq, ws, Wd = q4(W.bfloat16())
    assert torch.equal(Wd, W)
    y = ops.gemm_w4a8(wq, ws, x.bfloat16(), N, ops.EPI_F32)
    want = W[:, cols].t()
    bad = ((y - want).abs() > 1e-6 * want.abs()).nonzero()
    assert bad.numel() == 0, f"{bad.shape[0]} mismatches, first (m, n): {bad[:8].tolist()}"


def test_w4a8_block_scales_exact():
    """All-ones activations against e2m1 1.0 codes whose 32-k blocks carry distinct powers of two: Y[m][n] is the
    sum over blocks of 32 * 2^e[n][b], exact -- a scale applied to the wrong lane / block shows up per element."""
    torch.manual_seed(2)
    N, K, M = 16384, 1024, 32  # >= 128 column blocks: one split, no fp16 slabs between the MFMA and the output
    e = torch.randint(-6, 7, (N, K // 32), device=DEV).float()
    W = torch.exp2(e).repeat_interleave(32, dim=1)
    wq, ws, Wd = q4(W.bfloat16())
    assert torch.equal(Wd, W)
    y = ops.gemm_w4a8(wq, ws, torch.ones(M, K, device=DEV).bfloat16(), N, ops.EPI_F32)
    want = (32 * torch.exp2(e)).sum(1)[None].expand(M, N)
    bad = ((y - want).abs() > 1e-6 * want.abs()).nonzero()
    assert bad.numel() == 0, f"{bad.shape[0]} mismatches, first (m, n): {bad[:8].tolist()}"


@pytest.mark.parametrize("M", [17, 64, 65, 128, 129, 256])
@pytest.mark.parametrize("N,K,norm", [(4096, 4096, True), (6144, 4096, False), (32064, 3072, True),
                                      (1536, 8960, False), (4096, 14336, False), (28672, 4096, True)])
def test_w4a8_f32_matches_dequantised_reference(M, N, K, norm):
    torch.manual_seed(M + N)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    wq, ws, Wd = q4(W)
    ys = [ops.gemm_w4a8(wq, ws, x, N, ops.EPI_F32, norm=norm, eps=1e-6) for _ in range(2)]
    ref = deq_x(x, norm) @ Wd.t()
    assert rel_err(ys[0], ref) < 1e-3
    assert torch.equal(ys[0], ys[1])


def test_w4a8_block_scales_span_the_exponent_range():
    """Every 32-k block of every row at its own power of two (2^-20 .. 2^20): a block scale applied to the wrong
    lane, row or k range of the MFMA shows up as a large error."""
    assert ops.w8a8_eligible(16384, 4096, 200)
    torch.manual_seed(3)
    N, K, M = 16384, 4096, 200  # one split (fp16 split-K slabs would saturate on these magnitudes)
    e = torch.randint(-20, 21, (N, K // 32), device=DEV).float()
    W = (torch.randn(N, K, device=DEV) * torch.exp2(e).repeat_interleave(32, dim=1)).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, ws, Wd = q4(W)
    y = ops.gemm_w4a8(wq, ws, x, N, ops.EPI_F32)
    assert rel_err(y, deq_x(x) @ Wd.t()) < 1e-3


@pytest.mark.parametrize("M", [100, 256])
def test_w4a8_bias_and_residual(M):
    torch.manual_seed(5)
    N, K = 4096, 4096
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, ws, Wd = q4(W)
    bias = torch.randn(N, device=DEV)
    y = ops.gemm_w4a8(wq, ws, x, N, ops.EPI_BF16, bias=bias)
    assert rel_err(y, deq_x(x) @ Wd.t() + bias) < 1e-2
    r = torch.randn(M, N, device=DEV).bfloat16()
    ref = deq_x(x) @ Wd.t() + r.float()
    ops.gemm_w4a8(wq, ws, x, N, ops.EPI_RESID, out=r)
    assert rel_err(r, ref) < 1e-2


@pytest.mark.parametrize("act", ["silu", "gelu"])
@pytest.mark.parametrize("M,F,K", [(256, 14336, 4096), (130, 2048, 1024), (40, 1024, 3072)])
def test_w4a8_gateup_norm(act, M, F, K):
    torch.manual_seed(9)
    Wg = (torch.randn(F, K, device=DEV) * 0.02).bfloat16()
    Wu = (torch.randn(F, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.3 * torch.randn(K, device=DEV)).bfloat16()
    wq, ws, Wd = q4(interleave_tiles(fold_gain(Wg, g), fold_gain(Wu, g), tile=8))
    epi = ops.EPI_SILU if act == "silu" else ops.EPI_GELU
    y = ops.gemm_w4a8(wq, ws, x, 2 * F, epi, norm=True, eps=1e-5)
    gu = (deq_x(x, True, 1e-5) @ Wd.t()).view(M, F // 8, 2, 8)
    gg, u = gu[:, :, 0].reshape(M, F), gu[:, :, 1].reshape(M, F)
    a = torch.nn.functional.silu(gg) if act == "silu" else torch.nn.functional.gelu(gg, approximate="tanh")
    assert rel_err(y, a * u) < 1.5e-2


def _rot(x, c, s_):
    half = x.shape[-1] // 2
    return torch.cat([x[..., :half] * c - x[..., half:] * s_, x[..., half:] * c + x[..., :half] * s_], -1)


@pytest.mark.parametrize("kv", ["bf16", "fp8"])
def test_w4a8_qkv_rope_kv_append(kv):
    torch.manual_seed(8)
    H, Hkv, hd = 32, 8, 128
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
    wq, ws, Wd = q4(W[perm])
    ops.gemm_w4a8(wq, ws, x, qkv_dim, ops.EPI_QKV_ROPE, bias=bias[perm], out=q,
                  rope=dict(kc=kc, vtc=vt, slot=slot, pos=pos, cos_t=cos_t, sin_t=sin_t, H=H, Hkv=Hkv, hd=hd))
    inv_perm = torch.argsort(perm)
    ref = (deq_x(x) @ Wd[inv_perm].t() + bias).bfloat16().float()
    kn, vn = ops.unpack_kcache(kc), ops.unpack_vcache(vt)
    rt = (lambda t: t)  # noqa: E731
    if kv == "fp8":
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
def test_w4a8_engine_logits_near_oracle(name):
    """The fp4 engine at 1 row (W4A16: one short prompt prefills in <= 16 rows) and 64 / 256 rows (W4A8) against the
    fp32 oracle on the dequantised MXFP4 weights, with the per-row e4m3 rounding of every GEMM input above 16 rows;
    the real layer dimensions cut to 3 layers (see test_w8a8_gpu.py for why depth is tested relatively)."""
    cfg = dataclasses.replace(get_config(name), n_layers=3)
    eng = DecodeEngine(cfg, device="cuda", max_batch=256, max_context=128, keep_natural=True, seed=29,
                       weight_dtype="fp4")
    assert eng.w4a8 and eng.max_batch == 256
    wq = mxfp4_roundtrip_weights(eng.weights)
    ref = {"bf16": ReferenceModel(wq, memo_weights=True), "fp8": ReferenceModel(wq, memo_weights=True,
                                                                                act_dtype="fp8")}
    for m, rows in ((1, [0]), (64, [0, 63]), (256, [0, 255])):
        prompts = _prompts(m)
        got = eng.last_logits(prompts)
        oracle = ref["bf16" if m == 1 else "fp8"]
        for i in rows:
            want = oracle.forward(torch.tensor([eng.encode(prompts[i])], device="cuda"), last_only=True)[0, -1]
            cos = float(torch.nn.functional.cosine_similarity(got[i].float(), want, dim=0))
            assert cos > 0.98, (name, m, i, cos)
    eng.close()
    del ref
    torch.cuda.empty_cache()


def test_w4a8_engine_greedy_decode_256_rows():
    """256 rows decode through the graph-replayed W4A8 path: every row completes and the graph replay equals the
    eager forwards token for token."""
    cfg = dataclasses.replace(get_config("qwen2:1.5b"), n_layers=4)
    eng = DecodeEngine(cfg, device="cuda", max_batch=256, max_context=256, seed=3, weight_dtype="fp4",
                       steps_per_graph=4)
    prompts = _prompts(256)
    opts = [dict(temperature=0.0, repeat_penalty=1.0, eos_id=-1)] * 256
    a = eng.generate(prompts, 8, opts, use_graph=True)
    b = eng.generate(prompts, 8, opts, use_graph=False)
    assert all(r.eval_count == 8 for r in a)
    assert [r.tokens for r in a] == [r.tokens for r in b]
    eng.close()
