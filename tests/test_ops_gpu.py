"""Numerics of every HIP kernel against a plain PyTorch fp32 reference.

Shapes cover the study's variants: head_dim 96/128/256, GQA groups 1/4/6/7/8,
M = 1..256 rows, gate/up SiLU and GeLU-tanh epilogues, QKV bias, residual add.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.models.weights import fold_gain, interleave_tiles, pack_mfma_a, rope_pair_order  # noqa: E402

DEV = torch.device("cuda")


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("M", [1, 5, 16, 17, 33, 64])
@pytest.mark.parametrize("N,K", [(512, 256), (6144, 4096), (1024, 14336)])
def test_skinny_gemm_plain_bias(M, N, K):
    torch.manual_seed(0)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV)
    y = ops.skinny_gemm(pack_mfma_a(W), x, N, ops.EPI_BF16, bias=bias)
    ref = x.float() @ W.float().t() + bias
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("M", [1, 8, 32])
def test_skinny_gemm_resid_inplace(M):
    torch.manual_seed(1)
    N, K = 2048, 4096
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    ref = x.float() @ W.float().t() + r.float()
    ops.skinny_gemm(pack_mfma_a(W), x, N, ops.EPI_RESID, out=r)
    assert rel_err(r, ref) < 1e-2


@pytest.mark.parametrize("M", [1, 16, 64])
def test_skinny_gemm_fused_rmsnorm_prologue(M):
    torch.manual_seed(7)
    N, K = 1024, 3584
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (3 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.2 * torch.randn(K, device=DEV)).bfloat16()
    y = ops.skinny_gemm(pack_mfma_a(fold_gain(W, g)), x, N, ops.EPI_F32, norm=True, eps=1e-6)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-6) * g.float()
    assert rel_err(y, xn @ W.float().t()) < 1e-2


@pytest.mark.parametrize("M", [1, 20])
def test_skinny_gemm_fused_rmsnorm_gateup(M):
    torch.manual_seed(9)
    F, K = 2048, 4096
    Wg = (torch.randn(F, K, device=DEV) * 0.02).bfloat16()
    Wu = (torch.randn(F, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.3 * torch.randn(K, device=DEV)).bfloat16()
    y = ops.skinny_gemm(pack_mfma_a(interleave_tiles(fold_gain(Wg, g), fold_gain(Wu, g), tile=8)), x, 2 * F,
                        ops.EPI_SILU, norm=True, eps=1e-5)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    ref = torch.nn.functional.silu(xn @ Wg.float().t()) * (xn @ Wu.float().t())
    assert rel_err(y, ref) < 2e-2


def test_skinny_gemm_f32_logits():
    torch.manual_seed(2)
    N, K, M = 32064, 3072, 3
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    y = ops.skinny_gemm(pack_mfma_a(W), x, N, ops.EPI_F32)
    assert y.dtype == torch.float32
    assert rel_err(y, x.float() @ W.float().t()) < 1e-3


@pytest.mark.parametrize("act", ["silu", "gelu"])
@pytest.mark.parametrize("M", [1, 16, 40, 120])
def test_skinny_gemm_gateup(act, M):
    torch.manual_seed(3)
    F, K = 1536, 1024
    Wg = (torch.randn(F, K, device=DEV) * 0.03).bfloat16()
    Wu = (torch.randn(F, K, device=DEV) * 0.03).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    epi = ops.EPI_SILU if act == "silu" else ops.EPI_GELU
    y = ops.skinny_gemm(pack_mfma_a(interleave_tiles(Wg, Wu, tile=8)), x, 2 * F, epi)
    g = x.float() @ Wg.float().t()
    u = x.float() @ Wu.float().t()
    a = torch.nn.functional.silu(g) if act == "silu" else torch.nn.functional.gelu(g, approximate="tanh")
    assert y.shape == (M, F)
    assert rel_err(y, a * u) < 1.5e-2


@pytest.mark.parametrize("M", [17, 32, 48, 64, 65, 100, 128, 129, 200, 256])
@pytest.mark.parametrize("N,K,norm", [(32064, 3072, True), (256, 14336, False), (4096, 4096, True),
                                      (1920, 8960, False)])
def test_batched_gemm_matches_skinny_and_reference(M, N, K, norm):
    """The LDS-staged split-K path (16 < M <= 256): N not a multiple of the 128-row block, deep k-splits
    (N=256, K=14336 -> 56 partial ranges), fused norm; repeated launches check the self-resetting tickets."""
    torch.manual_seed(11)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.2 * torch.randn(K, device=DEV)).bfloat16() if norm else None
    assert ops.gemm_ws_bytes(N, K, M) > 0 or (M <= 32 and N < 8192)  # narrow N at M <= 32: skinny path
    Wf = fold_gain(W, g) if norm else W
    wp = pack_mfma_a(Wf)
    ys = [ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=norm, eps=1e-6) for _ in range(3)]
    y0 = ops.skinny_gemm(wp, x, N, ops.EPI_F32, norm=norm, eps=1e-6, batched=False) if M <= 64 else None
    xr = x.float()
    if norm:
        xr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6)
    ref = xr @ Wf.float().t()
    for y in ys:
        assert rel_err(y, ref) < 2e-3
        assert torch.equal(y, ys[0])  # deterministic reduction order
    if y0 is not None:  # the skinny kernel covers M <= 64
        assert rel_err(ys[0], y0) < 2e-3


@pytest.mark.parametrize("d", [1536, 2048, 3584, 4096])
def test_rmsnorm(d):
    x = torch.randn(7, d, device=DEV).bfloat16()
    g = (1 + 0.1 * torch.randn(d, device=DEV)).bfloat16()
    y = ops.rmsnorm(x, g, 1e-6)
    xf = x.float()
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * g.float()
    assert rel_err(y, ref) < 1e-2


def test_embed_scale():
    E = torch.randn(1000, 2048, device=DEV).bfloat16()
    tok = torch.tensor([3, 999, 0, 3], device=DEV, dtype=torch.int32)
    y = ops.embed(tok, E, 45.25)
    assert rel_err(y, E[tok.long()].float() * 45.25) < 1e-2


def _rope_tables(hd, T_max, theta=10000.0):
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(T_max, dtype=torch.float64)[:, None] * inv[None]
    return ang.cos().float().to(DEV), ang.sin().float().to(DEV)


def _rot(x, c, s_):
    half = x.shape[-1] // 2
    return torch.cat([x[..., :half] * c - x[..., half:] * s_, x[..., half:] * c + x[..., :half] * s_], -1)


@pytest.mark.parametrize("H,Hkv,hd", [(32, 8, 128), (12, 2, 128), (8, 1, 256), (32, 32, 96), (28, 4, 128)])
@pytest.mark.parametrize("M", [1, 5, 40, 128, 256])
@pytest.mark.parametrize("norm", [False, True])
def test_fused_qkv_rope_kv_append(H, Hkv, hd, M, norm):
    torch.manual_seed(8)
    K, T_max, S = 512, 256, max(64, M)
    qkv_dim = (H + 2 * Hkv) * hd
    W = (torch.randn(qkv_dim, K, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(qkv_dim, device=DEV)
    x = torch.randn(M, K, device=DEV).bfloat16()
    per = rope_pair_order(hd).to(DEV)
    perm = torch.cat([h * hd + per for h in range(H + Hkv)] + [torch.arange((H + Hkv) * hd, qkv_dim, device=DEV)])
    kc = torch.zeros(S, Hkv, T_max, hd, device=DEV).bfloat16()
    vt = torch.zeros(S, Hkv, hd, T_max, device=DEV).bfloat16()
    q = torch.zeros(M, H * hd, device=DEV).bfloat16()
    slot = torch.randperm(S, device=DEV)[:M].int()
    pos = torch.randint(0, T_max, (M,), device=DEV).int()
    cos_t, sin_t = _rope_tables(hd, T_max)
    g = (1 + 0.2 * torch.randn(K, device=DEV)).bfloat16() if norm else None
    Wp = pack_mfma_a(fold_gain(W[perm], g)) if norm else pack_mfma_a(W[perm])
    ops.qkv_rope(Wp, x, qkv_dim, q, kc, vt, slot, pos, cos_t, sin_t, H, Hkv, hd, bias=bias[perm], norm=norm, eps=1e-6)
    xr = x.float()
    if norm:
        xr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * g.float()
    ref = (xr @ W.float().t() + bias).bfloat16().float()
    kn, vn = ops.unpack_kcache(kc), ops.unpack_vcache(vt)  # fragment-major caches -> [S, Hkv, T, hd]
    for m in range(M):
        p, sl = int(pos[m]), int(slot[m])
        c, s_ = cos_t[p], sin_t[p]
        qh = ref[m, : H * hd].view(H, hd)
        kh = ref[m, H * hd:(H + Hkv) * hd].view(Hkv, hd)
        vh = ref[m, (H + Hkv) * hd:].view(Hkv, hd)
        assert rel_err(q[m].view(H, hd), _rot(qh, c, s_)) < 1e-2
        assert rel_err(kn[sl, :, p], _rot(kh, c, s_)) < 1e-2
        assert rel_err(vn[sl, :, p], vh) < 1e-2
    # nothing but the M appended positions was written
    assert int((kn != 0).any(-1).sum()) == M * Hkv and int((vn != 0).any(-1).sum()) == M * Hkv


def _attn_ref(q, K, V, L, G):
    H, hd = q.shape
    out = torch.empty(H, hd, device=q.device)
    for h in range(H):
        kh = h // G
        s = (q[h].float() @ K[kh][:L].float().t()) / math.sqrt(hd)
        out[h] = s.softmax(-1) @ V[kh][:L].float()
    return out


@pytest.mark.parametrize("H,Hkv,hd", [(32, 8, 128), (12, 2, 128), (8, 1, 256), (32, 32, 96), (28, 4, 128),
                                      (16, 16, 256)])
@pytest.mark.parametrize("lengths", [[1], [37, 130, 1, 600], [2048]])
def test_attention_split_combine(H, Hkv, hd, lengths):
    torch.manual_seed(4)
    T_max = 2048
    M = len(lengths)
    kc = torch.randn(M, Hkv, T_max, hd, device=DEV).bfloat16()
    vt = torch.randn(M, Hkv, hd, T_max, device=DEV).bfloat16()
    q = torch.randn(M, H * hd, device=DEV).bfloat16()
    slot = torch.arange(M, device=DEV, dtype=torch.int32)
    pos = torch.tensor([L - 1 for L in lengths], device=DEV, dtype=torch.int32)
    counters = torch.zeros(M * Hkv, device=DEV, dtype=torch.int32)
    kp, vp = ops.pack_kcache(kc), ops.pack_vcache(vt.transpose(-1, -2))  # the kernel's cache layouts
    for nsplit in (1, 3, 8, 16, 64, 2, 16):  # repeated nsplit: the in-kernel counters must reset
        out = ops.attention(q, kp, vp, slot, pos, H, Hkv, hd, nsplit, 1.0 / math.sqrt(hd), counters=counters)
        for m, L in enumerate(lengths):
            ref = _attn_ref(q[m].view(H, hd), kc[m].float(), vt[m].float().transpose(-1, -2), L, H // Hkv)
            assert rel_err(out[m].view(H, hd), ref) < 2e-2, (nsplit, m, L)
        assert int(counters.abs().sum()) == 0


def test_sample_greedy_and_topk():
    torch.manual_seed(5)
    M, V = 4, 151936
    logits = torch.randn(M, V, device=DEV)
    logits[0, 1234] = 50.0
    logits[1, 77] = 50.0
    tok = torch.zeros(M, device=DEV, dtype=torch.int32)
    pos = torch.full((M,), 10, device=DEV, dtype=torch.int32)
    gen = torch.zeros(M, 16, device=DEV, dtype=torch.int32)
    n_gen = torch.zeros(M, device=DEV, dtype=torch.int32)
    max_new = torch.full((M,), 8, device=DEV, dtype=torch.int32)
    done = torch.zeros(M, device=DEV, dtype=torch.int32)
    hist = torch.zeros(M * 64, device=DEV, dtype=torch.int32)
    slot = torch.arange(M, device=DEV, dtype=torch.int32)
    rows = [dict(temperature=0.0, top_p=1.0, repeat_penalty=1.0, top_k=40, repeat_last_n=64, eos_id=-1, seed=1),
            dict(temperature=0.8, top_p=0.9, repeat_penalty=1.1, top_k=40, repeat_last_n=64, eos_id=-1, seed=2),
            dict(temperature=1.0, top_p=1.0, repeat_penalty=1.0, top_k=1, repeat_last_n=0, eos_id=-1, seed=3),
            dict(temperature=1.0, top_p=0.5, repeat_penalty=1.0, top_k=5, repeat_last_n=0, eos_id=-1, seed=4)]
    params = ops.sample_params_tensor(rows, DEV)
    ref_arg = logits.argmax(-1).cpu()
    top5 = set(logits[3].topk(5).indices.cpu().tolist())
    ops.sample(logits.clone(), tok, pos, gen, n_gen, max_new, done, hist, slot, params, 2048)
    t = tok.cpu().tolist()
    assert t[0] == 1234
    assert t[1] == 77           # dominant logit survives temperature + top-p
    assert t[2] == int(ref_arg[2])  # top_k = 1 is greedy
    assert t[3] in top5
    assert n_gen.cpu().tolist() == [1, 1, 1, 1]
    assert pos.cpu().tolist() == [11, 11, 11, 11]
    assert gen[:, 0].cpu().tolist() == t


@pytest.mark.parametrize("V", [128256, 151936, 32064, 256000])
def test_sample_chunk_max_matches(V):
    """The chunk-maximum sampler draws the same token as the one-workgroup and two-stage kernels for the same
    logits, seeds and decode state: greedy, Ollama defaults with a repeat history (penalty > 1), a penalty < 1 (which
    raises history logits above their chunk maxima), top_k 256, top_p off, and a row with a planted history max."""
    torch.manual_seed(V % 97)
    M = 12
    base = torch.randn(M, V, device=DEV) * 3
    base[5, 777] = 40.0   # a dominant logit that is also in row 5's history (penalised)
    rows = []
    for i in range(M):
        kind = i % 6
        rows.append([dict(temperature=0.0, top_p=1.0, repeat_penalty=1.1, top_k=40, repeat_last_n=64),
                     dict(temperature=0.8, top_p=0.9, repeat_penalty=1.1, top_k=40, repeat_last_n=64),
                     dict(temperature=0.8, top_p=0.9, repeat_penalty=0.8, top_k=40, repeat_last_n=64),
                     dict(temperature=1.0, top_p=1.0, repeat_penalty=1.0, top_k=256, repeat_last_n=0),
                     dict(temperature=1.2, top_p=0.5, repeat_penalty=1.3, top_k=10, repeat_last_n=32),
                     dict(temperature=0.8, top_p=0.9, repeat_penalty=1.1, top_k=40, repeat_last_n=64)][kind])
        rows[-1].update(eos_id=-1, seed=1000 + i)
    params = ops.sample_params_tensor(rows, DEV)
    # a history of 20 generated ids per row, including the row's top logits (so the penalty matters)
    hist = torch.zeros(M, 64, device=DEV, dtype=torch.int32)
    top = base.topk(10, dim=-1).indices
    for i in range(M):
        ids = torch.cat([top[i, :6], torch.randint(0, V, (14,), device=DEV)]).to(torch.int32)
        hist[i, :20] = ids
    hist[5, 3] = 777
    results = []
    for mode in ("cm", "one", "split"):
        lg = base.clone()
        tok = torch.zeros(M, device=DEV, dtype=torch.int32)
        pos = torch.full((M,), 50, device=DEV, dtype=torch.int32)
        gen = torch.zeros(M, 32, device=DEV, dtype=torch.int32)
        n_gen = torch.full((M,), 20, device=DEV, dtype=torch.int32)
        max_new = torch.full((M,), 30, device=DEV, dtype=torch.int32)
        done = torch.zeros(M, device=DEV, dtype=torch.int32)
        h = hist.clone().view(-1)
        slot = torch.arange(M, device=DEV, dtype=torch.int32)
        cmax = base.view(M, V // 16, 16).amax(-1).contiguous() if mode == "cm" else None
        ops.sample(lg, tok, pos, gen, n_gen, max_new, done, h, slot, params, 2048, split=(mode == "split"), cmax=cmax)
        results.append((tok.cpu(), pos.cpu(), n_gen.cpu(), h.cpu()))
    for r in results[1:]:
        for a, b in zip(results[0], r):
            assert torch.equal(a, b)


def test_sample_distribution_matches_topk_softmax():
    """Sampling frequencies over many seeds follow softmax over the top-k (top_p off)."""
    torch.manual_seed(6)
    V, M = 5000, 64
    base = torch.randn(V) * 0.1
    base[:4] = torch.tensor([3.0, 2.5, 2.0, 1.0])
    logits = base.to(DEV).repeat(M, 1)
    counts = torch.zeros(4)
    for rep in range(16):
        tok = torch.zeros(M, device=DEV, dtype=torch.int32)
        z = lambda: torch.zeros(M, device=DEV, dtype=torch.int32)  # noqa: E731
        rows = [dict(temperature=1.0, top_p=1.0, repeat_penalty=1.0, top_k=3, repeat_last_n=0, eos_id=-1,
                     seed=rep * 1000 + i) for i in range(M)]
        ops.sample(logits.clone(), tok, z(), torch.zeros(M, 4, device=DEV, dtype=torch.int32), z(),
                   torch.full((M,), 4, device=DEV, dtype=torch.int32), z(), torch.zeros(M * 64, device=DEV,
                   dtype=torch.int32), torch.arange(M, device=DEV, dtype=torch.int32),
                   ops.sample_params_tensor(rows, DEV), 2048)
        for t in tok.cpu().tolist():
            assert t < 3
            counts[t] += 1
    p = torch.softmax(torch.tensor([3.0, 2.5, 2.0]), 0)
    freq = counts[:3] / counts.sum()
    assert torch.allclose(freq, p, atol=0.06), (freq, p)


@pytest.mark.parametrize("H,Hkv,hd", [(32, 8, 128), (32, 32, 96), (28, 4, 128), (16, 8, 64)])
@pytest.mark.parametrize("kv", ["bf16", "fp8"])
def test_attention_many_rows(H, Hkv, hd, kv):
    """Single-split attention over many (row, kv head) pairs (the decode batch shape): rows of different lengths,
    an idle row, bf16 and fp8 caches."""
    torch.manual_seed(21)
    T_max, M = 512, 200
    lengths = torch.randint(1, T_max, (M,)).tolist()
    kc = torch.randn(M, Hkv, T_max, hd, device=DEV)
    vt = torch.randn(M, Hkv, T_max, hd, device=DEV)
    if kv == "fp8":
        kc, vt = kc.to(torch.float8_e4m3fn).float(), vt.to(torch.float8_e4m3fn).float()
        kp = ops.pack_kcache(kc.to(torch.float8_e4m3fn).view(torch.uint8))
        vp = ops.pack_vcache(vt.to(torch.float8_e4m3fn).view(torch.uint8))
    else:
        kc, vt = kc.bfloat16().float(), vt.bfloat16().float()
        kp, vp = ops.pack_kcache(kc.bfloat16()), ops.pack_vcache(vt.bfloat16())
    q = torch.randn(M, H * hd, device=DEV).bfloat16()
    slot = torch.arange(M, device=DEV, dtype=torch.int32)
    slot[7] = -1  # an idle row: no output written, no cache read
    pos = torch.tensor([L - 1 for L in lengths], device=DEV, dtype=torch.int32)
    out = torch.full((M, H * hd), 7.0, device=DEV).bfloat16()
    ops.attention(q, kp, vp, slot, pos, H, Hkv, hd, 1, 1.0 / math.sqrt(hd), out=out)
    for m in range(0, M, 9):
        if m == 7:
            continue
        ref = _attn_ref(q[m].view(H, hd), kc[m], vt[m], lengths[m], H // Hkv)
        assert rel_err(out[m].view(H, hd), ref) < 2e-2, (m, lengths[m])


@pytest.mark.parametrize("H,Hkv", [(32, 8), (28, 4), (12, 2), (32, 32)])
@pytest.mark.parametrize("ring", [1])
def test_attention_ring(H, Hkv, ring):
    """The LDS-DMA ring body (persistent workgroups, loader waves streaming whole 32-position blocks) against the
    fp32 reference and the register kernel: 256 rows of different lengths (block-aligned and not), idle rows."""
    torch.manual_seed(22 + ring)
    hd, T_max, M = 128, 512, 256
    lengths = torch.randint(1, T_max, (M,)).tolist()
    lengths[3], lengths[4], lengths[5] = 32, 33, T_max
    kc = torch.randn(M, Hkv, T_max, hd, device=DEV).bfloat16().float()
    vt = torch.randn(M, Hkv, T_max, hd, device=DEV).bfloat16().float()
    kp, vp = ops.pack_kcache(kc.bfloat16()), ops.pack_vcache(vt.bfloat16())
    q = torch.randn(M, H * hd, device=DEV).bfloat16()
    slot = torch.arange(M, device=DEV, dtype=torch.int32)
    slot[7] = slot[200] = -1  # idle rows: zero output
    pos = torch.tensor([L - 1 for L in lengths], device=DEV, dtype=torch.int32)
    try:
        ops.set_attention_ring(0)
        base = ops.attention(q, kp, vp, slot, pos, H, Hkv, hd, 1, 1.0 / math.sqrt(hd))
        ops.set_attention_ring(ring)
        outs = []
        for _ in range(2):
            out = torch.full((M, H * hd), 7.0, device=DEV).bfloat16()
            ops.attention(q, kp, vp, slot, pos, H, Hkv, hd, 1, 1.0 / math.sqrt(hd), out=out)
            outs.append(out)
    finally:
        ops.set_attention_ring(1)  # the default
    out = outs[0]
    assert torch.equal(outs[0], outs[1])  # deterministic
    assert not out.isnan().any()
    assert float(out[7].float().abs().max()) == 0.0 and float(out[200].float().abs().max()) == 0.0
    live = [m for m in range(M) if m not in (7, 200)]
    assert rel_err(out[live].float(), base[live].float()) < 1e-2
    for m in list(range(0, M, 17)) + [3, 4, 5]:
        if m in (7, 200):
            continue
        ref = _attn_ref(q[m].view(H, hd), kc[m], vt[m], lengths[m], H // Hkv)
        assert rel_err(out[m].view(H, hd), ref) < 2e-2, (m, lengths[m])


@pytest.mark.parametrize("M", [1, 4, 16])
@pytest.mark.parametrize("N,K,epi,norm", [(1536, 8960, ops.EPI_RESID, False),     # qwen2:1.5b down (96 tiles)
                                          (1536, 1536, ops.EPI_RESID, False),     # qwen2:1.5b O
                                          (2048, 16384, ops.EPI_RESID, False),    # gemma:2b down
                                          (2048, 2048, ops.EPI_F32, True),        # fused RMSNorm, 128 tiles
                                          (2 * 1280, 2048, ops.EPI_SILU, True)])  # gate/up pairs, 160 tiles
def test_skinny_split_k_matches_fp32_and_unsplit(M, N, K, epi, norm):
    """Split-K skinny grids (narrow outputs at <= 16 rows: ks k-ranges per tile, last-arriver combine in fixed
    order) against the fp32 reference and against the unsplit kernel on the same inputs."""
    torch.manual_seed(N + K + M)
    W = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.2 * torch.randn(K, device=DEV)).bfloat16()
    Wf = fold_gain(W, g) if norm else W
    if epi == ops.EPI_SILU:
        Wp = pack_mfma_a(interleave_tiles(Wf[: N // 2], Wf[N // 2:], tile=8))
    else:
        Wp = pack_mfma_a(Wf)
    xr = x.float()
    if norm:
        xr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * g.float()
    if epi == ops.EPI_SILU:
        ref = torch.nn.functional.silu(xr @ W[: N // 2].float().t()) * (xr @ W[N // 2:].float().t())
    else:
        ref = xr @ W.float().t()
    outs = []
    for batched in (True, False):
        r0 = torch.randn(M, N, device=DEV).bfloat16() if epi == ops.EPI_RESID else None
        if r0 is not None:
            torch.manual_seed(5)
            r0 = torch.randn(M, N, device=DEV).bfloat16()
            out = r0.clone()
            ops.skinny_gemm(Wp, x, N, epi, out=out, norm=norm, eps=1e-6, batched=batched)
            want = ref + r0.float()
        else:
            out = ops.skinny_gemm(Wp, x, N, epi, norm=norm, eps=1e-6, batched=batched)
            want = ref
        assert rel_err(out, want) < 1e-2, (batched, rel_err(out, want))
        outs.append(out.float())
    if N // 16 < 192 and K // 32 > 128:
        assert ops.gemm_ws_bytes(N, K, M) > 0  # the split grid was taken with batched=True
    assert rel_err(outs[0], outs[1]) < 5e-3


@pytest.mark.parametrize("M", [1, 16])
@pytest.mark.parametrize("N,K", [(1536, 8960), (2048, 16384)])
def test_skinny_split_matches_unsplit(M, N, K):
    """The few-row split-K rule (narrow grids with long K: qwen2:1.5b / gemma:2b down projections at <= 16 rows) against
    the fp32 reference and the unsplit kernel (cain_gemm_set_skinny_split(0))."""
    torch.manual_seed(N + M)
    W = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    x = (2 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.2 * torch.randn(K, device=DEV)).bfloat16()
    Wp = pack_mfma_a(fold_gain(W, g))
    xr = x.float()
    xr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * g.float()
    ref = xr @ W.float().t()
    outs = []
    try:
        for mode in (1, 0):
            ops.set_skinny_split(mode)
            if mode == 1:
                assert ops.gemm_ws_bytes(N, K, M) > 0  # the split grid is taken
            out = ops.skinny_gemm(Wp, x, N, ops.EPI_F32, norm=True, eps=1e-6, batched=True)
            assert rel_err(out, ref) < 1e-2, (mode, rel_err(out, ref))
            outs.append(out.float())
    finally:
        ops.set_skinny_split(1)
    assert rel_err(outs[0], outs[1]) < 5e-3


@pytest.mark.parametrize("V", [151936, 32064, 600, 257])
@pytest.mark.parametrize("M", [1, 3, 64])
def test_split_sampler_draws_the_same_tokens(V, M):
    """The two-stage sampler (16 vocabulary slices per row, last-arriver merge) draws exactly the token of the
    one-workgroup kernel for the same logits, options and seed -- greedy, top-k 1..256, top-p, repeat penalty
    with a history -- and advances the decode state the same way."""
    torch.manual_seed(V + M)
    T_max = 2048

    def state():
        return dict(tok=torch.zeros(M, device=DEV, dtype=torch.int32),
                    pos=torch.full((M,), 10, device=DEV, dtype=torch.int32),
                    gen=torch.zeros(M, 32, device=DEV, dtype=torch.int32),
                    n_gen=torch.full((M,), 5, device=DEV, dtype=torch.int32),
                    max_new=torch.full((M,), 20, device=DEV, dtype=torch.int32),
                    done=torch.zeros(M, device=DEV, dtype=torch.int32),
                    hist=torch.randint(0, V, (M * 64,), device=DEV, dtype=torch.int32),
                    slot=torch.arange(M, device=DEV, dtype=torch.int32))

    for rep in range(6):
        logits = torch.randn(M, V, device=DEV) * (0.5 + rep)
        logits[:, :3] += 4.0  # a few dominant entries, with a tie at rep 0
        if rep == 0:
            logits[:, 7] = logits[:, 1]
        kinds = [(0.0, 40, 1.0), (0.8, 40, 0.9), (1.0, 1, 1.0), (1.2, 256, 0.95), (0.7, 0, 1.0), (1.0, 7, 0.5)]
        rows = [dict(temperature=kinds[i % 6][0], top_k=kinds[i % 6][1], top_p=kinds[i % 6][2],
                     repeat_penalty=1.1 if i % 2 else 1.0, repeat_last_n=64, eos_id=-1, seed=rep * 7919 + i)
                for i in range(M)]
        params = ops.sample_params_tensor(rows, DEV)
        out = []
        for split in (False, True):
            st = state()
            torch.manual_seed(rep)
            st["hist"] = torch.randint(0, V, (M * 64,), device=DEV, dtype=torch.int32, generator=None)
            ops.sample(logits.clone(), st["tok"], st["pos"], st["gen"], st["n_gen"], st["max_new"], st["done"],
                       st["hist"], st["slot"], params, T_max, split=split)
            out.append({k: v.cpu() for k, v in st.items()})
        for k in ("tok", "pos", "gen", "n_gen", "done", "hist"):
            assert torch.equal(out[0][k], out[1][k]), (rep, k)
    # greedy rows are the argmax (lowest index on ties)
    assert int(out[1]["tok"][0]) == int(torch.argmax(logits[0]).item()) or rows[0]["repeat_penalty"] != 1.0


@pytest.mark.parametrize("mode", ["one", "split", "cm"])
def test_sample_stop_ids_end_rows(mode):
    """A sampled token equal to any of a row's stop ids (beside eos_id) ends the row (done = 1, position kept), in
    every sampler kernel; a row whose stop ids miss the token goes on."""
    V, M = 32064, 4
    logits = torch.randn(M, V, device=DEV)
    win = [101, 202, 303, 404]
    for i, w in enumerate(win):
        logits[i, w] = 50.0  # greedy picks it
    rows = [dict(temperature=0.0, top_p=1.0, repeat_penalty=1.0, top_k=40, repeat_last_n=0, eos_id=-1, seed=1,
                 stop=st) for st in ([101], [7, 202], [1, 2, 303], [1, 2, 3])]
    z = lambda: torch.zeros(M, device=DEV, dtype=torch.int32)  # noqa: E731
    tok, n_gen, done = z(), z(), z()
    pos = torch.full((M,), 10, device=DEV, dtype=torch.int32)
    cmax = logits.view(M, V // 16, 16).amax(-1).contiguous() if mode == "cm" else None
    ops.sample(logits.clone(), tok, pos, torch.zeros(M, 8, device=DEV, dtype=torch.int32), n_gen,
               torch.full((M,), 8, device=DEV, dtype=torch.int32), done, torch.zeros(M * 64, device=DEV,
               dtype=torch.int32), torch.arange(M, device=DEV, dtype=torch.int32), ops.sample_params_tensor(rows, DEV),
               2048, split=(mode == "split"), cmax=cmax)
    assert tok.cpu().tolist() == win
    assert done.cpu().tolist() == [1, 1, 1, 0]
    assert pos.cpu().tolist() == [10, 10, 10, 11]
