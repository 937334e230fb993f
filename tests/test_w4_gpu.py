"""MXFP4-weight (W4A16) kernels of ``csrc/gemm_w4.hip`` against a plain PyTorch fp32 reference computed on the
dequantised weights (e2m1 code x e8m0 block scale), and the ``weight_dtype="fp4"`` engine against the torch oracle
on the same dequantised weights (``mxfp4_roundtrip_weights``)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.engine import DecodeEngine  # noqa: E402
from cain_amd.models import TINY  # noqa: E402
from cain_amd.models.reference import ReferenceModel  # noqa: E402
from cain_amd.models.weights import (dequantize_mxfp4, fold_gain, interleave_tiles,  # noqa: E402
                                     mxfp4_roundtrip_weights, pack_mxfp4, quantize_mxfp4, rope_pair_order)

DEV = torch.device("cuda")
N_VARS = 6  # gemm_w4.hip W4Var: 2 persistent stream shapes, 4 tile shapes


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def q4(w):
    c, s = quantize_mxfp4(w)
    wq, ws = pack_mxfp4(c, s)
    return wq, ws, dequantize_mxfp4(c, s)


@pytest.fixture(autouse=True)
def _rule_variant():
    ops.set_w4_variant(-1)
    yield
    ops.set_w4_variant(-1)
    ops.set_w4_occupancy(0)


def test_e2m1_convert_semantics():
    """One tile whose codes walk all 16 e2m1 values at 3 block scales: the kernel's dequantisation (the hardware
    convert) equals the packer's, element by element (x = unit rows picks single weights out)."""
    N, K = 16, 128
    codes = (torch.arange(N * K, device=DEV) % 16).to(torch.uint8).reshape(N, K)
    scales = torch.tensor([127, 120, 131, 100], device=DEV, dtype=torch.uint8).repeat(N, 1)
    wq, ws = pack_mxfp4(codes, scales)
    Wd = dequantize_mxfp4(codes, scales)
    eye = torch.eye(K, device=DEV).bfloat16()
    for m0 in range(0, K, 64):
        y = ops.gemm_w4(wq, ws, eye[m0:m0 + 64].contiguous(), N, ops.EPI_F32)
        assert torch.equal(y, Wd[:, m0:m0 + 64].t().contiguous()), m0


@pytest.mark.parametrize("M", [1, 7, 16, 17, 64])
@pytest.mark.parametrize("N,K", [(512, 256), (6144, 4096), (1024, 14336), (2048, 8960), (32064, 3072),
                                 (128256, 4096)])
def test_w4_gemm_f32_and_bias(M, N, K):
    torch.manual_seed(0)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, ws, Wd = q4(W)
    y = ops.gemm_w4(wq, ws, x, N, ops.EPI_F32)
    assert y.dtype == torch.float32
    assert rel_err(y, x.float() @ Wd.t()) < 1e-3
    bias = torch.randn(N, device=DEV)
    yb = ops.gemm_w4(wq, ws, x, N, ops.EPI_BF16, bias=bias)
    assert rel_err(yb, x.float() @ Wd.t() + bias) < 1e-2
    # the quantisation itself stays within MXFP4's error of the bf16 weights
    assert rel_err(y, x.float() @ W.float().t()) < 0.15


@pytest.mark.parametrize("var", range(N_VARS))
@pytest.mark.parametrize("M", [1, 5, 40])
@pytest.mark.parametrize("N", [1024, 2 * 16 * 1024 + 16])
def test_w4_every_variant(var, M, N):
    """Every kernel shape on a K that leaves partial chunks: 15 quads, uneven over 4 / 8 waves; the second N gives
    the persistent stream grid several tiles per workgroup (tile edges inside the ring, the last tile alone)."""
    torch.manual_seed(2)
    K = 1920
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, ws, Wd = q4(W)
    ops.set_w4_variant(var)
    y = ops.gemm_w4(wq, ws, x, N, ops.EPI_F32)
    assert rel_err(y, x.float() @ Wd.t()) < 1e-3, var
    # the fused RMSNorm (sums of squares from the first tile of each stream workgroup) and the residual epilogue
    yn = ops.gemm_w4(wq, ws, x, N, ops.EPI_F32, norm=True, eps=1e-6)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-6)
    assert rel_err(yn, xn @ Wd.t()) < 2e-3, var
    r = torch.randn(M, N, device=DEV).bfloat16()
    ref = x.float() @ Wd.t() + r.float()
    ops.gemm_w4(wq, ws, x, N, ops.EPI_RESID, out=r)
    assert rel_err(r, ref) < 1e-2, var


@pytest.mark.parametrize("occ", [1, 3])
def test_w4_stream_grid_occupancy(occ):
    """The persistent grid at other workgroup counts per CU (more tiles per workgroup)."""
    torch.manual_seed(4)
    N, K = 28672, 4096
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(1, K, device=DEV).bfloat16()
    wq, ws, Wd = q4(W)
    ops.set_w4_occupancy(occ)
    try:
        y = ops.gemm_w4(wq, ws, x, N, ops.EPI_F32)
    finally:
        ops.set_w4_occupancy(0)
    assert rel_err(y, x.float() @ Wd.t()) < 1e-3


@pytest.mark.parametrize("ks", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K,epi", [(2048, 16384, "resid"), (1536, 8960, "resid"), (2048, 2048, "f32_norm"),
                                     (4096, 3072, "silu"), (1024, 12288, "f32_norm")])
def test_w4_split_k_stream(ks, N, K, epi):
    """Split-K of the few-row stream kernel (narrow outputs: gemma:2b / qwen2:1.5b down and O, a gate/up, forced k
    ranges 1-4): every split count gives the fp32 result, RMSNorm applied by the last arriver, residual added
    once, and the tickets are left at zero for the next launch."""
    torch.manual_seed(ks + N)
    M = 1
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (3 * torch.randn(M, K, device=DEV)).bfloat16()
    n_out = N // 2 if epi == "silu" else N
    r = torch.randn(M, n_out, device=DEV).bfloat16()
    wq, ws, Wd = q4(W)
    ops.set_w4_split(ks)
    try:
        kq = K // 128
        want_ks = ks if ks > 1 and kq % ks == 0 and kq // ks >= (4 if kq < 24 else 8) else 1
        assert ops.w4_split(N, K, M, ops.EPI_F32) == want_ks
        if epi == "resid":
            ref = x.float() @ Wd.t() + r.float()
            ops.gemm_w4(wq, ws, x, N, ops.EPI_RESID, out=r)
            assert rel_err(r, ref) < 1e-2
        elif epi == "silu":
            h = x.float() @ Wd.t()
            hh = h.view(M, N // 16, 2, 8)  # interleaved 8-row blocks: gate rows, then up rows
            ref = (torch.nn.functional.silu(hh[:, :, 0]) * hh[:, :, 1]).reshape(M, n_out)
            y = ops.gemm_w4(wq, ws, x, N, ops.EPI_SILU)
            assert rel_err(y, ref) < 1e-2
        else:
            y = ops.gemm_w4(wq, ws, x, N, ops.EPI_F32, norm=True, eps=1e-6)
            xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-6)
            assert rel_err(y, xn @ Wd.t()) < 2e-3
        torch.cuda.synchronize()
        assert int(ops._W4_WS[x.device][:16384].count_nonzero()) == 0  # tickets reset
    finally:
        ops.set_w4_split(0)


def test_w4_split_rule_on_the_study_shapes():
    """The default rule splits only outputs of fewer 16-row tiles than CUs into ranges of >= 32 quads (the small
    models' down projections)."""
    n_cu = torch.cuda.get_device_properties(DEV).multi_processor_count
    if n_cu != 256:
        pytest.skip("rule values below are for 256 CUs")
    assert ops.w4_split(2048, 16384, 1, ops.EPI_RESID) == 2   # gemma:2b down: 128 tiles, 128 quads
    assert ops.w4_split(2048, 2048, 1, ops.EPI_RESID) == 1    # gemma:2b O: 16 quads (measured: no gain)
    assert ops.w4_split(1536, 8960, 1, ops.EPI_RESID) == 2    # qwen2:1.5b down: 96 tiles, 70 quads -> 2 x 35
    assert ops.w4_split(1536, 1536, 1, ops.EPI_RESID) == 1    # qwen2:1.5b O: 12 quads (measured slower split)
    assert ops.w4_split(4096, 14336, 1, ops.EPI_RESID) == 1   # llama3.1:8b down: 256 tiles
    assert ops.w4_split(6144, 4096, 1, ops.EPI_QKV_ROPE) == 1  # llama3.1:8b QKV: 384 tiles
    assert ops.w4_split(128256, 4096, 1, ops.EPI_F32) == 1    # LM head


@pytest.mark.parametrize("M", [1, 32])
def test_w4_resid_and_norm(M):
    torch.manual_seed(1)
    N, K = 2048, 4096
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (3 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.2 * torch.randn(K, device=DEV)).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    wq, ws, Wd = q4(W)
    ref = x.float() @ Wd.t() + r.float()
    ops.gemm_w4(wq, ws, x, N, ops.EPI_RESID, out=r)
    assert rel_err(r, ref) < 1e-2
    wq, ws, Wd = q4(fold_gain(W, g))
    y = ops.gemm_w4(wq, ws, x, N, ops.EPI_F32, norm=True, eps=1e-6)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-6)
    assert rel_err(y, xn @ Wd.t()) < 2e-3


@pytest.mark.parametrize("act", ["silu", "gelu"])
@pytest.mark.parametrize("M", [1, 16, 40])
def test_w4_gateup(act, M):
    torch.manual_seed(3)
    F, K = 1536, 1024
    Wg = (torch.randn(F, K, device=DEV) * 0.03).bfloat16()
    Wu = (torch.randn(F, K, device=DEV) * 0.03).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, ws, Wd = q4(interleave_tiles(Wg, Wu, tile=8))
    epi = ops.EPI_SILU if act == "silu" else ops.EPI_GELU
    y = ops.gemm_w4(wq, ws, x, 2 * F, epi)
    gu = (x.float() @ Wd.t()).view(M, F // 8, 2, 8)
    g, u = gu[:, :, 0].reshape(M, F), gu[:, :, 1].reshape(M, F)
    a = torch.nn.functional.silu(g) if act == "silu" else torch.nn.functional.gelu(g, approximate="tanh")
    assert y.shape == (M, F)
    assert rel_err(y, a * u) < 1.5e-2


def _rot(x, c, s_):
    half = x.shape[-1] // 2
    return torch.cat([x[..., :half] * c - x[..., half:] * s_, x[..., half:] * c + x[..., :half] * s_], -1)


@pytest.mark.parametrize("H,Hkv,hd", [(32, 8, 128), (8, 1, 256), (32, 32, 96)])
@pytest.mark.parametrize("M", [1, 40])
@pytest.mark.parametrize("kv8", [False, True])
@pytest.mark.parametrize("var,occ", [(-1, 0), (0, 0), (0, 1)])
def test_w4_qkv_rope_kv_append(H, Hkv, hd, M, kv8, var, occ):
    """The rule's kernel, and the 8-wave stream kernel (its epilogue sums each unit once into LDS, FOLD) with one
    tile per workgroup and, at one workgroup per CU, several (the double-buffered partial slabs reused)."""
    torch.manual_seed(8)
    if var >= 0 and M > 16:
        pytest.skip("the stream kernels take <= 16 rows")
    ops.set_w4_variant(var)
    ops.set_w4_occupancy(occ)
    K, T_max, S = 512, 256, 64
    qkv_dim = (H + 2 * Hkv) * hd
    W = (torch.randn(qkv_dim, K, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(qkv_dim, device=DEV)
    x = torch.randn(M, K, device=DEV).bfloat16()
    per = rope_pair_order(hd).to(DEV)
    perm = torch.cat([h * hd + per for h in range(H + Hkv)] + [torch.arange((H + Hkv) * hd, qkv_dim, device=DEV)])
    cdt = torch.uint8 if kv8 else torch.bfloat16
    kc = torch.zeros(S, Hkv, T_max, hd, device=DEV, dtype=cdt)
    vt = torch.zeros(S, Hkv, hd, T_max, device=DEV, dtype=cdt)
    q = torch.zeros(M, H * hd, device=DEV).bfloat16()
    slot = torch.randperm(S, device=DEV)[:M].int()
    pos = torch.randint(0, T_max, (M,), device=DEV).int()
    inv = 1.0 / (10000.0 ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(T_max, dtype=torch.float64)[:, None] * inv[None]
    cos_t, sin_t = ang.cos().float().to(DEV), ang.sin().float().to(DEV)
    c, s = quantize_mxfp4(W)
    Wd = dequantize_mxfp4(c, s)
    # block quantisation along K commutes with the row permutation
    wq, ws = pack_mxfp4(c[perm].contiguous(), s[perm].contiguous())
    ops.gemm_w4(wq, ws, x, qkv_dim, ops.EPI_QKV_ROPE, bias=bias[perm], out=q,
                rope=dict(kc=kc, vtc=vt, slot=slot, pos=pos, cos_t=cos_t, sin_t=sin_t, H=H, Hkv=Hkv, hd=hd))
    ref = (x.float() @ Wd.t() + bias).bfloat16().float()
    if kv8:
        kc, vt = kc.view(torch.float8_e4m3fn).float(), vt.view(torch.float8_e4m3fn).float()
    kn, vn = ops.unpack_kcache(kc), ops.unpack_vcache(vt)
    tol = 8e-2 if kv8 else 1e-2
    for m in range(M):
        p, sl = int(pos[m]), int(slot[m])
        cc, ss = cos_t[p], sin_t[p]
        assert rel_err(q[m].view(H, hd), _rot(ref[m, : H * hd].view(H, hd), cc, ss)) < 1e-2
        assert rel_err(kn[sl, :, p], _rot(ref[m, H * hd:(H + Hkv) * hd].view(Hkv, hd), cc, ss)) < tol
        assert rel_err(vn[sl, :, p], ref[m, (H + Hkv) * hd:].view(Hkv, hd)) < tol
    assert int((kn != 0).any(-1).sum()) == M * Hkv and int((vn != 0).any(-1).sum()) == M * Hkv
    ops.set_w4_occupancy(0)


@pytest.mark.parametrize("M,K", [(10, 1536), (16, 1536), (12, 2048), (6, 4096), (1, 1536)])
def test_w4_qkv_rope_rule_between_the_staging_sizes(M, K):
    """Rows x K between the 4-wave stream kernel's 28 KiB activation copy and the 8-wave one's 48 KiB (qwen2:1.5b's
    prefill chunks of 10-16 rows, llama3.1:8b's continuous batches of 4-6): the fused QKV epilogue has no 8-wave
    instance, so the rule takes the tile kernel (a round-6 regression ran these on the 4-wave kernel with a partial
    activation copy)."""
    torch.manual_seed(90 + M)
    H, Hkv, hd, T_max, S = 12, 2, 128, 64, 32
    qkv_dim = (H + 2 * Hkv) * hd
    W = (torch.randn(qkv_dim, K, device=DEV) * 0.03).bfloat16()
    bias = torch.randn(qkv_dim, device=DEV)
    x = torch.randn(M, K, device=DEV).bfloat16()
    per = rope_pair_order(hd).to(DEV)
    perm = torch.cat([h * hd + per for h in range(H + Hkv)] + [torch.arange((H + Hkv) * hd, qkv_dim, device=DEV)])
    c, s = quantize_mxfp4(W)
    wq, ws = pack_mxfp4(c[perm].contiguous(), s[perm].contiguous())
    inv = 1.0 / (10000.0 ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(T_max, dtype=torch.float64)[:, None] * inv[None]
    cos_t, sin_t = ang.cos().float().to(DEV), ang.sin().float().to(DEV)
    kc = torch.zeros(S, Hkv, T_max, hd, device=DEV).bfloat16()
    vt = torch.zeros(S, Hkv, hd, T_max, device=DEV).bfloat16()
    q = torch.zeros(M, H * hd, device=DEV).bfloat16()
    slot = torch.randperm(S, device=DEV)[:M].int()
    pos = torch.randint(0, T_max, (M,), device=DEV).int()
    ops.gemm_w4(wq, ws, x, qkv_dim, ops.EPI_QKV_ROPE, bias=bias[perm], out=q,
                rope=dict(kc=kc, vtc=vt, slot=slot, pos=pos, cos_t=cos_t, sin_t=sin_t, H=H, Hkv=Hkv, hd=hd))
    ref = (x.float() @ dequantize_mxfp4(c, s).t() + bias).bfloat16().float()
    kn, vn = ops.unpack_kcache(kc), ops.unpack_vcache(vt)
    for m in range(M):
        p, sl = int(pos[m]), int(slot[m])
        assert rel_err(q[m].view(H, hd), _rot(ref[m, : H * hd].view(H, hd), cos_t[p], sin_t[p])) < 1e-2, m
        assert rel_err(kn[sl, :, p], _rot(ref[m, H * hd:(H + Hkv) * hd].view(Hkv, hd), cos_t[p], sin_t[p])) < 1e-2
        assert rel_err(vn[sl, :, p], ref[m, (H + Hkv) * hd:].view(Hkv, hd)) < 1e-2


FP4_TINY = sorted(n for n, c in TINY.items() if not (c.d_model % 128 or c.q_dim % 128 or c.ffn % 128))


@pytest.mark.parametrize("name", FP4_TINY)
def test_fp4_engine_logits_match_oracle(name):
    """Prompts longer than one 64-row prefill chunk; oracle = the same model on the dequantised weights."""
    eng = DecodeEngine(name, device="cuda", max_batch=4, max_context=512, keep_natural=True, seed=3,
                       weight_dtype="fp4")
    assert eng.prefill_chunk == 64
    prompts = ["In 500 words, please give me information about Elizabeth II " * 3, "hi", "abc def ghi"]
    got = eng.last_logits(prompts)
    ref = ReferenceModel(mxfp4_roundtrip_weights(eng.weights))
    for i, p in enumerate(prompts):
        want = ref.forward(torch.tensor([eng.encode(p)], device="cuda"))[0, -1]
        cos = torch.nn.functional.cosine_similarity(got[i].float(), want.float(), dim=0)
        assert cos > 0.995, (name, i, float(cos))
    eng.close()


def test_fp4_engine_generate_graph_equals_eager():
    eng = DecodeEngine("tiny-llama3.1:8b", device="cuda", max_batch=8, max_context=256, seed=5, steps_per_graph=4,
                       weight_dtype="fp4")
    opts = [dict(temperature=0.8, seed=11 + i, eos_id=-1) for i in range(3)]
    prompts = ["In 100 words, please give me information about India", "hi", "abc"]
    a = eng.generate(prompts, 10, opts, use_graph=True)
    b = eng.generate(prompts, 10, opts, use_graph=False)
    assert [r.tokens for r in a] == [r.tokens for r in b]
    assert all(r.eval_count == 10 for r in a)
    eng.close()
