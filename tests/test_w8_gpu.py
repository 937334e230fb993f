"""fp8-weight (W8A16) kernels of ``csrc/gemm_w8.hip`` against a plain PyTorch fp32 reference computed on
the dequantised weights (q * scale), and the ``weight_dtype="fp8"`` engine against the torch oracle on the
same dequantised weights (``fp8_roundtrip_weights``)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.engine import DecodeEngine  # noqa: E402
from cain_amd.models import TINY  # noqa: E402
from cain_amd.models.reference import ReferenceModel  # noqa: E402
from cain_amd.models.weights import (dequantize_fp8_rows, fold_gain, fp8_roundtrip_weights,  # noqa: E402
                                     interleave_tiles, pack_mfma_a_fp8, quantize_fp8_rows, rope_pair_order)

DEV = torch.device("cuda")


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def q8(w):
    q, s = quantize_fp8_rows(w)
    return pack_mfma_a_fp8(q), s, dequantize_fp8_rows(q, s)


@pytest.mark.parametrize("M", [1, 7, 16, 17, 64])
@pytest.mark.parametrize("N,K", [(512, 256), (6144, 4096), (1024, 14336), (32064, 3072)])
def test_w8_gemm_f32_and_bias(M, N, K):
    torch.manual_seed(0)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, s, Wd = q8(W)
    y = ops.gemm_w8(wq, s, x, N, ops.EPI_F32)
    assert y.dtype == torch.float32
    assert rel_err(y, x.float() @ Wd.t()) < 1e-3
    bias = torch.randn(N, device=DEV)
    yb = ops.gemm_w8(wq, s, x, N, ops.EPI_BF16, bias=bias)
    assert rel_err(yb, x.float() @ Wd.t() + bias) < 1e-2
    # the quantisation itself stays close to the bf16 weights
    assert rel_err(y, x.float() @ W.float().t()) < 5e-2


@pytest.mark.parametrize("M", [1, 32])
def test_w8_resid_and_norm(M):
    torch.manual_seed(1)
    N, K = 2048, 4096
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = (3 * torch.randn(M, K, device=DEV)).bfloat16()
    g = (1 + 0.2 * torch.randn(K, device=DEV)).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    wq, s, Wd = q8(W)
    ref = x.float() @ Wd.t() + r.float()
    ops.gemm_w8(wq, s, x, N, ops.EPI_RESID, out=r)
    assert rel_err(r, ref) < 1e-2
    wq, s, Wd = q8(fold_gain(W, g))
    y = ops.gemm_w8(wq, s, x, N, ops.EPI_F32, norm=True, eps=1e-6)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-6)
    assert rel_err(y, xn @ Wd.t()) < 2e-3


@pytest.mark.parametrize("act", ["silu", "gelu"])
@pytest.mark.parametrize("M", [1, 16, 40])
def test_w8_gateup(act, M):
    torch.manual_seed(3)
    F, K = 1536, 1024
    Wg = (torch.randn(F, K, device=DEV) * 0.03).bfloat16()
    Wu = (torch.randn(F, K, device=DEV) * 0.03).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, s, Wd = q8(interleave_tiles(Wg, Wu, tile=8))
    epi = ops.EPI_SILU if act == "silu" else ops.EPI_GELU
    y = ops.gemm_w8(wq, s, x, 2 * F, epi)
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
def test_w8_qkv_rope_kv_append(H, Hkv, hd, M):
    torch.manual_seed(8)
    K, T_max, S = 512, 256, 64
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
    inv = 1.0 / (10000.0 ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(T_max, dtype=torch.float64)[:, None] * inv[None]
    cos_t, sin_t = ang.cos().float().to(DEV), ang.sin().float().to(DEV)
    qw, s = quantize_fp8_rows(W)
    Wd = dequantize_fp8_rows(qw, s)
    # per-row quantisation commutes with the row permutation
    ops.gemm_w8(pack_mfma_a_fp8(qw[perm]), s[perm].contiguous(), x, qkv_dim, ops.EPI_QKV_ROPE, bias=bias[perm],
                out=q, rope=dict(kc=kc, vtc=vt, slot=slot, pos=pos, cos_t=cos_t, sin_t=sin_t, H=H, Hkv=Hkv, hd=hd))
    ref = (x.float() @ Wd.t() + bias).bfloat16().float()
    kn, vn = ops.unpack_kcache(kc), ops.unpack_vcache(vt)
    for m in range(M):
        p, sl = int(pos[m]), int(slot[m])
        c, s_ = cos_t[p], sin_t[p]
        assert rel_err(q[m].view(H, hd), _rot(ref[m, : H * hd].view(H, hd), c, s_)) < 1e-2
        assert rel_err(kn[sl, :, p], _rot(ref[m, H * hd:(H + Hkv) * hd].view(Hkv, hd), c, s_)) < 1e-2
        assert rel_err(vn[sl, :, p], ref[m, (H + Hkv) * hd:].view(Hkv, hd)) < 1e-2
    assert int((kn != 0).any(-1).sum()) == M * Hkv and int((vn != 0).any(-1).sum()) == M * Hkv


@pytest.mark.parametrize("name", sorted(TINY))
def test_fp8_engine_logits_match_oracle(name):
    """Prompts longer than one 64-row prefill chunk; oracle = the same model on dequantised weights."""
    eng = DecodeEngine(name, device="cuda", max_batch=4, max_context=512, keep_natural=True, seed=3,
                       weight_dtype="fp8")
    assert eng.prefill_chunk == 64
    prompts = ["In 500 words, please give me information about Elizabeth II " * 3, "hi", "abc def ghi"]
    got = eng.last_logits(prompts)
    ref = ReferenceModel(fp8_roundtrip_weights(eng.weights))
    for i, p in enumerate(prompts):
        want = ref.forward(torch.tensor([eng.encode(p)], device="cuda"))[0, -1]
        cos = torch.nn.functional.cosine_similarity(got[i].float(), want.float(), dim=0)
        assert cos > 0.995, (name, i, float(cos))
    eng.close()


def test_fp8_engine_generate_graph_equals_eager():
    eng = DecodeEngine("tiny-llama3.1:8b", device="cuda", max_batch=8, max_context=256, seed=5, steps_per_graph=4,
                       weight_dtype="fp8")
    opts = [dict(temperature=0.8, seed=11 + i, eos_id=-1) for i in range(3)]
    prompts = ["In 100 words, please give me information about India", "hi", "abc"]
    a = eng.generate(prompts, 10, opts, use_graph=True)
    b = eng.generate(prompts, 10, opts, use_graph=False)
    assert [r.tokens for r in a] == [r.tokens for r in b]
    assert all(r.eval_count == 10 for r in a)
    eng.close()
