"""GGUF Q4_0 / Q4_K weight kernels of ``csrc/gemm_q4.hip`` against a plain PyTorch fp32 reference on the blocks'
values as llama.cpp decodes them (``gguf.py``'s decoders: the fp32 dequantised oracle), every epilogue, the fused
RMSNorm with and without a separate gain, multi-launch row counts, and the ``weight_dtype="q4_0" / "q4_k"`` engine
against the torch oracle on the same dequantised weights."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.engine import DecodeEngine  # noqa: E402
from cain_amd.models import TINY  # noqa: E402
from cain_amd.models.q4 import dequantize_q4, pack_q4, q4_fields, quantize_q4  # noqa: E402
from cain_amd.models.reference import ReferenceModel  # noqa: E402
from cain_amd.models.weights import interleave_tiles, roundtrip_weights, rope_pair_order  # noqa: E402

DEV = torch.device("cuda")


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def q4(w, fmt, gain=None):
    n, k = w.shape
    b = quantize_q4(w, fmt)
    wq, sb = pack_q4(q4_fields(b, fmt, n, k), fmt, gain)
    return wq, sb, dequantize_q4(b, fmt, n, k)


def _normed(x, eps=1e-6):
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)


@pytest.mark.parametrize("fmt", [0, 1])
def test_code_and_scale_semantics(fmt):
    """Unit activation rows pick single weights out: the kernel's codes, block scales and offsets equal the
    decoders' values element by element (up to fp32 rounding of s (128 + q) - (128 s + o))."""
    torch.manual_seed(fmt)
    N, K = 32, 512
    wq, sb, Wd = q4(torch.randn(N, K, device=DEV) * 0.05, fmt)
    eye = torch.eye(K, device=DEV).bfloat16()
    for m0 in range(0, K, 16):
        y = ops.gemm_q4(fmt, wq, sb, eye[m0:m0 + 16].contiguous(), N, ops.EPI_F32)
        assert torch.allclose(y, Wd[:, m0:m0 + 16].t(), rtol=1e-5, atol=1e-6), m0


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("M", [1, 3, 7, 16, 20])
@pytest.mark.parametrize("N,K", [(512, 256), (6144, 4096), (1024, 14336), (2048, 8960), (4096, 1536),
                                 (1024, 24576)])
def test_q4_f32_matches_reference(fmt, M, N, K):
    torch.manual_seed(M + K)
    W = torch.randn(N, K, device=DEV) * 0.02
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, sb, Wd = q4(W, fmt)
    y = ops.gemm_q4(fmt, wq, sb, x, N, ops.EPI_F32)
    assert rel_err(y, x.float() @ Wd.t()) < 1e-3
    # and the quantisation stays within its format's error of the original weights
    assert rel_err(y, x.float() @ W.t()) < 0.15


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("M", [1, 5])
def test_q4_bias_residual_norm_and_gain(fmt, M):
    torch.manual_seed(9 + M)
    N, K = 4096, 4096
    W = torch.randn(N, K, device=DEV) * 0.02
    x = (3 * torch.randn(M, K, device=DEV)).bfloat16()
    g = torch.rand(K, device=DEV) + 0.5
    wq, sb, Wd = q4(W, fmt)
    bias = torch.randn(N, device=DEV)
    yb = ops.gemm_q4(fmt, wq, sb, x, N, ops.EPI_BF16, bias=bias)
    assert rel_err(yb, x.float() @ Wd.t() + bias) < 1e-2
    r = torch.randn(M, N, device=DEV).bfloat16()
    ref = x.float() @ Wd.t() + r.float()
    ops.gemm_q4(fmt, wq, sb, x, N, ops.EPI_RESID, out=r)
    assert rel_err(r, ref) < 1e-2
    yn = ops.gemm_q4(fmt, wq, sb, x, N, ops.EPI_F32, norm=True, eps=1e-6)
    assert rel_err(yn, _normed(x) @ Wd.t()) < 1e-3
    # a GGUF file's gain kept separate from its blocks: applied to the activations while staging
    wqg, sbg, _ = q4(W, fmt, gain=g)
    yg = ops.gemm_q4(fmt, wqg, sbg, x, N, ops.EPI_F32, norm=True, eps=1e-6, gain=True)
    assert rel_err(yg, (_normed(x) * g) @ Wd.t()) < 5e-3


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("act", ["silu", "gelu"])
def test_q4_gateup_activation(fmt, act):
    torch.manual_seed(11)
    M, F, K = 2, 2048, 2048
    Wg, Wu = torch.randn(F, K, device=DEV) * 0.02, torch.randn(F, K, device=DEV) * 0.02
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq, sb, Wd = q4(interleave_tiles(Wg, Wu, tile=8), fmt)
    y = ops.gemm_q4(fmt, wq, sb, x, 2 * F, ops.EPI_SILU if act == "silu" else ops.EPI_GELU, norm=True)
    h = _normed(x) @ Wd.t()
    hh = h.view(M, F // 8, 2, 8)
    a = hh[:, :, 0].reshape(M, F)
    u = hh[:, :, 1].reshape(M, F)
    a = torch.nn.functional.silu(a) if act == "silu" else torch.nn.functional.gelu(a, approximate="tanh")
    assert rel_err(y, a * u) < 1.5e-2


def _rot(x, c, s_):
    half = x.shape[-1] // 2
    return torch.cat([x[..., :half] * c - x[..., half:] * s_, x[..., half:] * c + x[..., :half] * s_], -1)


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("H,Hkv,hd", [(32, 8, 128), (8, 1, 256)])
@pytest.mark.parametrize("M", [1, 4])
def test_q4_qkv_rope_kv_append(fmt, H, Hkv, hd, M):
    torch.manual_seed(8)
    K, T_max, S = 1024, 256, 64
    qkv_dim = (H + 2 * Hkv) * hd
    W = torch.randn(qkv_dim, K, device=DEV) * 0.05
    bias = torch.randn(qkv_dim, device=DEV)
    x = torch.randn(M, K, device=DEV).bfloat16()
    per = rope_pair_order(hd).to(DEV)
    perm = torch.cat([h * hd + per for h in range(H + Hkv)] + [torch.arange((H + Hkv) * hd, qkv_dim, device=DEV)])
    kc = torch.zeros(S, Hkv, T_max, hd, device=DEV, dtype=torch.bfloat16)
    vt = torch.zeros(S, Hkv, hd, T_max, device=DEV, dtype=torch.bfloat16)
    q = torch.zeros(M, H * hd, device=DEV).bfloat16()
    slot = torch.randperm(S, device=DEV)[:M].int()
    pos = torch.randint(0, T_max, (M,), device=DEV).int()
    inv = 1.0 / (10000.0 ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(T_max, dtype=torch.float64)[:, None] * inv[None]
    cos_t, sin_t = ang.cos().float().to(DEV), ang.sin().float().to(DEV)
    wq, sb, Wd_perm = q4(W[perm].contiguous(), fmt)  # blocks along K: quantising the permuted rows is the same
    Wd = torch.empty_like(Wd_perm)
    Wd[perm] = Wd_perm
    ops.gemm_q4(fmt, wq, sb, x, qkv_dim, ops.EPI_QKV_ROPE, bias=bias[perm], out=q,
                rope=dict(kc=kc, vtc=vt, slot=slot, pos=pos, cos_t=cos_t, sin_t=sin_t, H=H, Hkv=Hkv, hd=hd))
    ref = (x.float() @ Wd.t() + bias).bfloat16().float()
    kn, vn = ops.unpack_kcache(kc), ops.unpack_vcache(vt)
    for m in range(M):
        p, sl = int(pos[m]), int(slot[m])
        cc, ss = cos_t[p], sin_t[p]
        assert rel_err(q[m].view(H, hd), _rot(ref[m, : H * hd].view(H, hd), cc, ss)) < 1e-2
        assert rel_err(kn[sl, :, p], _rot(ref[m, H * hd:(H + Hkv) * hd].view(Hkv, hd), cc, ss)) < 1e-2
        assert rel_err(vn[sl, :, p], ref[m, (H + Hkv) * hd:].view(Hkv, hd)) < 1e-2


Q4_TINY = sorted(n for n, c in TINY.items() if not (c.d_model % 256 or c.q_dim % 256 or c.ffn % 256))


@pytest.mark.parametrize("wd", ["q4_0", "q4_k"])
@pytest.mark.parametrize("name", Q4_TINY)
def test_q4_engine_logits_match_oracle(wd, name):
    """Prompts longer than one prefill chunk; oracle = the same model on gguf.py's dequantised blocks."""
    eng = DecodeEngine(name, device="cuda", max_batch=4, max_context=512, keep_natural=True, seed=3, weight_dtype=wd)
    prompts = ["In 500 words, please give me information about Elizabeth II " * 3, "hi", "abc def ghi"]
    got = eng.last_logits(prompts)
    ref = ReferenceModel(roundtrip_weights(eng.weights, wd))
    for i, p in enumerate(prompts):
        want = ref.forward(torch.tensor([eng.encode(p)], device="cuda"))[0, -1]
        cos = torch.nn.functional.cosine_similarity(got[i].float(), want.float(), dim=0)
        assert cos > 0.995, (wd, name, i, float(cos))
    eng.close()


def test_q4_engine_generate_graph_equals_eager():
    eng = DecodeEngine("tiny-llama3.1:8b", device="cuda", max_batch=4, max_context=256, seed=5, steps_per_graph=4,
                       weight_dtype="q4_k")
    opts = [dict(temperature=0.8, seed=11 + i, eos_id=-1) for i in range(3)]
    prompts = ["In 100 words, please give me information about India", "hi", "abc"]
    a = eng.generate(prompts, 10, opts, use_graph=True)
    b = eng.generate(prompts, 10, opts, use_graph=False)
    assert [r.tokens for r in a] == [r.tokens for r in b]
    eng.close()


@pytest.mark.parametrize("family,arch", [("llama", "llama"), ("gemma", "gemma")])
@pytest.mark.parametrize("ttype,wd", [("Q4_K", "q4_k"), ("Q4_0", "q4_0")])
def test_gguf_file_runs_its_blocks_as_stored(family, arch, ttype, wd, tmp_path):
    """A GGUF file of Q4_K / Q4_0 weights on weight_dtype q4_k / q4_0: the engine packs the file's blocks as stored
    (norm gains applied to the activations, not folded into the values) and its logits match the fp32 oracle of the
    file's decoded weights (transformers-free: gguf.py's decoders)."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).parent))
    from hf_fixtures import make_checkpoint

    from cain_amd.models.gguf import export_gguf, load_gguf
    from cain_amd.models.hf import load_pretrained

    make_checkpoint(family, tmp_path / "hf", scale=4.0)
    _, mw, _ = load_pretrained(tmp_path / "hf", dtype=torch.float32)
    for lw in mw.layers:  # non-unit gains: the separate-gain path must apply them
        lw.attn_norm = lw.attn_norm + 0.3 * torch.rand_like(lw.attn_norm)
        lw.mlp_norm = lw.mlp_norm + 0.3 * torch.rand_like(lw.mlp_norm)
    export_gguf(mw, tmp_path / "m.gguf", arch, tensor_type=ttype)
    eng = DecodeEngine.from_pretrained(str(tmp_path / "m.gguf"), device="cuda", max_batch=2, max_context=256,
                                       weight_dtype=wd)
    assert eng._packed.get("q4_gain") and eng.weights.native["requantized"] == []
    _, mg, _ = load_gguf(tmp_path / "m.gguf", dtype=torch.float32)
    ref = ReferenceModel(mg)
    ids = [[1, 5, 9, 33, 100, 7, 64], [1, 200, 3]]
    got = eng.last_logits(ids)
    for i, p in enumerate(ids):
        want = ref.forward(torch.tensor([p]))[0, -1]
        cos = torch.nn.functional.cosine_similarity(got[i].float().cpu(), want.float(), dim=0)
        assert cos > 0.999, (family, wd, i, float(cos))
    eng.close()
