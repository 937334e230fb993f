"""MXFP4 (e2m1 + e8m0 block-32) weight quantisation and the W4A16 fragment packing (CPU; the kernels are in
test_w4_gpu.py)."""
import pytest
import torch

from cain_amd.models import TINY
from cain_amd.models.config import MODELS, get_config
from cain_amd.models.weights import (E2M1_VALUES, dequantize_mxfp4, mxfp4_roundtrip_weights, pack_for_engine,
                                     pack_mxfp4, quantize_mxfp4, random_weights, unpack_mxfp4)


def test_quantize_mxfp4_grid_scales_and_error():
    torch.manual_seed(0)
    w = (torch.randn(96, 512) * 0.02 * torch.linspace(0.1, 3, 96)[:, None]).bfloat16()
    w[7, 64:96] = 0  # an all-zero block
    c, s = quantize_mxfp4(w)
    assert c.dtype == torch.uint8 and s.dtype == torch.uint8 and c.shape == (96, 512) and s.shape == (96, 16)
    assert int(c.max()) <= 15 and int(s.min()) >= 1  # e >= -126: a normal fp32 scale
    d = dequantize_mxfp4(c, s)
    assert torch.equal(d.bfloat16().float(), d)  # exact in bf16
    assert float(d[7, 64:96].abs().max()) == 0.0
    # every element is an e2m1 value times its block's power of two
    mag = (d.reshape(96, 16, 32).abs() / torch.exp2(s.float() - 127)[..., None])
    assert bool(torch.isin(mag, torch.tensor(E2M1_VALUES)).all())
    rel = (d - w.float()).norm(dim=1) / w.float().norm(dim=1).clamp_min(1e-12)
    assert float(rel.mean()) < 0.13  # Gaussian blocks: ~11 % (the MSE-best of the two candidate scales)
    # the per-block choice never does worse than the no-saturation scale alone
    e0 = torch.ceil(torch.log2(w.float().reshape(96, 16, 32).abs().amax(2) / 6)).clamp(-126, 127)
    assert bool(((s.float() - 127 == e0) | (s.float() - 127 == e0 - 1) | (e0 < -126)).all())


def test_pack_mxfp4_layout_roundtrip():
    c, s = quantize_mxfp4(torch.randn(48, 384))
    wq, ws = pack_mxfp4(c, s)
    assert wq.shape == (3, 3, 64, 16) and ws.shape == (3, 3, 64) and wq.dtype == ws.dtype == torch.uint8
    c2, s2 = unpack_mxfp4(wq, ws)
    assert torch.equal(c2, c) and torch.equal(s2, s)
    for t, p, g, r, sl, b, h in [(0, 0, 0, 0, 0, 0, 0), (2, 1, 3, 5, 2, 1, 1), (1, 2, 2, 15, 3, 3, 0)]:
        row, k = 16 * t + r, 128 * p + 32 * g + 8 * sl + 2 * b + h
        assert (int(wq[t, p, 16 * g + r, 4 * sl + b]) >> (4 * h)) & 15 == int(c[row, k])
        assert int(ws[t, p, 16 * g + r]) == int(s[row, 4 * p + g])  # one scale block per lane
    with pytest.raises(ValueError):
        pack_mxfp4(c[:, :320], s[:, :10])


@pytest.mark.parametrize("name", ["tiny-llama3.1:8b", "tiny-gemma:2b", "tiny-qwen2:1.5b"])
def test_pack_for_engine_fp4(name):
    cfg = get_config(name)
    mw = random_weights(cfg, seed=1)
    rt = mxfp4_roundtrip_weights(mw)
    pk = pack_for_engine(mw, weight_dtype="fp4")
    assert pk["weight_dtype"] == "fp4"
    lp = pk["layers"][0]
    for k, n, kk in [("wqkv", cfg.qkv_dim, cfg.d_model), ("wo", cfg.d_model, cfg.q_dim),
                     ("wgu", 2 * cfg.ffn, cfg.d_model), ("wdown", cfg.d_model, cfg.ffn)]:
        assert lp[k].shape == (n // 16, kk // 128, 64, 16)
        assert lp["s" + k[1:]].shape == (n // 16, kk // 128, 64)
    wd = dequantize_mxfp4(*unpack_mxfp4(lp["wdown"], lp["sdown"]))
    assert torch.equal(wd.bfloat16(), rt.layers[0].w_down)
    assert pk["lm_head"].shape == (cfg.vocab // 16, cfg.d_model // 128, 64, 16)
    assert pk["lm_head_scale"].shape == (cfg.vocab // 16, cfg.d_model // 128, 64)


def test_real_models_fit_w4_kernel_constraints():
    for cfg in MODELS.values():
        assert cfg.d_model % 128 == 0 and cfg.q_dim % 128 == 0 and cfg.ffn % 128 == 0, cfg.name


def test_torch_backend_fp4_uses_dequantised_oracle():
    from cain_amd.engine import DecodeEngine
    from cain_amd.models.reference import ReferenceModel

    eng = DecodeEngine("tiny-llama3.1:8b", device="cpu", max_batch=2, max_context=128, seed=2, weight_dtype="fp4")
    assert eng.backend == "torch"
    got = eng.last_logits(["hello world"])[0]
    want = ReferenceModel(mxfp4_roundtrip_weights(eng.weights)).forward(
        torch.tensor([eng.encode("hello world")]))[0, -1]
    assert torch.allclose(got.float(), want.float())
    big = DecodeEngine("tiny-llama3.1:8b", device="cpu", max_batch=200, max_context=64, weight_dtype="fp4")
    assert big.max_batch == 64
    odd = [n for n, c in TINY.items() if c.d_model % 128 or c.q_dim % 128 or c.ffn % 128]
    for n in odd:
        with pytest.raises(ValueError):
            DecodeEngine(n, device="cpu", weight_dtype="fp4")


def _nonunit_gains(mw, seed=4):
    g = torch.Generator().manual_seed(seed)
    cfg = mw.cfg

    def gain(t):
        v = 1.0 + 0.6 * torch.randn(t.shape, generator=g)  # effective gains spread over ~[-0.8, 2.8]
        return (v - 1.0 if cfg.norm_add_one else v).to(t.dtype)

    for lw in mw.layers:
        lw.attn_norm, lw.mlp_norm = gain(lw.attn_norm), gain(lw.mlp_norm)
    mw.final_norm = gain(mw.final_norm)
    return mw


@pytest.mark.parametrize("name", ["tiny-llama3.1:8b", "tiny-gemma:2b"])
def test_fp4_oracle_quantises_the_gain_folded_weights(name):
    """the oracle's MXFP4 block scales are taken over W diag(g), exactly the matrix the engine packs, so
    the oracle matches the packed bytes for NON-unit norm gains too (it used to quantise W and keep g separate)."""
    from cain_amd.models.weights import effective_gain, fold_gain, qkv_row_permutation

    cfg = get_config(name)
    mw = _nonunit_gains(random_weights(cfg, seed=1))
    rt = mxfp4_roundtrip_weights(mw)
    assert torch.equal(effective_gain(cfg, rt.layers[0].attn_norm).float(), torch.ones(cfg.d_model))
    pk = pack_for_engine(mw, weight_dtype="fp4")
    lp = pk["layers"][0]
    perm = qkv_row_permutation(cfg)
    wqkv = dequantize_mxfp4(*unpack_mxfp4(lp["wqkv"], lp["sqkv"])).bfloat16()
    assert torch.equal(wqkv, rt.layers[0].wqkv[perm])
    wgu = dequantize_mxfp4(*unpack_mxfp4(lp["wgu"], lp["sgu"])).bfloat16()
    f = cfg.ffn
    assert torch.equal(wgu.reshape(f // 8, 2, 8, -1)[:, 0].reshape(f, -1), rt.layers[0].w_gate)
    assert torch.equal(wgu.reshape(f // 8, 2, 8, -1)[:, 1].reshape(f, -1), rt.layers[0].w_up)
    lm = dequantize_mxfp4(*unpack_mxfp4(pk["lm_head"], pk["lm_head_scale"])).bfloat16()
    assert torch.equal(lm, rt.lm_head)
    # and the old oracle (quantise W, keep g) is a different matrix once the gains are not 1
    ga = effective_gain(cfg, mw.layers[0].attn_norm)
    old = fold_gain(dequantize_mxfp4(*quantize_mxfp4(mw.layers[0].wqkv)).bfloat16(), ga)
    assert not torch.equal(old, rt.layers[0].wqkv)


def test_fp8_oracle_quantises_the_gain_folded_weights():
    from cain_amd.models.weights import dequantize_fp8_rows, fp8_roundtrip_weights, unpack_mfma_a_fp8

    cfg = get_config("tiny-llama3.1:8b")
    mw = _nonunit_gains(random_weights(cfg, seed=2))
    rt = fp8_roundtrip_weights(mw)
    pk = pack_for_engine(mw, weight_dtype="fp8")
    lp = pk["layers"][0]
    f = cfg.ffn
    wgu = dequantize_fp8_rows(unpack_mfma_a_fp8(lp["wgu"]), lp["sgu"]).bfloat16()
    assert torch.equal(wgu.reshape(f // 8, 2, 8, -1)[:, 0].reshape(f, -1), rt.layers[0].w_gate)
