"""fp8 (e4m3) weight quantisation and the W8A16 fragment packing (CPU; the kernels are in test_w8_gpu.py)."""
import pytest
import torch

from cain_amd.models import TINY
from cain_amd.models.config import get_config
from cain_amd.models.weights import (FP8_MAX, dequantize_fp8_rows, fp8_roundtrip_weights, pack_for_engine,
                                     pack_mfma_a_fp8, quantize_fp8_rows, random_weights, unpack_mfma_a_fp8)


def test_quantize_rows_pow2_scales_and_error():
    torch.manual_seed(0)
    w = (torch.randn(96, 512) * 0.02 * torch.linspace(0.1, 3, 96)[:, None]).bfloat16()
    q, s = quantize_fp8_rows(w)
    assert q.dtype == torch.float8_e4m3fn and s.dtype == torch.float32
    assert torch.equal(torch.exp2(torch.log2(s).round()), s)  # powers of two
    amax = q.float().abs().amax(1)
    assert bool(((amax > FP8_MAX / 2 - 16) & (amax <= FP8_MAX)).all())  # top binade used
    wd = dequantize_fp8_rows(q, s)
    assert torch.equal(wd.bfloat16().float(), wd)  # exact in bf16
    rel = (wd - w.float()).norm(dim=1) / w.float().norm(dim=1)
    assert float(rel.max()) < 0.04


def test_pack_fp8_layout():
    q, _ = quantize_fp8_rows(torch.randn(48, 192))
    p = pack_mfma_a_fp8(q)
    assert p.shape == (3, 3, 64, 16) and p.dtype == torch.uint8
    assert torch.equal(unpack_mfma_a_fp8(p).view(torch.uint8), q.view(torch.uint8))
    qb = q.view(torch.uint8)
    for t, kp, g, r, h, j in [(0, 0, 0, 0, 0, 0), (2, 1, 3, 5, 1, 6), (1, 2, 2, 15, 0, 7)]:
        assert p[t, kp, g * 16 + r, h * 8 + j] == qb[16 * t + r, 64 * kp + 32 * h + 8 * g + j]
    with pytest.raises(ValueError):
        pack_mfma_a_fp8(q[:, :160])


@pytest.mark.parametrize("name", ["tiny-llama3.1:8b", "tiny-gemma:2b", "tiny-qwen2:1.5b"])
def test_pack_for_engine_fp8(name):
    cfg = get_config(name)
    mw = random_weights(cfg, seed=1)
    rt = fp8_roundtrip_weights(mw)
    pk = pack_for_engine(mw, weight_dtype="fp8")
    assert pk["weight_dtype"] == "fp8"
    lp = pk["layers"][0]
    for k, n, kk in [("wqkv", cfg.qkv_dim, cfg.d_model), ("wo", cfg.d_model, cfg.q_dim),
                     ("wgu", 2 * cfg.ffn, cfg.d_model), ("wdown", cfg.d_model, cfg.ffn)]:
        assert lp[k].shape == (n // 16, kk // 64, 64, 16)
        assert lp["s" + k[1:]].shape == (n,)
    # the packed down projection dequantises to the oracle's round-tripped weight
    wd = dequantize_fp8_rows(unpack_mfma_a_fp8(lp["wdown"]), lp["sdown"])
    assert torch.equal(wd.bfloat16(), rt.layers[0].w_down)
    assert pk["lm_head"].shape == (cfg.vocab // 16, cfg.d_model // 64, 64, 16)
    assert pk["lm_head_scale"].shape == (cfg.vocab,)
    with pytest.raises(ValueError):
        pack_for_engine(mw, weight_dtype="int4")


def test_tiny_models_fit_w8_kernel_constraints():
    for name in TINY:
        cfg = get_config(name)
        assert cfg.d_model % 64 == 0 and cfg.q_dim % 64 == 0 and cfg.ffn % 64 == 0


def test_torch_backend_fp8_uses_dequantised_oracle():
    from cain_amd.engine import DecodeEngine
    from cain_amd.models.reference import ReferenceModel

    eng = DecodeEngine("tiny-llama3.1:8b", device="cpu", max_batch=2, max_context=128, seed=2, weight_dtype="fp8")
    assert eng.backend == "torch" and eng.max_batch == 2 and eng.prefill_chunk == 64
    got = eng.last_logits(["hello world"])[0]
    want = ReferenceModel(fp8_roundtrip_weights(eng.weights)).forward(torch.tensor([eng.encode("hello world")]))[0, -1]
    assert torch.allclose(got.float(), want.float())
    bf = ReferenceModel(eng.weights).forward(torch.tensor([eng.encode("hello world")]))[0, -1]
    assert not torch.equal(got.float(), bf.float())  # the fp8 engine is not silently the bf16 model
    with pytest.raises(ValueError):
        DecodeEngine("tiny-llama3.1:8b", device="cpu", weight_dtype="int4")
    big = DecodeEngine("tiny-llama3.1:8b", device="cpu", max_batch=200, max_context=64, weight_dtype="fp8")
    assert big.max_batch == 64
