"""GGUF Q4_0 / Q4_K blocks for the native Q4 kernel (models/q4.py, ops/csrc/gemm_q4.hip), CPU checks: the block
quantisers write ggml's layouts (Q4_0 byte-identical to the numpy reference quantiser), the field extraction is
bit-exact against gguf.py's decoders, and an emulation of the kernel's arithmetic on the PACKED bytes -- its lane
layout, nibble order and scale indexing, T_b = sum x (128 + q) and the (128 s + o) X_b correction -- reproduces the
fp32 product with the dequantised weights."""
import numpy as np
import pytest
import torch

from cain_amd.models import gguf
from cain_amd.models.q4 import (dequantize_q4, pack_q4, q4_fields, quant_pack_q4, quantize_q4, quantize_q4_0,
                                quantize_q4_k)


def test_q4_0_matches_the_reference_quantiser():
    torch.manual_seed(0)
    w = torch.randn(32, 512) * 0.02
    ours = quantize_q4_0(w).reshape(-1).numpy()
    theirs = gguf.quantize_q4_0(w.numpy())
    assert np.array_equal(ours, theirs)


@pytest.mark.parametrize("fmt", [0, 1])
def test_quantisers_round_trip_through_the_gguf_decoders(fmt):
    torch.manual_seed(fmt)
    w = torch.randn(48, 1024) * 0.02
    wd = dequantize_q4(quantize_q4(w, fmt), fmt, 48, 1024)
    rel = float((wd - w).norm() / w.norm())
    assert rel < (0.12 if fmt == 0 else 0.10), rel


@pytest.mark.parametrize("fmt", [0, 1])
def test_fields_are_exact(fmt):
    """codes and scales from q4_fields rebuild the decoders' values exactly (Q4_0: d (q - 8); Q4_K: d sc q - dmin m)."""
    torch.manual_seed(3)
    n, k = 32, 768
    b = quantize_q4(torch.randn(n, k) * 0.05, fmt)
    f = q4_fields(b, fmt, n, k)
    q = f["codes"].float().reshape(n, k // 32, 32)
    if fmt == 0:
        w = f["d"].float()[..., None] * (q - 8)
    else:
        d = f["d"].float().repeat_interleave(8, 1)[..., None]
        dm = f["dmin"].float().repeat_interleave(8, 1)[..., None]
        w = d * f["sc"].float()[..., None] * q - dm * f["m"].float()[..., None]
    assert torch.equal(w.reshape(n, k), dequantize_q4(b, fmt, n, k))


def emulate(wq, sbuf, fmt, x, n, k):
    """The kernel's arithmetic on the packed bytes (gemm_q4.hip step): per 128-k quad p, MFMA s (block 4p + s) and
    lane group g the codes of k = 128p + 32s + 8g + j come from dword s, byte j & 3, nibble j >> 2; T = sum x (128 +
    q); out = sum_b s_b T_b - (128 s_b + o_b) X_b with the scales read at the kernel's offsets."""
    nt, kq = n // 16, k // 128
    m = x.shape[0]
    by = wq.reshape(nt, kq, 4, 16, 16)                     # [t, p, g, r, 16 bytes]
    dw = by.reshape(nt, kq, 4, 16, 4, 4)                   # [t, p, g, r, s, byte]
    lo, hi = dw & 15, dw >> 4
    q = torch.cat([lo, hi], -1).long()                     # j = h * 4 + b
    # codes[t, r, p, s, g, j] -> weight row 16t + r, k = 128p + 32s + 8g + j
    codes = q.permute(0, 3, 1, 4, 2, 5).reshape(n, k)
    sc16 = sbuf[: n * k // 16].view(torch.int16).reshape(nt, kq, 16, 4).permute(0, 2, 1, 3).reshape(n, k // 32)
    if fmt == 0:
        s = sc16.view(torch.float16).float()
        o = 8 * s
    else:
        dd = sbuf[n * k // 16: n * k // 16 + n * k // 64].view(torch.int32).reshape(nt, k // 256, 16)
        dd = dd.permute(0, 2, 1).reshape(n, k // 256)
        d = (dd & 0xFFFF).to(torch.int16).view(torch.float16).float().repeat_interleave(8, 1)
        dmin = ((dd >> 16) & 0xFFFF).to(torch.int16).view(torch.float16).float().repeat_interleave(8, 1)
        s = d * (sc16 & 0xFF).float()
        o = dmin * ((sc16 >> 8) & 0xFF).float()
    xb = x.float().reshape(m, k // 32, 32)
    T = torch.einsum("mbj,nbj->mnb", xb, (128 + codes).float().reshape(n, k // 32, 32))
    X = xb.sum(-1)                                          # [m, b]
    return (T * s[None]).sum(-1) - torch.einsum("nb,mb->mn", 128 * s + o, X)


@pytest.mark.parametrize("fmt", [0, 1])
def test_packed_layout_and_kernel_arithmetic(fmt):
    torch.manual_seed(7 + fmt)
    n, k, m = 64, 1024, 3
    w = torch.randn(n, k) * 0.02
    x = torch.randn(m, k).bfloat16()
    b = quantize_q4(w, fmt)
    wq, sbuf = pack_q4(q4_fields(b, fmt, n, k), fmt)
    assert wq.shape == (n // 16, k // 128, 64, 16)
    assert sbuf.numel() == n * k // 16 + (n * k // 64 if fmt else 0)
    got = emulate(wq, sbuf, fmt, x, n, k)
    ref = x.float() @ dequantize_q4(b, fmt, n, k).t()
    assert float((got - ref).abs().max() / ref.abs().max()) < 1e-5


def test_gain_is_appended_after_the_scales():
    w = torch.randn(32, 512) * 0.02
    g = torch.rand(512) + 0.5
    _, s0 = quant_pack_q4(w, 1)
    _, s1 = quant_pack_q4(w, 1, gain=g)
    assert torch.equal(s1[: s0.numel()], s0)
    assert torch.equal(s1[s0.numel():].view(torch.float32), g)


@pytest.mark.parametrize("wd", ["q4_0", "q4_k"])
def test_cpu_engine_runs_the_q4_oracle(wd):
    """weight_dtype q4_0 / q4_k on the torch backend: the oracle multiplies by the dequantised ggml blocks of the
    gain-folded weights (weights.roundtrip_weights), and generation runs."""
    from cain_amd.engine import DecodeEngine
    from cain_amd.models.q4 import Q4_FORMATS, q4_roundtrip

    eng = DecodeEngine("tiny-llama3.1:8b", device="cpu", max_batch=2, max_context=64, weight_dtype=wd, seed=1)
    r = eng.generate(["hello there"], 4, [dict(temperature=0.0, eos_id=-1)])[0]
    assert r.eval_count == 4
    w = eng.weights.layers[0].wo
    assert torch.equal(eng.ref.mw.layers[0].wo, q4_roundtrip(w, Q4_FORMATS[wd]))


def test_engine_rejects_q4_on_widths_not_a_multiple_of_256():
    from cain_amd.engine import DecodeEngine

    with pytest.raises(ValueError, match="multiples of 256"):
        DecodeEngine("tiny-qwen2:1.5b", device="cpu", max_batch=1, max_context=64, weight_dtype="q4_k")


@pytest.mark.parametrize("family,arch", [("llama", "llama"), ("gemma", "gemma")])
@pytest.mark.parametrize("ttype,fmt", [("Q4_K", 1), ("Q4_0", 0)])
def test_gguf_blocks_are_kept_as_stored(family, arch, ttype, fmt, tmp_path):
    """a GGUF file whose weights are Q4_K / Q4_0 runs its blocks as stored -- gguf_q4_native's
    blocks decode to exactly the values load_gguf_weights decodes (after the same row operations: Llama q / k
    un-permuted, q / k / v concatenated), so nothing is re-quantised."""
    from hf_fixtures import make_checkpoint

    from cain_amd.models.gguf import GGUFFile, export_gguf, load_gguf
    from cain_amd.models.hf import load_pretrained
    from cain_amd.models.q4 import gguf_q4_native

    make_checkpoint(family, tmp_path / "hf", scale=4.0)
    _, mw, _ = load_pretrained(tmp_path / "hf", dtype=torch.float32)
    export_gguf(mw, tmp_path / "m.gguf", arch, tensor_type=ttype)
    cfg, mg, _ = load_gguf(tmp_path / "m.gguf", dtype=torch.float32)
    nat = gguf_q4_native(GGUFFile(tmp_path / "m.gguf"), cfg, fmt)
    assert nat["requantized"] == []

    def dq(b):
        return dequantize_q4(b, fmt, b.shape[0], b.shape[1] * (256 if fmt else 32))

    for lw, nl in zip(mg.layers, nat["layers"]):
        for name in ("wqkv", "wo", "w_gate", "w_up", "w_down"):
            assert torch.equal(dq(nl[name]), getattr(lw, name)), name
    assert torch.equal(dq(nat["lm_head"]), mg.lm_head)
