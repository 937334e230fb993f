"""GGUF 4-bit weights (llama.cpp's Q4_0 and Q4_K) for the native Q4 kernel (``ops/csrc/gemm_q4.hip``).

The reference's models are Ollama pulls whose default builds are Q4_0 / Q4_K_M GGUF files
(/root/reference/README.md:29-30; tags at /root/reference/experiment/RunnerConfig.py:80).  Round 5 dequantised such
files and re-quantised them to MXFP4, a different 4-bit grid.  Here the block VALUES stay exactly as the file stores
them and only their layout changes:

* ``q4_fields``: ggml block bytes -> codes (uint8 0..15 per weight) plus the block scales -- Q4_0: fp16 ``d`` per 32;
  Q4_K: 6-bit ``sc`` / ``m`` per 32 and fp16 ``d`` / ``dmin`` per 256 (decoded as ggml's ``get_scale_min_k4``,
  ``gguf._k_scale_min``);
* ``pack_q4``: the fields -> the kernel's tile layout (gemm_q4.hip header), one byte buffer of scales
  ``[sc: N K / 16][Q4_K (d, dmin): N K / 64][optional fp32 gain: K]``;
* ``quantize_q4_0`` / ``quantize_q4_k``: weights -> ggml block bytes (random-init models in a GGUF format: the
  bench's ``--weights q4_0 / q4_k`` rows), ``dequantize_q4``: bytes -> fp32 (gguf.py's decoders, the oracle).

Q4_K's quantiser is a plain min/max fit (per 32: scale (max - min) / 15, min -min; per 256: d, dmin = the largest
/ 63), not llama.cpp's iterative ``make_qkx2_quants`` search: the kernel runs whatever valid blocks a file holds,
and random weights only need valid blocks of the right layout.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from .gguf import _k_scale_min, dequantize

Q4_FORMATS = {"q4_0": 0, "q4_k": 1}  # gemm_q4.hip Q4F_*
_BLOCK_BYTES = {0: 18, 1: 144}
_BLOCK_ELEMS = {0: 32, 1: 256}
GGML_TYPE = {0: 2, 1: 12}  # ggml type ids of Q4_0 / Q4_K


def _fp16_bytes(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.float16).contiguous().view(torch.uint8).reshape(*x.shape, 2)


def quantize_q4_0(w: torch.Tensor) -> torch.Tensor:
    """ggml Q4_0 blocks of ``w`` [N, K] (K % 32 == 0) as uint8 [N, K / 32, 18] (ggml's quantize_row_q4_0_ref: d =
    the signed value of largest magnitude / -8, q = clamp(floor(x / d + 8.5), 0, 15), low nibbles the first 16)."""
    n, k = w.shape
    x = w.float().reshape(n, k // 32, 32)
    idx = x.abs().argmax(-1, keepdim=True)
    d = torch.gather(x, -1, idx) / -8.0  # ggml takes the codes with the fp32 d, then stores d as fp16
    inv = torch.where(d != 0, 1.0 / torch.where(d != 0, d, torch.ones_like(d)), torch.zeros_like(d))
    q = torch.clamp(torch.floor(x * inv + 8.5), 0, 15).to(torch.uint8)
    qs = q[..., :16] | (q[..., 16:] << 4)
    return torch.cat([_fp16_bytes(d[..., 0]), qs], -1).contiguous()


def quantize_q4_k(w: torch.Tensor) -> torch.Tensor:
    """Q4_K blocks of ``w`` [N, K] (K % 256 == 0) as uint8 [N, K / 256, 144]: [d fp16][dmin fp16][12 bytes of 6-bit
    (sc, m) pairs][128 bytes of codes], w = d sc q - dmin m (see the module doc for the fit)."""
    n, k = w.shape
    x = w.float().reshape(n, k // 256, 8, 32)
    mn = torch.clamp(x.amin(-1), max=0.0)                    # [n, sb, 8]
    mx = x.amax(-1)
    scale = torch.clamp(mx - mn, min=0.0) / 15.0
    mins = -mn
    d = scale.amax(-1) / 63.0                                 # [n, sb]
    dmin = mins.amax(-1) / 63.0
    d16, dmin16 = d.to(torch.float16).float(), dmin.to(torch.float16).float()
    safe = lambda v: torch.where(v > 0, v, torch.ones_like(v))  # noqa: E731
    sc = torch.where(d16[..., None] > 0, torch.round(scale / safe(d16)[..., None]), torch.zeros_like(scale))
    m = torch.where(dmin16[..., None] > 0, torch.round(mins / safe(dmin16)[..., None]), torch.zeros_like(mins))
    sc, m = sc.clamp(0, 63), m.clamp(0, 63)
    s = d16[..., None] * sc                                   # effective per-32 scale and offset
    o = dmin16[..., None] * m
    q = torch.where(s[..., None] > 0, torch.round((x + o[..., None]) / safe(s)[..., None]), torch.zeros_like(x))
    q = q.clamp(0, 15).to(torch.uint8)                        # [n, sb, 8, 32]
    sci, mi = sc.to(torch.uint8), m.to(torch.uint8)
    scales = torch.cat([sci[..., :4] | ((sci[..., 4:] >> 4) << 6), mi[..., :4] | ((mi[..., 4:] >> 4) << 6),
                        (sci[..., 4:] & 0x0F) | ((mi[..., 4:] & 0x0F) << 4)], -1)  # inverse of _k_scale_min
    qp = q.reshape(n, k // 256, 4, 2, 32)                     # 4 groups of 64: sub-block 2g low, 2g + 1 high
    qs = (qp[..., 0, :] | (qp[..., 1, :] << 4)).reshape(n, k // 256, 128)
    return torch.cat([_fp16_bytes(d), _fp16_bytes(dmin), scales, qs], -1).contiguous()


def quantize_q4(w: torch.Tensor, fmt: int) -> torch.Tensor:
    return quantize_q4_0(w) if fmt == 0 else quantize_q4_k(w)


def dequantize_q4(blocks: torch.Tensor, fmt: int, n: int, k: int) -> torch.Tensor:
    """fp32 [N, K] values of ggml block bytes (the decoders of ``gguf.py``: the kernel's oracle)."""
    return dequantize(blocks.reshape(-1), GGML_TYPE[fmt], n * k).reshape(n, k)


def q4_fields(blocks: torch.Tensor, fmt: int, n: int, k: int) -> Dict[str, torch.Tensor]:
    """ggml block bytes (any shape holding N K / elems blocks, rows in order) -> codes uint8 [N, K] in 0..15 and the
    scale fields: Q4_0 ``d`` fp16 [N, K / 32]; Q4_K ``sc`` / ``m`` uint8 [N, K / 32], ``d`` / ``dmin`` fp16
    [N, K / 256].  Bit-exact: no value is recomputed."""
    bb, be = _BLOCK_BYTES[fmt], _BLOCK_ELEMS[fmt]
    b = blocks.reshape(n, k // be, bb)
    if fmt == 0:
        qs = b[..., 2:18]
        codes = torch.cat([qs & 15, qs >> 4], -1).reshape(n, k)
        return {"codes": codes.contiguous(), "d": b[..., 0:2].contiguous().view(torch.float16)[..., 0]}
    sc, mn = _k_scale_min(b[..., 4:16].reshape(-1, 12))
    qs = b[..., 16:144].reshape(n, k // 256, 4, 32)
    codes = torch.stack([qs & 15, qs >> 4], 3).reshape(n, k)  # [sb, group, low / high, 32] = element order
    return {"codes": codes.contiguous(), "sc": sc.to(torch.uint8).reshape(n, k // 32),
            "m": mn.to(torch.uint8).reshape(n, k // 32),
            "d": b[..., 0:2].contiguous().view(torch.float16)[..., 0],
            "dmin": b[..., 2:4].contiguous().view(torch.float16)[..., 0]}


def pack_q4(fields: Dict[str, torch.Tensor], fmt: int, gain: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor,
                                                                                                      torch.Tensor]:
    """``q4_fields`` -> (codes uint8 [N / 16, K / 128, 64, 16], scale buffer uint8) in gemm_q4.hip's layout: lane
    l = 16 g + r of quad p holds row 16 t + r, k = 128 p + 32 s + 8 g + j at dword s, byte j & 3, nibble j >> 2; the
    scale buffer is [per (t, p, r): 4 x 2 bytes of block scales][Q4_K: per (t, super-block, r) (d, dmin)][gain]."""
    codes = fields["codes"]
    n, k = codes.shape
    if n % 16 or k % 256:
        raise ValueError(f"pack_q4 needs N % 16 == 0 and K % 256 == 0, got {tuple(codes.shape)}")
    nt, kq = n // 16, k // 128
    t = codes.reshape(nt, 16, kq, 4, 4, 2, 4)              # [t, r, p, s, g, h, b]
    t = t.permute(0, 2, 4, 1, 3, 6, 5)                     # [t, p, g, r, s, b, h]
    wq = (t[..., 0] | (t[..., 1] << 4)).contiguous().reshape(nt, kq, 64, 16)

    def tiles(x16: torch.Tensor) -> torch.Tensor:          # [N, K / 32] 16-bit -> [t, p, r, 4 blocks] bytes
        return x16.reshape(nt, 16, kq, 4).permute(0, 2, 1, 3).contiguous().view(torch.uint8).reshape(-1)

    if fmt == 0:
        parts = [tiles(fields["d"].contiguous().view(torch.int16))]
    else:
        scm = fields["sc"].to(torch.int16) | (fields["m"].to(torch.int16) << 8)
        dd = torch.stack([fields["d"], fields["dmin"]], -1).contiguous().view(torch.int32)[..., 0]  # [N, K / 256]
        parts = [tiles(scm), dd.reshape(nt, 16, k // 256).permute(0, 2, 1).contiguous().view(torch.uint8).reshape(-1)]
    if gain is not None:
        parts.append(gain.float().contiguous().view(torch.uint8).reshape(-1))
    return wq, torch.cat(parts).contiguous()


def quant_pack_q4(w: torch.Tensor, fmt: int, gain: Optional[torch.Tensor] = None):
    """Quantise ``w`` [N, K] to ggml blocks and pack them: (codes, scale buffer)."""
    n, k = w.shape
    return pack_q4(q4_fields(quantize_q4(w, fmt), fmt, n, k), fmt, gain)


def q4_roundtrip(w: torch.Tensor, fmt: int) -> torch.Tensor:
    """The values a Q4 engine multiplies by: dequant(quant(w)), in w's dtype (the torch oracle)."""
    n, k = w.shape
    return dequantize_q4(quantize_q4(w, fmt), fmt, n, k).to(w.dtype)


def gguf_q4_native(g, cfg, fmt: int, device="cpu") -> Dict[str, object]:
    """A GGUF file's GEMM weights as ggml blocks of ``fmt`` (uint8 [N, K / elems, bytes]) in the engine's natural
    row order -- the same row operations as ``gguf.load_gguf_weights`` (Llama q / k un-permuted, q / k / v
    concatenated, Phi-3's fused gate/up split), applied to whole rows of blocks, so no value changes.  Tensors the
    file stores in another type (a Q4_K_M file's Q6_K tensors, an F16 output head) are quantised to ``fmt`` from
    their decoded values and listed under ``requantized``.  Result: {"fmt", "layers": [{wqkv, wo, w_gate, w_up,
    w_down}], "lm_head", "requantized"}, attached to ``ModelWeights.native`` for ``pack_for_engine``."""
    import numpy as np

    from .gguf import unpermute_qk

    arch = g.metadata["general.architecture"]
    bb, be = _BLOCK_BYTES[fmt], _BLOCK_ELEMS[fmt]
    requant = []

    def blocks(name: str) -> torch.Tensor:
        t = g.tensors[name]
        n, k = t.shape
        if t.type == GGML_TYPE[fmt]:
            return torch.from_numpy(np.array(g.raw(name))).to(device).reshape(n, k // be, bb)
        requant.append(f"{name} ({t.type_name})")
        return quantize_q4(g.tensor(name, device=device, dtype=torch.float32), fmt)

    f = cfg.ffn
    layers = []
    for i in range(cfg.n_layers):
        p = f"blk.{i}."
        if g.has(p + "attn_qkv.weight"):
            qkv = blocks(p + "attn_qkv.weight")
        else:
            q, kk = blocks(p + "attn_q.weight"), blocks(p + "attn_k.weight")
            if arch == "llama":
                q, kk = unpermute_qk(q, cfg.n_heads), unpermute_qk(kk, cfg.n_kv_heads)
            qkv = torch.cat([q, kk, blocks(p + "attn_v.weight")], 0)
        if g.has(p + "ffn_gate.weight"):
            gate, up = blocks(p + "ffn_gate.weight"), blocks(p + "ffn_up.weight")
        else:  # phi3: ffn_up = [gate; up]
            gu = blocks(p + "ffn_up.weight")
            gate, up = gu[:f].contiguous(), gu[f:].contiguous()
        layers.append({"wqkv": qkv.contiguous(), "wo": blocks(p + "attn_output.weight"), "w_gate": gate,
                       "w_up": up, "w_down": blocks(p + "ffn_down.weight")})
    lm = blocks("output.weight") if g.has("output.weight") else blocks("token_embd.weight")
    return {"fmt": fmt, "layers": layers, "lm_head": lm, "requantized": requant}


def pack_native(blocks: torch.Tensor, fmt: int, gain: Optional[torch.Tensor] = None,
                rows: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Pack ggml blocks [N, K / elems, bytes] (rows reordered by ``rows`` first) for the kernel, the RMSNorm gain
    appended unfolded (a file's values stay exact)."""
    n = blocks.shape[0]
    k = blocks.shape[1] * _BLOCK_ELEMS[fmt]
    b = blocks if rows is None else blocks[rows]
    return pack_q4(q4_fields(b.contiguous(), fmt, n, k), fmt, gain)
