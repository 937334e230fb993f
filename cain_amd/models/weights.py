"""Random-init weights and their HBM layouts.

There is no network for checkpoints, so weights are seeded random tensors of
each architecture's exact shapes (N(0, 0.02) like HF init; norm gains 1).

Two layouts:

* **natural** — ``nn.Linear`` ``[out, in]`` row-major; consumed by the torch
  oracle (``reference.py``) and by prefill GEMMs on the library path.
* **packed** — the decode engine's MFMA-fragment-major layout
  ``[N/16][K/32][64 lanes][8 bf16]``: the 16-byte A-operand fragment of lane
  ``l`` of ``v_mfma_f32_16x16x32_bf16`` for output rows ``16t..16t+15`` and
  reduction slice ``32s..32s+31`` is element ``(t, s, l)``.  One wave
  load instruction therefore reads 1 KiB of contiguous HBM (8 full lines),
  which is what a weight-streaming GEMV wants (cdna_hip_programming.md §5
  'GEMV / M ≤ 16' row).  Gate/up are interleaved by 8-row blocks so every
  16-row tile holds 8 gate rows and the 8 matching up rows and the GEMM applies
  the activation in its epilogue.  Gemma's ``(1 + w)`` norm gain is folded into the stored gain.  Q/K rows
  are permuted per head (``rope_pair_order``) so every 16-row tile holds 8
  complete RoPE pairs and the QKV GEMM can rotate in its epilogue.
* **packed fp8** (``weight_dtype="fp8"``, the W8A16 decode option) — the same
  row orders, each row quantised to OCP e4m3 with one fp32 scale
  (``quantize_fp8_rows``), bytes laid out ``[N/16][K/64][64 lanes][16]`` for
  ``ops/csrc/gemm_w8.hip`` (``pack_mfma_a_fp8``).  The reference's models are
  4-bit GGUF quantisations served by Ollama; fp8 is the gfx950
  native narrow weight type.
* **packed MXFP4** (``weight_dtype="fp4"``, the reference's 4-bit precision
  class) — e2m1 elements with one e8m0 scale per 32 k of a row
  (``quantize_mxfp4``), bytes laid out ``[N/16][K/128][64 lanes][16]`` plus
  scale bytes ``[N/16][K/128][64]`` for ``ops/csrc/gemm_w4.hip``
  (``pack_mxfp4``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from .config import ModelConfig

INIT_STD = 0.02


def pack_mfma_a(w: torch.Tensor) -> torch.Tensor:
    """[N, K] → [N/16, K/32, 64, 8] (lane = g*16 + r; k = 32s + 8g + j)."""
    n, k = w.shape
    if n % 16 or k % 32:
        raise ValueError(f"pack_mfma_a needs N%16==0 and K%32==0, got {tuple(w.shape)}")
    t = w.reshape(n // 16, 16, k // 32, 4, 8)          # [t, r, s, g, j]
    t = t.permute(0, 2, 3, 1, 4)                        # [t, s, g, r, j]
    return t.contiguous().reshape(n // 16, k // 32, 64, 8)


def unpack_mfma_a(p: torch.Tensor) -> torch.Tensor:
    nt, ns = p.shape[0], p.shape[1]
    t = p.reshape(nt, ns, 4, 16, 8).permute(0, 3, 1, 2, 4)  # [t, r, s, g, j]
    return t.contiguous().reshape(nt * 16, ns * 32)


FP8_MAX = 448.0  # largest finite OCP e4m3 value


def quantize_fp8_rows(w: torch.Tensor):
    """Per-output-row symmetric e4m3 quantisation: (q [N, K] float8_e4m3fn, scale [N] fp32), W ~= q * scale.

    Scales are powers of two (the row's amax lands in e4m3's top binade): relative precision is e4m3's
    either way, and q * scale is then exact in bf16, so ``fp8_roundtrip_weights`` gives the torch oracle
    exactly the weights the fp8 kernels multiply by."""
    wf = w.float()
    amax = wf.abs().amax(dim=1).clamp_min(1e-30)
    scale = torch.exp2(torch.ceil(torch.log2(amax / FP8_MAX)))
    q = (wf / scale[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q, scale.contiguous()


def dequantize_fp8_rows(q: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    return q.float() * scale.float()[:, None]


def pack_mfma_a_fp8(q: torch.Tensor) -> torch.Tensor:
    """e4m3 [N, K] -> uint8 [N/16, K/64, 64, 16]: lane = g*16 + r holds bytes h*8 + j = element
    (16t + r, 64p + 32h + 8g + j) -- the two k-slices of one ``v_mfma_f32_16x16x32_bf16`` A fragment pair."""
    n, k = q.shape
    if n % 16 or k % 64:
        raise ValueError(f"pack_mfma_a_fp8 needs N%16==0 and K%64==0, got {tuple(q.shape)}")
    t = q.view(torch.uint8).reshape(n // 16, 16, k // 64, 2, 4, 8)  # [t, r, p, h, g, j]
    t = t.permute(0, 2, 4, 1, 3, 5)                                   # [t, p, g, r, h, j]
    return t.contiguous().reshape(n // 16, k // 64, 64, 16)


def pack_mfma_a_fp8_k128(q: torch.Tensor) -> torch.Tensor:
    """e4m3 [N, K] -> uint8 [N/16, K/64, 64, 16] for the W8A8 wide kernel (ops/csrc/wgemm8.hip): lane = g*16 + r
    holds bytes j = element (16t + r, 64p + 16g + j); two consecutive 1-KiB blocks (p = 2s, 2s + 1) are the
    32-B A operands of one v_mfma_scale_f32_16x16x128_f8f6f4 over k 128s .. 128s + 127."""
    n, k = q.shape
    if n % 16 or k % 128:
        raise ValueError(f"pack_mfma_a_fp8_k128 needs N%16==0 and K%128==0, got {tuple(q.shape)}")
    t = q.view(torch.uint8).reshape(n // 16, 16, k // 64, 4, 16)    # [t, r, p, g, j]
    return t.permute(0, 2, 3, 1, 4).contiguous().reshape(n // 16, k // 64, 64, 16)


def unpack_mfma_a_fp8(p: torch.Tensor) -> torch.Tensor:
    nt, kp = p.shape[0], p.shape[1]
    t = p.reshape(nt, kp, 4, 16, 2, 8).permute(0, 3, 1, 4, 2, 5)   # [t, r, p, h, g, j]
    return t.contiguous().reshape(nt * 16, kp * 64).view(torch.float8_e4m3fn)


#: e2m1 magnitudes by 3-bit code (OCP MX: sign bit 3, 2 exponent bits, 1 mantissa bit)
E2M1_VALUES = (0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0)
_E2M1_BOUNDS = (0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5.0)  # round-to-nearest decision points between the magnitudes
MX_BLOCK = 32


def quantize_mxfp4(w: torch.Tensor):
    """OCP MXFP4 quantisation along K: (codes uint8 [N, K] in 0..15, e8m0 scale bytes uint8 [N, K/32]).

    Each 32-element block of a row shares a power-of-two scale 2^e, stored biased (e + 127, clamped to e >= -126
    so the decoded scale is a normal fp32).  Per block the scale is the better (smaller squared error) of
    e0 = ceil(log2(amax / 6)) -- the block's largest magnitude lands in (3, 6], nothing saturates -- and e0 - 1,
    which resolves the small elements twice as finely and saturates the largest at 6 (chosen for ~1/3 of Gaussian
    blocks: 11.8 -> 11.1 % relative error).  Elements round to the nearest e2m1 value of w / 2^e."""
    n, k = w.shape
    if k % MX_BLOCK:
        raise ValueError(f"quantize_mxfp4 needs K % {MX_BLOCK} == 0, got {tuple(w.shape)}")
    wf = w.float().reshape(n, k // MX_BLOCK, MX_BLOCK)
    amax = wf.abs().amax(dim=2)
    e0 = torch.ceil(torch.log2(amax / 6.0))
    e0 = torch.where(amax > 0, e0, torch.full_like(e0, -126.0)).clamp(-126, 127)
    bounds = torch.tensor(_E2M1_BOUNDS, device=w.device, dtype=torch.float32)
    vals = torch.tensor(E2M1_VALUES, device=w.device, dtype=torch.float32)

    def rnd(e):
        sc = torch.exp2(e)[..., None]
        y = wf / sc
        mag = torch.bucketize(y.abs().clamp(max=6.0), bounds)
        err = ((vals[mag] * sc - y.abs() * sc) ** 2).sum(dim=2)
        return mag.to(torch.uint8) | ((y < 0).to(torch.uint8) << 3), err

    c0, err0 = rnd(e0)
    e1 = (e0 - 1).clamp(-126, 127)
    c1, err1 = rnd(e1)
    pick = err1 < err0
    codes = torch.where(pick[..., None], c1, c0)
    e = torch.where(pick, e1, e0)
    return codes.reshape(n, k).contiguous(), (e + 127).to(torch.uint8).contiguous()


def dequantize_mxfp4(codes: torch.Tensor, scales: torch.Tensor) -> torch.Tensor:
    """fp32 [N, K] values of ``quantize_mxfp4``'s output (exactly representable in bf16)."""
    n, k = codes.shape
    vals = torch.tensor(E2M1_VALUES, device=codes.device, dtype=torch.float32)
    c = codes.long()
    v = vals[c & 7] * torch.where((c & 8) != 0, -1.0, 1.0)
    sc = torch.exp2(scales.float() - 127.0)
    return (v.reshape(n, k // MX_BLOCK, MX_BLOCK) * sc[..., None]).reshape(n, k)


def pack_mxfp4(codes: torch.Tensor, scales: torch.Tensor):
    """MXFP4 codes [N, K] + e8m0 scales [N, K/32] -> the few-row kernel's layout (ops/csrc/gemm_w4.hip):
    (wq uint8 [N/16, K/128, 64, 16], ws uint8 [N/16, K/128, 64]).  Lane l = 16g + r of quad p holds row 16t + r,
    k = 128p + 32g + 8s + 2b + h at byte 4s + b, nibble h (0 low) -- one whole scale block per lane -- and
    ws[t, p, l] is that block's scale byte."""
    n, k = codes.shape
    if n % 16 or k % 128:
        raise ValueError(f"pack_mxfp4 needs N%16==0 and K%128==0, got {tuple(codes.shape)}")
    t = codes.reshape(n // 16, 16, k // 128, 4, 4, 4, 2)              # [t, r, p, g, s, b, h]
    t = t.permute(0, 2, 3, 1, 4, 5, 6)                                  # [t, p, g, r, s, b, h]
    byte = t[..., 0] | (t[..., 1] << 4)
    wq = byte.contiguous().reshape(n // 16, k // 128, 64, 16)
    s = scales.reshape(n // 16, 16, k // 128, 4).permute(0, 2, 3, 1)  # [t, p, g, r]
    return wq, s.contiguous().reshape(n // 16, k // 128, 64)


def unpack_mxfp4(wq: torch.Tensor, ws: torch.Tensor):
    """Inverse of ``pack_mxfp4``: (codes [N, K], scales [N, K/32])."""
    nt, kq = wq.shape[0], wq.shape[1]
    lo, hi = wq & 15, wq >> 4
    t = torch.stack([lo, hi], dim=-1).reshape(nt, kq, 4, 16, 4, 4, 2)  # [t, p, g, r, s, b, h]
    codes = t.permute(0, 3, 1, 2, 4, 5, 6).contiguous().reshape(nt * 16, kq * 128)
    s = ws.reshape(nt, kq, 4, 16).permute(0, 3, 1, 2).contiguous().reshape(nt * 16, kq * 4)
    return codes, s


def rope_pair_order(hd: int) -> torch.Tensor:
    """Row order inside one q/k head for the fused QKV-RoPE epilogue: 16-row tile i holds
    rotation pairs j = 8i..8i+7 as rows [j..j+8) followed by [j+hd/2 .. j+hd/2+8)."""
    half = hd // 2
    idx = []
    for i in range(hd // 16):
        idx += list(range(8 * i, 8 * i + 8)) + list(range(half + 8 * i, half + 8 * i + 8))
    return torch.tensor(idx, dtype=torch.long)


def qkv_row_permutation(cfg: ModelConfig) -> torch.Tensor:
    """Permutation of the fused QKV rows (q heads, k heads permuted per head; v unchanged)."""
    hd = cfg.head_dim
    per_head = rope_pair_order(hd)
    parts = [h * hd + per_head for h in range(cfg.n_heads + cfg.n_kv_heads)]
    parts.append(torch.arange((cfg.n_heads + cfg.n_kv_heads) * hd, cfg.qkv_dim))
    return torch.cat(parts)


def interleave_tiles(a: torch.Tensor, b: torch.Tensor, tile: int = 16) -> torch.Tensor:
    """Rows of a and b interleaved by ``tile``-row blocks: [a0, b0, a1, b1, ...]."""
    n, k = a.shape
    return torch.stack([a.reshape(n // tile, tile, k), b.reshape(n // tile, tile, k)], dim=1).reshape(2 * n, k)


@dataclass
class LayerWeights:
    attn_norm: torch.Tensor
    wqkv: torch.Tensor
    bqkv: Optional[torch.Tensor]
    wo: torch.Tensor
    mlp_norm: torch.Tensor
    w_gate: torch.Tensor
    w_up: torch.Tensor
    w_down: torch.Tensor


@dataclass
class ModelWeights:
    cfg: ModelConfig
    embed: torch.Tensor                 # [V, d] natural
    final_norm: torch.Tensor
    lm_head: torch.Tensor               # [V, d] (aliases embed when tied)
    layers: List[LayerWeights]
    packed: Dict[str, object] = field(default_factory=dict)
    # weights kept in a file's quantised form (models/q4.py gguf_q4_native: GGUF Q4_0 / Q4_K blocks), packed as
    # stored by pack_for_engine when the engine's weight_dtype is that format
    native: Dict[str, object] = field(default_factory=dict)

    @property
    def device(self) -> torch.device:
        return self.embed.device


def random_weights(cfg: ModelConfig, device="cpu", dtype=torch.bfloat16, seed: int = 0) -> ModelWeights:
    g = torch.Generator(device=device)
    g.manual_seed(seed)

    def rnd(*shape, std=INIT_STD):
        return (torch.randn(*shape, generator=g, device=device, dtype=torch.float32) * std).to(dtype)

    def gain():
        # Gemma stores w with the model computing (1 + w): init w = 0 so the effective gain is 1
        if cfg.norm_add_one:
            return torch.zeros(cfg.d_model, device=device, dtype=dtype)
        return torch.ones(cfg.d_model, device=device, dtype=dtype)

    d = cfg.d_model
    layers = []
    for _ in range(cfg.n_layers):
        layers.append(LayerWeights(
            attn_norm=gain(),
            wqkv=rnd(cfg.qkv_dim, d),
            bqkv=rnd(cfg.qkv_dim, std=0.1) if cfg.qkv_bias else None,
            wo=rnd(d, cfg.q_dim),
            mlp_norm=gain(),
            w_gate=rnd(cfg.ffn, d),
            w_up=rnd(cfg.ffn, d),
            w_down=rnd(d, cfg.ffn),
        ))
    embed = rnd(cfg.vocab, d)
    lm_head = embed if cfg.tie_embeddings else rnd(cfg.vocab, d)
    return ModelWeights(cfg, embed, gain(), lm_head, layers)


def effective_gain(cfg: ModelConfig, w: torch.Tensor) -> torch.Tensor:
    return (w.float() + 1.0).to(w.dtype) if cfg.norm_add_one else w


def fold_gain(w: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """W diag(g): the RMSNorm gain that feeds a GEMM folded into its weight columns (fp32 product, one
    bf16 rounding).  RMSNorm(x) W^T = inv(x) * (x (W diag(g))^T), so the fused kernels only need the
    per-row sum of squares of x (gemm.hip, NORM)."""
    return (w.float() * g.float()[None, :]).to(w.dtype)


def _unit_gain(cfg: ModelConfig, g: torch.Tensor) -> torch.Tensor:
    """The stored RMSNorm gain whose effective gain is 1 (0 under Gemma's (1 + w) convention)."""
    return torch.zeros_like(g) if cfg.norm_add_one else torch.ones_like(g)


def _roundtrip(mw: ModelWeights, rt) -> ModelWeights:
    """Copy of ``mw`` whose GEMM weights are ``rt`` of exactly the matrices the engine quantises: each norm gain
    folded into the weight it feeds first (``fold_gain``, as ``pack_for_engine``), the gains then set to 1 -- so a
    block / row scale sees W diag(g), not W, for any gains.  The LM head is untied from the embedding table, which
    the engine keeps in bf16."""
    cfg = mw.cfg
    layers = []
    for lw in mw.layers:
        ga, gm = effective_gain(cfg, lw.attn_norm), effective_gain(cfg, lw.mlp_norm)
        layers.append(LayerWeights(attn_norm=_unit_gain(cfg, lw.attn_norm), wqkv=rt(fold_gain(lw.wqkv, ga)),
                                   bqkv=lw.bqkv, wo=rt(lw.wo), mlp_norm=_unit_gain(cfg, lw.mlp_norm),
                                   w_gate=rt(fold_gain(lw.w_gate, gm)), w_up=rt(fold_gain(lw.w_up, gm)),
                                   w_down=rt(lw.w_down)))
    lm = rt(fold_gain(mw.lm_head, effective_gain(cfg, mw.final_norm)))
    return ModelWeights(cfg, mw.embed, _unit_gain(cfg, mw.final_norm), lm, layers)


def fp8_roundtrip_weights(mw: ModelWeights) -> ModelWeights:
    """The torch oracle of a ``weight_dtype="fp8"`` engine: dequant(quant_fp8_rows(W diag(g))) in bf16, unit
    gains (``_roundtrip``)."""
    return _roundtrip(mw, lambda w: dequantize_fp8_rows(*quantize_fp8_rows(w)).to(w.dtype))


def mxfp4_roundtrip_weights(mw: ModelWeights) -> ModelWeights:
    """The torch oracle of a ``weight_dtype="fp4"`` engine: dequant(quant_mxfp4(W diag(g))) in bf16, unit gains
    (``_roundtrip``): the block scales of the oracle and of the engine are taken over the same gain-folded
    matrix, so non-unit norm gains are pinned too (tests/test_fp4_pack.py, tests/test_w4_gpu.py)."""
    return _roundtrip(mw, lambda w: dequantize_mxfp4(*quantize_mxfp4(w)).to(w.dtype))


def q4_roundtrip_weights(mw: ModelWeights, weight_dtype: str) -> ModelWeights:
    """The torch oracle of a ``weight_dtype="q4_0" / "q4_k"`` engine: the ggml blocks of W diag(g), dequantised by
    gguf.py's decoders (``_roundtrip``; models/q4.py)."""
    from .q4 import Q4_FORMATS, q4_roundtrip

    fmt = Q4_FORMATS[weight_dtype]
    if mw.native.get("fmt") == fmt:
        return mw  # a GGUF file's blocks run as stored: the loaded (decoded) weights are the values, gains separate
    return _roundtrip(mw, lambda w: q4_roundtrip(w, fmt))


def roundtrip_weights(mw: ModelWeights, weight_dtype: str) -> ModelWeights:
    """The weights a ``weight_dtype`` engine multiplies by, for the torch oracle."""
    if weight_dtype == "fp8":
        return fp8_roundtrip_weights(mw)
    if weight_dtype == "fp4":
        return mxfp4_roundtrip_weights(mw)
    if weight_dtype in ("q4_0", "q4_k"):
        return q4_roundtrip_weights(mw, weight_dtype)
    return mw


# q4_0 / q4_k: llama.cpp's GGUF block formats (models/q4.py, ops/csrc/gemm_q4.hip), Ollama's default builds
WEIGHT_DTYPES = ("bf16", "fp8", "fp4", "q4_0", "q4_k")


def pack_for_engine(mw: ModelWeights, free_natural: bool = False, weight_dtype: str = "bf16",
                    w8a8: bool = False) -> Dict[str, object]:
    """Build the decode engine's packed tensors (see module doc); norm gains are folded into the GEMM
    weights they feed (attn_norm -> wqkv, mlp_norm -> gate/up, final_norm -> lm_head).

    ``weight_dtype="fp8"``: every GEMM weight (LM head included) is quantised per row after the gain
    fold; each matrix entry becomes the fp8 packing and its scales are stored under ``s<name>``.  With
    ``w8a8`` the same e4m3 bytes are also stored in the W8A8 wide kernel's packing under ``<name>8``.
    ``weight_dtype="fp4"``: MXFP4 (``quantize_mxfp4``), the ``pack_mxfp4`` bytes under ``<name>`` and the e8m0
    scale bytes under ``s<name>``.  ``weight_dtype="q4_0" / "q4_k"``: ggml blocks of the gain-folded weights
    (models/q4.py), the ``pack_q4`` codes under ``<name>`` and its scale buffer under ``s<name>``."""
    if weight_dtype not in WEIGHT_DTYPES:
        raise ValueError(f"weight_dtype must be one of {WEIGHT_DTYPES}, got {weight_dtype!r}")
    cfg = mw.cfg
    fp8 = weight_dtype == "fp8"
    fp4 = weight_dtype == "fp4"
    q4 = weight_dtype in ("q4_0", "q4_k")
    perm = qkv_row_permutation(cfg).to(mw.device)

    native = None
    if q4:
        from .q4 import Q4_FORMATS, pack_native
        if mw.native.get("fmt") == Q4_FORMATS[weight_dtype]:
            native = mw.native
    if native is not None:
        # a GGUF file's blocks as stored: row operations only (QKV RoPE order, gate/up interleave), the norm gains
        # appended to the scale buffers of the GEMMs they feed instead of folded in (runtime.hip q4_gain)
        fmt = native["fmt"]
        layers = []
        for lw, nl in zip(mw.layers, native["layers"]):
            ga = effective_gain(cfg, lw.attn_norm).float()
            gm = effective_gain(cfg, lw.mlp_norm).float()
            lp: Dict[str, object] = {"bqkv": None if lw.bqkv is None else lw.bqkv.float()[perm].contiguous()}
            lp["wqkv"], lp["sqkv"] = pack_native(nl["wqkv"], fmt, ga, rows=perm)
            lp["wo"], lp["so"] = pack_native(nl["wo"], fmt)
            g_, u_ = nl["w_gate"], nl["w_up"]
            gu = interleave_tiles(g_.reshape(g_.shape[0], -1), u_.reshape(u_.shape[0], -1), tile=8)
            lp["wgu"], lp["sgu"] = pack_native(gu.reshape(-1, *g_.shape[1:]), fmt, gm)
            lp["wdown"], lp["sdown"] = pack_native(nl["w_down"], fmt)
            layers.append(lp)
        packed = {"layers": layers, "weight_dtype": weight_dtype, "q4_gain": True}
        packed["lm_head"], packed["lm_head_scale"] = pack_native(native["lm_head"], fmt,
                                                                 effective_gain(cfg, mw.final_norm).float())
        mw.packed = packed
        return packed

    def put(dst: Dict[str, object], name: str, w: torch.Tensor) -> None:
        if q4:
            from .q4 import Q4_FORMATS, quant_pack_q4
            dst[name], dst["s" + name[1:]] = quant_pack_q4(w, Q4_FORMATS[weight_dtype])
        elif fp4:
            dst[name], dst["s" + name[1:]] = pack_mxfp4(*quantize_mxfp4(w))
        elif fp8:
            q, sc = quantize_fp8_rows(w)
            dst[name], dst["s" + name[1:]] = pack_mfma_a_fp8(q), sc
            if w8a8:
                dst[name + "8"] = pack_mfma_a_fp8_k128(q)
        else:
            dst[name] = pack_mfma_a(w)

    layers = []
    for lw in mw.layers:
        ga = effective_gain(cfg, lw.attn_norm)
        gm = effective_gain(cfg, lw.mlp_norm)
        lp: Dict[str, object] = {"bqkv": None if lw.bqkv is None else lw.bqkv.float()[perm].contiguous()}
        put(lp, "wqkv", fold_gain(lw.wqkv[perm], ga))
        put(lp, "wo", lw.wo)
        wgu = interleave_tiles(fold_gain(lw.w_gate, gm), fold_gain(lw.w_up, gm), tile=8)
        put(lp, "wgu", wgu)
        put(lp, "wdown", lw.w_down)
        layers.append(lp)
        if free_natural:
            lw.wqkv = lw.wo = lw.w_gate = lw.w_up = lw.w_down = None
    packed: Dict[str, object] = {"layers": layers, "weight_dtype": weight_dtype}
    lm = fold_gain(mw.lm_head, effective_gain(cfg, mw.final_norm))
    put(packed, "wlm_head", lm)
    del lm
    packed["lm_head"] = packed.pop("wlm_head")
    if fp8 or fp4 or q4:
        packed["lm_head_scale"] = packed.pop("slm_head")
        if w8a8:
            packed["lm_head8"] = packed.pop("wlm_head8")
    if free_natural and not cfg.tie_embeddings:
        mw.lm_head = None
    mw.packed = packed
    return packed
