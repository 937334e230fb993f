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


def pack_for_engine(mw: ModelWeights, free_natural: bool = False) -> Dict[str, object]:
    """Build the decode engine's packed tensors (see module doc); norm gains are folded into the GEMM
    weights they feed (attn_norm -> wqkv, mlp_norm -> gate/up, final_norm -> lm_head)."""
    cfg = mw.cfg
    perm = qkv_row_permutation(cfg).to(mw.device)
    layers = []
    for lw in mw.layers:
        ga = effective_gain(cfg, lw.attn_norm)
        gm = effective_gain(cfg, lw.mlp_norm)
        layers.append({
            "wqkv": pack_mfma_a(fold_gain(lw.wqkv[perm], ga)),
            "bqkv": None if lw.bqkv is None else lw.bqkv.float()[perm].contiguous(),
            "wo": pack_mfma_a(lw.wo),
            "wgu": pack_mfma_a(interleave_tiles(fold_gain(lw.w_gate, gm), fold_gain(lw.w_up, gm), tile=8)),
            "wdown": pack_mfma_a(lw.w_down),
        })
        if free_natural:
            lw.wqkv = lw.wo = lw.w_gate = lw.w_up = lw.w_down = None
    packed = {
        "layers": layers,
        "lm_head": pack_mfma_a(fold_gain(mw.lm_head, effective_gain(cfg, mw.final_norm))),
    }
    if free_natural and not cfg.tie_embeddings:
        mw.lm_head = None
    mw.packed = packed
    return packed
