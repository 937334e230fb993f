"""Torch-eager oracle of the seven decoder architectures.

Plain PyTorch, fp32 compute by default, natural weight layout.  It is the
numerics reference every HIP kernel and the fused engine are tested against
(SURVEY §4 item 4), and it is the CPU path of the engine (tests, CI).

Covered variants: GQA/MQA/MHA, head_dim 96/128/256,
QKV bias (Qwen2), GeGLU-tanh vs SwiGLU, Gemma's ``(1 + w)`` RMSNorm gain and
``sqrt(d)`` embedding scale, tied embeddings, Llama-3 RoPE scaling, NeoX
("rotate_half") RoPE.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from .config import ModelConfig, rope_inv_freq
from .weights import ModelWeights, effective_gain


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def rope_cos_sin(cfg: ModelConfig, positions: torch.Tensor):
    inv = torch.tensor(rope_inv_freq(cfg), dtype=torch.float64, device=positions.device)
    ang = positions.to(torch.float64)[..., None] * inv            # [..., hd/2]
    return torch.cos(ang).float(), torch.sin(ang).float()


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [..., hd] with cos/sin [..., hd/2] broadcastable (rotate_half convention)."""
    h = x.shape[-1] // 2
    x1, x2 = x[..., :h], x[..., h:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def activation(cfg: ModelConfig, g: torch.Tensor) -> torch.Tensor:
    if cfg.act == "gelu_tanh":
        return F.gelu(g, approximate="tanh")
    return F.silu(g)


class ReferenceModel:
    """Full-sequence causal forward: tokens [B, T] → logits [B, T, V] (fp32)."""

    def __init__(self, mw: ModelWeights, compute_dtype=torch.float32):
        self.mw = mw
        self.cfg = mw.cfg
        self.dt = compute_dtype

    def embed(self, tokens: torch.Tensor) -> torch.Tensor:
        x = self.mw.embed[tokens].to(self.dt)
        if self.cfg.embed_scale:
            x = x * torch.tensor(math.sqrt(self.cfg.d_model), dtype=torch.bfloat16).to(self.dt)
        return x

    def layer(self, x: torch.Tensor, li: int, positions: torch.Tensor, attn_mask: Optional[torch.Tensor] = None):
        cfg, lw = self.cfg, self.mw.layers[li]
        B, T, _ = x.shape
        h = rms_norm(x, effective_gain(cfg, lw.attn_norm), cfg.norm_eps).to(self.dt)
        qkv = h @ lw.wqkv.to(self.dt).t()
        if lw.bqkv is not None:
            qkv = qkv + lw.bqkv.to(self.dt)
        q, k, v = qkv.split([cfg.q_dim, cfg.kv_dim, cfg.kv_dim], dim=-1)
        q = q.view(B, T, cfg.n_heads, cfg.head_dim)
        k = k.view(B, T, cfg.n_kv_heads, cfg.head_dim)
        v = v.view(B, T, cfg.n_kv_heads, cfg.head_dim)
        cos, sin = rope_cos_sin(cfg, positions)                     # [B, T, hd/2]
        q = apply_rope(q.float(), cos[:, :, None], sin[:, :, None]).to(self.dt)
        k = apply_rope(k.float(), cos[:, :, None], sin[:, :, None]).to(self.dt)
        k = k.repeat_interleave(cfg.group, dim=2)
        v = v.repeat_interleave(cfg.group, dim=2)
        att = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) / math.sqrt(cfg.head_dim)
        causal = torch.ones(T, T, dtype=torch.bool, device=x.device).tril()
        mask = causal if attn_mask is None else causal & attn_mask
        att = att.masked_fill(~mask, float("-inf")).softmax(-1)
        o = torch.einsum("bhqk,bkhd->bqhd", att, v.float()).reshape(B, T, cfg.q_dim).to(self.dt)
        x = x + (o @ lw.wo.to(self.dt).t())
        h = rms_norm(x, effective_gain(cfg, lw.mlp_norm), cfg.norm_eps).to(self.dt)
        g = h @ lw.w_gate.to(self.dt).t()
        u = h @ lw.w_up.to(self.dt).t()
        a = (activation(cfg, g.float()) * u.float()).to(self.dt)
        return x + a @ lw.w_down.to(self.dt).t()

    @torch.no_grad()
    def forward(self, tokens: torch.Tensor, positions: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, T = tokens.shape
        if positions is None:
            positions = torch.arange(T, device=tokens.device).expand(B, T)
        x = self.embed(tokens)
        for li in range(self.cfg.n_layers):
            x = self.layer(x, li, positions)
        x = rms_norm(x, effective_gain(self.cfg, self.mw.final_norm), self.cfg.norm_eps).to(self.dt)
        return (x @ self.mw.lm_head.to(self.dt).t()).float()

    @torch.no_grad()
    def greedy(self, prompt: torch.Tensor, n_new: int) -> torch.Tensor:
        """Greedy continuation of prompt [B, T] (recomputes the prefix each step; tests only)."""
        toks = prompt
        out = []
        for _ in range(n_new):
            nxt = self.forward(toks)[:, -1].argmax(-1)
            out.append(nxt)
            toks = torch.cat([toks, nxt[:, None]], dim=1)
        return torch.stack(out, dim=1)
