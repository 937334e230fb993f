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


def fp8_kv_roundtrip(t: torch.Tensor) -> torch.Tensor:
    """A KV value as the fp8 cache holds it: rounded to bf16, then to e4m3 (saturating at +-448), widened."""
    return t.to(torch.bfloat16).float().clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float()


def fp8_act_roundtrip(t: torch.Tensor) -> torch.Tensor:
    """Per-row e4m3 quantisation of a bf16 GEMM input, widened: e4m3(x / s) * s with s = amax / 448."""
    xb = t.to(torch.bfloat16).float()
    amax = xb.abs().amax(-1, keepdim=True)
    s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    return (xb / s).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float() * s


class ReferenceModel:
    """Causal forward: tokens [B, T] → logits [B, T, V] (fp32).

    ``compute_dtype=torch.bfloat16`` is the PyTorch bf16-eager baseline of the numerics tests: the HIP engine's
    error against the fp32 oracle must stay within a small factor of this baseline's on the same weights.

    ``cache`` (a list, one ``[k, v]`` per layer, filled on first use) turns it into an incremental decoder:
    the CPU serving path of the engine uses it so a generation costs one token of compute per step.
    ``memo_weights`` keeps the compute-dtype copies of the weights (CPU serving: no per-call conversion)."""

    def __init__(self, mw: ModelWeights, compute_dtype=torch.float32, memo_weights: bool = False,
                 kv_dtype: str = "bf16", act_dtype: str = "bf16"):
        self.mw = mw
        self.cfg = mw.cfg
        self.dt = compute_dtype
        # "fp8": K (after RoPE) and V pass through bf16 -> e4m3 as the engine's fp8 KV cache stores them
        self.kv_fp8 = kv_dtype == "fp8"
        # "fp8": every GEMM input is quantised per row to e4m3 as the W8A8 kernels do (ops/csrc/wgemm8.hip
        # quant_rows_kernel: bf16 row, scale amax / 448; the RMSNorm factor from the unquantised row)
        self.act_fp8 = act_dtype == "fp8"
        self._memo = {} if memo_weights else None

    def _w(self, t: torch.Tensor) -> torch.Tensor:
        if self._memo is None:
            return t.to(self.dt)
        key = id(t)
        w = self._memo.get(key)
        if w is None:
            w = self._memo[key] = t.to(self.dt)
        return w

    def _in(self, t: torch.Tensor) -> torch.Tensor:
        """A GEMM input as the kernels see it (per-row e4m3 with act_dtype="fp8")."""
        return fp8_act_roundtrip(t).to(self.dt) if self.act_fp8 else t

    def _norm_in(self, x: torch.Tensor, gain: torch.Tensor) -> torch.Tensor:
        h = rms_norm(x, gain, self.cfg.norm_eps)
        if self.act_fp8:  # quantised row times the exact RMSNorm factor of the bf16 row
            xb = x.to(torch.bfloat16).float()
            h = fp8_act_roundtrip(x) * torch.rsqrt(xb.pow(2).mean(-1, keepdim=True) + self.cfg.norm_eps) * gain.float()
        return h.to(self.dt)

    def embed(self, tokens: torch.Tensor) -> torch.Tensor:
        x = self.mw.embed[tokens].to(self.dt)
        if self.cfg.embed_scale:
            x = x * torch.tensor(math.sqrt(self.cfg.d_model), dtype=torch.bfloat16).to(self.dt)
        return x

    def layer(self, x: torch.Tensor, li: int, positions: torch.Tensor, attn_mask: Optional[torch.Tensor] = None,
              cache: Optional[list] = None):
        cfg, lw = self.cfg, self.mw.layers[li]
        B, T, _ = x.shape
        h = self._norm_in(x, effective_gain(cfg, lw.attn_norm))
        qkv = h @ self._w(lw.wqkv).t()
        if lw.bqkv is not None:
            qkv = qkv + lw.bqkv.to(self.dt)
        q, k, v = qkv.split([cfg.q_dim, cfg.kv_dim, cfg.kv_dim], dim=-1)
        q = q.view(B, T, cfg.n_heads, cfg.head_dim)
        k = k.view(B, T, cfg.n_kv_heads, cfg.head_dim)
        v = v.view(B, T, cfg.n_kv_heads, cfg.head_dim)
        cos, sin = rope_cos_sin(cfg, positions)                     # [B, T, hd/2]
        q = apply_rope(q.float(), cos[:, :, None], sin[:, :, None]).to(self.dt)
        k = apply_rope(k.float(), cos[:, :, None], sin[:, :, None]).to(self.dt)
        if self.kv_fp8:
            k, v = fp8_kv_roundtrip(k).to(self.dt), fp8_kv_roundtrip(v).to(self.dt)
        past = 0
        if cache is not None:
            if len(cache) > li:
                past = cache[li][0].shape[1]
                k = torch.cat([cache[li][0], k], dim=1)
                v = torch.cat([cache[li][1], v], dim=1)
                cache[li] = [k, v]
            else:
                cache.append([k, v])
        k = k.repeat_interleave(cfg.group, dim=2)
        v = v.repeat_interleave(cfg.group, dim=2)
        att = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) / math.sqrt(cfg.head_dim)
        causal = torch.ones(T, past + T, dtype=torch.bool, device=x.device).tril(diagonal=past)
        mask = causal if attn_mask is None else causal & attn_mask
        att = att.masked_fill(~mask, float("-inf")).softmax(-1)
        o = torch.einsum("bhqk,bkhd->bqhd", att, v.float()).reshape(B, T, cfg.q_dim).to(self.dt)
        x = x + (self._in(o) @ self._w(lw.wo).t())
        h = self._norm_in(x, effective_gain(cfg, lw.mlp_norm))
        g = h @ self._w(lw.w_gate).t()
        u = h @ self._w(lw.w_up).t()
        a = (activation(cfg, g.float()) * u.float()).to(self.dt)
        return x + self._in(a) @ self._w(lw.w_down).t()

    @torch.no_grad()
    def forward(self, tokens: torch.Tensor, positions: Optional[torch.Tensor] = None,
                cache: Optional[list] = None, last_only: bool = False) -> torch.Tensor:
        B, T = tokens.shape
        if positions is None:
            past = cache[0][0].shape[1] if cache else 0
            positions = torch.arange(past, past + T, device=tokens.device).expand(B, T)
        x = self.embed(tokens)
        for li in range(self.cfg.n_layers):
            x = self.layer(x, li, positions, cache=cache)
        if last_only:
            x = x[:, -1:]
        x = self._norm_in(x, effective_gain(self.cfg, self.mw.final_norm))
        if self.dt != torch.float32:
            # reduced-precision eager baseline (tests' relative numerics criterion): bf16 everywhere the engine keeps
            # bf16, but fp32 logits like the engine's LM head (fp32 accumulation, no bf16 rounding of the logits)
            return x.float() @ self.mw.lm_head.float().t()
        return (x @ self._w(self.mw.lm_head).t()).float()

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
