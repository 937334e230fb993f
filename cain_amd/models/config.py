"""Architecture configs of the study's seven models (the ``model`` factor).

Identities: reference experiment/RunnerConfig.py:80 (Ollama tags) and the
notebook's display names (data-analysis/analysis-visualization.ipynb:229-237).
Dimensions are the public HF configs of those checkpoints (SURVEY §2.7 [ext]);
with random-init weights only the shapes matter.  ``tiny_*`` configs keep the
same structural features (GQA group, head_dim, QKV bias, GeGLU, tied
embeddings, llama-3 RoPE scaling) at test size.
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, replace
from functools import lru_cache
from pathlib import Path
from typing import Dict, Optional, Tuple


@dataclass(frozen=True)
class RopeScaling:
    """Llama-3.1 frequency-dependent scaling."""
    factor: float = 8.0
    low_freq_factor: float = 1.0
    high_freq_factor: float = 4.0
    original_max_position: int = 8192


@dataclass(frozen=True)
class ModelConfig:
    name: str
    display_name: str
    n_layers: int
    d_model: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    ffn: int
    vocab: int
    act: str = "silu"                 # "silu" (SwiGLU) | "gelu_tanh" (GeGLU)
    tie_embeddings: bool = False
    qkv_bias: bool = False
    rope_theta: float = 10000.0
    rope_scaling: Optional[RopeScaling] = None
    norm_eps: float = 1e-5
    norm_add_one: bool = False        # Gemma: x * (1 + w)
    embed_scale: bool = False         # Gemma: embeddings * sqrt(d_model)
    max_context: int = 8192
    bos_id: int = 1
    eos_id: int = 2
    # per-frequency divisors of the inverse frequencies (GGUF's rope_freqs tensor: llama.cpp bakes Llama 3.1's
    # scaling into it); applied instead of rope_scaling when set
    rope_freq_factors: Optional[Tuple[float, ...]] = None
    # further stop ids beside eos_id (at most 3 reach the sampler): a checkpoint's other end ids and its chat
    # template's turn-end tokens (hf.py / gguf.py), as Ollama stops on its templates' stop strings
    stop_ids: Tuple[int, ...] = ()
    # the architecture family of a loaded checkpoint (llama, mistral, qwen2, gemma, phi3; "" for the built-in tags)
    family: str = ""

    @property
    def group(self) -> int:
        return self.n_heads // self.n_kv_heads

    @property
    def q_dim(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.n_kv_heads * self.head_dim

    @property
    def qkv_dim(self) -> int:
        return self.q_dim + 2 * self.kv_dim

    def n_params(self) -> int:
        d, L = self.d_model, self.n_layers
        per_layer = d * self.qkv_dim + self.q_dim * d + 3 * d * self.ffn + 2 * d
        if self.qkv_bias:
            per_layer += self.qkv_dim
        emb = self.vocab * d
        head = 0 if self.tie_embeddings else self.vocab * d
        return L * per_layer + emb + head + d

    def weight_bytes(self, dtype_bytes: int = 2) -> int:
        """Bytes streamed per decode step (every weight once, lm_head included)."""
        return self.n_params() * dtype_bytes

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.n_layers * self.kv_dim * dtype_bytes

    def as_dict(self) -> Dict:
        return asdict(self)


MODELS: Dict[str, ModelConfig] = {
    "qwen2:1.5b": ModelConfig("qwen2:1.5b", "Qwen 2 1.5B", 28, 1536, 12, 2, 128, 8960, 151936,
                              tie_embeddings=True, qkv_bias=True, rope_theta=1e6, norm_eps=1e-6,
                              bos_id=151643, eos_id=151645, max_context=32768),
    "gemma:2b": ModelConfig("gemma:2b", "Gemma 1.1 2B", 18, 2048, 8, 1, 256, 16384, 256000, act="gelu_tanh",
                            tie_embeddings=True, rope_theta=1e4, norm_eps=1e-6, norm_add_one=True,
                            embed_scale=True, bos_id=2, eos_id=1),
    "phi3:3.8b": ModelConfig("phi3:3.8b", "Phi 3 3B", 32, 3072, 32, 32, 96, 8192, 32064, rope_theta=1e4,
                             norm_eps=1e-5, bos_id=1, eos_id=32000, max_context=4096),
    "qwen2:7b": ModelConfig("qwen2:7b", "Qwen 2 7B", 28, 3584, 28, 4, 128, 18944, 152064, qkv_bias=True,
                            rope_theta=1e6, norm_eps=1e-6, bos_id=151643, eos_id=151645, max_context=32768),
    "gemma:7b": ModelConfig("gemma:7b", "Gemma 1.1 7B", 28, 3072, 16, 16, 256, 24576, 256000, act="gelu_tanh",
                            tie_embeddings=True, rope_theta=1e4, norm_eps=1e-6, norm_add_one=True,
                            embed_scale=True, bos_id=2, eos_id=1),
    "mistral:7b": ModelConfig("mistral:7b", "Mistral 0.3 7B", 32, 4096, 32, 8, 128, 14336, 32768,
                              rope_theta=1e6, norm_eps=1e-5, max_context=32768),
    "llama3.1:8b": ModelConfig("llama3.1:8b", "Llama 3.1 8B", 32, 4096, 32, 8, 128, 14336, 128256,
                               rope_theta=5e5, rope_scaling=RopeScaling(), norm_eps=1e-5,
                               bos_id=128000, eos_id=128009, max_context=131072),
}

#: model factor order used by the reference config (experiment/RunnerConfig.py:80)
STUDY_ORDER = ["llama3.1:8b", "gemma:2b", "gemma:7b", "phi3:3.8b", "qwen2:1.5b", "qwen2:7b", "mistral:7b"]


def _tiny(base: str, **kw) -> ModelConfig:
    b = MODELS[base]
    d = dict(n_layers=2, d_model=256, ffn=512, vocab=1024, max_context=1024, bos_id=1, eos_id=2)
    d.update(kw)
    return replace(b, name=f"tiny-{base}", display_name=f"tiny {b.display_name}", **d)


TINY: Dict[str, ModelConfig] = {
    # same head_dim / group / features as the full models, shrunk widths
    "tiny-llama3.1:8b": _tiny("llama3.1:8b", n_heads=4, n_kv_heads=1, head_dim=64 * 2),
    "tiny-qwen2:1.5b": _tiny("qwen2:1.5b", n_heads=6, n_kv_heads=1, head_dim=128, d_model=384),
    "tiny-gemma:2b": _tiny("gemma:2b", n_heads=2, n_kv_heads=1, head_dim=256),
    "tiny-phi3:3.8b": _tiny("phi3:3.8b", n_heads=4, n_kv_heads=4, head_dim=96, d_model=384),
    "tiny-qwen2:7b": _tiny("qwen2:7b", n_heads=7, n_kv_heads=1, head_dim=128, d_model=448),
    "tiny-gemma:7b": _tiny("gemma:7b", n_heads=2, n_kv_heads=2, head_dim=256),
    "tiny-mistral:7b": _tiny("mistral:7b", n_heads=4, n_kv_heads=1, head_dim=128),
}


def get_config(name: str) -> ModelConfig:
    """The tag's architecture: a checkpoint registered under it in ``CAIN_CHECKPOINTS`` (``hf.py``) first, else
    the built-in config."""
    import os

    if os.environ.get("CAIN_CHECKPOINTS"):
        from .hf import checkpoint_for

        path = checkpoint_for(name)
        if path:
            return _checkpoint_config(name, path)
    if name in MODELS:
        return MODELS[name]
    if name in TINY:
        return TINY[name]
    # Ollama accepts "name:tag" and "name:tag-quant"; strip a quant suffix
    base = name.split("-")[0]
    if base in MODELS:
        return MODELS[base]
    raise KeyError(f"unknown model {name!r}; known: {sorted(MODELS) + sorted(TINY)}")


@lru_cache(maxsize=64)
def _checkpoint_config(name: str, path: str) -> ModelConfig:
    from .hf import checkpoint_config

    return checkpoint_config(Path(path), name=name)


def rope_inv_freq(cfg: ModelConfig):
    """Inverse frequencies (numpy float64), with Llama-3 scaling or explicit per-frequency factors when configured."""
    import numpy as np

    hd = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (np.arange(0, hd, 2, dtype=np.float64) / hd))
    if cfg.rope_freq_factors is not None:
        fac = np.asarray(cfg.rope_freq_factors, dtype=np.float64)
        if fac.shape != inv.shape:
            raise ValueError(f"rope_freq_factors has {fac.size} entries, head_dim {hd} needs {inv.size}")
        return inv / fac
    rs = cfg.rope_scaling
    if rs is None:
        return inv
    low_wl = rs.original_max_position / rs.low_freq_factor
    high_wl = rs.original_max_position / rs.high_freq_factor
    out = np.empty_like(inv)
    for i, f in enumerate(inv):
        wl = 2 * math.pi / f
        if wl < high_wl:
            out[i] = f
        elif wl > low_wl:
            out[i] = f / rs.factor
        else:
            smooth = (rs.original_max_position / wl - rs.low_freq_factor) / (rs.high_freq_factor - rs.low_freq_factor)
            out[i] = (1 - smooth) * f / rs.factor + smooth * f
    return out
