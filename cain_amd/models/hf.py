"""Hugging Face checkpoints for the seven study architectures: ``config.json`` + ``*.safetensors`` (+ ``tokenizer.json``).

The reference serves real models through Ollama (``/root/reference/experiment/RunnerConfig.py:80``, the Ollama tags;
``README.md:29-30``).  The engine here defaults to seeded random weights of each architecture's exact shapes (there is
no network for checkpoints), and this module is how a user points it at real ones instead:

* ``config_from_hf`` maps a ``config.json`` (Llama / Mistral / Qwen2 / Gemma / Phi-3; transformers 4.x keys
  ``rope_theta`` + ``rope_scaling`` and 5.x ``rope_parameters``) onto ``ModelConfig``;
* ``load_hf_weights`` reads the safetensors shards (``safe_open``: no pickle) into ``ModelWeights``, natural layout:
  q / k / v (or Phi-3's fused ``qkv_proj``) concatenated into ``wqkv``, Phi-3's fused ``gate_up_proj`` split, the LM
  head tied to the embedding table when the checkpoint has none;
* ``load_pretrained`` returns config, weights and the checkpoint's ``tokenizer.json`` tokenizer;
* ``CAIN_CHECKPOINTS="tag=/path,tag2=/path2"`` registers checkpoints (directories, or GGUF files: ``gguf.py``)
  under model tags: every place that builds an
  engine from a tag (``DecodeEngine(tag)``, the Ollama-compatible server, the study, ``bench.py``) and
  ``get_config(tag)`` then use the checkpoint.

The torch oracle (``reference.py``) follows the transformers conventions (rotate-half RoPE on the checkpoint's q / k
row order, Gemma's ``(1 + w)`` gain and bf16 ``sqrt(d)`` embedding scale, Llama-3 frequency scaling), and
``pack_for_engine`` permutes q / k rows itself, so checkpoint tensors are used as stored.  ``tests/test_hf_checkpoint.py``
pins the oracle's logits on loaded checkpoints against transformers' own model classes, per architecture.

Not supported (refused with an error, not approximated): RoPE types other than default / llama3 (linear, dynamic,
YaRN, Phi-3 long-rope), partial rotary embeddings, MLP or output-projection biases.  A sliding attention window
shorter than the model's context caps the engine's context at the window, inside which attention is exact.
"""
from __future__ import annotations

import json
import os
import re
from pathlib import Path
from typing import Dict, List, Optional, Tuple, Union

import torch

from .config import ModelConfig, RopeScaling
from .weights import LayerWeights, ModelWeights

PathLike = Union[str, os.PathLike]

# transformers architectures -> the study family they implement (the tags' families in config.MODELS)
ARCHITECTURES = {
    "LlamaForCausalLM": "llama",
    "MistralForCausalLM": "mistral",
    "Qwen2ForCausalLM": "qwen2",
    "GemmaForCausalLM": "gemma",
    "Phi3ForCausalLM": "phi3",
}
# the model classes' own defaults where a config.json may omit the key (transformers writes only non-defaults)
_TIE_DEFAULT = {"llama": False, "mistral": False, "qwen2": False, "gemma": True, "phi3": False}
_GELU_TANH = ("gelu_pytorch_tanh", "gelu_tanh", "gelu_new", "gelu")  # HF Gemma runs the tanh form for all of them


def _read_config(path: PathLike) -> Dict:
    p = Path(path)
    return json.loads((p / "config.json" if p.is_dir() else p).read_text())


def _family(hf: Dict) -> str:
    mt = hf.get("model_type")
    if mt in _TIE_DEFAULT:
        return mt
    for a in hf.get("architectures") or []:
        if a in ARCHITECTURES:
            return ARCHITECTURES[a]
    raise ValueError(f"unsupported architecture: model_type={mt!r}, architectures={hf.get('architectures')!r}; "
                     f"supported: {sorted(ARCHITECTURES)}")


def _rope(hf: Dict) -> Tuple[float, Optional[RopeScaling]]:
    """(theta, Llama-3 scaling or None) from either config generation."""
    rp = dict(hf.get("rope_parameters") or {})
    rs = dict(hf.get("rope_scaling") or {})
    theta = float(rp.get("rope_theta", hf.get("rope_theta") or 10000.0))
    spec = rs or rp
    kind = spec.get("rope_type", spec.get("type", "default")) or "default"
    prf = float(spec.get("partial_rotary_factor", hf.get("partial_rotary_factor") or 1.0))
    if prf != 1.0:
        raise NotImplementedError(f"partial rotary embeddings (factor {prf}) are not supported")
    if kind == "default":
        return theta, None
    if kind == "llama3":
        return theta, RopeScaling(factor=float(spec["factor"]), low_freq_factor=float(spec["low_freq_factor"]),
                                  high_freq_factor=float(spec["high_freq_factor"]),
                                  original_max_position=int(spec["original_max_position_embeddings"]))
    raise NotImplementedError(f"RoPE type {kind!r} is not supported (default and llama3 are)")


def _first(v, default: int) -> int:
    if v is None:
        return default
    return int(v[0]) if isinstance(v, (list, tuple)) else int(v)


def _last(v, default: int) -> int:
    """The stop id of a list of end ids: the last (Llama 3.1 Instruct: [end_of_text, eom, eot] -> eot, the turn end
    Ollama stops on; the engine keeps one stop id per request)."""
    if v is None:
        return default
    return int(v[-1]) if isinstance(v, (list, tuple)) else int(v)


def config_from_hf(hf: Union[Dict, PathLike], name: Optional[str] = None,
                   tensor_names: Optional[List[str]] = None) -> ModelConfig:
    """``ModelConfig`` of a transformers ``config.json`` (a dict, the file or its directory).  ``tensor_names`` (the
    checkpoint's tensors, when known) settle what the config may leave implicit: a tied LM head (no
    ``lm_head.weight``) and QKV biases (``q_proj.bias``)."""
    if not isinstance(hf, dict):
        if name is None:
            p = Path(hf)
            name = (p if p.is_dir() else p.parent).name
        hf = _read_config(hf)
    fam = _family(hf)
    d = int(hf["hidden_size"])
    n_heads = int(hf["num_attention_heads"])
    n_kv = int(hf.get("num_key_value_heads") or n_heads)
    head_dim = int(hf.get("head_dim") or d // n_heads)
    act_name = hf.get("hidden_activation") or hf.get("hidden_act") or "silu"
    if fam == "gemma" or act_name in ("gelu_pytorch_tanh", "gelu_tanh", "gelu_new"):
        if act_name not in _GELU_TANH:
            raise NotImplementedError(f"activation {act_name!r} is not supported")
        act = "gelu_tanh"
    elif act_name == "silu":
        act = "silu"
    else:
        raise NotImplementedError(f"activation {act_name!r} is not supported (silu, gelu-tanh are)")
    for key in ("mlp_bias",):
        if hf.get(key):
            raise NotImplementedError(f"{key}=true is not supported")
    names = set(tensor_names or [])
    if names:
        tie = "lm_head.weight" not in names
        qkv_bias = any(n.endswith("self_attn.q_proj.bias") or n.endswith("self_attn.qkv_proj.bias") for n in names)
    else:
        tie = bool(hf.get("tie_word_embeddings", _TIE_DEFAULT[fam]))
        qkv_bias = fam == "qwen2" or bool(hf.get("attention_bias", False))
    theta, scaling = _rope(hf)
    max_ctx = int(hf.get("max_position_embeddings") or 8192)
    window = hf.get("sliding_window")
    # transformers applies the window for Mistral and Phi-3 whenever it is set, for Qwen2 only with use_sliding_window
    uses_window = window and (fam in ("mistral", "phi3") or hf.get("use_sliding_window"))
    if uses_window and int(window) < max_ctx:
        max_ctx = int(window)  # attention is exact inside the window; the engine's context stops at it
    return ModelConfig(
        name=name or fam, display_name=name or fam, n_layers=int(hf["num_hidden_layers"]), d_model=d,
        n_heads=n_heads, n_kv_heads=n_kv, head_dim=head_dim, ffn=int(hf["intermediate_size"]),
        vocab=int(hf["vocab_size"]), act=act, tie_embeddings=tie, qkv_bias=qkv_bias, rope_theta=theta,
        rope_scaling=scaling, norm_eps=float(hf.get("rms_norm_eps", 1e-6)), norm_add_one=fam == "gemma",
        embed_scale=fam == "gemma", max_context=max_ctx, bos_id=_first(hf.get("bos_token_id"), 1),
        eos_id=_last(hf.get("eos_token_id"), 2), stop_ids=_other_ends(hf.get("eos_token_id")), family=fam)


def _other_ends(v) -> Tuple[int, ...]:
    """The end ids of a list besides the one ``_last`` picks."""
    return tuple(int(x) for x in v[:-1]) if isinstance(v, (list, tuple)) else ()


# turn-end tokens of the families' chat templates, on which Ollama's templates stop
# in priority order (with_stop_ids keeps 3 beside eos_id): Llama 3.x's eot / eom / end_of_text first, as llama.cpp's
# end-of-generation set has them
TURN_END_TOKENS = ("<|eot_id|>", "<|eom_id|>", "<|end_of_text|>", "<|end|>", "<end_of_turn>", "<|im_end|>",
                   "<|endoftext|>", "</s>")


def with_stop_ids(cfg: ModelConfig, extra_ids) -> ModelConfig:
    """``cfg`` with ``extra_ids`` added to its stop ids (kept distinct from eos_id, order kept, first 3)."""
    import dataclasses

    ids = []
    for i in list(cfg.stop_ids) + [int(x) for x in extra_ids]:
        if i != cfg.eos_id and i >= 0 and i not in ids:
            ids.append(i)
    return dataclasses.replace(cfg, stop_ids=tuple(ids[:3]))


def template_stop_ids(tok) -> List[int]:
    """Ids of the turn-end tokens a tokenizer knows (``TURN_END_TOKENS``)."""
    out = []
    for t in TURN_END_TOKENS:
        i = tok.tok.token_to_id(t) if tok is not None and hasattr(tok, "tok") else None
        if i is not None:
            out.append(int(i))
    return out


def _shards(path: Path) -> List[Path]:
    idx = path / "model.safetensors.index.json"
    if idx.exists():
        return [path / f for f in sorted(set(json.loads(idx.read_text())["weight_map"].values()))]
    files = sorted(path.glob("*.safetensors"))
    if not files:
        raise FileNotFoundError(f"no *.safetensors in {path}")
    return files


class _Tensors:
    """Lazy view of a checkpoint's tensors over its safetensors shards (``safe_open``: no code runs from the file)."""

    def __init__(self, path: Path):
        from safetensors import safe_open

        self._where: Dict[str, Path] = {}
        self._open = safe_open
        for f in _shards(path):
            with safe_open(str(f), framework="pt") as h:
                for k in h.keys():
                    self._where[k] = f

    def names(self) -> List[str]:
        return list(self._where)

    def get(self, name: str) -> torch.Tensor:
        f = self._where.get(name)
        if f is None:
            raise KeyError(f"checkpoint has no tensor {name!r}")
        with self._open(str(f), framework="pt") as h:
            return h.get_tensor(name)

    def has(self, name: str) -> bool:
        return name in self._where


def load_hf_weights(path: PathLike, cfg: Optional[ModelConfig] = None, device="cpu",
                    dtype: torch.dtype = torch.bfloat16) -> ModelWeights:
    """``ModelWeights`` (natural layout, ``dtype``) of a checkpoint directory (or a GGUF file: models/gguf.py)."""
    p = Path(path)
    if is_gguf(p):
        from .gguf import GGUFFile, config_from_gguf, load_gguf_weights

        g = GGUFFile(p)
        return load_gguf_weights(g, cfg or config_from_gguf(g, name=p.stem), device=device, dtype=dtype)
    t = _Tensors(p)
    if cfg is None:
        cfg = config_from_hf(_read_config(p), name=p.name, tensor_names=t.names())
    pre = "model."

    def w(name: str) -> torch.Tensor:
        return t.get(name).to(device=device, dtype=dtype)

    def check(name: str, x: torch.Tensor, shape) -> torch.Tensor:
        if tuple(x.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(x.shape)}, the config implies {tuple(shape)}")
        return x

    d, qd, kd, f = cfg.d_model, cfg.q_dim, cfg.kv_dim, cfg.ffn
    layers = []
    for i in range(cfg.n_layers):
        lp = f"{pre}layers.{i}."
        if t.has(lp + "self_attn.qkv_proj.weight"):
            wqkv = w(lp + "self_attn.qkv_proj.weight")
            bqkv = w(lp + "self_attn.qkv_proj.bias") if t.has(lp + "self_attn.qkv_proj.bias") else None
        else:
            wqkv = torch.cat([w(lp + f"self_attn.{k}_proj.weight") for k in "qkv"], 0)
            bqkv = (torch.cat([w(lp + f"self_attn.{k}_proj.bias") for k in "qkv"], 0)
                    if t.has(lp + "self_attn.q_proj.bias") else None)
        if t.has(lp + "self_attn.o_proj.bias") or t.has(lp + "mlp.down_proj.bias"):
            raise NotImplementedError("output-projection / MLP biases are not supported")
        if t.has(lp + "mlp.gate_up_proj.weight"):
            gu = check(lp + "mlp.gate_up_proj.weight", w(lp + "mlp.gate_up_proj.weight"), (2 * f, d))
            w_gate, w_up = gu[:f].contiguous(), gu[f:].contiguous()  # HF Phi3MLP: gate first, then up
        else:
            w_gate, w_up = w(lp + "mlp.gate_proj.weight"), w(lp + "mlp.up_proj.weight")
        if (bqkv is not None) != cfg.qkv_bias:
            raise ValueError(f"layer {i}: QKV bias {'present' if bqkv is not None else 'absent'}, config says "
                             f"qkv_bias={cfg.qkv_bias}")
        layers.append(LayerWeights(
            attn_norm=check(lp + "input_layernorm.weight", w(lp + "input_layernorm.weight"), (d,)),
            wqkv=check(lp + "qkv", wqkv, (qd + 2 * kd, d)),
            bqkv=None if bqkv is None else check(lp + "qkv bias", bqkv, (qd + 2 * kd,)),
            wo=check(lp + "self_attn.o_proj.weight", w(lp + "self_attn.o_proj.weight"), (d, qd)),
            mlp_norm=check(lp + "post_attention_layernorm.weight", w(lp + "post_attention_layernorm.weight"), (d,)),
            w_gate=check(lp + "gate", w_gate, (f, d)), w_up=check(lp + "up", w_up, (f, d)),
            w_down=check(lp + "mlp.down_proj.weight", w(lp + "mlp.down_proj.weight"), (d, f))))
    embed = check("embed_tokens", w(pre + "embed_tokens.weight"), (cfg.vocab, d))
    if t.has("lm_head.weight") and not cfg.tie_embeddings:
        lm_head = check("lm_head.weight", w("lm_head.weight"), (cfg.vocab, d))
    else:
        lm_head = embed
    return ModelWeights(cfg, embed, check("norm", w(pre + "norm.weight"), (d,)), lm_head, layers)


def load_tokenizer(path: PathLike, cfg: Optional[ModelConfig] = None):
    """The checkpoint's ``tokenizer.json`` (``HFTokenizer``), or None when it has none."""
    from .tokenizer import HFTokenizer

    if is_gguf(path):
        from .gguf import GGUFFile, load_gguf_tokenizer

        return load_gguf_tokenizer(GGUFFile(path), cfg)
    f = Path(path) / "tokenizer.json"
    if not f.exists():
        return None
    tok = HFTokenizer(str(f), bos_id=cfg.bos_id if cfg else None)
    tok.chat_template, tok.special_tokens = _chat_template(Path(path))
    return tok


def _chat_template(path: Path) -> Tuple[Optional[str], Dict[str, str]]:
    """(chat template, special-token strings) of a checkpoint directory: ``chat_template.jinja`` or
    ``tokenizer_config.json``'s ``chat_template`` (a string, or named templates: "default" is used)."""
    tc = path / "tokenizer_config.json"
    conf = json.loads(tc.read_text()) if tc.exists() else {}
    special = {}
    for k in ("bos_token", "eos_token", "unk_token", "pad_token"):
        v = conf.get(k)
        if isinstance(v, dict):
            v = v.get("content")
        if isinstance(v, str):
            special[k] = v
    tmpl = conf.get("chat_template")
    if isinstance(tmpl, list):
        named = {t.get("name"): t.get("template") for t in tmpl if isinstance(t, dict)}
        tmpl = named.get("default") or next(iter(named.values()), None)
    jf = path / "chat_template.jinja"
    if jf.exists():
        tmpl = jf.read_text()
    return (tmpl if isinstance(tmpl, str) and tmpl else None), special


def load_pretrained(path: PathLike, name: Optional[str] = None, device="cpu",
                    dtype: torch.dtype = torch.bfloat16):
    """(config, weights, tokenizer or None) of a checkpoint directory or a GGUF file."""
    p = Path(path)
    if is_gguf(p):
        from .gguf import load_gguf

        return load_gguf(p, name=name or p.stem, device=device, dtype=dtype)
    cfg = checkpoint_config(p, name=name or p.name)
    w = load_hf_weights(p, cfg, device=device, dtype=dtype)
    return cfg, w, load_tokenizer(p, cfg)


def is_gguf(path: PathLike) -> bool:
    from .gguf import is_gguf as _is_gguf

    return _is_gguf(path)


def checkpoint_config(path: PathLike, name: Optional[str] = None) -> ModelConfig:
    """The ``ModelConfig`` of a checkpoint directory or GGUF file."""
    p = Path(path)
    if is_gguf(p):
        from .gguf import GGUFFile, config_from_gguf

        return config_from_gguf(GGUFFile(p), name=name or p.stem)
    cfg = config_from_hf(p, name=name, tensor_names=_Tensors(p).names())
    gc = p / "generation_config.json"  # the generation end ids (Llama 3.1 Instruct: end_of_text, eom, eot)
    if gc.exists():
        ends = json.loads(gc.read_text()).get("eos_token_id")
        cfg = with_stop_ids(cfg, ends if isinstance(ends, list) else [ends] if ends is not None else [])
    return with_stop_ids(cfg, template_stop_ids(load_tokenizer(p)))


def registered_checkpoints() -> Dict[str, str]:
    """``CAIN_CHECKPOINTS="tag=/path,..."`` as a dict (model tag -> checkpoint directory)."""
    out: Dict[str, str] = {}
    for spec in filter(None, (s.strip() for s in os.environ.get("CAIN_CHECKPOINTS", "").split(","))):
        tag, sep, path = spec.partition("=")
        if not sep or not tag or not path:
            raise ValueError(f"CAIN_CHECKPOINTS entry {spec!r} is not tag=/path")
        out[tag.strip()] = path.strip()
    return out


def checkpoint_for(tag: str) -> Optional[str]:
    """The checkpoint registered for ``tag``: a path, or ``ollama`` / ``ollama:<models dir>`` for the GGUF blob a
    local Ollama installation serves under that tag (``ollama_blob``)."""
    path = registered_checkpoints().get(tag)
    if path and (path == "ollama" or path.startswith("ollama:")):
        return str(ollama_blob(tag, path[7:] or None))
    return path


def ollama_blob(tag: str, models_dir: Optional[PathLike] = None) -> Path:
    """The GGUF model blob Ollama stores for ``tag`` (``name[:tag]``, default tag ``latest``; a ``namespace/name``
    or ``host/namespace/name`` prefix as Ollama writes it): the manifest at
    ``<models>/manifests/<host>/<namespace>/<name>/<tag>`` names its layers; the one of media type
    ``application/vnd.ollama.image.model`` is ``<models>/blobs/sha256-<hex>``.  ``models_dir`` defaults to
    ``$OLLAMA_MODELS`` or ``~/.ollama/models``.  JSON only: nothing from the store is executed."""
    root = Path(models_dir or os.environ.get("OLLAMA_MODELS") or Path.home() / ".ollama" / "models").expanduser()
    name, _, version = tag.partition(":")
    parts = name.split("/")
    host, ns = "registry.ollama.ai", "library"
    if len(parts) == 2:
        ns, name = parts
    elif len(parts) >= 3:
        host, ns, name = parts[0], parts[1], "/".join(parts[2:])
    manifest = root / "manifests" / host / ns / name / (version or "latest")
    if not manifest.is_file():
        raise FileNotFoundError(f"no Ollama manifest for {tag!r} at {manifest}")
    layers = json.loads(manifest.read_text()).get("layers") or []
    model = [lay for lay in layers if str(lay.get("mediaType", "")).endswith(".image.model")]
    if not model:
        raise ValueError(f"Ollama manifest {manifest} has no model layer")
    digest = str(model[0].get("digest", ""))
    if not re.fullmatch(r"sha256:[0-9a-f]{64}", digest):
        raise ValueError(f"Ollama manifest {manifest}: malformed model digest {digest!r}")
    blob = root / "blobs" / digest.replace(":", "-")
    if not blob.is_file():
        raise FileNotFoundError(f"Ollama blob {blob} (for {tag!r}) is missing")
    return blob
