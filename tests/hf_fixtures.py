"""Tiny Hugging Face checkpoints of the five study families, written by transformers itself (``save_pretrained``,
safetensors), with non-trivial norm gains and QKV biases so the loader's gain / bias conventions are exercised.

Shapes follow the engine's tiny configs (``models/config.py`` TINY): the same head_dim / GQA group / features at
test size, vocabularies of 1,024 (a multiple of 64, as the HIP LM head wants)."""
from __future__ import annotations

from pathlib import Path
from typing import Dict

import torch

LLAMA3_ROPE = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
               "original_max_position_embeddings": 8192, "rope_theta": 500000.0}

# family -> (transformers config class, model class, config kwargs)
FAMILIES: Dict[str, tuple] = {
    "llama": ("LlamaConfig", "LlamaForCausalLM",
              dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=1, head_dim=128,
                   rope_parameters=LLAMA3_ROPE, max_position_embeddings=131072, rms_norm_eps=1e-5,
                   tie_word_embeddings=False)),
    "mistral": ("MistralConfig", "MistralForCausalLM",
                dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=1,
                     head_dim=128, rope_parameters={"rope_type": "default", "rope_theta": 1e6},
                     max_position_embeddings=32768, sliding_window=None, rms_norm_eps=1e-5)),
    "qwen2": ("Qwen2Config", "Qwen2ForCausalLM",
              dict(hidden_size=384, intermediate_size=512, num_attention_heads=6, num_key_value_heads=1, head_dim=128,
                   rope_parameters={"rope_type": "default", "rope_theta": 1e6}, max_position_embeddings=32768,
                   rms_norm_eps=1e-6, tie_word_embeddings=True, use_sliding_window=False)),
    "gemma": ("GemmaConfig", "GemmaForCausalLM",
              dict(hidden_size=256, intermediate_size=512, num_attention_heads=2, num_key_value_heads=1, head_dim=256,
                   hidden_activation="gelu_pytorch_tanh", rope_parameters={"rope_type": "default", "rope_theta": 1e4},
                   max_position_embeddings=8192, rms_norm_eps=1e-6)),
    "phi3": ("Phi3Config", "Phi3ForCausalLM",
             dict(hidden_size=384, intermediate_size=512, num_attention_heads=4, num_key_value_heads=4,
                  rope_parameters={"rope_type": "default", "rope_theta": 1e4, "partial_rotary_factor": 1.0},
                  max_position_embeddings=4096, sliding_window=None, rms_norm_eps=1e-5, pad_token_id=0)),
}


def make_checkpoint(family: str, path: Path, n_layers: int = 2, vocab: int = 1024, seed: int = 0,
                    scale: float = 1.0):
    """Write a random tiny checkpoint of ``family`` to ``path``; returns the transformers model (fp32, eval).
    ``scale`` multiplies the linear weights' init std (larger logits make the parity check sharper)."""
    import transformers

    cfg_cls, model_cls, kw = FAMILIES[family]
    kw = dict(kw, vocab_size=vocab, num_hidden_layers=n_layers, bos_token_id=1, eos_token_id=2,
              initializer_range=0.02 * scale)
    cfg = getattr(transformers, cfg_cls)(**kw)
    cfg._attn_implementation = "eager"
    torch.manual_seed(seed)
    model = getattr(transformers, model_cls)(cfg).eval()
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if name.endswith("norm.weight"):
                # gains around 1 (Gemma stores w of (1 + w): around 0)
                base = 0.0 if family == "gemma" else 1.0
                p.copy_(base + 0.2 * torch.randn(p.shape, generator=g))
            elif name.endswith(".bias"):
                p.copy_(0.1 * torch.randn(p.shape, generator=g))
    path.mkdir(parents=True, exist_ok=True)
    model.save_pretrained(str(path))
    return model


CHAT_TOKENS = ["<|system|>", "<|user|>", "<|assistant|>"]
# a llama-3-like template: BOS, one marker per turn, the assistant marker as the generation prompt
CHAT_TEMPLATE = ("{{ bos_token }}{% for m in messages %}{{ '<|' + m['role'] + '|>' }} {{ m['content'] }} {% endfor %}"
                 "{% if add_generation_prompt %}<|assistant|>{% endif %}")


def write_tokenizer(path: Path, vocab: int = 1024, bos_token: str = "<s>", chat: bool = False) -> None:
    """A word-level ``tokenizer.json`` whose template prepends ``bos_token`` (as Llama 3's and Gemma's do); with
    ``chat`` also turn-marker tokens and a ``tokenizer_config.json`` carrying ``CHAT_TEMPLATE``."""
    import json

    from tokenizers import Tokenizer, models, pre_tokenizers, processors

    special = [bos_token, "</s>"] + (CHAT_TOKENS if chat else [])
    words = ["<unk>", bos_token, "</s>"] + special[2:]
    words += [f"w{i}" for i in range(vocab - len(words))]
    tok = Tokenizer(models.WordLevel({w: i for i, w in enumerate(words)}, unk_token="<unk>"))
    tok.pre_tokenizer = pre_tokenizers.WhitespaceSplit()
    tok.post_processor = processors.TemplateProcessing(single=f"{bos_token} $A", special_tokens=[(bos_token, 1)])
    tok.add_special_tokens(special)
    tok.save(str(path / "tokenizer.json"))
    if chat:
        (path / "tokenizer_config.json").write_text(json.dumps({"bos_token": bos_token, "eos_token": "</s>",
                                                                "chat_template": CHAT_TEMPLATE}))


def hf_logits(model, tokens: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
    with torch.no_grad():
        return model(input_ids=tokens, position_ids=positions).logits.float()
