"""Model zoo, layouts, tokenizer and the torch-eager engine backend on CPU."""
import numpy as np
import pytest
import torch

from cain_amd.engine import DecodeEngine
from cain_amd.engine.engine import sample_host
from cain_amd.models import MODELS, STUDY_ORDER, TINY, get_config, random_weights
from cain_amd.models.config import rope_inv_freq
from cain_amd.models.reference import ReferenceModel
from cain_amd.models.tokenizer import SyntheticTokenizer, tokens_for_words
from cain_amd.models.weights import (interleave_tiles, pack_mfma_a, qkv_row_permutation, rope_pair_order,
                                     unpack_mfma_a)

# public HF parameter counts of the checkpoints (billions, 2 d.p.)
PARAMS_B = {"qwen2:1.5b": 1.54, "gemma:2b": 2.51, "phi3:3.8b": 3.82, "qwen2:7b": 7.62, "gemma:7b": 8.54,
            "mistral:7b": 7.25, "llama3.1:8b": 8.03}


def test_model_zoo_matches_study():
    assert sorted(STUDY_ORDER) == sorted(MODELS)
    for name, b in PARAMS_B.items():
        assert round(MODELS[name].n_params() / 1e9, 2) == b, name
    assert {c.group for c in MODELS.values()} == {1, 4, 6, 7, 8}
    assert {c.head_dim for c in MODELS.values()} == {96, 128, 256}
    assert get_config("llama3.1:8b-instruct-q4_0").name == "llama3.1:8b"
    with pytest.raises(KeyError):
        get_config("nope:1b")


def test_llama3_rope_scaling_bands():
    cfg = MODELS["llama3.1:8b"]
    inv = rope_inv_freq(cfg)
    base = 1.0 / (cfg.rope_theta ** (np.arange(0, 128, 2) / 128))
    assert inv[0] == pytest.approx(base[0])            # high frequency untouched
    assert inv[-1] == pytest.approx(base[-1] / 8.0)    # low frequency scaled by factor 8
    assert np.all(inv <= base + 1e-15)


def test_layouts_are_permutations():
    w = torch.randn(64, 96)
    assert torch.equal(unpack_mfma_a(pack_mfma_a(w)), w)
    for hd in (64, 96, 128, 256):
        p = rope_pair_order(hd)
        assert sorted(p.tolist()) == list(range(hd))
    cfg = MODELS["qwen2:7b"]
    perm = qkv_row_permutation(cfg)
    assert sorted(perm.tolist()) == list(range(cfg.qkv_dim))
    a, b = torch.zeros(16, 4), torch.ones(16, 4)
    il = interleave_tiles(a, b, tile=8)
    assert il[:8].sum() == 0 and il[8:16].sum() == 32 and il[16:24].sum() == 0


def test_tokenizer_counts_and_stability():
    t = SyntheticTokenizer(32000, 1, 2)
    ids = t.encode("In 100 words, please give me information about India")
    assert ids[0] == 1 and ids == t.encode("In 100 words, please give me information about India")
    assert all(16 <= i < 32000 for i in ids[1:])
    text = t.decode(list(range(100, 500)))
    assert 0.6 < len(text.split()) / 400 < 0.9   # ~3/4 of tokens start a word
    assert tokens_for_words(100) == 134 and tokens_for_words(1000) == 1334


@pytest.mark.parametrize("name", ["tiny-gemma:2b", "tiny-phi3:3.8b", "tiny-qwen2:7b"])
def test_reference_model_is_causal(name):
    cfg = TINY[name]
    m = ReferenceModel(random_weights(cfg, seed=1))
    t = torch.randint(0, cfg.vocab, (1, 9))
    full = m.forward(t)
    prefix = m.forward(t[:, :5])
    assert torch.allclose(full[:, :5], prefix, atol=1e-4)


def test_torch_engine_generate_and_options():
    eng = DecodeEngine("tiny-llama3.1:8b", device="cpu")
    r = eng.generate(["In 10 words, please give me information about India", "hi"], [5, 3],
                     [dict(temperature=0.0), dict(temperature=0.8, seed=3)])
    assert [x.eval_count for x in r] == [5, 3]
    j = r[0].ollama_json()
    assert j["eval_count"] == 5 and j["prompt_eval_count"] == len(r[0].prompt_tokens) and j["done"]
    r2 = eng.generate(["hi"], 3, [dict(temperature=0.8, seed=3)])
    assert r2[0].tokens == r[1].tokens  # seeded sampling is reproducible


def test_sample_host_pipeline():
    rng = np.random.default_rng(0)
    logits = torch.tensor([0.0, 5.0, 4.9, -1.0])
    o = dict(temperature=0.0, top_k=40, top_p=0.9, repeat_penalty=1.1, repeat_last_n=64)
    assert sample_host(logits, [], o, rng) == 1
    assert sample_host(logits, [1], o, rng) == 2  # repeat penalty demotes the recent token
    o.update(temperature=1.0, top_k=1)
    assert sample_host(logits, [], o, rng) == 1


@pytest.mark.parametrize("name", ["tiny-gemma:2b", "tiny-qwen2:7b", "tiny-llama3.1:8b"])
def test_reference_model_kv_cache_matches_full_forward(name):
    cfg = TINY[name]
    m = ReferenceModel(random_weights(cfg, seed=1), memo_weights=True)
    t = torch.randint(0, cfg.vocab, (1, 12))
    full = m.forward(t)
    cache: list = []
    inc = torch.cat([m.forward(t[:, :7], cache=cache), m.forward(t[:, 7:9], cache=cache),
                     m.forward(t[:, 9:], cache=cache)], 1)
    assert torch.allclose(inc, full, atol=1e-4)
    assert len(cache) == cfg.n_layers and cache[0][0].shape[1] == 12


def test_attention_split_rule(monkeypatch):
    """engine.attention_splits: few (row, kv head) pairs split over positions (<= 8, >= 4 blocks of 32 per split at
    full context); a single pair (gemma:2b's MQA at batch 1) takes up to 16 splits of >= 3 blocks; many pairs fill
    ~256 workgroups; the A/B overrides apply."""
    from cain_amd.engine.engine import attention_splits

    monkeypatch.delenv("CAIN_ATTN_FEW_SPLITS", raising=False)
    monkeypatch.delenv("CAIN_ATTN_MIN_BLOCKS", raising=False)
    assert attention_splits(1, 1, 1536) == 16   # gemma:2b, one row
    assert attention_splits(1, 2, 1536) == 8    # qwen2:1.5b
    assert attention_splits(1, 8, 1536) == 8    # llama3.1:8b
    assert attention_splits(1, 32, 1536) == 2   # phi3:3.8b (MHA: 32 pairs)
    assert attention_splits(1, 1, 512) == 5     # short context: >= 3 blocks per split
    assert attention_splits(256, 8, 1536) == 1  # the headline's 2,048 pairs
    monkeypatch.setenv("CAIN_ATTN_FEW_SPLITS", "4")
    assert attention_splits(1, 1, 1536) == 4 and attention_splits(1, 8, 1536) == 4
