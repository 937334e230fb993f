"""Hugging Face checkpoints (models/hf.py) on CPU: config mapping, loading, and the torch oracle's logits on a loaded
checkpoint against transformers' own model classes -- an implementation independent of this repository's, per
study family (Llama 3.1 with its RoPE scaling, Mistral, Qwen2 with QKV biases and a tied head, Gemma with its
(1 + w) gains, sqrt(d) scale and GeGLU, Phi-3 with fused qkv / gate_up)."""
import dataclasses

import pytest
import torch

from hf_fixtures import FAMILIES, hf_logits, make_checkpoint, write_tokenizer

from cain_amd.engine import DecodeEngine
from cain_amd.models import MODELS, get_config
from cain_amd.models.hf import config_from_hf, load_hf_weights, load_pretrained, registered_checkpoints
from cain_amd.models.reference import ReferenceModel

pytest.importorskip("transformers")


@pytest.mark.parametrize("family", sorted(FAMILIES))
def test_oracle_matches_transformers_on_a_loaded_checkpoint(family, tmp_path):
    model = make_checkpoint(family, tmp_path, scale=4.0)
    cfg, mw, tok = load_pretrained(tmp_path, dtype=torch.float32)
    assert tok is None
    assert cfg.n_layers == 2 and cfg.vocab == 1024
    g = torch.Generator().manual_seed(3)
    tokens = torch.randint(3, 1024, (2, 12), generator=g)
    # positions past Llama 3.1's low-frequency wavelength bound, so its RoPE scaling changes the rotations
    positions = (torch.arange(12) + (3000 if family == "llama" else 0)).expand(2, 12)
    ours = ReferenceModel(mw).forward(tokens, positions=positions)
    theirs = hf_logits(model, tokens, positions)
    err = float((ours - theirs).abs().max() / theirs.abs().max())
    assert theirs.abs().max() > 0.5, "logits too small to compare"
    # transformers forms the RoPE angle pos * inv_freq in fp32 (the oracle in fp64): ~2e-4 rad of angle at
    # position 3,000, 5e-5 of the logits here; at positions 0-11 the llama error is 1e-6
    tol = 1e-4 if family == "llama" else 2e-5
    assert err < tol, f"{family}: max relative logit error {err:.2e}"
    if family == "llama":  # negative control: the same checkpoint without the Llama-3 scaling is 100x further off
        unscaled = dataclasses.replace(mw, cfg=dataclasses.replace(cfg, rope_scaling=None))
        off = ReferenceModel(unscaled).forward(tokens, positions=positions)
        assert float((off - theirs).abs().max() / theirs.abs().max()) > 1e-3


def test_gemma_checkpoint_keeps_the_stored_gain_convention(tmp_path):
    make_checkpoint("gemma", tmp_path)
    cfg, mw, _ = load_pretrained(tmp_path, dtype=torch.float32)
    assert cfg.norm_add_one and cfg.embed_scale and cfg.act == "gelu_tanh" and cfg.tie_embeddings
    assert abs(float(mw.layers[0].attn_norm.mean())) < 0.2  # w of (1 + w), not 1 + w
    assert mw.lm_head is mw.embed


def test_phi3_fused_projections_are_split_gate_first(tmp_path):
    model = make_checkpoint("phi3", tmp_path)
    _, mw, _ = load_pretrained(tmp_path, dtype=torch.float32)
    gu = model.model.layers[1].mlp.gate_up_proj.weight
    assert torch.equal(mw.layers[1].w_gate, gu[:512]) and torch.equal(mw.layers[1].w_up, gu[512:])
    assert torch.equal(mw.layers[1].wqkv, model.model.layers[1].self_attn.qkv_proj.weight)


def test_qwen2_biases_and_tied_head(tmp_path):
    model = make_checkpoint("qwen2", tmp_path)
    cfg, mw, _ = load_pretrained(tmp_path, dtype=torch.float32)
    assert cfg.qkv_bias and cfg.tie_embeddings
    a = model.model.layers[0].self_attn
    assert torch.equal(mw.layers[0].bqkv, torch.cat([a.q_proj.bias, a.k_proj.bias, a.v_proj.bias]))


def test_bf16_load_is_the_checkpoint_rounded_once(tmp_path):
    make_checkpoint("llama", tmp_path)
    _, m32, _ = load_pretrained(tmp_path, dtype=torch.float32)
    _, m16, _ = load_pretrained(tmp_path)
    assert m16.layers[0].wqkv.dtype == torch.bfloat16
    assert torch.equal(m16.layers[0].wqkv, m32.layers[0].wqkv.to(torch.bfloat16))


def test_sharded_checkpoint_loads(tmp_path):
    """A multi-shard checkpoint (model.safetensors.index.json), as the 7-8 B models are published."""
    import transformers

    make_checkpoint("mistral", tmp_path / "one")
    model = transformers.MistralForCausalLM.from_pretrained(str(tmp_path / "one"))
    model.save_pretrained(str(tmp_path / "sharded"), max_shard_size="200KB")
    assert (tmp_path / "sharded" / "model.safetensors.index.json").exists()
    a = load_hf_weights(tmp_path / "one", dtype=torch.float32)
    b = load_hf_weights(tmp_path / "sharded", dtype=torch.float32)
    for la, lb in zip(a.layers, b.layers):
        assert torch.equal(la.wqkv, lb.wqkv) and torch.equal(la.w_down, lb.w_down)


# public config.json fields of the study's checkpoints (architecture fields only)
PUBLIC = {
    "llama3.1:8b": dict(model_type="llama", hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                        num_attention_heads=32, num_key_value_heads=8, vocab_size=128256, rms_norm_eps=1e-5,
                        rope_theta=500000.0, max_position_embeddings=131072, tie_word_embeddings=False,
                        rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                      "high_freq_factor": 4.0, "original_max_position_embeddings": 8192},
                        bos_token_id=128000, eos_token_id=[128001, 128008, 128009], hidden_act="silu"),
    "qwen2:1.5b": dict(model_type="qwen2", hidden_size=1536, intermediate_size=8960, num_hidden_layers=28,
                       num_attention_heads=12, num_key_value_heads=2, vocab_size=151936, rms_norm_eps=1e-6,
                       rope_theta=1e6, max_position_embeddings=32768, tie_word_embeddings=True,
                       sliding_window=32768, use_sliding_window=False, hidden_act="silu"),
    "qwen2:7b": dict(model_type="qwen2", hidden_size=3584, intermediate_size=18944, num_hidden_layers=28,
                     num_attention_heads=28, num_key_value_heads=4, vocab_size=152064, rms_norm_eps=1e-6,
                     rope_theta=1e6, max_position_embeddings=32768, tie_word_embeddings=False,
                     sliding_window=131072, use_sliding_window=False, hidden_act="silu"),
    "gemma:2b": dict(model_type="gemma", hidden_size=2048, intermediate_size=16384, num_hidden_layers=18,
                     num_attention_heads=8, num_key_value_heads=1, head_dim=256, vocab_size=256000,
                     rms_norm_eps=1e-6, rope_theta=10000.0, max_position_embeddings=8192, hidden_act="gelu",
                     hidden_activation="gelu_pytorch_tanh"),
    "gemma:7b": dict(model_type="gemma", hidden_size=3072, intermediate_size=24576, num_hidden_layers=28,
                     num_attention_heads=16, num_key_value_heads=16, head_dim=256, vocab_size=256000,
                     rms_norm_eps=1e-6, rope_theta=10000.0, max_position_embeddings=8192, hidden_act="gelu"),
    "phi3:3.8b": dict(model_type="phi3", hidden_size=3072, intermediate_size=8192, num_hidden_layers=32,
                      num_attention_heads=32, num_key_value_heads=32, vocab_size=32064, rms_norm_eps=1e-5,
                      rope_theta=10000.0, rope_scaling=None, max_position_embeddings=4096, sliding_window=2047,
                      tie_word_embeddings=False, hidden_act="silu"),
    "mistral:7b": dict(model_type="mistral", hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                       num_attention_heads=32, num_key_value_heads=8, vocab_size=32768, rms_norm_eps=1e-5,
                       rope_theta=1e6, max_position_embeddings=32768, sliding_window=None, hidden_act="silu"),
}
ARCH_FIELDS = ("n_layers", "d_model", "n_heads", "n_kv_heads", "head_dim", "ffn", "vocab", "act", "tie_embeddings",
               "qkv_bias", "rope_theta", "rope_scaling", "norm_eps", "norm_add_one", "embed_scale")


@pytest.mark.parametrize("tag", sorted(PUBLIC))
def test_builtin_configs_match_the_public_checkpoints(tag):
    """The random-init zoo (config.MODELS) has the architecture the published config.json describes."""
    got = config_from_hf(PUBLIC[tag], name=tag)
    want = MODELS[tag]
    for f in ARCH_FIELDS:
        assert getattr(got, f) == getattr(want, f), (tag, f, getattr(got, f), getattr(want, f))
    assert got.n_params() == want.n_params()


def test_phi3_window_caps_the_context():
    assert config_from_hf(PUBLIC["phi3:3.8b"]).max_context == 2047
    assert config_from_hf(PUBLIC["qwen2:7b"]).max_context == 32768  # use_sliding_window false


@pytest.mark.parametrize("rope, msg", [({"rope_type": "yarn", "factor": 4.0}, "yarn"),
                                       ({"rope_type": "longrope"}, "longrope"),
                                       ({"rope_type": "default", "partial_rotary_factor": 0.5}, "partial")])
def test_unsupported_rope_is_refused(rope, msg):
    hf = dict(PUBLIC["mistral:7b"], rope_scaling=rope)
    with pytest.raises(NotImplementedError, match=msg):
        config_from_hf(hf)


def test_unsupported_architecture_is_refused():
    with pytest.raises(ValueError, match="unsupported architecture"):
        config_from_hf(dict(PUBLIC["mistral:7b"], model_type="gpt2", architectures=["GPT2LMHeadModel"]))


def test_tokenizer_json_is_used_with_its_bos_template(tmp_path):
    make_checkpoint("llama", tmp_path)
    write_tokenizer(tmp_path)
    cfg, mw, tok = load_pretrained(tmp_path)
    ids = tok.encode("w5 w7 w9")
    assert ids == [1, 8, 10, 12]
    assert tok.encode("w5", add_bos=False) == [8]
    assert tok.decode(ids) == "w5 w7 w9"
    assert tok.piece(8) == "w5"


def test_registered_checkpoint_drives_tag_engines(tmp_path, monkeypatch):
    """CAIN_CHECKPOINTS="tag=path": get_config and DecodeEngine(tag) (hence the server, study and bench) use the
    checkpoint; the CPU engine's greedy tokens follow transformers' greedy decode on it."""
    model = make_checkpoint("qwen2", tmp_path / "ck", scale=4.0)
    write_tokenizer(tmp_path / "ck")
    monkeypatch.setenv("CAIN_CHECKPOINTS", f"my-qwen:tiny={tmp_path / 'ck'}")
    assert registered_checkpoints() == {"my-qwen:tiny": str(tmp_path / "ck")}
    cfg = get_config("my-qwen:tiny")
    assert (cfg.d_model, cfg.n_heads, cfg.head_dim, cfg.qkv_bias, cfg.tie_embeddings) == (384, 6, 128, True, True)
    eng = DecodeEngine("my-qwen:tiny", device="cpu", max_batch=1, max_context=64)
    assert eng.cfg.name == "my-qwen:tiny"
    prompt = "w10 w20 w30 w40"
    ids = eng.encode(prompt)
    assert ids[0] == 1 and len(ids) == 5
    res = eng.generate([prompt], 6, [dict(temperature=0.0, eos_id=-1)])[0]
    with torch.no_grad():
        hf = model.generate(torch.tensor([ids]), max_new_tokens=6, do_sample=False, eos_token_id=None,
                            pad_token_id=0)[0, len(ids):].tolist()
    assert res.tokens == hf
    assert res.text == eng.tokenizer.decode(hf)


def test_from_pretrained_engine(tmp_path):
    make_checkpoint("gemma", tmp_path)
    eng = DecodeEngine.from_pretrained(str(tmp_path), device="cpu", max_batch=2, max_context=64, name="g")
    assert eng.cfg.name == "g" and eng.cfg.norm_add_one
    out = eng.generate(["a", "b"], 3, [dict(temperature=0.0, eos_id=-1)] * 2)
    assert [len(r.tokens) for r in out] == [3, 3]


def test_bad_registration_is_an_error(monkeypatch):
    monkeypatch.setenv("CAIN_CHECKPOINTS", "no-path-here")
    with pytest.raises(ValueError, match="tag=/path"):
        registered_checkpoints()


def test_server_serves_a_checkpoint(tmp_path, monkeypatch):
    """``serve --checkpoint TAG=PATH``: the Ollama-compatible server lists, describes and decodes the checkpoint
    (greedy tokens = transformers' greedy decode; response text from its tokenizer.json)."""
    import http.client
    import json

    from cain_amd.client import OllamaClient
    from cain_amd.serve import EngineBackend, ServerThread
    from cain_amd.serve.server import register_checkpoints

    monkeypatch.setenv("CAIN_CHECKPOINTS", "")  # restored after the test (register_checkpoints writes it)
    model = make_checkpoint("gemma", tmp_path / "g", scale=4.0)
    write_tokenizer(tmp_path / "g", bos_token="<bos>")
    assert register_checkpoints([f"gemma-real:2b={tmp_path / 'g'}"]) == ["gemma-real:2b"]
    be = EngineBackend(["gemma-real:2b"], device="cpu", max_batch=2, max_context=64)
    with ServerThread(be) as s:
        c = OllamaClient(s.url)
        assert c.tags() == ["gemma-real:2b"]
        host, port = s.url.split("//")[1].split(":")
        conn = http.client.HTTPConnection(host, int(port))
        conn.request("POST", "/api/show", body=json.dumps({"model": "gemma-real:2b"}))
        info = json.loads(conn.getresponse().read())
        conn.close()
        assert info["model_info"]["checkpoint"] == str(tmp_path / "g")
        assert info["model_info"]["head_dim"] == 256
        assert info["template"] == "" and 'stop "</s>"' in info["parameters"]  # eos 2 = </s>
        r = c.generate("gemma-real:2b", "w3 w4 w5", options={"temperature": 0, "num_predict": 5})
    ids = be.engine("gemma-real:2b").encode("w3 w4 w5")
    with torch.no_grad():
        want = model.generate(torch.tensor([ids]), max_new_tokens=5, do_sample=False, eos_token_id=None,
                              pad_token_id=0)[0, len(ids):].tolist()
    assert r.eval_count == 5
    assert r.text == be.engine("gemma-real:2b").tokenizer.decode(want)


def test_chat_template_renders_like_transformers_and_the_server_applies_it(tmp_path, monkeypatch):
    """Ollama wraps /api/generate prompts in the model's template (unless raw) and /api/chat messages always: the
    checkpoint's tokenizer_config.json template renders as transformers' apply_chat_template does, and the server
    decodes the templated ids (greedy tokens = transformers' generate on them)."""
    from hf_fixtures import CHAT_TEMPLATE
    from transformers import PreTrainedTokenizerFast

    from cain_amd.client import OllamaClient
    from cain_amd.serve import EngineBackend, ServerThread

    model = make_checkpoint("llama", tmp_path / "ck", scale=4.0)
    write_tokenizer(tmp_path / "ck", chat=True)
    _, _, tok = load_pretrained(tmp_path / "ck")
    assert tok.chat_template == CHAT_TEMPLATE
    msgs = [{"role": "system", "content": "w7 w8"}, {"role": "user", "content": "w3 w4 w5"}]
    ref = PreTrainedTokenizerFast(tokenizer_file=str(tmp_path / "ck" / "tokenizer.json"), bos_token="<s>",
                                  eos_token="</s>", chat_template=CHAT_TEMPLATE)
    assert tok.render_chat(msgs) == ref.apply_chat_template(msgs, tokenize=False, add_generation_prompt=True)
    ids = tok.encode(tok.render_chat(msgs), add_bos=False)
    assert ids == ref.apply_chat_template(msgs, tokenize=True, add_generation_prompt=True, return_dict=False)
    assert ids[0] == 1 and ids.count(1) == 1  # one BOS: the template's

    monkeypatch.setenv("CAIN_CHECKPOINTS", f"llama-chat:tiny={tmp_path / 'ck'}")
    be = EngineBackend(["llama-chat:tiny"], device="cpu", max_batch=2, max_context=64)
    with ServerThread(be) as s:
        c = OllamaClient(s.url)
        r = c.generate("llama-chat:tiny", "w3 w4 w5", options={"temperature": 0, "num_predict": 4}, system="w7 w8")
        raw = c.generate("llama-chat:tiny", "w3 w4 w5", options={"temperature": 0, "num_predict": 4}, raw=True)
        chat = c.chat("llama-chat:tiny", msgs, options={"temperature": 0, "num_predict": 4})
    assert r.prompt_eval_count == len(ids) and chat.prompt_eval_count == len(ids)
    assert chat.text == r.text
    with torch.no_grad():
        want = model.generate(torch.tensor([ids]), max_new_tokens=4, do_sample=False, eos_token_id=None,
                              pad_token_id=0)[0, len(ids):].tolist()
    assert r.text == tok.decode(want)
    assert raw.prompt_eval_count == len(tok.encode("w3 w4 w5"))  # raw: the prompt as given, BOS from the file


def test_stop_ids_from_generation_config_and_template_tokens(tmp_path, monkeypatch):
    """A checkpoint's other end ids (generation_config.json) and its tokenizer's turn-end tokens become stop ids;
    a generation ends on them ("stop"), unless the caller forces the length (eos_id -1, as the study and bench do)."""
    import json

    from cain_amd.models.hf import checkpoint_config

    make_checkpoint("mistral", tmp_path, scale=4.0)
    write_tokenizer(tmp_path, chat=True)
    tj = json.loads((tmp_path / "tokenizer.json").read_text())
    tj["added_tokens"].append({"id": 40, "content": "<|eot_id|>", "single_word": False, "lstrip": False,
                               "rstrip": False, "normalized": False, "special": True})
    tj["model"]["vocab"] = {("<|eot_id|>" if i == 40 else w): i for w, i in tj["model"]["vocab"].items()}
    (tmp_path / "tokenizer.json").write_text(json.dumps(tj))
    (tmp_path / "generation_config.json").write_text(json.dumps({"eos_token_id": [2, 33]}))
    cfg = checkpoint_config(tmp_path, name="m")
    assert cfg.eos_id == 2 and cfg.stop_ids == (33, 40)
    eng = DecodeEngine.from_pretrained(str(tmp_path), device="cpu", max_batch=1, max_context=64)
    assert eng.cfg.stop_ids == (33, 40)
    free = eng.generate(["w5 w6"], 8, [dict(temperature=0.0, eos_id=-1)])[0]
    assert len(free.tokens) == 8 and free.done_reason == "length"
    k = 3
    stop_at = free.tokens[k]
    first = free.tokens.index(stop_at)
    got = eng.generate(["w5 w6"], 8, [dict(temperature=0.0, eos_id=-1, stop_ids=[stop_at])])[0]
    assert got.tokens == free.tokens[:first + 1] and got.done_reason == "stop"


def test_stream_decoder_holds_split_characters():
    """Streamed pieces concatenate to the full decode, also when a character's UTF-8 bytes span tokens (a byte-level
    vocabulary of single bytes here), and for the synthetic tokenizer (its decode strips the first space)."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers

    from cain_amd.models.tokenizer import HFTokenizer, StreamDecoder, SyntheticTokenizer

    alphabet = pre_tokenizers.ByteLevel.alphabet()
    tok = Tokenizer(models.BPE({c: i for i, c in enumerate(sorted(alphabet))}, []))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    t = HFTokenizer.from_tokenizer(tok)
    text = "energy é 世界 ok"
    ids = t.encode(text, add_bos=False)
    assert len(ids) == len(text.encode("utf-8"))  # one token per byte: 世 and 界 span three tokens each
    d = StreamDecoder(t)
    pieces = [d.push([i]) for i in ids]
    assert "".join(pieces) == text and all("�" not in p for p in pieces)
    assert pieces[0] == "e"
    syn = SyntheticTokenizer(1024)
    sd = StreamDecoder(syn)
    gen = [17, 18, 19, 20, 21, 22]
    assert "".join(sd.push(gen[i:i + 2]) for i in range(0, 6, 2)) + sd.flush() == syn.decode(gen)
    # a length cutoff inside a character: the held-back bytes come out at flush, and the stream equals the response
    cut = ids[:ids.index(t.encode("世", add_bos=False)[0]) + 2]
    d2 = StreamDecoder(t)
    pieces = [d2.push([i]) for i in cut]
    assert "".join(pieces) + d2.flush() == t.decode(cut)
    # each push decodes a window from the previous chunk's start, not the whole sequence
    seen = []
    orig = t.decode
    t.decode = lambda x: seen.append(len(x)) or orig(x)
    d3 = StreamDecoder(t)
    out = "".join(d3.push([i]) for i in ids) + d3.flush()
    t.decode = orig
    assert out == text and max(seen) <= 8 < len(ids)


def test_streamed_response_concatenates_to_the_final_text(tmp_path, monkeypatch):
    """/api/generate with stream: the NDJSON pieces join to the same text the non-streamed response carries."""
    from cain_amd.client import OllamaClient
    from cain_amd.serve import EngineBackend, ServerThread

    make_checkpoint("qwen2", tmp_path / "ck", scale=4.0)
    write_tokenizer(tmp_path / "ck")
    monkeypatch.setenv("CAIN_CHECKPOINTS", f"q:tiny={tmp_path / 'ck'}")
    be = EngineBackend(["q:tiny"], device="cpu", max_batch=2, max_context=64)
    with ServerThread(be) as s:
        c = OllamaClient(s.url)
        pieces = []
        st = c.generate("q:tiny", "w3 w4", stream=True, options={"temperature": 0, "num_predict": 6},
                        on_chunk=pieces.append)
        full = c.generate("q:tiny", "w3 w4", options={"temperature": 0, "num_predict": 6})
    assert st.eval_count == 6 and "".join(pieces) == full.text


def test_template_errors_are_http_400(tmp_path, monkeypatch):
    """A chat template that raises (raise_exception, as real templates do on unsupported roles) is the request's
    error (HTTP 400 with Ollama's {"error": ...}), not a server failure."""
    import json

    from cain_amd.client import OllamaClient, OllamaError
    from cain_amd.serve import EngineBackend, ServerThread

    make_checkpoint("gemma", tmp_path / "ck")
    write_tokenizer(tmp_path / "ck", chat=True)
    conf = json.loads((tmp_path / "ck" / "tokenizer_config.json").read_text())
    conf["chat_template"] = ("{% for m in messages %}{% if m['role'] == 'system' %}"
                             "{{ raise_exception('System role not supported') }}{% endif %}{{ m['content'] }}{% endfor %}")
    (tmp_path / "ck" / "tokenizer_config.json").write_text(json.dumps(conf))
    monkeypatch.setenv("CAIN_CHECKPOINTS", f"g:tiny={tmp_path / 'ck'}")
    be = EngineBackend(["g:tiny"], device="cpu", max_batch=1, max_context=64)
    with ServerThread(be) as s:
        c = OllamaClient(s.url)
        with pytest.raises(OllamaError, match="System role not supported"):
            c.generate("g:tiny", "w3", system="w4", options={"num_predict": 2})
        assert c.generate("g:tiny", "w3", options={"temperature": 0, "num_predict": 2}).eval_count == 2
