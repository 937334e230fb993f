"""GGUF files (models/gguf.py) on CPU.

* Block decoders: every quantised type against a per-element scalar decoder written from ggml's reference loops
  (``dequantize_row_*``), on random blocks; Q8_0 / Q4_0 also through this module's quantisers.  No independent GGUF
  implementation is importable here, so these pin the vectorisation, not the format against llama.cpp (parity
  unpinned, documented in gguf.py).
* Conventions: the q / k un-permutation against transformers' own GGUF processor; Gemma's stored 1 + w.
* End to end, per family: a transformers checkpoint written as GGUF with llama.cpp's conventions (``export_gguf``)
  and read back gives the oracle logits transformers computes on the original checkpoint.
"""
import dataclasses

import numpy as np
import pytest
import torch

from hf_fixtures import FAMILIES, hf_logits, make_checkpoint

from cain_amd.engine import DecodeEngine
from cain_amd.models.gguf import (GGML_TYPES, TYPE_ID, GGUFFile, dequantize, export_gguf, load_gguf, permute_qk,
                                  quantize_q4_0, quantize_q8_0, unpermute_qk, write_gguf)
from cain_amd.models.hf import load_pretrained
from cain_amd.models.reference import ReferenceModel

pytest.importorskip("transformers")
GGUF_ARCH = {"llama": "llama", "mistral": "llama", "qwen2": "qwen2", "gemma": "gemma", "phi3": "phi3"}


# ------------------------------------------------------------------ scalar reference decoders (ggml loop order)
def _h(b, i):
    return float(np.frombuffer(bytes(b[i:i + 2]), np.float16)[0])


def _scale_min_k4(j, q):
    if j < 4:
        return q[j] & 63, q[j + 4] & 63
    return (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4), (q[j + 4] >> 4) | ((q[j] >> 6) << 4)


def ref_block(name, b):
    b = [int(x) for x in b]
    y = [0.0] * GGML_TYPES[TYPE_ID[name]][1]
    if name in ("Q4_0", "Q4_1"):
        d = _h(b, 0)
        m = _h(b, 2) if name == "Q4_1" else 0.0
        qs = b[4:] if name == "Q4_1" else b[2:]
        off = 0 if name == "Q4_1" else 8
        for j in range(16):
            y[j] = ((qs[j] & 0xF) - off) * d + m
            y[j + 16] = ((qs[j] >> 4) - off) * d + m
    elif name in ("Q5_0", "Q5_1"):
        d = _h(b, 0)
        m = _h(b, 2) if name == "Q5_1" else 0.0
        p = 4 if name == "Q5_1" else 2
        qh = int.from_bytes(bytes(b[p:p + 4]), "little")
        qs = b[p + 4:]
        off = 0 if name == "Q5_1" else 16
        for j in range(16):
            xh0 = ((qh >> j) << 4) & 0x10
            xh1 = (qh >> (j + 12)) & 0x10
            y[j] = (((qs[j] & 0xF) | xh0) - off) * d + m
            y[j + 16] = (((qs[j] >> 4) | xh1) - off) * d + m
    elif name == "Q8_0":
        d = _h(b, 0)
        for j in range(32):
            y[j] = d * (b[2 + j] - 256 if b[2 + j] > 127 else b[2 + j])
    elif name in ("Q4_K", "Q5_K"):
        d, dmin, sc = _h(b, 0), _h(b, 2), b[4:16]
        qh = b[16:48] if name == "Q5_K" else None
        ql = b[48:176] if name == "Q5_K" else b[16:144]
        u1, u2, is_, yi, qi = 1, 2, 0, 0, 0
        for _ in range(4):
            s1, m1 = _scale_min_k4(is_, sc)
            s2, m2 = _scale_min_k4(is_ + 1, sc)
            for l in range(32):
                h = (16 if qh[l] & u1 else 0) if qh else 0
                y[yi + l] = d * s1 * ((ql[qi + l] & 0xF) + h) - dmin * m1
            for l in range(32):
                h = (16 if qh[l] & u2 else 0) if qh else 0
                y[yi + 32 + l] = d * s2 * ((ql[qi + l] >> 4) + h) - dmin * m2
            qi += 32
            yi += 64
            is_ += 2
            u1 <<= 2
            u2 <<= 2
    elif name == "Q2_K":
        sc, qs = b[0:16], b[16:80]
        d, dmin = _h(b, 80), _h(b, 82)
        is_, yi = 0, 0
        for n in range(2):
            q = qs[32 * n: 32 * n + 32]
            for j in range(4):
                shift = 2 * j
                for half16 in range(2):
                    s = sc[is_]
                    is_ += 1
                    for l in range(16):
                        y[yi + 16 * half16 + l] = d * (s & 0xF) * ((q[16 * half16 + l] >> shift) & 3) - dmin * (s >> 4)
                yi += 32
    elif name == "Q3_K":
        hm, qs, raw = b[0:32], b[32:96], b[96:108]
        d = _h(b, 108)
        aux = [int.from_bytes(bytes(raw[4 * i:4 * i + 4]), "little") for i in range(3)]
        k1, k2, tmp = 0x03030303, 0x0F0F0F0F, aux[2]
        aux = [(aux[0] & k2) | (((tmp >> 0) & k1) << 4), (aux[1] & k2) | (((tmp >> 2) & k1) << 4),
               ((aux[0] >> 4) & k2) | (((tmp >> 4) & k1) << 4), ((aux[1] >> 4) & k2) | (((tmp >> 6) & k1) << 4)]
        scales = [((a >> (8 * i)) & 0xFF) for a in aux for i in range(4)]
        m, is_, yi = 1, 0, 0
        for n in range(2):
            q = qs[32 * n: 32 * n + 32]
            shift = 0
            for j in range(4):
                for half16 in range(2):
                    dl = d * (scales[is_] - 32)
                    is_ += 1
                    for l in range(16):
                        ll = 16 * half16 + l
                        y[yi + ll] = dl * (((q[ll] >> shift) & 3) - (0 if hm[ll] & m else 4))
                yi += 32
                shift += 2
                m <<= 1
    elif name == "Q6_K":
        ql, qh = b[0:128], b[128:192]
        sc = [x - 256 if x > 127 else x for x in b[192:208]]
        d = _h(b, 208)
        for n in range(2):
            for l in range(32):
                is_ = l // 16
                q1 = ((ql[64 * n + l] & 0xF) | (((qh[32 * n + l] >> 0) & 3) << 4)) - 32
                q2 = ((ql[64 * n + l + 32] & 0xF) | (((qh[32 * n + l] >> 2) & 3) << 4)) - 32
                q3 = ((ql[64 * n + l] >> 4) | (((qh[32 * n + l] >> 4) & 3) << 4)) - 32
                q4 = ((ql[64 * n + l + 32] >> 4) | (((qh[32 * n + l] >> 6) & 3) << 4)) - 32
                y[128 * n + l] = d * sc[8 * n + is_] * q1
                y[128 * n + l + 32] = d * sc[8 * n + is_ + 2] * q2
                y[128 * n + l + 64] = d * sc[8 * n + is_ + 4] * q3
                y[128 * n + l + 96] = d * sc[8 * n + is_ + 6] * q4
    return np.array(y, np.float32)


def _random_blocks(name, n, seed=0):
    rng = np.random.default_rng(seed)
    _, bs, bb = GGML_TYPES[TYPE_ID[name]]
    raw = rng.integers(0, 256, (n, bb), dtype=np.uint8)
    fp16_at = {"Q6_K": [208], "Q2_K": [80, 82], "Q3_K": [108]}.get(
        name, [0, 2] if name in ("Q4_1", "Q5_1", "Q4_K", "Q5_K") else [0])
    for p in fp16_at:  # finite, moderate half-precision scales
        raw[:, p:p + 2] = np.frombuffer(rng.uniform(-2, 2, n).astype(np.float16).tobytes(), np.uint8).reshape(n, 2)
    return raw


@pytest.mark.parametrize("name", ["Q4_0", "Q4_1", "Q5_0", "Q5_1", "Q8_0", "Q2_K", "Q3_K", "Q4_K", "Q5_K", "Q6_K"])
def test_block_decoders_match_the_scalar_reference(name):
    raw = _random_blocks(name, 6)
    bs = GGML_TYPES[TYPE_ID[name]][1]
    got = dequantize(raw.reshape(-1), TYPE_ID[name], 6 * bs).numpy().reshape(6, bs)
    for i in range(6):
        np.testing.assert_allclose(got[i], ref_block(name, raw[i]), rtol=1e-6, atol=1e-6, err_msg=name)


def test_q8_0_and_q4_0_round_trip():
    x = np.random.default_rng(1).normal(0, 1, 32 * 64).astype(np.float32)
    y8 = dequantize(quantize_q8_0(x), TYPE_ID["Q8_0"], x.size).numpy()
    y4 = dequantize(quantize_q4_0(x), TYPE_ID["Q4_0"], x.size).numpy()
    amax = np.abs(x.reshape(-1, 32)).max(1, keepdims=True)
    assert np.all(np.abs(y8 - x).reshape(-1, 32) <= amax / 127 * 0.5 + 1e-3 * amax)
    # Q4_0's 16 levels run -8 d .. 7 d around the signed maximum: half a step inside, one step at the far end
    assert np.all(np.abs(y4 - x).reshape(-1, 32) <= amax / 8 + 1e-3 * amax)
    # the block's largest-magnitude element is exact up to the fp16 scale (Q4_0 maps it to -8 * d)
    i = np.abs(x.reshape(-1, 32)).argmax(1)
    np.testing.assert_allclose(y4.reshape(-1, 32)[np.arange(64), i], x.reshape(-1, 32)[np.arange(64), i], rtol=1e-3)


def test_container_round_trip(tmp_path):
    rng = np.random.default_rng(2)
    a = rng.normal(0, 1, (64, 96)).astype(np.float32)
    meta = {"general.architecture": "llama", "general.name": "t", "x.int": 7, "x.big": 2 ** 40, "x.neg": -3,
            "x.float": 0.5, "x.bool": True, "x.strs": ["a", "bb", ""], "x.ints": [1, -2, 3], "x.floats": [0.25, 1.5]}
    T = {"f32": (a, "F32"), "f16": (a, "F16"), "bf16": (a, "BF16"), "q8": (a, "Q8_0"), "q4": (a, "Q4_0"),
         "vec": (a[0], "F32")}
    write_gguf(tmp_path / "t.gguf", meta, T)
    g = GGUFFile(tmp_path / "t.gguf")
    for k, v in meta.items():
        assert g.metadata[k] == v, k
    assert g.version == 3 and g.tensors["q8"].shape == (64, 96) and g.tensors["vec"].shape == (96,)
    at = torch.from_numpy(a)
    assert torch.equal(g.tensor("f32"), at)
    assert torch.equal(g.tensor("f16"), at.half().float())
    assert torch.equal(g.tensor("bf16"), at.bfloat16().float())
    assert torch.equal(g.tensor("q8"), dequantize(quantize_q8_0(a), TYPE_ID["Q8_0"], a.size).reshape(a.shape))
    assert float((g.tensor("q4") - at).abs().max()) < 0.6
    with pytest.raises(NotImplementedError):  # an IQ type
        dequantize(np.zeros(64, np.uint8), 16, 256)


def test_tensor_slices_cover_block_boundaries(tmp_path, monkeypatch):
    """GGUFFile.tensor dequantises in slices of whole blocks: the slices join exactly."""
    import cain_amd.models.gguf as G

    a = np.random.default_rng(3).normal(0, 1, (40, 512)).astype(np.float32)
    write_gguf(tmp_path / "s.gguf", {"general.architecture": "llama"}, {"k": (a, "Q4_0"), "f": (a, "F16")})
    whole = GGUFFile(tmp_path / "s.gguf")
    ref_k, ref_f = whole.tensor("k"), whole.tensor("f")
    monkeypatch.setattr(G, "SLICE_ELEMS", 1000)  # not a multiple of the 32-element block or of a row
    assert torch.equal(GGUFFile(tmp_path / "s.gguf").tensor("k"), ref_k)
    assert torch.equal(GGUFFile(tmp_path / "s.gguf").tensor("f"), ref_f)


def test_qk_permutation_matches_transformers():
    from transformers.modeling_gguf_pytorch_utils import LlamaTensorProcessor

    w = torch.randn(8 * 64, 32)
    for heads in (8, 2):
        p = permute_qk(w[: heads * 64], heads)
        theirs = LlamaTensorProcessor()._reverse_permute_weights(p.numpy(), heads, heads)
        assert np.array_equal(unpermute_qk(p, heads).numpy(), theirs)
        assert torch.equal(unpermute_qk(p, heads), w[: heads * 64])
        assert not torch.equal(p, w[: heads * 64])


@pytest.mark.parametrize("family", sorted(FAMILIES))
def test_gguf_export_and_load_match_transformers(family, tmp_path):
    """HF checkpoint -> GGUF (llama.cpp conventions, F32) -> load_gguf: the oracle's logits equal transformers' on
    the original checkpoint (Llama 3.1's scaling travels as a rope_freqs tensor)."""
    model = make_checkpoint(family, tmp_path / "hf", scale=4.0)
    _, mw, _ = load_pretrained(tmp_path / "hf", dtype=torch.float32)
    export_gguf(mw, tmp_path / "m.gguf", GGUF_ARCH[family], tensor_type="F32")
    cfg, mg, tok = load_gguf(tmp_path / "m.gguf", dtype=torch.float32)
    assert tok is None and cfg.name == "m"
    assert (cfg.n_layers, cfg.d_model, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.ffn, cfg.vocab) == \
        (mw.cfg.n_layers, mw.cfg.d_model, mw.cfg.n_heads, mw.cfg.n_kv_heads, mw.cfg.head_dim, mw.cfg.ffn, mw.cfg.vocab)
    assert (cfg.tie_embeddings, cfg.qkv_bias, cfg.norm_add_one) == (mw.cfg.tie_embeddings, mw.cfg.qkv_bias,
                                                                    mw.cfg.norm_add_one)
    assert (cfg.rope_freq_factors is not None) == (family == "llama")
    assert torch.equal(mg.layers[1].wqkv, mw.layers[1].wqkv)  # un-permuted back to the checkpoint's row order
    if family == "gemma":
        raw = GGUFFile(tmp_path / "m.gguf").tensor("blk.0.attn_norm.weight")
        assert torch.allclose(raw - 1.0, mw.layers[0].attn_norm, atol=1e-6)  # stored 1 + w (transformers subtracts 1)
    tokens = torch.randint(3, 1024, (2, 10), generator=torch.Generator().manual_seed(5))
    positions = (torch.arange(10) + (3000 if family == "llama" else 0)).expand(2, 10)
    theirs = hf_logits(model, tokens, positions)
    ours = ReferenceModel(mg).forward(tokens, positions=positions)
    err = float((ours - theirs).abs().max() / theirs.abs().max())
    assert err < (1e-4 if family == "llama" else 2e-5), f"{family}: {err:.2e}"


def test_q8_0_gguf_is_close_and_engine_loads_it(tmp_path, monkeypatch):
    """A Q8_0 file through CAIN_CHECKPOINTS: get_config / DecodeEngine(tag) use it; logits near the fp32 model's."""
    model = make_checkpoint("mistral", tmp_path / "hf", scale=4.0)
    _, mw, _ = load_pretrained(tmp_path / "hf", dtype=torch.float32)
    export_gguf(mw, tmp_path / "q8.gguf", "llama", tensor_type="Q8_0")
    monkeypatch.setenv("CAIN_CHECKPOINTS", f"mistral-q8:tiny={tmp_path / 'q8.gguf'}")
    eng = DecodeEngine("mistral-q8:tiny", device="cpu", max_batch=1, max_context=64)
    assert eng.cfg.name == "mistral-q8:tiny" and eng.cfg.n_kv_heads == 1
    tokens = torch.randint(3, 1024, (1, 8), generator=torch.Generator().manual_seed(6))
    theirs = hf_logits(model, tokens, torch.arange(8)[None])[0, -1]
    ours = eng.last_logits([tokens[0].tolist()])[0]
    rel = float((ours - theirs).norm() / theirs.norm())
    assert rel < 0.03, rel


@pytest.mark.parametrize("arch", ["qwen2", "llama"])
def test_gguf_tokenizer_through_transformers_converter(arch, tmp_path):
    """A byte-level BPE vocabulary stored the GGUF way (tokens, merges; Qwen2's and Llama 3's kind) comes back as a
    working tokenizer."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    text = ["In 100 words, please give me information about India", "energy of remote and on device inference"] * 20
    tok.train_from_iterator(text, trainers.BpeTrainer(vocab_size=300, special_tokens=["<|endoftext|>"],
                                                      initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    import json
    spec = json.loads(tok.to_str())
    vocab = spec["model"]["vocab"]
    tokens = [t for t, _ in sorted(vocab.items(), key=lambda kv: kv[1])]
    merges = [m if isinstance(m, str) else " ".join(m) for m in spec["model"]["merges"]]
    model = make_checkpoint("qwen2" if arch == "qwen2" else "llama", tmp_path / "hf")
    _, mw, _ = load_pretrained(tmp_path / "hf")
    fields = {"tokenizer.ggml.model": "gpt2", "tokenizer.ggml.tokens": tokens, "tokenizer.ggml.merges": merges,
              "tokenizer.ggml.token_type": [1] * len(tokens)}
    export_gguf(mw, tmp_path / "t.gguf", arch, tokenizer_fields=fields)
    _, _, gt = load_gguf(tmp_path / "t.gguf")
    s = "please give me information about remote energy"
    ids = gt.encode(s, add_bos=False)
    assert ids == tok.encode(s).ids
    assert gt.decode(ids) == s
    # byte-level BPE files add no BOS unless tokenizer.ggml.add_bos_token says so (llama.cpp's rule; Llama-3 files
    # set it, Qwen2 files do not)
    assert gt.encode(s, add_bos=True) == ids
    fields.update({"tokenizer.ggml.bos_token_id": 0, "tokenizer.ggml.add_bos_token": True})
    export_gguf(mw, tmp_path / "b.gguf", arch, tokenizer_fields=fields)
    _, _, gb = load_gguf(tmp_path / "b.gguf")
    assert gb.encode(s, add_bos=True) == [0] + ids and gb.encode(s, add_bos=False) == ids
    del model


def test_ollama_store_blob_drives_the_tag(tmp_path, monkeypatch):
    """CAIN_CHECKPOINTS="qwen2:1.5b=ollama:<models dir>": the tag resolves through a local Ollama store (manifest ->
    model layer -> sha256 blob, a GGUF file) and the engine decodes it as transformers decodes the original."""
    import hashlib
    import json

    from cain_amd.models import get_config
    from cain_amd.models.hf import ollama_blob

    model = make_checkpoint("qwen2", tmp_path / "hf", scale=4.0)
    _, mw, _ = load_pretrained(tmp_path / "hf", dtype=torch.float32)
    store = tmp_path / "ollama"
    (store / "blobs").mkdir(parents=True)
    export_gguf(mw, tmp_path / "m.gguf", "qwen2", tensor_type="F32")
    data = (tmp_path / "m.gguf").read_bytes()
    digest = hashlib.sha256(data).hexdigest()
    (store / "blobs" / f"sha256-{digest}").write_bytes(data)
    man = store / "manifests" / "registry.ollama.ai" / "library" / "qwen2" / "1.5b"
    man.parent.mkdir(parents=True)
    man.write_text(json.dumps({"schemaVersion": 2, "layers": [
        {"mediaType": "application/vnd.ollama.image.template", "digest": "sha256:" + "0" * 64, "size": 1},
        {"mediaType": "application/vnd.ollama.image.model", "digest": f"sha256:{digest}", "size": len(data)}]}))
    assert ollama_blob("qwen2:1.5b", store) == store / "blobs" / f"sha256-{digest}"
    with pytest.raises(FileNotFoundError):
        ollama_blob("qwen2:7b", store)
    bad = store / "manifests" / "registry.ollama.ai" / "library" / "evil" / "latest"
    bad.parent.mkdir(parents=True)
    bad.write_text(json.dumps({"layers": [{"mediaType": "application/vnd.ollama.image.model",
                                           "digest": "sha256:../../../etc/passwd"}]}))
    with pytest.raises(ValueError, match="malformed"):
        ollama_blob("evil", store)
    ns = store / "manifests" / "registry.ollama.ai" / "someone" / "tiny" / "latest"
    ns.parent.mkdir(parents=True)
    ns.write_text(man.read_text())
    assert ollama_blob("someone/tiny", store) == ollama_blob("qwen2:1.5b", store)

    monkeypatch.setenv("CAIN_CHECKPOINTS", f"qwen2:1.5b=ollama:{store}")
    cfg = get_config("qwen2:1.5b")
    assert (cfg.d_model, cfg.n_layers, cfg.qkv_bias) == (384, 2, True)  # the blob's, not the built-in 1.5B
    eng = DecodeEngine("qwen2:1.5b", device="cpu", max_batch=1, max_context=64)
    ids = [5, 9, 33, 100]
    got = eng.generate([ids], 5, [dict(temperature=0.0, eos_id=-1)])[0].tokens
    with torch.no_grad():
        want = model.generate(torch.tensor([ids]), max_new_tokens=5, do_sample=False, eos_token_id=None,
                              pad_token_id=0)[0, len(ids):].tolist()
    assert got == want


@pytest.mark.parametrize("arch", ["llama", "gemma", "phi3"])
def test_gguf_sentencepiece_vocabulary(arch, tmp_path):
    """A SentencePiece-style vocabulary (tokenizer.ggml.model "llama": pieces with U+2581, byte fallback pieces,
    scores, token types) as Mistral / Gemma / Phi-3 GGUF files carry it: the converter builds a tokenizer that
    round-trips text, also without a padding id in the file."""
    toks = ["<unk>", "<s>", "</s>"] + [f"<0x{i:02X}>" for i in range(256)] + \
        ["\u2581", "\u2581w", "o", "r", "d", "\u2581word", "\u2581the", "t", "h", "e", "\u2581t", "\u2581energy", "n",
         "g", "y", "\u2581e"]
    n_norm = len(toks) - 259
    fields = {"tokenizer.ggml.model": "llama", "tokenizer.ggml.tokens": toks,
              "tokenizer.ggml.scores": [0.0] * 259 + [-float(i) for i in range(n_norm)],
              "tokenizer.ggml.token_type": [2, 3, 3] + [6] * 256 + [1] * n_norm}
    make_checkpoint({"llama": "mistral"}.get(arch, arch), tmp_path / "hf")
    _, mw, _ = load_pretrained(tmp_path / "hf")
    export_gguf(mw, tmp_path / "t.gguf", arch, tokenizer_fields=fields)
    _, _, tok = load_gguf(tmp_path / "t.gguf")
    ids = tok.encode("the word energy", add_bos=False)
    assert ids and max(ids) < len(toks)
    # SentencePiece vocabularies get llama.cpp's default BOS (no add_bos_token key in the file): the converters attach
    # no post-processor, so the tokenizer prepends it itself (raw prompts reached Gemma without BOS)
    fields["tokenizer.ggml.bos_token_id"] = 1
    export_gguf(mw, tmp_path / "b.gguf", arch, tokenizer_fields=fields)
    _, _, tb = load_gguf(tmp_path / "b.gguf")
    with_bos = tb.encode("the word energy", add_bos=True)
    assert with_bos[0] == 1 and with_bos[1:] == ids and with_bos.count(1) == 1
    fields["tokenizer.ggml.add_bos_token"] = False
    export_gguf(mw, tmp_path / "n.gguf", arch, tokenizer_fields=fields)
    assert load_gguf(tmp_path / "n.gguf")[2].encode("the word energy", add_bos=True) == ids
    if arch != "phi3":
        assert tok.decode(ids) == "the word energy"
    # phi3: transformers' Phi-3 converter lays Phi-3's own added tokens (ids 32000+) and normaliser over the vocabulary;
    # on this 275-piece toy vocabulary it drops the word boundaries, so only loading and encoding are checked here


@pytest.mark.parametrize("arch, their", [("llama", "llama"), ("qwen2", "qwen2"), ("phi3", "phi3"), ("gemma", "gemma2")])
def test_metadata_keys_match_transformers_gguf_mapping(arch, their):
    """The GGUF metadata keys config_from_gguf reads are the ones transformers' GGUF loader maps onto the same
    config fields (transformers.integrations.ggml.GGUF_CONFIG_MAPPING; gemma 1 files use gemma 2's key names)."""
    from transformers.integrations.ggml import GGUF_CONFIG_MAPPING

    ours = {"block_count": "num_hidden_layers", "context_length": "max_position_embeddings",
            "embedding_length": "hidden_size", "feed_forward_length": "intermediate_size",
            "attention.head_count": "num_attention_heads", "attention.head_count_kv": "num_key_value_heads",
            "rope.freq_base": "rope_theta", "attention.layer_norm_rms_epsilon": "rms_norm_eps"}
    m = GGUF_CONFIG_MAPPING[their]
    for key, field in ours.items():
        assert m.get(key) == field, (arch, key, m.get(key))
    # and the exporter writes exactly those keys under the architecture's prefix
    cfg = get_config_for_test(arch)
    md = GGUFMeta(cfg, arch)
    for key in ours:
        assert f"{arch}.{key}" in md


def get_config_for_test(arch):
    from cain_amd.models import TINY

    return TINY[{"llama": "tiny-llama3.1:8b", "qwen2": "tiny-qwen2:1.5b", "phi3": "tiny-phi3:3.8b",
                 "gemma": "tiny-gemma:2b"}[arch]]


def GGUFMeta(cfg, arch):  # noqa: N802 - the metadata export_gguf writes, read back
    import tempfile
    from pathlib import Path

    from cain_amd.models import random_weights

    with tempfile.TemporaryDirectory() as td:
        p = Path(td) / "m.gguf"
        export_gguf(random_weights(cfg, dtype=torch.float32), p, arch, tensor_type="F16")
        return GGUFFile(p).metadata


def test_convert_cli_round_trip(tmp_path):
    """python -m cain_amd convert <hf dir> <out.gguf>: the written file loads back to the checkpoint's logits."""
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    model = make_checkpoint("llama", tmp_path / "hf", scale=4.0)
    r = subprocess.run([sys.executable, "-m", "cain_amd", "convert", str(tmp_path / "hf"), str(tmp_path / "o.gguf"),
                        "--type", "F32"], capture_output=True, text=True, cwd=str(root), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "architecture: llama" in r.stdout
    _, mg, _ = load_gguf(tmp_path / "o.gguf", dtype=torch.float32)
    tokens = torch.randint(3, 1024, (1, 8), generator=torch.Generator().manual_seed(2))
    pos = torch.arange(8)[None]
    theirs = hf_logits(model, tokens, pos)
    ours = ReferenceModel(mg).forward(tokens, positions=pos)
    assert float((ours - theirs).abs().max() / theirs.abs().max()) < 2e-5


def test_convert_cli_writes_the_tokenizer_and_context(tmp_path):
    """convert carries a byte-level BPE tokenizer.json (tokens, merges, BOS rule, chat template) into the
    GGUF's tokenizer.ggml.* metadata and writes the checkpoint's max_position_embeddings, so the file is complete for
    llama.cpp-style loaders; it loads back to the same encodings here."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, processors, trainers

    from cain_amd.models.gguf import GGUFFile

    root = Path(__file__).resolve().parent.parent
    make_checkpoint("llama", tmp_path / "hf")
    conf = json.loads((tmp_path / "hf" / "config.json").read_text())
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    text = ["In 100 words, please give me information about India", "energy of remote and on device inference"] * 20
    tok.train_from_iterator(text, trainers.BpeTrainer(vocab_size=300, special_tokens=["<s>", "</s>"],
                                                      initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    tok.post_processor = processors.TemplateProcessing(single="<s> $A", special_tokens=[("<s>", 0)])
    tok.save(str(tmp_path / "hf" / "tokenizer.json"))
    conf.update(bos_token_id=0, eos_token_id=1, max_position_embeddings=4096)
    (tmp_path / "hf" / "config.json").write_text(json.dumps(conf))
    r = subprocess.run([sys.executable, "-m", "cain_amd", "convert", str(tmp_path / "hf"), str(tmp_path / "o.gguf"),
                        "--type", "F16"], capture_output=True, text=True, cwd=str(root), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "tokenizer gpt2" in r.stdout
    md = GGUFFile(tmp_path / "o.gguf").metadata
    assert md["llama.context_length"] == 4096
    assert md["tokenizer.ggml.add_bos_token"] is True and md["tokenizer.ggml.bos_token_id"] == 0
    _, _, gt = load_gguf(tmp_path / "o.gguf")
    s = "please give me information about remote energy"
    assert gt.encode(s, add_bos=True) == tok.encode(s).ids
    assert gt.encode(s, add_bos=False) == tok.encode(s, add_special_tokens=False).ids
