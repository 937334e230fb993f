"""End-to-end HIP engine vs the torch-eager oracle on every architecture family (tiny shapes),
plus hipGraph replay determinism and full-size smoke for the flagship model."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd.engine import DecodeEngine  # noqa: E402
from cain_amd.models import TINY  # noqa: E402
from cain_amd.models.reference import ReferenceModel  # noqa: E402

PROMPTS = ["In 100 words, please give me information about India",
           "In 500 words, please give me information about Elizabeth II, Queen of the United Kingdom and more",
           "hi"]


@pytest.mark.parametrize("name", sorted(TINY))
def test_engine_logits_match_oracle(name):
    eng = DecodeEngine(name, device="cuda", max_batch=4, max_context=256, keep_natural=True, seed=3)
    got = eng.last_logits(PROMPTS)
    ref = ReferenceModel(eng.weights)
    for i, p in enumerate(PROMPTS):
        ids = torch.tensor([eng.encode(p)], device="cuda")
        want = ref.forward(ids)[0, -1]
        cos = torch.nn.functional.cosine_similarity(got[i].float(), want.float(), dim=0)
        assert cos > 0.995, (name, i, float(cos))
    eng.close()


@pytest.mark.parametrize("name", ["tiny-llama3.1:8b", "tiny-gemma:2b", "tiny-qwen2:1.5b"])
def test_graph_replay_equals_eager_steps(name):
    eng = DecodeEngine(name, device="cuda", max_batch=4, max_context=256, seed=5, steps_per_graph=4)
    opts = [dict(temperature=0.8, seed=11 + i, eos_id=-1) for i in range(3)]
    a = eng.generate(PROMPTS, 10, opts, use_graph=True)
    b = eng.generate(PROMPTS, 10, opts, use_graph=False)
    assert [r.tokens for r in a] == [r.tokens for r in b]
    assert all(r.eval_count == 10 for r in a)
    g = eng.generate(PROMPTS, 6, [dict(temperature=0.0, eos_id=-1)] * 3)
    g2 = eng.generate(PROMPTS, 6, [dict(temperature=0.0, eos_id=-1)] * 3)
    assert [r.tokens for r in g] == [r.tokens for r in g2]
    eng.close()


@pytest.mark.parametrize("name", ["tiny-llama3.1:8b", "tiny-qwen2:1.5b", "tiny-gemma:2b"])
def test_chunk_max_sampler_same_tokens(name):
    """Few-row decode with the chunk-maximum sampler (the LM head writes 16-column maxima) generates exactly the
    tokens of the two-stage sampler: sampled (Ollama defaults, repeat penalty) and greedy rows."""
    from cain_amd import ops
    opts = [dict(seed=21, eos_id=-1), dict(temperature=0.0, eos_id=-1), dict(repeat_penalty=0.9, seed=5, eos_id=-1)]
    out = []
    saved = ops.sample_cm_mode()
    for cm in (3, 1, 0):  # the lean chunk-maximum kernel, the round-3 one, the two-stage kernel
        ops.set_sample_cm(cm)
        eng = DecodeEngine(name, device="cuda", max_batch=4, max_context=256, seed=7, steps_per_graph=4)
        out.append([r.tokens for r in eng.generate(PROMPTS, 24, opts)])
        eng.close()
    ops.set_sample_cm(saved)
    assert out[0] == out[2] and out[1] == out[2]


@pytest.mark.parametrize("dtype", ["fp8", "fp4", "q4_0", "q4_k"])
def test_lean_sampler_on_every_lm_head_format(dtype):
    """Single-stream decode on every few-row weight format: the fp8 / MXFP4 / Q4 LM heads write the chunk maxima,
    and the lean chunk-maximum sampler generates exactly the tokens of the two-stage sampler (which reads the full
    logits)."""
    from cain_amd import ops
    opts = [dict(seed=21, eos_id=-1)]
    out = []
    saved = ops.sample_cm_mode()
    for cm in (3, 0):
        ops.set_sample_cm(cm)
        eng = DecodeEngine("tiny-llama3.1:8b", device="cuda", max_batch=1, max_context=256, seed=7,
                           steps_per_graph=4, weight_dtype=dtype)
        out.append([r.tokens for r in eng.generate(PROMPTS[:1], 32, opts)])
        eng.close()
    ops.set_sample_cm(saved)
    assert out[0] == out[1]


def test_chunk_max_sampler_wide_batch_same_tokens():
    """80 rows (the wide GEMM path: its unsplit LM-head epilogue writes the chunk maxima): the chunk-maximum sampler
    generates exactly the tokens of the one-workgroup-per-row sampler."""
    from cain_amd import ops
    prompts = [f"In {50 + i} words, please give me information about topic {i}" for i in range(80)]
    opts = [dict(seed=100 + i, eos_id=-1) if i % 3 else dict(temperature=0.0, eos_id=-1) for i in range(80)]
    out = []
    saved = ops.sample_cm_mode()
    for cm in (3, 1, 0):
        ops.set_sample_cm(cm)
        eng = DecodeEngine("tiny-llama3.1:8b", device="cuda", max_batch=80, max_context=256, seed=7, steps_per_graph=4)
        out.append([r.tokens for r in eng.generate(prompts, 12, opts)])
        eng.close()
    ops.set_sample_cm(saved)
    assert out[0] == out[2] and out[1] == out[2]


def test_greedy_first_token_matches_oracle():
    eng = DecodeEngine("tiny-mistral:7b", device="cuda", max_batch=4, max_context=256, keep_natural=True, seed=9)
    ref = ReferenceModel(eng.weights)
    res = eng.generate(PROMPTS, 1, [dict(temperature=0.0, repeat_penalty=1.0, eos_id=-1)] * 3)
    for i, p in enumerate(PROMPTS):
        lg = ref.forward(torch.tensor([eng.encode(p)], device="cuda"))[0, -1]
        top2 = lg.topk(2)
        if float(top2.values[0] - top2.values[1]) > 1e-2:  # unambiguous argmax
            assert res[i].tokens[0] == int(top2.indices[0])
    eng.close()


def test_eos_stops_row():
    eng = DecodeEngine("tiny-llama3.1:8b", device="cuda", max_batch=2, max_context=256, seed=1)
    first = eng.generate(["abc"], 1, [dict(temperature=0.0, eos_id=-1)])[0].tokens[0]
    r = eng.generate(["abc", "abc def"], 5, [dict(temperature=0.0, eos_id=first), dict(temperature=0.0, eos_id=-1)])
    assert r[0].tokens == [first] and r[0].done_reason == "stop"
    assert len(r[1].tokens) == 5
    eng.close()


@pytest.mark.slow
def test_flagship_llama_smoke():
    eng = DecodeEngine("llama3.1:8b", device="cuda", max_batch=2, max_context=512, seed=0)
    r = eng.generate(PROMPTS[:2], 16, [dict(eos_id=-1)] * 2)
    assert [x.eval_count for x in r] == [16, 16]
    assert all(0 <= t < eng.cfg.vocab for x in r for t in x.tokens)
    eng.close()


@pytest.mark.parametrize("name,rows", [("tiny-llama3.1:8b", 100), ("tiny-gemma:7b", 100), ("tiny-llama3.1:8b", 200)])
def test_wide_batch_and_long_prefill_match_oracle(name, rows):
    """100 / 200 rows: decode GEMMs on the batched (LDS-staged, NB = 8 / 16) path, prefill in 128-row chunks."""
    eng = DecodeEngine(name, device="cuda", max_batch=rows, max_context=512, keep_natural=True, seed=4)
    long = " ".join(f"word{i}" for i in range(160))  # > 128 prompt tokens: several prefill chunks
    prompts = [f"In {i} words, please give me information about topic {i}" for i in range(rows - 1)] + [long]
    got = eng.last_logits(prompts)
    ref = ReferenceModel(eng.weights)
    for i in (0, 37, rows - 2, rows - 1):
        want = ref.forward(torch.tensor([eng.encode(prompts[i])], device="cuda"))[0, -1]
        cos = torch.nn.functional.cosine_similarity(got[i].float(), want.float(), dim=0)
        assert cos > 0.995, (name, i, float(cos))
    r = eng.generate(prompts, 4, [dict(temperature=0.8, seed=i, eos_id=-1) for i in range(rows)])
    assert all(x.eval_count == 4 for x in r)
    eng.close()


def _teacher_forced_agreement(eng, ref, prompts, n_new, rows, tie=0.05):
    """Greedy generation through the hipGraph decode loop, then the oracle run over prompt + generated tokens
    (teacher forcing): at every step the engine's token must be the oracle's argmax unless the oracle's margin
    between its argmax and the engine's token is a near-tie at the bf16 error level of the stack (``tie`` x the
    logits' std: a 32-layer random-init stack carries ~10 % relative logit error, cf. test_fullsize_gpu).
    Returns (exact steps, total steps)."""
    res = eng.generate(prompts, n_new, [dict(temperature=0.0, repeat_penalty=1.0, eos_id=-1)] * len(prompts))
    exact = total = 0
    for i in rows:
        p_ids = eng.encode(prompts[i])
        toks = res[i].tokens
        assert len(toks) == n_new
        seq = torch.tensor([p_ids + toks[:-1]], device="cuda")
        lg = ref.forward(seq)[0, len(p_ids) - 1:]  # logits that predicted each generated token
        for s, t in enumerate(toks):
            best = int(lg[s].argmax())
            total += 1
            if best == t:
                exact += 1
            else:
                margin = float(lg[s, best] - lg[s, t])
                assert margin < tie * float(lg[s].std()), (i, s, best, t, margin)
    return exact, total


@pytest.mark.parametrize("name", ["tiny-llama3.1:8b", "tiny-gemma:2b", "tiny-qwen2:1.5b", "tiny-phi3:3.8b"])
def test_greedy_decode_tracks_oracle_token_by_token(name):
    """end-to-end greedy decode of a random-init model against the torch path for N steps (KV
    appends, RoPE at every position, the sampler's argmax, graph replay); disagreements only at near-ties."""
    eng = DecodeEngine(name, device="cuda", max_batch=4, max_context=256, keep_natural=True, seed=13,
                       steps_per_graph=8)
    ref = ReferenceModel(eng.weights)
    exact, total = _teacher_forced_agreement(eng, ref, PROMPTS, 48, range(len(PROMPTS)))
    assert exact / total > 0.9, (exact, total)
    eng.close()


def test_greedy_decode_tracks_oracle_full_size():
    """Full-size greedy decode: the engine's tokens disagree with the fp32 oracle's teacher-forced argmax no
    more often than a PyTorch bf16-eager model's argmax does on the same sequences (relative criterion,
    tests/numerics.py), and only at near-ties."""
    from numerics import eager_bf16

    eng = DecodeEngine("llama3.1:8b", device="cuda", max_batch=4, max_context=256, keep_natural=True, seed=13,
                       steps_per_graph=16)
    ref = ReferenceModel(eng.weights, memo_weights=True)
    exact, total = _teacher_forced_agreement(eng, ref, PROMPTS[:2], 64, range(2), tie=0.3)
    eager = eager_bf16(eng.weights)
    base_bad = 0
    res = eng.generate(PROMPTS[:2], 64, [dict(temperature=0.0, repeat_penalty=1.0, eos_id=-1)] * 2)
    for i in range(2):
        p_ids = eng.encode(PROMPTS[i])
        seq = torch.tensor([p_ids + res[i].tokens[:-1]], device="cuda")
        a = ref.forward(seq)[0, len(p_ids) - 1:].argmax(-1)
        b = eager.forward(seq)[0, len(p_ids) - 1:].argmax(-1)
        base_bad += int((a != b).sum())
    assert total - exact <= 1.25 * base_bad + 2, (total - exact, base_bad, total)
    eng.close()
    del ref, eager
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name,dtype,cus", [("tiny-llama3.1:8b", "bf16", 128), ("tiny-qwen2:1.5b", "bf16", 64),
                                            ("llama3.1:8b", "fp4", 64), ("qwen2:1.5b", "bf16", 128)])
def test_cu_limited_engine_matches_full_device(name, dtype, cus):
    """DecodeEngine(cu_limit=n): the kernels run on a CU-masked stream with grids sized for n CUs (the batch-1 energy
    lever, tools/cu_sweep.py); same logits and greedy tokens as the whole device, and the launch-sizing budget is
    back to the device's after every call."""
    from cain_amd import ops
    from cain_amd.models import get_config, random_weights

    full = torch.cuda.get_device_properties(0).multi_processor_count
    w = random_weights(get_config(name), device="cuda", seed=9)
    kw = dict(device="cuda", max_batch=1, max_context=512, seed=9, weights=w, keep_natural=True, weight_dtype=dtype)
    a = DecodeEngine(name, **kw)
    b = DecodeEngine(name, cu_limit=cus, **kw)
    assert b.cu_limit == cus and ops.cu_budget() == full
    la, lb = a.last_logits(PROMPTS[:1]), b.last_logits(PROMPTS[:1])
    # grids sized for fewer CUs split the k sums differently: rounding-level differences, which 32 random-init
    # layers amplify to a few percent (tests/numerics.py), hence the looser bound at full size
    tol = 1e-2 if name.startswith("tiny") else 5e-2
    assert float((la.float() - lb.float()).norm() / la.float().norm()) < tol
    ga = a.generate(PROMPTS[:1], 12, [dict(temperature=0.0, top_k=1, eos_id=-1)])[0]
    gb = b.generate(PROMPTS[:1], 12, [dict(temperature=0.0, top_k=1, eos_id=-1)])[0]
    # (greedy paths of a random-init 32-layer model part at near-ties after a few tokens: the full-size cases pin
    # the first token, taken from the logits compared above)
    n_same = 4 if name.startswith("tiny") else 1
    assert gb.eval_count == 12 and ga.tokens[:n_same] == gb.tokens[:n_same]
    assert ops.cu_budget() == full
    a.close()
    b.close()
