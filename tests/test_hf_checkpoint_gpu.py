"""The HIP engine on Hugging Face checkpoints (models/hf.py): next-token logits against transformers' fp32 model of
the same checkpoint, per study family, with the relative criterion of tests/numerics.py (the engine at most 1.25x
as far from fp32 as a PyTorch bf16-eager model on the engine's bf16 weights).  The checkpoints carry non-unit
norm gains and QKV biases (hf_fixtures.make_checkpoint), which the engine folds / adds in its GEMM epilogues."""
import pytest
import torch

from hf_fixtures import FAMILIES, make_checkpoint
from numerics import assert_within_eager, eager_bf16, rel

from cain_amd.engine import DecodeEngine

pytest.importorskip("transformers")
pytestmark = pytest.mark.gpu

PROMPTS = [[1, 17, 230, 5, 999, 64, 3, 410], [1, 88, 2, 700], [1, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]]


@pytest.mark.parametrize("family", sorted(FAMILIES))
@pytest.mark.parametrize("weights", ["bf16", "fp4"])
def test_hip_engine_on_a_checkpoint(family, weights, tmp_path):
    model = make_checkpoint(family, tmp_path, scale=4.0)
    eng = DecodeEngine.from_pretrained(str(tmp_path), device="cuda", max_batch=4, max_context=128,
                                       keep_natural=True, weight_dtype=weights)
    got = eng.last_logits(PROMPTS).float().cpu()
    from cain_amd.models.weights import roundtrip_weights

    # fp4: the oracle and the eager baseline multiply by the dequantised MXFP4 weights, as the kernels do
    base = roundtrip_weights(eng.weights, weights)
    eager = eager_bf16(base)
    err, err_eager = [], []
    for i, p in enumerate(PROMPTS):
        toks = torch.tensor([p])
        if weights == "bf16":
            with torch.no_grad():
                want = model(input_ids=toks).logits[0, -1].float()
        else:
            from cain_amd.models.reference import ReferenceModel
            want = ReferenceModel(base).forward(toks.cuda())[0, -1].float().cpu()
        ref_e = eager.forward(toks.cuda())[0, -1].float().cpu()
        err.append(rel(got[i], want))
        err_eager.append(rel(ref_e, want))
    assert_within_eager(err, err_eager, f"{family} {weights}")
    eng.close()


@pytest.mark.parametrize("weights", ["bf16", "fp4"])
def test_hip_engine_on_a_gguf_file(weights, tmp_path):
    """A Q4_0 GGUF file (llama.cpp conventions: permuted q / k rows, Llama 3.1 scaling as rope_freqs) on the HIP
    engine, against the oracle on the same dequantised weights."""
    from cain_amd.models.gguf import export_gguf
    from cain_amd.models.hf import load_pretrained
    from cain_amd.models.reference import ReferenceModel
    from cain_amd.models.weights import roundtrip_weights

    make_checkpoint("llama", tmp_path / "hf", scale=4.0)
    _, mw, _ = load_pretrained(tmp_path / "hf", dtype=torch.float32)
    export_gguf(mw, tmp_path / "m.gguf", "llama", tensor_type="Q4_0")
    eng = DecodeEngine.from_pretrained(str(tmp_path / "m.gguf"), device="cuda", max_batch=4, max_context=128,
                                       keep_natural=True, weight_dtype=weights)
    assert eng.cfg.rope_freq_factors is not None
    got = eng.last_logits(PROMPTS).float().cpu()
    base = roundtrip_weights(eng.weights, weights)
    ref, eager = ReferenceModel(base), eager_bf16(base)
    err, err_eager = [], []
    for i, p in enumerate(PROMPTS):
        toks = torch.tensor([p], device="cuda")
        want = ref.forward(toks)[0, -1].float().cpu()
        err.append(rel(got[i], want))
        err_eager.append(rel(eager.forward(toks)[0, -1].float().cpu(), want))
    assert_within_eager(err, err_eager, f"gguf {weights}")
    eng.close()
