"""Diagnose qwen2:1.5b fp4 last-token logits against the oracle under kernel switches (round-6 debugging)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cain_amd import ops  # noqa: E402
from cain_amd.engine import DecodeEngine  # noqa: E402
from cain_amd.models.reference import ReferenceModel  # noqa: E402
from cain_amd.models.weights import mxfp4_roundtrip_weights  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "qwen2:1.5b"
prompt = "In 100 words, please give me information about India"
eng = DecodeEngine(name, device="cuda", max_batch=256, max_context=128, keep_natural=True, seed=17, weight_dtype="fp4")
ref = ReferenceModel(mxfp4_roundtrip_weights(eng.weights), memo_weights=True)
toks = torch.tensor([eng.encode(prompt)], device="cuda")
want = ref.forward(toks, last_only=True)[0, -1]


def cos(tag):
    g = eng.last_logits([prompt])[0].float()
    c = float(torch.nn.functional.cosine_similarity(g, want, dim=0))
    print(f"{tag:40s} cos {c:.5f}  n_tok {toks.shape[1]}", flush=True)


cos("default")
ops.set_sample_cm(0)
cos("sample_cm 0 (no chunk maxima)")
ops.set_sample_cm(3)
ops.set_w4_split(1)
cos("w4 split off")
ops.set_w4_split(0)
for v in range(6):
    ops.set_w4_variant(v)
    cos(f"w4 variant {v}")
ops.set_w4_variant(-1)
cos("default again")
