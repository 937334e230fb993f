"""How far a GGUF Q4_K model moves when the engine re-quantises it to MXFP4 ("the current path
quantified"), against the other quantisation steps, on the fp32 torch oracle (cain_amd.models.reference).

W0 = the architecture's seeded random bf16 weights; Q = the Q4_K blocks of W0 as a GGUF file stores them
(q4_roundtrip_weights: the values Ollama runs and the q4_k engine runs as stored); M(Q) = MXFP4 re-quantisation of
those values (what weight_dtype="fp4" runs on a Q4_K file); M(W0) = MXFP4 of the original weights.  Per pair:
relative error of the last-token logits over 8 prompts, and greedy-token agreement over 256 steps -- teacher-forced
(both models fed the reference model's greedy tokens; argmax agreement per position) and free-running (the step of
the first disagreement).

    python tools/q4k_requant_error.py [--models qwen2:1.5b,llama3.1:8b] [--steps 256]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cain_amd.models import TINY  # noqa: E402
from cain_amd.models.config import MODELS  # noqa: E402
from cain_amd.models.reference import ReferenceModel  # noqa: E402
from cain_amd.models.tokenizer import get_tokenizer  # noqa: E402
from cain_amd.models.weights import mxfp4_roundtrip_weights, q4_roundtrip_weights, random_weights  # noqa: E402

TOPICS = ["India", "World War II", "Elizabeth II", "United States", "Cristiano Ronaldo", "The Beatles", "Barack Obama",
          "Lady Gaga"]


def rel(a, b):
    return float((a - b).norm() / b.norm())


@torch.no_grad()
def greedy(ref, prompt, n):
    cache = []
    lg = ref.forward(prompt, cache=cache, last_only=True)[:, -1]
    out = []
    for _ in range(n):
        t = lg.argmax(-1)
        out.append(t)
        lg = ref.forward(t[:, None], cache=cache)[:, -1]
    return torch.stack(out, 1)


@torch.no_grad()
def teacher_forced_argmax(ref, seq):
    return ref.forward(seq)[:, :-1].argmax(-1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="qwen2:1.5b,llama3.1:8b")
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--out", default=None)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    dev = a.device
    rows = []
    for name in a.models.split(","):
        cfg = MODELS.get(name) or TINY[name]
        tok = get_tokenizer(cfg)
        w0 = random_weights(cfg, device=dev, seed=11)
        wq = q4_roundtrip_weights(w0, "q4_k")
        variants = {"W0 (bf16)": w0, "Q (Q4_K as stored)": wq, "M(Q) (Q4_K re-quantised to MXFP4)":
                    mxfp4_roundtrip_weights(wq), "M(W0) (MXFP4 of bf16)": mxfp4_roundtrip_weights(w0)}
        refs = {k: ReferenceModel(v) for k, v in variants.items()}
        prompts = [torch.tensor([tok.encode(f"In 100 words, please give me information about {t}")], device=dev)
                   for t in TOPICS]
        last = {k: torch.stack([r.forward(p, last_only=True)[0, -1] for p in prompts]) for k, r in refs.items()}
        # the reference trajectory: Q's greedy continuation of the first prompt
        seq_q = torch.cat([prompts[0], greedy(refs["Q (Q4_K as stored)"], prompts[0], a.steps)], 1)
        tf = {k: teacher_forced_argmax(r, seq_q)[0, prompts[0].shape[1] - 1:] for k, r in refs.items()}
        free = {k: greedy(r, prompts[0], a.steps)[0] for k, r in refs.items()}
        for test, base in (("M(Q) (Q4_K re-quantised to MXFP4)", "Q (Q4_K as stored)"),
                           ("Q (Q4_K as stored)", "W0 (bf16)"), ("M(W0) (MXFP4 of bf16)", "W0 (bf16)")):
            agree = float((tf[test] == tf[base]).float().mean())
            diff = (free[test] != free[base]).nonzero()
            first = int(diff[0, 0]) if diff.numel() else a.steps
            r = dict(model=name, test=test, base=base, logit_rel_err=round(rel(last[test], last[base]), 5),
                     teacher_forced_argmax_agreement=round(agree, 4), free_running_first_divergence=first,
                     steps=a.steps)
            rows.append(r)
            print(json.dumps(r), flush=True)
        del refs, variants, w0, wq
        torch.cuda.empty_cache()
    if a.out:
        Path(a.out).write_text("\n".join(json.dumps(r) for r in rows) + "\n")


if __name__ == "__main__":
    main()
