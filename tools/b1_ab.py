#!/usr/bin/env python3
"""Batch-1 decode throughput per model, as bench.py's single-stream rows measure it (forced length, graph-replayed,
median of --trials generations), for A/B runs of two kernel-library builds on ONE box:

    CAIN_KERNELS_LIB=ab/libcain_kernels_r5.so python tools/b1_ab.py --label r5 ; python tools/b1_ab.py --label new

run alternately (boxes differ by 1-3 %, profiles/r4).  One JSON line per (model, dtype) with the label.
"""
import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cain_amd.engine import DecodeEngine  # noqa: E402
from cain_amd.models.tokenizer import tokens_for_words  # noqa: E402

ALL7 = "llama3.1:8b,qwen2:1.5b,gemma:2b,phi3:3.8b,qwen2:7b,gemma:7b,mistral:7b"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default=ALL7)
    ap.add_argument("--dtype", default="fp4")
    ap.add_argument("--words", type=int, default=1000)
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--label", default=os.environ.get("CAIN_KERNELS_LIB", "default"))
    ap.add_argument("--out", default=None, help="append the JSON lines to this file too")
    ap.add_argument("--sample-cm", type=int, default=None,
                    help="sampler A/B: cain_amd.ops.set_sample_cm mode (3 = the lean chunk-maximum kernel)")
    ap.add_argument("--w4-split", type=int, default=None,
                    help="A/B: force k ranges per tile of the MXFP4 stream GEMMs wherever the shape allows "
                         "(cain_amd.ops.set_w4_split; 0 = the rule)")
    a = ap.parse_args()
    if a.w4_split is not None:
        from cain_amd import ops

        ops.set_w4_split(a.w4_split)
    if a.sample_cm is not None:
        from cain_amd import ops

        ops.set_sample_cm(a.sample_cm)
    n_tok = tokens_for_words(a.words)
    opts = dict(eos_id=-1)
    for model in filter(None, a.models.split(",")):
        for dtype in a.dtype.split(","):
            eng = DecodeEngine(model, device="cuda", max_batch=1, max_context=1536, weight_dtype=dtype,
                               steps_per_graph=16, seed=1234)
            eng.generate(["warm up"], 32, [dict(opts, seed=7)])
            rates = []
            for t in range(a.trials):
                torch.cuda.synchronize()
                time.sleep(0.5)
                t0 = time.perf_counter()
                r = eng.generate([f"In {a.words} words, please give me information about topic {t}"], n_tok,
                                 [dict(opts, seed=8 + t)])[0]
                torch.cuda.synchronize()
                rates.append(r.eval_count / (time.perf_counter() - t0))
            rec = {"label": a.label, "sample_cm": a.sample_cm, "w4_split": a.w4_split, "model": model, "dtype": dtype, "tok_per_s": round(statistics.median(rates), 1),
                   "trials": [round(x, 1) for x in rates], "tokens": n_tok}
            print(json.dumps(rec), flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(json.dumps(rec) + "\n")
            del eng
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
