#!/usr/bin/env python3
"""Batch-1 decode on MXFP4 weights with the W4 stream kernel's split-K off and on (csrc/gemm_w4.hip w4_split),
interleaved on one GPU: single-stream tok/s per model (median of --trials generations of --tokens forced tokens,
graph-replayed, as bench.py's single-stream rows).  One JSON line per (model, split setting, trial round).

    python tools/w4_split_ab.py [--models qwen2:1.5b,gemma:2b,phi3:3.8b] [--tokens 512] [--trials 3] [--rounds 2]
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cain_amd import ops  # noqa: E402
from cain_amd.engine import DecodeEngine  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="qwen2:1.5b,gemma:2b,phi3:3.8b")
    ap.add_argument("--tokens", type=int, default=512)
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--cap", type=int, default=0,
                    help="compare the rule (cap 1) with a pair budget of cap x CUs instead of split off vs rule")
    ap.add_argument("--min-quads", type=int, default=0,
                    help="compare the rule (32) with this shortest k range (in quads) instead of split off vs rule")
    a = ap.parse_args()
    opts = dict(eos_id=-1, seed=7)
    for model in filter(None, a.models.split(",")):
        for rnd in range(a.rounds):
            settings = (("cap1", f"cap{a.cap}") if a.cap else ("minq32", f"minq{a.min_quads}") if a.min_quads
                        else (1, 0))  # 1 = off, 0 = the rule
            for split in settings:
                if isinstance(split, str) and split.startswith("cap"):
                    ops.set_w4_split(0)
                    ops.set_w4_split_cap(int(split[3:]))
                elif isinstance(split, str):
                    ops.set_w4_split(0)
                    ops.set_w4_split_min_quads(int(split[4:]))
                else:
                    ops.set_w4_split(split)
                eng = DecodeEngine(model, device="cuda", max_batch=1, max_context=1024, weight_dtype="fp4",
                                   steps_per_graph=16, seed=1)
                eng.generate(["warm up"], 32, [opts])
                rates = []
                for t in range(a.trials):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    r = eng.generate([f"In 500 words, please give me information about topic {t}"], a.tokens, [opts])[0]
                    torch.cuda.synchronize()
                    rates.append(r.eval_count / (time.perf_counter() - t0))
                cfg = eng.cfg
                label = split if isinstance(split, str) else ("rule" if split == 0 else "off")
                print(json.dumps({"model": model, "round": rnd, "split": label,
                                  "tok_per_s": round(statistics.median(rates), 1),
                                  "o_ks": ops.w4_split(cfg.d_model, cfg.q_dim, 1, ops.EPI_RESID) if split != 1 else 1,
                                  "down_ks": ops.w4_split(cfg.d_model, cfg.ffn, 1, ops.EPI_RESID) if split != 1 else 1}),
                      flush=True)
                eng.close()
                del eng
                torch.cuda.empty_cache()
    ops.set_w4_split(0)
    ops.set_w4_split_cap(1)
    ops.set_w4_split_min_quads(32)
    return 0


if __name__ == "__main__":
    sys.exit(main())
