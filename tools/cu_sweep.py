#!/usr/bin/env python3
"""Batch-1 energy lever: the reference's one-request protocol (/root/reference/experiment/RunnerConfig.py:120-131)
on a CU-limited stream (DecodeEngine(cu_limit=n): runtime.hip cain_stream_create_cu_limited + grids sized for n
CUs), tok/s and GPU J/token per CU count.  A batch-1 decode streams weights at a few TB/s from a few hundred
workgroups; fewer CUs may hold most of that rate at a lower board power.

Per (model, weights) one engine per CU count shares the random weights; trials run interleaved over the CU counts
(trial t of every count, then trial t + 1), each after ``--settle`` s of rest, each its own energy window.  One JSON
line per (model, weights, cus) with the median tok/s and J/token, and ``vs_full`` ratios against the whole device.

    python3 tools/cu_sweep.py --cases llama3.1:8b:fp4,qwen2:1.5b:bf16 --cus 256,192,128,64 --out gpurun_out/cu.jsonl
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="llama3.1:8b:fp4,llama3.1:8b:bf16,qwen2:1.5b:bf16,gemma:2b:fp4")
    ap.add_argument("--cus", default="256,192,128,64")
    ap.add_argument("--words", type=int, default=1000)
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--settle", type=float, default=2.0)
    ap.add_argument("--out", default="gpurun_out/cu_sweep.jsonl")
    ns = ap.parse_args()

    import torch

    from cain_amd.energy import EnergyMeter
    from cain_amd.engine import DecodeEngine
    from cain_amd.models.tokenizer import tokens_for_words
    from cain_amd.models.weights import random_weights
    from cain_amd.models import get_config

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    full = torch.cuda.get_device_properties(dev).multi_processor_count
    cus = [int(c) for c in ns.cus.split(",")]
    n_tok = tokens_for_words(ns.words)
    meter = EnergyMeter(devices=[0], period_ms=100.0, keep_samples=False, sources=("gpu",))
    Path(ns.out).parent.mkdir(parents=True, exist_ok=True)
    out = open(ns.out, "a")
    for case in filter(None, ns.cases.split(",")):
        model, dtype = case.rsplit(":", 1)
        w = random_weights(get_config(model), device=dev, seed=1)
        engs = {c: DecodeEngine(model, device=dev, max_batch=1, max_context=1536, seed=1, weights=w, keep_natural=True,
                                weight_dtype=dtype, cu_limit=0 if c >= full else c) for c in cus}
        prompt = f"In {ns.words} words, please give me information about energy efficiency"
        for c, e in engs.items():
            e.generate([prompt], 32, [dict(eos_id=-1, seed=3)])
        meter.measure_idle(2.0)
        rates = {c: [] for c in cus}
        jpt = {c: [] for c in cus}
        watts = {c: [] for c in cus}
        for t in range(ns.trials):
            for c, e in engs.items():
                torch.cuda.synchronize()
                time.sleep(ns.settle)
                meter.start()
                t0 = time.perf_counter()
                r = e.generate([prompt], n_tok, [dict(eos_id=-1, seed=10 + t)])[0]
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                rd = meter.stop()
                rates[c].append(r.eval_count / dt)
                jpt[c].append(rd.gpu_energy_j / max(1, r.eval_count))
                watts[c].append(rd.gpu_power_w)
                print(f"[cu_sweep] {model} {dtype} cus={c} trial {t}: {rates[c][-1]:.1f} tok/s "
                      f"{jpt[c][-1]:.4f} J/tok {watts[c][-1]:.0f} W", file=sys.stderr, flush=True)
        base = cus[0] if full not in cus else full
        med = {c: (statistics.median(rates[c]), statistics.median(jpt[c]), statistics.median(watts[c])) for c in cus}
        for c in cus:
            rec = dict(model=model, weights=dtype, cus=c, tok_per_s=round(med[c][0], 2), J_per_token=round(med[c][1], 4),
                       gpu_power_W=round(med[c][2], 1), idle_power_W=round(meter.idle_power_w, 1),
                       tok_per_s_vs_full=round(med[c][0] / med[base][0], 4),
                       J_per_token_vs_full=round(med[c][1] / med[base][1], 4), trials=ns.trials, words=ns.words,
                       tokens=n_tok)
            print(json.dumps(rec), flush=True)
            out.write(json.dumps(rec) + "\n")
            out.flush()
        for e in engs.values():
            e.close()
        del engs, w
        torch.cuda.empty_cache()
    meter.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
