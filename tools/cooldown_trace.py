#!/usr/bin/env python3
"""Board power after a 1,000-word on-device run: how long the MI355X takes to return to its idle floor, the
evidence the study's cooldown is set on (the reference rests 90 s between runs,
/root/reference/experiment/RunnerConfig.py:55).

For each model: settle, measure the idle floor (board power from the amd-smi energy counter, this device only), run
one batch-1 generation of the full request length (the study's on-device arm), then keep sampling for ``--tail``
seconds.  Power is the energy counter's slope over ``--bin`` second bins.  Reported per model:

* ``settle_s[p]``: seconds after the generation ends until the ``--window`` s rolling mean first falls within p % of
  idle (p = 2, 5, 10);
* ``recover_s[p]``: the same, but staying within p % for the rest of the tail (nan if a later excursion -- the
  board's own ~1-2 s steps back to ~290 W, seen in idle windows too -- breaks it);
* the trace itself (``--csv``: t after the end of generation, W).

    python3 tools/cooldown_trace.py --models llama3.1:8b,qwen2:1.5b,gemma:2b --out gpurun_out/cooldown.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def power_bins(points, t0_ns: int, t1_ns: int, bin_s: float):
    """(t_mid_ns, W) from cumulative (t_ns, J) points in [t0, t1], one value per bin of bin_s seconds."""
    pts = [(t, j) for t, j in points if t0_ns <= t <= t1_ns]
    out = []
    if len(pts) < 2:
        return out
    step = int(bin_s * 1e9)
    i = 0
    edge = pts[0][0]
    while True:
        j0 = i
        while i + 1 < len(pts) and pts[i + 1][0] <= edge + step:
            i += 1
        if i == j0:
            if i + 1 >= len(pts):
                break
            i += 1  # a gap longer than one bin: take the next point
        (ta, ja), (tb, jb) = pts[j0], pts[i]
        if tb > ta:
            out.append(((ta + tb) // 2, (jb - ja) / ((tb - ta) * 1e-9)))
        edge = tb
        if i + 1 >= len(pts):
            break
    return out


def recover_time(series, t_end_ns: int, idle_w: float, pct: float, window_s: float) -> float:
    """Seconds after t_end until the rolling window_s mean stays <= idle * (1 + pct/100) to the end of the series
    (nan if it never does)."""
    after = [(t, w) for t, w in series if t >= t_end_ns]
    if not after:
        return float("nan")
    lim = idle_w * (1 + pct / 100.0)
    win = int(window_s * 1e9)
    means = []
    for k, (t, _) in enumerate(after):
        vals = [w for tt, w in after[k:] if tt < t + win]
        if after[-1][0] < t + win // 2:
            break
        means.append((t, sum(vals) / len(vals)))
    last_bad = None
    for t, m in means:
        if m > lim:
            last_bad = t
    if not means:
        return float("nan")
    if last_bad is None:
        return 0.0
    nxt = [t for t, _ in means if t > last_bad]
    return (nxt[0] - t_end_ns) * 1e-9 if nxt else float("nan")


def settle_time(series, t_end_ns: int, idle_w: float, pct: float, window_s: float) -> float:
    """Seconds after t_end until the rolling window_s mean first falls to <= idle * (1 + pct/100) (nan: never)."""
    after = [(t, w) for t, w in series if t >= t_end_ns]
    lim = idle_w * (1 + pct / 100.0)
    win = int(window_s * 1e9)
    for k, (t, _) in enumerate(after):
        if after[-1][0] < t + win // 2:
            break
        vals = [w for tt, w in after[k:] if tt < t + win]
        if sum(vals) / len(vals) <= lim:
            return (t - t_end_ns) * 1e-9
    return float("nan")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="llama3.1:8b,qwen2:1.5b,gemma:2b")
    ap.add_argument("--weights", default="bf16")
    ap.add_argument("--words", type=int, default=1000)
    ap.add_argument("--settle", type=float, default=30.0, help="rest before each idle measurement (s)")
    ap.add_argument("--idle", type=float, default=5.0, help="idle measurement window (s)")
    ap.add_argument("--tail", type=float, default=45.0, help="sampling after the generation (s)")
    ap.add_argument("--bin", type=float, default=0.25)
    ap.add_argument("--window", type=float, default=1.0)
    ap.add_argument("--out", default="gpurun_out/cooldown.json")
    ap.add_argument("--csv", default="gpurun_out/cooldown_trace.csv")
    ns = ap.parse_args()

    import torch

    from cain_amd.energy import EnergyMeter
    from cain_amd.engine import DecodeEngine
    from cain_amd.models.tokenizer import tokens_for_words

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    meter = EnergyMeter(devices=[0], period_ms=50.0, fast_period_ms=1.0, keep_samples=False, sources=("gpu",))
    n_tok = tokens_for_words(ns.words)
    results, rows = [], []
    for model in filter(None, ns.models.split(",")):
        eng = DecodeEngine(model, device=dev, max_batch=1, max_context=1536, seed=1, weight_dtype=ns.weights)
        prompt = f"In {ns.words} words, please give me information about energy efficiency"
        eng.generate([prompt], 32, [dict(eos_id=-1, seed=3)])  # graphs captured, clocks warm
        torch.cuda.synchronize()
        time.sleep(ns.settle)
        idle_w = meter.measure_idle(ns.idle)
        t_gen0 = time.monotonic_ns()
        r = eng.generate([prompt], n_tok, [dict(eos_id=-1, seed=5)])[0]
        torch.cuda.synchronize()
        t_end = time.monotonic_ns()
        time.sleep(ns.tail)
        t_tail = time.monotonic_ns()
        pts = meter.sampler.trace(0)
        series = power_bins(pts, t_gen0 - int(2e9), t_tail, ns.bin)
        gen_w = [w for t, w in series if t_gen0 <= t <= t_end]
        rec = {p: recover_time(series, t_end, idle_w, p, ns.window) for p in (2, 5, 10)}
        settle = {p: settle_time(series, t_end, idle_w, p, ns.window) for p in (2, 5, 10)}
        res = dict(model=model, weights=ns.weights, tokens=r.eval_count, gen_s=round((t_end - t_gen0) * 1e-9, 3),
                   idle_W=round(idle_w, 1), gen_mean_W=round(sum(gen_w) / max(1, len(gen_w)), 1),
                   first_bin_after_W=round(next((w for t, w in series if t >= t_end), float("nan")), 1),
                   settle_s={str(k): (None if v != v else round(v, 2)) for k, v in settle.items()},
                   recover_s={str(k): (None if v != v else round(v, 2)) for k, v in rec.items()},
                   tail_s=ns.tail, bin_s=ns.bin, window_s=ns.window)
        print(json.dumps(res), flush=True)
        results.append(res)
        rows += [(model, round((t - t_end) * 1e-9, 3), round(w, 1)) for t, w in series]
        eng.close()
        del eng
        torch.cuda.empty_cache()
        meter.sampler.trim(t_tail)
    meter.close()
    Path(ns.out).parent.mkdir(parents=True, exist_ok=True)
    Path(ns.out).write_text(json.dumps(results, indent=1) + "\n")
    with open(ns.csv, "w") as f:
        f.write("model,t_after_end_s,power_W\n")
        for m, t, w in rows:
            f.write(f"{m},{t},{w}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
