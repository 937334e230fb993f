#!/usr/bin/env python3
"""Headline benchmark: on-device LLM generation throughput and energy per token.

Metric (BASELINE.json): "Joules/generated-token (on-device vs remote) +
tokens/sec, per model/length".  This bench measures the on-device arm of the
flagship config — llama3.1:8b, 1000-word requests (⌈4/3·1000⌉ = 1334 forced
tokens), bf16, random-init weights, synthetic prompts built
from the reference's own topics list — on N GPUs of one node, one process per
GPU (weak scaling: every rank runs the same per-GPU trial batch).

A *step* is one batch of ``--batch`` concurrent trials on every GPU: prefill of
the prompts, then the full generation of 1334 tokens per trial with Ollama's
default sampling (temperature 0.8, top-k 40, top-p 0.9, repeat penalty 1.1),
EOS disabled so every trial produces the requested length.  ``value`` is the
whole-job generated tokens/s; the JSON also reports measured GPU energy per
generated token from the amd-smi counters (``J_per_token``; idle-subtracted
variant too).  Baseline: the reference's llama3.1:8b on-device 1000-word cell,
est. 19.2 tok/s and 0.574 J/token on a MacBook Pro M2.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--model M] [--words W] [--batch B (default 256)]
       (multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ..., or plain
       ``python bench.py --gpus N``, which spawns the N ranks itself before anything touches a GPU)

After the timed steps and a ``--settle`` every rank also runs the reference's one-request-at-a-time protocol
(batch 1; reference experiment/RunnerConfig.py:120-131): the median of ``--single-trials`` full-length
generations, each in its own energy window, for the bench model on bf16 (``single_stream_tok_per_s`` /
``single_stream_J_per_token``), fp8 e4m3 (``single_stream_fp8_*``) and MXFP4 weights (``single_stream_fp4_*``,
the reference's 4-bit precision class: Ollama serves 4-bit builds), for ``--single-models`` (default
qwen2:1.5b, gemma:2b) on bf16 and MXFP4 and for ``--single-fp4-models`` (default phi3:3.8b, qwen2:7b, gemma:7b,
mistral:7b) on MXFP4: ``single_stream_by_model``, all 7 study models, with each cell's BASELINE.md numbers.
"""
from __future__ import annotations

import argparse
import csv
import json
import math
import os
import socket
import statistics
import subprocess
import sys
import time
from pathlib import Path

BASELINE = {  # BASELINE.md §2, on_device rows: (est. tok/s, est. J/token) per requested length
    ("llama3.1:8b", 100): (7.9, 0.483), ("llama3.1:8b", 500): (14.9, 0.726), ("llama3.1:8b", 1000): (19.2, 0.574),
    ("qwen2:1.5b", 100): (12.8, 0.180), ("qwen2:1.5b", 500): (43.5, 0.081), ("qwen2:1.5b", 1000): (76.5, 0.056),
    ("gemma:2b", 100): (12.1, 0.212), ("gemma:2b", 500): (34.3, 0.132), ("gemma:2b", 1000): (67.2, 0.077),
    ("phi3:3.8b", 100): (8.8, 0.401), ("phi3:3.8b", 500): (15.6, 0.619), ("phi3:3.8b", 1000): (25.3, 0.398),
    ("qwen2:7b", 100): (6.2, 1.105), ("qwen2:7b", 500): (15.2, 0.703), ("qwen2:7b", 1000): (25.1, 0.436),
    ("gemma:7b", 100): (8.0, 0.496), ("gemma:7b", 500): (17.4, 0.651), ("gemma:7b", 1000): (32.7, 0.329),
    ("mistral:7b", 100): (7.1, 0.653), ("mistral:7b", 500): (15.9, 0.648), ("mistral:7b", 1000): (28.3, 0.366),
}


def topics():
    p = Path(__file__).resolve().parent / "experiments" / "topics.csv"
    try:
        with open(p, newline="") as fh:
            return [r["Topic"] for r in csv.DictReader(fh)]
    except OSError:
        return ["United States", "India", "Elizabeth II", "World War II"]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv) -> int:
    """``--gpus N`` without a launcher: start N ranks of this script (one per GPU, LOCAL_RANK = GPU) as child
    processes -- this process never initialises HIP -- and return the worst exit code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3.1:8b")
    ap.add_argument("--words", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=256, help="concurrent trials per GPU (trial batching, <= 256)")
    ap.add_argument("--context", type=int, default=1536)
    ap.add_argument("--steps-per-graph", type=int, default=16)
    ap.add_argument("--no-energy", action="store_true")
    ap.add_argument("--weights", choices=("bf16", "fp8", "fp4", "q4_0", "q4_k"), default="bf16",
                    help="GEMM weight storage: bf16 (headline), fp8 e4m3 per-row scaled (W8A8 above 16 rows, W8A16 "
                         "below) or MXFP4 (W4A16 with bf16 activations at <= 16 rows, W4A8 with per-row e4m3 "
                         "activations above: --w4a8-min-rows)")
    ap.add_argument("--kv", choices=("bf16", "fp8"), default="bf16",
                    help="KV-cache storage: bf16 (headline) or fp8 e4m3 (half the attention bytes; separate config)")
    ap.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                    help="cpu: the torch oracle backend over gloo (tests of the multi-rank plumbing; tiny models)")
    ap.add_argument("--settle", type=float, default=8.0, help="seconds of rest before the idle-power baseline")
    ap.add_argument("--no-single", action="store_true", help="skip the batch-1 (single-stream) measurement")
    ap.add_argument("--single-trials", type=int, default=3, help="batch-1 generations per (model, dtype); median")
    ap.add_argument("--single-settle", type=float, default=1.0, help="seconds of rest before each batch-1 trial")
    ap.add_argument("--single-models", default="qwen2:1.5b,gemma:2b",
                    help="other models measured at batch 1 (bf16 and MXFP4 weights), comma-separated")
    ap.add_argument("--single-fp4-models", default="phi3:3.8b,qwen2:7b,gemma:7b,mistral:7b",
                    help="models measured at batch 1 on MXFP4 weights only (the reference's 4-bit class), "
                         "comma-separated: with --single-models and the bench model, the 7 study models")
    ap.add_argument("--single-q4", default="q4_k",
                    help="GGUF 4-bit block formats (q4_0, q4_k; comma-separated, empty: none) also measured at batch "
                         "1 on all 7 models: Ollama's default builds run natively (csrc/gemm_q4.hip)")
    ap.add_argument("--checkpoint", default=None,
                    help="a Hugging Face checkpoint directory or GGUF file for --model (default: random-init weights of "
                         "the model's architecture; models/hf.py, models/gguf.py)")
    ap.add_argument("--w4a8-min-rows", type=int, default=0,
                    help="MXFP4: rows above which forwards run W4A8 instead of W4A16 (0: the runtime's default, 16)")
    ns = ap.parse_args()

    if ns.checkpoint:  # before any engine (and inherited by spawned ranks): --model's engines load the checkpoint
        os.environ["CAIN_CHECKPOINTS"] = ",".join(filter(None, [os.environ.get("CAIN_CHECKPOINTS", ""),
                                                                f"{ns.model}={ns.checkpoint}"]))
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and ns.gpus > 1:
        return spawn_ranks(ns.gpus, sys.argv[1:])
    world = int(world_env or "1")
    if world != ns.gpus:
        raise SystemExit(f"bench.py: --gpus {ns.gpus} but the launcher started WORLD_SIZE={world} ranks")

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = ns.device == "cpu"
    if world > 1:
        if cpu:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == world
    if cpu:
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)

    from cain_amd.engine import DecodeEngine

    if ns.w4a8_min_rows and not cpu:
        from cain_amd import ops
        ops.set_w4a8_min_rows(ns.w4a8_min_rows)
    from cain_amd.models.tokenizer import tokens_for_words

    n_tok = tokens_for_words(ns.words)
    eng = DecodeEngine(ns.model, device=dev, max_batch=ns.batch, max_context=ns.context, seed=1234 + rank,
                       steps_per_graph=ns.steps_per_graph, weight_dtype=ns.weights, kv_dtype=ns.kv)
    if eng.max_batch < ns.batch:
        raise SystemExit(f"--batch {ns.batch} exceeds the engine's row limit {eng.max_batch} for --weights {ns.weights}")
    tps = topics()
    opts = {"eos_id": -1}  # forced length: random weights never emit a meaningful EOS

    def prompts(step):
        return [f"In {ns.words} words, please give me information about {tps[(step * ns.batch + i + rank * 7) % len(tps)]}"
                for i in range(ns.batch)]

    def one_step(step):
        res = eng.generate(prompts(step), n_tok, [dict(opts, seed=step * 100003 + i + 1) for i in range(ns.batch)])
        return sum(r.eval_count for r in res)

    def sync():
        if not cpu:
            torch.cuda.synchronize(dev)

    def progress(what: str) -> None:  # stderr heartbeat (long runs must keep writing; the JSON stays on stdout)
        if rank == 0:
            print(f"[bench] {what} {time.strftime('%H:%M:%S')}", file=sys.stderr, flush=True)

    for w in range(ns.warmup):
        one_step(-1 - w)
        progress(f"warmup {w + 1}/{ns.warmup}")

    meter = None
    if not ns.no_energy and not cpu:
        try:
            from cain_amd.energy import EnergyMeter
            # host CPU + RAM energy is shared by every rank of the node: each rank is charged its share
            meter = EnergyMeter(devices=[local], period_ms=100.0, keep_samples=False, sources=("gpu", "cpu", "ram"),
                                host_share=1.0 / int(os.environ.get("LOCAL_WORLD_SIZE", world)))
            # the board stays ~15 % above its idle floor for seconds after a burst: settle first
            sync()
            time.sleep(max(0.0, ns.settle))
            meter.measure_idle(2.0)
        except Exception as exc:  # energy is auxiliary to the throughput metric
            print(f"[bench] energy meter unavailable: {exc}", file=sys.stderr)
            meter = None
        one_step(-100)  # back to a warm steady state before the timed region

    def barrier():
        if world > 1:
            dist.barrier()
        sync()

    barrier()
    if meter:
        meter.start()
    t0 = time.perf_counter()
    toks = 0
    for s in range(ns.steps):
        toks += one_step(s)
        progress(f"step {s + 1}/{ns.steps}")
    barrier()
    dt = time.perf_counter() - t0
    reading = meter.stop() if meter else None

    # ---- batch 1, the reference's one-request-at-a-time protocol (outside the timed region): after a settle, the
    # median of --single-trials generations of the full request length per (model, weight dtype), each with its
    # own energy window; the bench model on bf16 / fp8 / MXFP4 weights (fp4: the reference's 4-bit precision class)
    # and the --single-models on bf16 / fp4.
    single = {}  # (model, dtype) -> (median tok/s, median J/token)

    def single_stream(model: str, dtype: str, engine=None):
        own = engine is None
        e1 = engine or DecodeEngine(model, device=dev, max_batch=1, max_context=ns.context, seed=1234 + rank,
                                    steps_per_graph=ns.steps_per_graph, weight_dtype=dtype, kv_dtype=ns.kv)
        e1.generate(prompts(-7)[:1], min(n_tok, 32), [dict(opts, seed=7)])  # warm the batch-1 graphs
        rates, jpt = [], []
        for t in range(ns.single_trials):
            barrier()
            time.sleep(ns.single_settle)
            if meter:
                meter.start()
            t1 = time.perf_counter()
            r1 = e1.generate(prompts(-8 - t)[:1], n_tok, [dict(opts, seed=8 + t)])[0]
            sync()
            dt1 = time.perf_counter() - t1
            rd1 = meter.stop() if meter else None
            rates.append(r1.eval_count / dt1)
            jpt.append(rd1.gpu_energy_j / max(1, r1.eval_count) if rd1 is not None else float("nan"))
        if own:
            e1.close()
            del e1
            if not cpu:
                torch.cuda.empty_cache()
        progress(f"single stream {model} {dtype}: {statistics.median(rates):.1f} tok/s")
        return statistics.median(rates), statistics.median(jpt)

    cases = []
    if not ns.no_single:
        cases = [(ns.model, "bf16")]
        if not cpu and ns.weights == "bf16":
            cases += [(ns.model, "fp8"), (ns.model, "fp4")]
            cases += [(m, dt) for m in filter(None, ns.single_models.split(",")) if m != ns.model
                      for dt in ("bf16", "fp4")]
            cases += [(m, "fp4") for m in filter(None, ns.single_fp4_models.split(","))
                      if m != ns.model and (m, "fp4") not in cases]
            q4s = [q for q in filter(None, ns.single_q4.split(",")) if q in ("q4_0", "q4_k")]
            cases += [(m, q) for q in q4s for m in dict.fromkeys(c[0] for c in cases)]
        sync()
        time.sleep(max(0.0, ns.settle))  # the board returns toward idle after the batched steps
    for model, dtype in cases:
        try:
            single[(model, dtype)] = single_stream(model, dtype, eng if (model, dtype) == (ns.model, ns.weights) else None)
        except Exception as exc:  # auxiliary measurement
            print(f"[bench] single stream {model} {dtype} unavailable: {exc}", file=sys.stderr)
            single[(model, dtype)] = (float("nan"), float("nan"))

    flat = [v for c in cases for v in single[c]]
    vals = torch.tensor([dt, float(toks), reading.gpu_energy_j if reading else float("nan"),
                         reading.idle_subtracted_j if reading else float("nan"),
                         reading.total_energy_j if reading else float("nan"),
                         meter.idle_power_w if meter and getattr(meter, "idle_power_w", None) else float("nan")] + flat,
                        dtype=torch.float64, device=dev)
    if world > 1:
        allv = [torch.zeros_like(vals) for _ in range(world)]
        dist.all_gather(allv, vals)
        allv = torch.stack(allv).cpu()
    else:
        allv = vals[None].cpu()
    t_max = float(allv[:, 0].max())
    tokens = float(allv[:, 1].sum())
    energy = float(allv[:, 2].sum())
    energy_idle_sub = float(allv[:, 3].sum())
    energy_total = float(allv[:, 4].sum())
    idle_w = float(allv[:, 5].mean())
    ss = {c: (float(allv[:, 6 + 2 * i].mean()), float(allv[:, 7 + 2 * i].mean())) for i, c in enumerate(cases)}

    def rnd(v, nd):
        return None if math.isnan(v) else round(v, nd)

    def ss_get(model, dtype, j):
        return rnd(ss.get((model, dtype), (float("nan"), float("nan")))[j], 4 if j else 2)
    value = tokens / t_max
    base_tps, base_jpt = BASELINE.get((ns.model, ns.words), (None, None))
    if rank == 0:
        out = {
            "metric": "tokens/sec (on-device generation; also J/generated-token)",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": ns.steps,
            "warmup": ns.warmup,
            "ms_per_step": round(1000 * t_max / ns.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base_tps, 2) if base_tps else None,
            "dtype": ("bf16" if ns.weights == "bf16" else
                      f"bf16 activations, GGUF {ns.weights.upper()} weights (the blocks' exact values, W4A16)"
                      if ns.weights in ("q4_0", "q4_k") else
                      (f"MXFP4 (e2m1 + e8m0 block-32) weights; GEMM activations per-row e4m3 above "
                       f"{max(16, ns.w4a8_min_rows)} rows (W4A8: this {ns.batch}-row run), bf16 at or below (W4A16)"
                       if getattr(eng, "w4a8", False) and ns.batch > max(16, ns.w4a8_min_rows) else
                       "bf16 activations, MXFP4 (e2m1 + e8m0 block-32) weights (W4A16)") if ns.weights == "fp4" else
                      "fp8-e4m3 weights and per-row e4m3 GEMM activations (W8A8), bf16 elsewhere"
                      if getattr(eng, "w8a8", False) else "bf16 activations, fp8-e4m3 weights")
                     + (", fp8-e4m3 KV cache" if ns.kv == "fp8" else ""),
            "device": "cpu (torch oracle)" if cpu else "MI355X",
            "data": ("synthetic (reference topics.csv prompts, random-init weights)" if not ns.checkpoint else
                     f"synthetic prompts (reference topics.csv), checkpoint weights ({os.path.basename(ns.checkpoint)})"),
            "config": {"model": ns.model, "global_batch": ns.batch * world, "seq_len": n_tok,
                       "parallelism": f"dp{world}", "words": ns.words, "trials_per_gpu": ns.batch,
                       "sampling": "ollama defaults (T=0.8, top_k=40, top_p=0.9, repeat_penalty=1.1), eos disabled"},
            "tokens_generated": int(tokens),
            "J_per_token": round(energy / tokens, 5) if not math.isnan(energy) else None,
            "J_per_token_idle_subtracted": (round(energy_idle_sub / tokens, 5)
                                            if not math.isnan(energy_idle_sub) else None),
            "J_per_token_incl_host": (round(energy_total / tokens, 5) if not math.isnan(energy_total) else None),
            "host_energy_source": reading.cpu_energy_source if reading else None,
            "avg_gpu_power_W": round(energy / t_max / world, 1) if not math.isnan(energy) else None,
            "idle_power_W": rnd(idle_w, 1),
            "single_stream_trials": ns.single_trials,
            "single_stream_tok_per_s": ss_get(ns.model, "bf16", 0),
            "single_stream_J_per_token": ss_get(ns.model, "bf16", 1),
            "single_stream_fp8_tok_per_s": ss_get(ns.model, "fp8", 0),
            "single_stream_fp8_J_per_token": ss_get(ns.model, "fp8", 1),
            "single_stream_fp4_tok_per_s": ss_get(ns.model, "fp4", 0),
            "single_stream_fp4_J_per_token": ss_get(ns.model, "fp4", 1),
            "single_stream_q4_k_tok_per_s": ss_get(ns.model, "q4_k", 0),
            "single_stream_q4_k_J_per_token": ss_get(ns.model, "q4_k", 1),
            "single_stream_by_model": {
                m: {dt: {"tok_per_s": ss_get(m, dt, 0), "J_per_token": ss_get(m, dt, 1)}
                    for dt in ("bf16", "fp8", "fp4", "q4_0", "q4_k") if (m, dt) in ss}
                | {"baseline": dict(zip(("tok_per_s", "J_per_token"), BASELINE.get((m, ns.words), (None, None))))}
                for m in dict.fromkeys(c[0] for c in cases)},
            "baseline": {"tok_per_s": base_tps, "J_per_token": base_jpt, "hardware": "MacBook Pro M2 (est.)"},
            "vs_baseline_J_per_token": (round(base_jpt / (energy / tokens), 2)
                                        if base_jpt and not math.isnan(energy) and energy > 0 else None),
            "single_stream_vs_baseline_J_per_token": (round(base_jpt / ss_get(ns.model, "bf16", 1), 3)
                                                      if base_jpt and ss_get(ns.model, "bf16", 1) else None),
            "single_stream_fp4_vs_baseline_J_per_token": (round(base_jpt / ss_get(ns.model, "fp4", 1), 3)
                                                          if base_jpt and ss_get(ns.model, "fp4", 1) else None),
            # wide-batch GEMM plans in use: N x K @ rows -> k-splits x ring variant (csrc/wgemm.hip)
            "wgemm_plans": {f"{t['n']}x{t['k']}@{t['m']}": f"{t['ks']}x{t['variant']}"
                            for t in getattr(eng, "wgemm_plans", [])},
        }
        print(json.dumps(out), flush=True)
    if meter:
        meter.close()
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
