#!/usr/bin/env python3
"""Named GPU run sets: every GPU call of the build is ``python3 tools/gpu_manifest.py <set>`` -- one manifest
instead of one shell script per call (round 3 left 45 ``tools/r3*.sh``; their findings are in profiles/r3/README.md
and the git history).  Each set is a list of steps ``(name, time limit s, command)`` run in order by
tools/gpu_steps.sh, which logs each step to gpurun_out/<set>/<name>.log and stops the set after a crash or time
limit.  ``python3 tools/gpu_manifest.py --list`` prints the sets.

Conventions: kernel statistics come from ``rocprofv3 --kernel-trace --stats`` of graph-replayed bench runs
(per-kernel averages include no host time); bench A/Bs run the variants interleaved on one box (DVFS and
box-to-box spread are ~1-3 %)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PY = "python3"
TEST = f"{PY} -u -m pytest -x -q --timeout 300 --timeout-method thread"
B1 = f"{PY} bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy"


def prof(tag: str, args: str, limit: int = 300):
    """A rocprof kernel-stats step of bench.py (the trace CSV itself is dropped, the stats CSV kept)."""
    return (f"prof_{tag}", limit,
            f"rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_{tag} -o run -- "
            f"{PY} bench.py {args} && find gpurun_out/prof_{tag} -name '*kernel_trace.csv' -delete")


#: every llama3.1:8b wide-GEMM shape on the 256-column kernel (csrc/wgemm256.hip), default split counts
PL_V5 = "6144:4096:256:0:5,4096:4096:256:0:5,28672:4096:256:0:5,4096:14336:256:0:5,128256:4096:256:0:5"

SETS = {
    # round 4: MXFP4 weights (gemm_w4.hip) -- kernels vs fp32, engine vs oracle, then the single-stream rates
    "r4_fp4": [
        ("w4_tests", 600, f"{TEST} tests/test_w4_gpu.py"),
        ("engine_tests", 600, f"{TEST} tests/test_engine_gpu.py tests/test_w8_gpu.py"),
        ("b1_llama_fp4", 300, f"{B1} --weights fp4"),
        ("b1_llama_bf16", 300, B1),
        ("b1_qwen_fp4", 300, f"{B1} --weights fp4 --model qwen2:1.5b"),
        ("b1_gemma_fp4", 300, f"{B1} --weights fp4 --model gemma:2b"),
        prof("b1_llama_fp4", "--batch 1 --steps 1 --warmup 1 --no-energy --no-single --weights fp4"),
    ],
    # round 4: the persistent stream MXFP4 kernel
    "r4_fp4b": [
        ("w4_tests", 600, f"{TEST} tests/test_w4_gpu.py"),
        ("b1_llama_fp4", 300, f"{B1} --weights fp4"),
        ("b1_qwen_fp4", 300, f"{B1} --weights fp4 --model qwen2:1.5b"),
        ("b1_gemma_fp4", 300, f"{B1} --weights fp4 --model gemma:2b"),
        prof("b1_llama_fp4b", "--batch 1 --steps 1 --warmup 1 --no-energy --no-single --weights fp4"),
    ],
    # in-graph few-row GEMM microbenchmarks (every MXFP4 kernel shape vs fp8 / bf16)
    "r4_w4bench2": [
        ("w4_tests", 600, f"{TEST} tests/test_w4_gpu.py"),
        ("w4bench_llama", 400, f"{PY} tools/w4_bench.py --variants rule,0,1,2,3,4,5"),
        ("b1_llama_fp4", 300, f"{B1} --weights fp4"),
    ],
    "r4_fp4c": [
        ("w4_tests", 600, f"{TEST} tests/test_w4_gpu.py"),
        ("w4bench_llama", 400, f"{PY} tools/w4_bench.py --variants rule,0,1,2 --dtypes fp4"),
        ("b1_llama_fp4", 300, f"{B1} --weights fp4"),
        ("b1_qwen_fp4", 300, f"{B1} --weights fp4 --model qwen2:1.5b"),
        prof("b1_llama_fp4c", "--batch 1 --steps 1 --warmup 1 --no-energy --no-single --weights fp4"),
    ],
    "r4_norm": [
        ("norm_on", 300, f"{PY} tools/w4_bench.py --variants 1,3,4 --norm on --dtypes fp4,fp8"),
        ("norm_off", 300, f"{PY} tools/w4_bench.py --variants 1,3,4 --norm off --dtypes fp4,fp8"),
    ],
    "r4_w4bench": [
        ("w4bench_llama", 400, f"{PY} tools/w4_bench.py --variants rule,0,1,2,3,4,5 --occ 0"),
        ("w4bench_occ", 300, f"{PY} tools/w4_bench.py --variants 0,2 --occ 1,3,4 --dtypes fp4"),
        ("w4bench_qwen", 300, f"{PY} tools/w4_bench.py --model qwen2:1.5b --variants rule,0,2,3,4,5"),
    ],
    # the whole GPU suite (what the driver runs at round end)
    # pruned variants / env switches and the scaled fp16 split-K slabs: the affected kernels' tests, then the headline
    "r4_prune": [
        ("prune_tests", 900, f"{TEST} tests/test_wgemm_gpu.py tests/test_ops_gpu.py tests/test_w8a8_gpu.py "
                             f"tests/test_engine_gpu.py"),
        ("bench", 400, f"{PY} bench.py --gpus 1 --steps 10 --warmup 3"),
    ],
    # headline A/B, interleaved: the round-3 library (ab/libcain_kernels_head.so: unscaled fp16 slabs, before the
    # pruning), the tree without the slab scaling (ab/libcain_kernels_noscale.so) and the tree
    "r4_slab_ab": [(f"hl_{tag}_{i}", 300, f"{env}{PY} bench.py --steps 3 --warmup 1 --no-single --no-energy")
                   for i in range(2) for tag, env in (("head", "CAIN_KERNELS_LIB=ab/libcain_kernels_head.so "),
                                                      ("noscale", "CAIN_KERNELS_LIB=ab/libcain_kernels_noscale.so "),
                                                      ("new", ""))],
    # batch-1 energy lever: CU-limited streams (tools/cu_sweep.py), after the engine's CU-limit test
    "r4_cu": [
        ("cu_tests", 300, f"{TEST} tests/test_engine_gpu.py -k cu_limited"),
        ("cu_sweep", 900, f"{PY} tools/cu_sweep.py --out gpurun_out/r4_cu/cu_sweep.jsonl"),
    ],
    # board power after a 1,000-word on-device run (the study's cooldown evidence)
    "r4_cooldown": [("cooldown", 600, f"{PY} tools/cooldown_trace.py --out gpurun_out/r4_cooldown/cooldown.json "
                                      f"--csv gpurun_out/r4_cooldown/cooldown_trace.csv")],
    # W4A8: MXFP4 weights at trial-batch widths (wgemm8.hip FP4)
    "r4_w4a8": [
        ("w4a8_tests", 600, f"{TEST} tests/test_w4a8_gpu.py"),
        ("b256_fp4", 400, f"{PY} bench.py --weights fp4 --steps 3 --warmup 1 --no-single --no-energy"),
        prof("b256_fp4", "--weights fp4 --steps 1 --warmup 1 --no-single --no-energy"),
    ],
    # the GPU suite in two calls (a gpurun call is limited to 20 min)
    "suite_a": [("kernels", 1100, f"{PY} -u -m pytest -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py "
                                  f"tests/test_wgemm_gpu.py tests/test_w4_gpu.py tests/test_w4a8_gpu.py "
                                  f"tests/test_w8_gpu.py tests/test_w8a8_gpu.py tests/test_kv8_gpu.py")],
    "suite_b": [("engine", 1100, f"{PY} -u -m pytest -q --timeout 600 --timeout-method thread tests/test_engine_gpu.py "
                                 f"tests/test_continuous_gpu.py tests/test_energy_gpu.py tests/test_fullsize_gpu.py")],
    # round-end evidence: the driver's bench command, then kernel stats of the headline and of batch-1 fp4
    "r4_final": [
        ("bench", 900, f"{PY} bench.py --gpus 1 --steps 20 --warmup 5"),
        prof("headline_final", "--steps 1 --warmup 1 --no-single --no-energy"),
        prof("b1_llama_fp4_final", "--batch 1 --steps 1 --warmup 1 --no-energy --no-single --weights fp4"),
    ],
    # separate precision configurations of the headline workload (bf16 stays the headline), then the smoke test
    "r4_configs": [
        ("cfg_fp4", 300, f"{PY} bench.py --weights fp4 --steps 3 --warmup 1 --no-single"),
        ("cfg_fp4_kv8", 300, f"{PY} bench.py --weights fp4 --kv fp8 --steps 3 --warmup 1 --no-single"),
        ("smoke", 300, f"{PY} -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"),
    ],
    # W4A16 vs W4A8 at mid widths (MXFP4 engines; runtime default: W4A8 above 64 rows)
    "r4_w4a8_cross": [(f"b{b}_t{t}", 240, f"{PY} bench.py --weights fp4 --batch {b} --steps 2 --warmup 1 --no-single "
                                          f"--no-energy --w4a8-min-rows {t}")
                      for b in (24, 48, 64) for t in (16, 64)],
    # decode steps per captured graph (host launches per generation), headline, interleaved
    "r4_spg": [(f"spg{k}_{i}", 240, f"{PY} bench.py --steps 3 --warmup 1 --no-single --no-energy --steps-per-graph {k}")
               for i in range(2) for k in (16, 32, 64)],
    # wave-per-row activation quantiser (wgemm8.hip quant_rows_wave_kernel) vs the 256-thread one, fp4 256 rows
    "r4_quant_ab": [("quant_tests", 300, f"{TEST} tests/test_w8a8_gpu.py tests/test_w4a8_gpu.py")]
    + [(f"q_{tag}_{i}", 240, f"{env}{PY} bench.py --weights fp4 --steps 3 --warmup 1 --no-single --no-energy")
       for i in range(2) for tag, env in (("head", "CAIN_KERNELS_LIB=ab/libcain_kernels_head.so "), ("new", ""))],
    # round 5: deterministic W4 row sums + the gain-folded fp4 oracle at full size, then batch-1 fp4 rates
    "r5_check": [
        ("w4_tests", 600, f"{TEST} tests/test_w4_gpu.py"),
        ("fp4_gains", 600, f"{TEST} tests/test_fullsize_gpu.py -k nonunit"),
        ("b1_llama_fp4", 300, f"{B1} --weights fp4"),
        ("b1_qwen_fp4", 300, f"{B1} --weights fp4 --model qwen2:1.5b"),
    ],
    # round 5: the reference's design on MXFP4 weights (both arms fp4), n = 10, 10 s cooldown, one session per call
    "r5_fp4_study": [("study", 1150, "CAIN_STUDY_WEIGHTS=fp4 STUDY_NAME=fp4_r5 COOLDOWN_MS=10000 REPS=10 "
                                     "IDLE_SETTLE_S=12 bash tools/study_chunk.sh 960")],
    # its second replicate (another seed): n = 20 per cell with the first
    "r5_fp4_study_b": [("study", 1150, "CAIN_STUDY_WEIGHTS=fp4 STUDY_NAME=fp4_r5b SEED=2026 COOLDOWN_MS=10000 REPS=10 "
                                       "IDLE_SETTLE_S=12 bash tools/study_chunk.sh 960")],
    # its third replicate (n = 30 per cell with the first two)
    "r5_fp4_study_c": [("study", 1150, "CAIN_STUDY_WEIGHTS=fp4 STUDY_NAME=fp4_r5c SEED=2027 COOLDOWN_MS=10000 REPS=10 "
                                       "IDLE_SETTLE_S=12 bash tools/study_chunk.sh 960")],
    # round 5: the 256-column wide GEMM (wgemm256.hip): numerics first (a new kernel), then isolated shape timings
    # against the 128-column ring, then the headline with every llama shape on it (interleaved with the default)
    "r5_w256": [
        ("w256_tests", 300, f"{TEST} tests/test_wgemm256_gpu.py"),
        ("wgemm_bench", 300, f"{PY} tools/wgemm_bench.py --rows 256 --variants 0,5 --no-lt --no-old "
                             f"--splits 256:16,256:8,192:16"),
    ] + [(f"hl_{tag}_{i}", 240, f"{env}{PY} bench.py --steps 3 --warmup 1 --no-single --no-energy")
         for i in range(2) for tag, env in (("v0", ""), ("v5", f"CAIN_WGEMM_PLANS={PL_V5} "))],
    # 256-column kernel after the fixed-operand X X^T: numerics, isolated timings, PMC of both kernels
    "r5_w256b": [
        ("w256_tests", 300, f"{TEST} tests/test_wgemm256_gpu.py"),
        ("wgemm_bench", 300, f"{PY} tools/wgemm_bench.py --rows 256 --variants 0,5 --no-lt --no-old"),
        ("pmc", 300, "bash tools/pmc_wgemm.sh r5_w256b/pmc --rows 256 --variants 0,5 --only gateup,down,o"),
    ],
    # ablations of both wide kernels: full / DMA only / MFMA only (old: 0, 8, 9; 256-column: 5, 6, 7), kernel stats
    "r5_w256_abl": [
        ("abl", 300, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_w256_abl/prof -o run -- "
                     f"{PY} tools/wgemm_bench.py --rows 256 --variants 0,8,9,5,6,7 --no-lt --no-old "
                     "--splits 256:16 --only gateup,down,o"),
    ],
    # the 256-column kernel with 64-deep X stages (whole 128-B lines): numerics, ablations, headline A/B
    "r5_w256c": [
        ("w256_tests", 300, f"{TEST} tests/test_wgemm256_gpu.py"),
        ("abl", 300, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_w256c/prof -o run -- "
                     f"{PY} tools/wgemm_bench.py --rows 256 --variants 0,8,9,5,6,7 --no-lt --no-old "
                     "--splits 256:16"),
    ] + [(f"hl_{tag}_{i}", 240, f"{env}{PY} bench.py --steps 3 --warmup 1 --no-single --no-energy")
         for i in range(1) for tag, env in (("v0", ""), ("v5", f"CAIN_WGEMM_PLANS={PL_V5} "))],
    "r5_w256d": [
        ("w256_tests", 300, f"{TEST} tests/test_wgemm256_gpu.py"),
        ("hl_v11", 240, f"CAIN_WGEMM_PLANS={PL_V5.replace(':5', ':11')} {PY} bench.py --steps 3 --warmup 1 --no-single "
                        "--no-energy"),
        ("abl", 300, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_w256d/prof -o run -- "
                     f"{PY} tools/wgemm_bench.py --rows 256 --variants 0,5,11 --no-lt --no-old "
                     "--splits 256:16 --only gateup,down,o,qkv"),
    ],
    # batch-1 QKV: where its 9 us go (the RoPE / KV-append epilogue, the fused norm, the kernel shape)
    "r5_qkv": [
        ("w4_qkv", 300, f"{PY} tools/w4_bench.py --roles qkv,qkv_plain,qkv_plain_nonorm,o --variants rule,0,1,2 "
                        "--dtypes fp4"),
    ],
    # batch 1: the attention merge with its partial outputs loaded beside (m, l); QKV diagnostics; rates; kernel stats
    "r5_b1": [
        ("attn_tests", 300, f"{TEST} tests/test_ops_gpu.py -k 'attention or sample'"),
        ("w4_qkv", 300, f"{PY} tools/w4_bench.py --roles qkv,qkv_plain,qkv_plain_nonorm,o --variants rule,0,1,2 "
                        "--dtypes fp4"),
        ("b1_llama_fp4", 300, f"{B1} --weights fp4"),
        ("b1_qwen_fp4", 300, f"{B1} --weights fp4 --model qwen2:1.5b"),
        prof("b1_llama_fp4_r5", "--batch 1 --steps 1 --warmup 1 --no-energy --no-single --weights fp4"),
    ],
    # attention merge: partial outputs loaded beside (m, l) (tree) vs round 4's two round trips (ab/ library),
    # interleaved on one box; then the driver's bench command (7-model single-stream table)
    "r5_attn_ab": [prof(f"b1_attn_{tag}_{i}", "--batch 1 --steps 1 --warmup 1 --no-energy --no-single --weights fp4")
                   if tag == "new" else
                   (f"prof_b1_attn_{tag}_{i}", 300,
                    f"CAIN_KERNELS_LIB=ab/libcain_kernels_attnold.so rocprofv3 --kernel-trace --stats --output-format csv "
                    f"-d gpurun_out/prof_b1_attn_{tag}_{i} -o run -- {PY} bench.py --batch 1 --steps 1 --warmup 1 "
                    f"--no-energy --no-single --weights fp4 && find gpurun_out/prof_b1_attn_{tag}_{i} "
                    f"-name '*kernel_trace.csv' -delete")
                   for i in range(2) for tag in ("old", "new")],
    # batch-1 fp4: the 8-wave stream kernel on QKV (one 128-k quad round per wave, FOLD epilogue, no spill) and a
    # 16-wave one (variant 6 then; removed after this A/B: profiles/r5/README.md) on QKV / O / down against the
    # rule's kernels, every model's shapes, interleaved twice
    "r5_qkv8": [("w4_tests", 400, f"{TEST} tests/test_w4_gpu.py")] + [
        (f"w4b_{m.replace(':', '_')}_{i}", 240,
         f"{PY} tools/w4_bench.py --model {m} --roles qkv,o,down --variants rule,0,6 --dtypes fp4")
        for i in range(2) for m in ("llama3.1:8b", "qwen2:7b", "mistral:7b", "phi3:3.8b", "gemma:7b", "qwen2:1.5b",
                                     "gemma:2b")],
    # batch-1 fp4 GEMMs with the weights cold (decode), Infinity-Cache-hot (8 copies) and cache-hot (1 copy): what a
    # prefetch of the next kernel's weights could buy
    "r5_mall": [(f"w4_mall_{m.replace(':', '_')}", 240, f"{PY} tools/w4_bench.py --model {m} --roles qkv,o,gateup,down "
                 f"--variants rule --dtypes fp4 --copies 0,8,1,0") for m in ("llama3.1:8b", "qwen2:1.5b")],
    "suite": [("gpu_suite", 1500, f"{PY} -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread")],
    # the driver's bench command
    "bench": [("bench", 900, f"{PY} bench.py --gpus 1 --steps 20 --warmup 5")],
    # round-5 evidence: the driver's bench command (7-model single stream, must fit the driver's 540 s), kernel stats
    # of the headline and of batch-1 fp4, the smoke test
    "r5_final": [
        ("bench", 900, f"{PY} bench.py --gpus 1 --steps 20 --warmup 5"),
        prof("headline_r5", "--steps 1 --warmup 1 --no-single --no-energy"),
        ("smoke", 300, f"{PY} -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"),
    ],
    # ---- round 6 (its one-off call scripts are folded in here; the reverted experiments' patches and data are under
    # profiles/r6/<name>/)
    # the lean chunk-maximum sampler: its tests, the per-phase trace, batch-1 A/B against the round-3 kernel
    # (profiles/r6/sampler/)
    "r6_lean": [("lean_tests", 300, f"{TEST} tests/test_sample_lean_gpu.py"),
                ("lean_trace", 200, f"{PY} -u tools/sample_lean_trace.py")] + [
        (f"b1_cm{mode}_{i}", 300, f"{PY} -u tools/b1_ab.py --models llama3.1:8b,qwen2:1.5b --dtype fp4 --trials 3 "
         f"--sample-cm {mode} --label cm{mode} --out gpurun_out/r6_lean/b1.jsonl")
        for i in range(2) for mode in (1, 3)],
    # batch-1 kernel statistics on MXFP4 (profiles/r6/prof/, profiles/r6/sampler/)
    "r6_b1_prof": [(f"prof_b1_{m.replace(':', '_')}", 300,
                    f"rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_b1_prof/{m.replace(':', '_')} "
                    f"-o b1 -- {PY} tools/b1_ab.py --models {m} --dtype fp4 --trials 1 --label prof && find "
                    f"gpurun_out/r6_b1_prof -name '*kernel_trace.csv' -delete")
                   for m in ("llama3.1:8b", "qwen2:1.5b", "gemma:2b")],
    # PMC counters of the batch-1 gate/up GEMM, MXFP4 against GGUF Q4_0 (profiles/r6/q4/pmc_gateup_fp4_vs_q4_0.json):
    # 8 SQ counters in one pass, no trace domain beside the kernel trace
    "r6_pmc_q4": [(f"pmc_{dt}", 120,
                   f"rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES "
                   f"SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace --stats -d gpurun_out/r6_pmc_q4/{dt} -o pmc -- "
                   f"{PY} tools/w4_bench.py --roles gateup --dtypes {dt} --variants rule") for dt in ("fp4", "q4_0")],
    # batch-1 rates of the seven models on MXFP4 and Q4_K, one box (profiles/r6/b1_fp4_7models_final.jsonl)
    "r6_b1_seven": [(f"b1_{dt}", 900, f"{PY} -u tools/b1_ab.py --dtype {dt} --trials 3 --label {dt} "
                     f"--out gpurun_out/r6_b1_seven/b1.jsonl") for dt in ("fp4", "q4_k")],
    # the same-box per-shape regression table (tools/shape_baseline.py; baselines/): record it, and check a
    # build against it before any batch-1 A/B is believed
    "r6_shapes": [("record", 900, f"{PY} -u tools/shape_baseline.py record --out gpurun_out/r6_shapes/b1_shapes_mi355x.json")],
    "shapes_check": [("check", 900, f"{PY} -u tools/shape_baseline.py check baselines/b1_shapes_mi355x.json")],
    # the final tree: the GPU suite and the smoke test (profiles/r6/tests/)
    "r6_final": [("gpu_suite", 900, f"{PY} -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"),
                 ("smoke", 200, f"{PY} -u -c 'import __graft_entry__ as g; g.smoke()'")],
}


def main(argv) -> int:
    if not argv or argv[0] in ("-h", "--help", "--list"):
        for k, steps in SETS.items():
            print(k, ":", ", ".join(s[0] for s in steps))
        return 0
    steps = [s for name in argv for s in SETS[name]]
    specs = [f"{n}|{t}|{c}" for n, t, c in steps]
    env = dict(os.environ, TMPDIR="/tmp")
    return subprocess.call(["bash", str(ROOT / "tools" / "gpu_steps.sh"), "_".join(argv)] + specs, cwd=str(ROOT),
                           env=env)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
