#!/usr/bin/env python3
"""Where a wide-batch GEMM's time goes (csrc/wgemm.hip, diagnostic variant 7 = the default ring + timestamps).

For each decode projection of a model at 256 rows: the call's event time (kernel + split-K reduce launch) with
the default variant, and from the stamped variant per workgroup (lane 0 of compute wave 0 and of loader wave 8):
start, stage 0 ready (first ring barrier passed), stage nst/2 ready, loop end, slab stores drained (ks > 1) or
epilogue stores drained (ks = 1), end -- s_memrealtime ticks (10 ns) relative to the first workgroup's start,
median / max over workgroups -- and the shader clock (s_memtime ticks / realtime).

    python tools/wgemm_trace.py [--model llama3.1:8b] [--only o,down] [--rows 256]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cain_amd import ops  # noqa: E402
from cain_amd.models.config import get_config  # noqa: E402
from cain_amd.models.weights import pack_mfma_a  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1:8b")
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--only", default="")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="0", help="ring variants (0 default, 5 loader-wave sums of squares)")
    ns = ap.parse_args()
    cfg = get_config(ns.model)
    dev = torch.device("cuda")
    lib = ops.load()
    lib.cain_wgemm_set_variant.argtypes = [ops.ci]
    lib.cain_wgemm_set_stamps.argtypes = [ctypes.c_void_p]
    M = ns.rows
    shapes = [("qkv", cfg.qkv_dim, cfg.d_model, ops.EPI_BF16, True),
              ("o", cfg.d_model, cfg.q_dim, ops.EPI_RESID, False),
              ("gateup", 2 * cfg.ffn, cfg.d_model, ops.EPI_SILU, True),
              ("down", cfg.d_model, cfg.ffn, ops.EPI_RESID, False),
              ("lm_head", cfg.vocab, cfg.d_model, ops.EPI_F32, True)]
    stamps = torch.zeros(4096 * 16, device=dev, dtype=torch.int64)
    for name, N, K, epi, norm in shapes:
        if ns.only and name not in ns.only.split(","):
            continue
        wbytes = N * K * 2
        ncopy = max(2, -(-(512 << 20) // wbytes))
        torch.manual_seed(0)
        Wp = [pack_mfma_a((torch.randn(N, K, device=dev) * 0.02).bfloat16()) for _ in range(ncopy)]
        x = (2 * torch.randn(M, K, device=dev)).bfloat16()
        n_out = N // 2 if epi in (ops.EPI_SILU, ops.EPI_GELU) else N
        out = torch.zeros(M, n_out, device=dev, dtype=torch.float32 if epi == ops.EPI_F32 else torch.bfloat16)

        def run(i):
            ops.skinny_gemm(Wp[i % ncopy], x, N, epi, out=out, norm=norm, eps=1e-6)

        def timeit():
            for i in range(3):
                run(i)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(ns.iters):
                run(i)
            b.record()
            torch.cuda.synchronize()
            return a.elapsed_time(b) * 1000.0 / ns.iters

        for var in [int(v) for v in ns.variants.split(",")]:
            lib.cain_wgemm_set_variant(var)
            y = ops.skinny_gemm(Wp[0], x, N, ops.EPI_F32, norm=norm, eps=1e-6)
            lib.cain_wgemm_set_variant(0)
            y0 = ops.skinny_gemm(Wp[0], x, N, ops.EPI_F32, norm=norm, eps=1e-6)
            print(f"{name} variant {var}: max |y - y(variant 0)| / max|y0| = "
                  f"{float((y - y0).abs().max() / y0.abs().max()):.3e}", flush=True)
            report(name, N, K, M, var, run, timeit, stamps, lib)
        del Wp
        torch.cuda.empty_cache()
    return 0


STAMPED = {0: 7}  # variant -> its timestamped build (csrc/wgemm.hip wg_launch_v)


def report(name, N, K, M, var, run, timeit, stamps, lib):
    if True:
        lib.cain_wgemm_set_variant(var)
        t_def = timeit()
        lib.cain_wgemm_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
        lib.cain_wgemm_set_variant(STAMPED[var])
        t_st = timeit()
        stamps.zero_()
        run(1)
        torch.cuda.synchronize()
        lib.cain_wgemm_set_variant(0)
        lib.cain_wgemm_set_stamps(None)
        plan = ops.wide_gemm_plan(N, K, M)
        s = stamps.view(-1, 2, 8)
        live = s[:, 0, 0] != 0
        s = s[live].double()
        t0 = s[:, :, 0].min()
        rel = (s - t0) * 0.01  # us (100 MHz realtime)
        clk = (s[:, 0, 7] - s[:, 0, 1]) / (s[:, 0, 6] - s[:, 0, 0]).clamp(min=1) * 0.1  # GHz
        print(f"{name} variant {var} N={N} K={K} M={M} plan={plan} grid={int(live.sum())}: call {t_def:.2f} us "
              f"(stamped {t_st:.2f}); clock median {clk.median():.2f} GHz")
        labels = ["start", "stage0", "mid", "loop_end", "drained", "end"]
        idx = [0, 2, 3, 4, 5, 6]
        for wv, role in ((0, "compute"), (1, "loader")):
            cells = []
            for lab, j in zip(labels, idx):
                col = rel[:, wv, j]
                if role == "loader" and j >= 5:
                    continue
                cells.append(f"{lab} {col.median():6.2f}/{col.max():6.2f}")
            print(f"   {role:8s} " + "  ".join(cells) + "   (median/max us)")
        dur = rel[:, 0, 6] - rel[:, 0, 0]
        loop = rel[:, 0, 4] - rel[:, 0, 2]
        print(f"   per-WG: duration {dur.median():.2f}/{dur.max():.2f}  fill (start->stage0) "
              f"{(rel[:, 0, 2] - rel[:, 0, 0]).median():.2f}  loop {loop.median():.2f}  "
              f"epilogue {(rel[:, 0, 5] - rel[:, 0, 4]).median():.2f} us", flush=True)


if __name__ == "__main__":
    sys.exit(main())
