#!/usr/bin/env python3
"""Wide-batch GEMM A/B on one GPU: the LDS-DMA ring kernel (csrc/wgemm.hip) vs the previous batched kernel
(csrc/gemm.hip bgemm) vs hipBLASLt (torch.mm), on the decode projections of a model at M rows.

Weights rotate over enough copies that every call streams from HBM (> 2x the 256 MiB Infinity Cache), as in
a real decode step where each layer's weights are read once.  Prints one JSON line per (shape, M, path):
us per call and effective weight TB/s; plus the numerics of the wide kernel vs an fp32 reference.

    python tools/wgemm_bench.py [--model llama3.1:8b] [--rows 128,256] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cain_amd import ops  # noqa: E402
from cain_amd.models.config import get_config  # noqa: E402
from cain_amd.models.weights import pack_mfma_a  # noqa: E402


def shapes(cfg):
    return [("qkv", cfg.qkv_dim, cfg.d_model, ops.EPI_BF16, True),
            ("o", cfg.d_model, cfg.q_dim, ops.EPI_RESID, False),
            ("gateup", 2 * cfg.ffn, cfg.d_model, ops.EPI_SILU, True),
            ("down", cfg.d_model, cfg.ffn, ops.EPI_RESID, False),
            ("lm_head", cfg.vocab, cfg.d_model, ops.EPI_F32, True)]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1:8b")
    ap.add_argument("--rows", default="128,256")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--no-lt", action="store_true")
    ap.add_argument("--no-old", action="store_true")
    ap.add_argument("--variants", default="0", help="ring variants to time (csrc/wgemm.hip wg_launch_v)")
    ap.add_argument("--splits", default="", help="split plans target:ksmax,... to time (default plan only)")
    ns = ap.parse_args()
    cfg = get_config(ns.model)
    dev = torch.device("cuda")
    lib = ops.load()
    lib.cain_wgemm_set_min_m.argtypes = [ops.ci]
    lib.cain_wgemm_set_variant.argtypes = [ops.ci]
    lib.cain_wgemm_set_split.argtypes = [ops.ci, ops.ci]

    variants = [int(v) for v in ns.variants.split(",")]
    splits = [tuple(int(y) for y in x.split(":")) for x in ns.splits.split(",") if x] or [(256, 8)]
    rows = [int(r) for r in ns.rows.split(",")]
    for name, N, K, epi, norm in shapes(cfg):
        if ns.only and name not in ns.only.split(","):
            continue
        wbytes = N * K * 2
        ncopy = max(2, -(-(512 << 20) // wbytes))
        torch.manual_seed(0)
        W = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(ncopy)]
        Wp = [pack_mfma_a(w) for w in W]
        for M in rows:
            x = (2 * torch.randn(M, K, device=dev)).bfloat16()
            n_out = N // 2 if epi in (ops.EPI_SILU, ops.EPI_GELU) else N
            out = torch.zeros(M, n_out, device=dev, dtype=torch.float32 if epi == ops.EPI_F32 else torch.bfloat16)

            def run(i):
                ops.skinny_gemm(Wp[i % ncopy], x, N, epi, out=out, norm=norm, eps=1e-6)

            def timeit(fn):
                for i in range(3):
                    fn(i)
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for i in range(ns.iters):
                    fn(i)
                b.record()
                torch.cuda.synchronize()
                return a.elapsed_time(b) * 1000.0 / ns.iters

            res = {"model": ns.model, "shape": name, "N": N, "K": K, "M": M}
            # numerics of the wide path (F32 epilogue, one copy)
            lib.cain_wgemm_set_min_m(64)
            y = ops.skinny_gemm(Wp[0], x, N, ops.EPI_F32, norm=norm, eps=1e-6)
            xr = x.float()
            if norm:
                xr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6)
            ref = xr @ W[0].float().t()
            res["rel_err"] = float((y - ref).norm() / ref.norm())
            for v in variants:
                for tgt, ksm in splits:
                    lib.cain_wgemm_set_variant(v)
                    lib.cain_wgemm_set_split(tgt, ksm)
                    key = "wide_us" if (v, tgt, ksm) == (variants[0],) + splits[0] else f"wide_v{v}_s{tgt}x{ksm}_us"
                    res[key] = timeit(run)
            lib.cain_wgemm_set_variant(variants[0])
            lib.cain_wgemm_set_split(*splits[0])
            if not ns.no_old:
                lib.cain_wgemm_set_min_m(0)
                res["old_us"] = timeit(run)
                lib.cain_wgemm_set_min_m(64)
            if not ns.no_lt:
                xo = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                res["hipblaslt_us"] = timeit(lambda i: torch.mm(x, W[i % ncopy].t(), out=xo))
            for k in [k for k in list(res) if k.endswith("_us")]:
                if k in res:
                    res[k.replace("_us", "_TBps")] = round(wbytes / (res[k] * 1e-6) / 1e12, 3)
                    res[k] = round(res[k], 2)
            print(json.dumps(res), flush=True)
        del W, Wp
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
