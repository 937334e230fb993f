#!/usr/bin/env python3
"""Per-kernel microbenchmarks on the flagship shapes (llama3.1:8b unless --model).

Reports time per call and effective HBM bandwidth (weight bytes / time) for each
GEMM role at several row counts and waves-per-workgroup choices, the attention
kernel at several context lengths, and the sampler.  Interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24); prints a JSON summary line per
measurement so results can be copied into profiles/.
"""
from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from cain_amd import ops  # noqa: E402
from cain_amd.models import get_config  # noqa: E402


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1:8b")
    ap.add_argument("--rows", default="1,16,64")
    ap.add_argument("--waves", default="0,4,8,16")
    ap.add_argument("--gemm-only", action="store_true")
    ap.add_argument("--norm", action="store_true", help="fused RMSNorm on qkv/gateup/lm_head (as in the model)")
    ap.add_argument("--roles", default="qkv,o,gateup,down,lm_head")
    ap.add_argument("--attn-only", action="store_true")
    ap.add_argument("--attn", default="1:128,1:1400,16:700,64:1400,128:700,128:1400",
                    help="attention cases M:L (rows : context length)")
    ap.add_argument("--attn-splits", default="auto", help="comma list of split counts ('auto' = the engine's)")
    ap.add_argument("--attn-tmax", type=int, default=1536)
    ap.add_argument("--attn-kv", choices=("bf16", "fp8"), default="bf16", help="KV-cache element type")
    ns = ap.parse_args()
    cfg = get_config(ns.model)
    dev = torch.device("cuda")
    d, F, V = cfg.d_model, cfg.ffn, cfg.vocab
    # a weight copy per role (random bytes: timing only); sized > Infinity Cache in aggregate
    roles = {
        "qkv": (cfg.qkv_dim, d, ops.EPI_BF16),
        "o": (d, cfg.q_dim, ops.EPI_RESID),
        "gateup": (2 * F, d, ops.EPI_SILU),
        "down": (d, F, ops.EPI_RESID),
        "lm_head": (V, d, ops.EPI_F32),
    }
    # several copies per role so consecutive calls stream > 600 MB (defeats the 256 MB Infinity Cache,
    # as a real decode step does: it streams every weight once)
    W = {}
    for k, (n, k_, _) in roles.items():
        ncopy = max(1, math.ceil(600e6 / (n * k_ * 2)))
        W[k] = [torch.randn(n // 16, k_ // 32, 64, 8, device=dev).bfloat16() for _ in range(ncopy)]
    roles = {r: v for r, v in roles.items() if r in ns.roles.split(",")}
    W = {r: W[r] for r in roles}
    res = []
    if ns.attn_only:
        ns.rows = ""
        ns.gemm_only = False
    for M in [int(x) for x in ns.rows.split(",") if x]:
        for role, (n, k, epi) in roles.items():
            x = torch.randn(M, k, device=dev).bfloat16()
            out = torch.zeros(M, n // 2 if epi == ops.EPI_SILU else n, device=dev,
                              dtype=torch.float32 if epi == ops.EPI_F32 else torch.bfloat16)
            ss = torch.zeros(64, device=dev)
            g = torch.ones(k, device=dev).bfloat16() if ns.norm and role in ("qkv", "gateup", "lm_head") else None
            variants = [(False, int(w)) for w in ns.waves.split(",")]
            if ops.gemm_ws_bytes(n, k, M) > 0:
                variants = [(False, 0), (True, 0)] if M <= 64 else [(True, 0)]  # skinny kernel: M <= 64
            for batched, wv in variants:
                it = [0]

                def run():
                    w = W[role][it[0] % len(W[role])]
                    it[0] += 1
                    ops.skinny_gemm(w, x, n, epi, out=out, waves=wv, batched=batched, norm=g is not None)
                us = timeit(run)
                gbs = n * k * 2 / us / 1e3
                r = dict(kind="gemm", model=cfg.name, role=role, M=M, N=n, K=k, waves=wv, us=round(us, 2),
                         TBps=round(gbs / 1e3, 3), path="batched" if batched else "skinny")
                res.append(r)
                print(json.dumps(r), flush=True)
    if ns.gemm_only:
        return
    # attention (random bytes in the fragment-major cache layout: timing only)
    T_max = ns.attn_tmax
    from cain_amd.engine.engine import attention_splits
    for case in ns.attn.split(","):
        M, L = (int(x) for x in case.split(":"))
        kc = torch.randn(M, cfg.n_kv_heads, T_max, cfg.head_dim, device=dev).bfloat16()
        vt = torch.randn(M, cfg.n_kv_heads, cfg.head_dim, T_max, device=dev).bfloat16()
        esz = 2
        if ns.attn_kv == "fp8":  # e4m3 bytes (uint8 storage selects the kernel's fp8 path)
            kc, vt = kc.to(torch.float8_e4m3fn).view(torch.uint8), vt.to(torch.float8_e4m3fn).view(torch.uint8)
            esz = 1
        q = torch.randn(M, cfg.q_dim, device=dev).bfloat16()
        slot = torch.arange(M, device=dev, dtype=torch.int32)
        pos = torch.full((M,), L - 1, device=dev, dtype=torch.int32)
        cnt = torch.zeros(M * cfg.n_kv_heads, device=dev, dtype=torch.int32)
        out = torch.empty(M, cfg.q_dim, device=dev).bfloat16()
        for sp in ns.attn_splits.split(","):
            ns_ = attention_splits(M, cfg.n_kv_heads, T_max) if sp == "auto" else int(sp)
            po = torch.empty(M * cfg.n_heads * ns_ * cfg.head_dim, device=dev)
            pm = torch.empty(ops.attention_ml_floats(M, cfg.n_heads, cfg.n_kv_heads, ns_), device=dev)
            us = timeit(lambda: ops.attention(q, kc, vt, slot, pos, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, ns_,
                                              1 / math.sqrt(cfg.head_dim), out=out, part_o=po, part_ml=pm,
                                              counters=cnt))
            kv_bytes = 2 * M * cfg.n_kv_heads * L * cfg.head_dim * esz
            r = dict(kind="attention", model=cfg.name, kv=ns.attn_kv, M=M, L=L, T_max=T_max, nsplit=ns_, split_arg=sp,
                     us=round(us, 2), TBps=round(kv_bytes / us / 1e6, 3))
            res.append(r)
            print(json.dumps(r), flush=True)
        del kc, vt
    if ns.attn_only:
        return
    # sampler
    for M in (1, 16, 64):
        lg = torch.randn(M, V, device=dev)
        z = lambda: torch.zeros(M, device=dev, dtype=torch.int32)  # noqa: E731
        tok, pos, n_gen, done = z(), z(), z(), z()
        gen = torch.zeros(M, 4096, device=dev, dtype=torch.int32)
        hist = torch.zeros(M * 64, device=dev, dtype=torch.int32)
        mx = torch.full((M,), 1 << 30, device=dev, dtype=torch.int32)
        slot = torch.arange(M, device=dev, dtype=torch.int32)
        prm = ops.sample_params_tensor([dict(temperature=0.8, top_p=0.9, repeat_penalty=1.1, top_k=40,
                                             repeat_last_n=64, eos_id=-1, seed=i) for i in range(M)], dev)

        def run():
            n_gen.zero_()
            ops.sample(lg, tok, pos, gen, n_gen, mx, done, hist, slot, prm, 1 << 30)
        us = timeit(run)
        r = dict(kind="sample", model=cfg.name, M=M, V=V, us=round(us, 2))
        res.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
