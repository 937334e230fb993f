#!/usr/bin/env python3
"""In-graph microbenchmark of the few-row weight-streaming GEMMs: MXFP4 (gemm_w4.hip, every kernel shape), fp8
(gemm_w8.hip) and bf16 (gemm.hip) on a model's projection shapes at one row.

Each case captures `reps` calls into one hipGraph (torch.cuda.CUDAGraph) rotating over enough weight copies to
exceed the 256 MiB Infinity Cache, replays it, and reports time per call and weight bytes / time -- the
graph-replayed per-kernel cost the decode step sees (boundary included), not an isolated launch.
usage: python3 tools/w4_bench.py [--model llama3.1:8b] [--rows 1] [--variants rule,0,1,2,3,4,5] [--occ 0]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from cain_amd import ops  # noqa: E402
from cain_amd.models import get_config  # noqa: E402


def graph_time(fn, reps: int = 40, iters: int = 5) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn(0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (iters * reps) * 1e3  # us per call


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1:8b")
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--variants", default="rule,0,1,2,3,4,5")
    ap.add_argument("--occ", default="0")
    ap.add_argument("--dtypes", default="fp4,fp8,bf16")
    ap.add_argument("--norm", choices=("model", "on", "off"), default="model",
                    help="fused RMSNorm: as in the model (QKV / gate-up / LM head), or forced on / off for every role")
    ap.add_argument("--roles", default="qkv,o,gateup,down,lm_head")
    ap.add_argument("--copies", default="0",
                    help="weight copies rotated per call, comma list: 0 = enough to exceed the 256 MiB Infinity Cache "
                         "(cold, as in decode); 1 = one copy (cache-hot); e.g. 8 = Infinity-Cache-hot, beyond L2")
    ns = ap.parse_args()
    cfg = get_config(ns.model)
    dev = torch.device("cuda")
    d, F = cfg.d_model, cfg.ffn
    roles = {"qkv": (cfg.qkv_dim, d, ops.EPI_QKV_ROPE, True), "o": (d, cfg.q_dim, ops.EPI_RESID, False),
             "gateup": (2 * F, d, ops.EPI_SILU, True), "down": (d, F, ops.EPI_RESID, False),
             "lm_head": (cfg.vocab, d, ops.EPI_F32, True),
             # the QKV shape without its RoPE / KV-append epilogue (bf16 output), with and without the fused norm
             "qkv_plain": (cfg.qkv_dim, d, ops.EPI_BF16, True), "qkv_plain_nonorm": (cfg.qkv_dim, d, ops.EPI_BF16, False)}
    M = ns.rows
    x = torch.randn(M, max(d, F, cfg.q_dim), device=dev).bfloat16()
    # the fused QKV epilogue's operands: RoPE tables, fragment-major caches, one slot / position per row
    T_max, hd = 1536, cfg.head_dim
    ang = torch.arange(T_max, device=dev, dtype=torch.float32)[:, None] * torch.rand(hd // 2, device=dev)[None]
    rope = dict(kc=torch.zeros(M, cfg.n_kv_heads, T_max, hd, device=dev).bfloat16(),
                vtc=torch.zeros(M, cfg.n_kv_heads, hd, T_max, device=dev).bfloat16(),
                slot=torch.arange(M, device=dev, dtype=torch.int32), pos=torch.full((M,), 700, device=dev, dtype=torch.int32),
                cos_t=ang.cos().contiguous(), sin_t=ang.sin().contiguous(), H=cfg.n_heads, Hkv=cfg.n_kv_heads, hd=hd)
    for role, (N, K, epi, norm) in roles.items():
        if role not in ns.roles.split(","):
            continue
        norm = norm if ns.norm == "model" else ns.norm == "on"
        xk = x[:, :K].contiguous()
        n_out = N // 2 if epi in (ops.EPI_SILU, ops.EPI_GELU) else N
        if epi == ops.EPI_QKV_ROPE:
            n_out = cfg.q_dim
        out = torch.zeros(M, n_out, device=dev, dtype=torch.float32 if epi == ops.EPI_F32 else torch.bfloat16)
        rp = rope if epi == ops.EPI_QKV_ROPE else None
        for dt, cp in [(dt, cp) for dt in ns.dtypes.split(",") for cp in ns.copies.split(",")]:
            bpp = {"fp4": 0.5 + 1 / 32, "fp8": 1.0, "bf16": 2.0, "q4_0": 0.5 + 1 / 16, "q4_k": 0.5 + 1 / 16 + 1 / 64}[dt]
            wbytes = int(N * K * bpp)
            ncopy = int(cp) if int(cp) > 0 else max(2, min(16, (768 << 20) // max(1, wbytes) + 1))
            if dt == "fp4":
                ws = [(torch.randint(0, 256, (N // 16, K // 128, 64, 16), device=dev, dtype=torch.uint8),
                       torch.randint(118, 122, (N // 16, K // 128, 64), device=dev, dtype=torch.uint8))
                      for _ in range(ncopy)]
                for v in ns.variants.split(","):
                    for occ in ns.occ.split(","):
                        ops.set_w4_variant(-1 if v == "rule" else int(v))
                        ops.set_w4_occupancy(int(occ))
                        used = ops.w4_variant(N, K, M, epi) if v == "rule" else int(v)

                        def fn(i, ws=ws):
                            wq, sc = ws[i % len(ws)]
                            ops.gemm_w4(wq, sc, xk, N, epi, out=out, norm=norm, rope=rp)
                        us = graph_time(fn)
                        print(json.dumps(dict(role=role, dtype=dt, N=N, K=K, M=M, variant=v, used=used, occ=int(occ), norm=norm,
                                              copies=ncopy, us=round(us, 2), TBps=round(wbytes / us / 1e6, 2))), flush=True)
                ops.set_w4_variant(-1)
                ops.set_w4_occupancy(0)
            elif dt in ("q4_0", "q4_k"):
                fmt = 1 if dt == "q4_k" else 0
                nsb = N * K // 16 + (N * K // 64 if fmt else 0)
                # random codes, scales 0x3c00 (fp16 1.0) / (sc, m) = (1, 0) and (d, dmin) = (1, 0): finite values
                def rnd_sb():
                    sb = torch.zeros(nsb, device=dev, dtype=torch.uint8)
                    if fmt == 0:
                        sb.view(torch.int16)[:] = 0x2c00
                    else:
                        sb[: N * K // 16].view(torch.int16)[:] = 1
                        sb[N * K // 16:].view(torch.int32)[:] = 0x2c00
                    return sb
                ws = [(torch.randint(0, 256, (N // 16, K // 128, 64, 16), device=dev, dtype=torch.uint8), rnd_sb())
                      for _ in range(ncopy)]

                def fn(i, ws=ws):
                    wq, sb = ws[i % len(ws)]
                    ops.gemm_q4(fmt, wq, sb, xk, N, epi, out=out, norm=norm, rope=rp)
                us = graph_time(fn)
                print(json.dumps(dict(role=role, dtype=dt, N=N, K=K, M=M, us=round(us, 2),
                                      TBps=round(wbytes / us / 1e6, 2))), flush=True)
            elif dt == "fp8":
                ws = [(torch.randint(0, 120, (N // 16, K // 64, 64, 16), device=dev, dtype=torch.uint8),
                       torch.full((N,), 0.01, device=dev)) for _ in range(ncopy)]

                def fn(i, ws=ws):
                    wq, sc = ws[i % len(ws)]
                    ops.gemm_w8(wq, sc, xk, N, epi, out=out, norm=norm, rope=rp)
                us = graph_time(fn)
                print(json.dumps(dict(role=role, dtype=dt, N=N, K=K, M=M, us=round(us, 2),
                                      TBps=round(wbytes / us / 1e6, 2))), flush=True)
            else:
                ws = [torch.randn(N // 16, K // 32, 64, 8, device=dev).bfloat16() for _ in range(ncopy)]

                def fn(i, ws=ws):
                    if rp is not None:
                        ops.qkv_rope(ws[i % len(ws)], xk, N, out, rp["kc"], rp["vtc"], rp["slot"], rp["pos"],
                                     rp["cos_t"], rp["sin_t"], rp["H"], rp["Hkv"], rp["hd"], norm=norm)
                    else:
                        ops.skinny_gemm(ws[i % len(ws)], xk, N, epi, out=out, norm=norm)
                us = graph_time(fn)
                print(json.dumps(dict(role=role, dtype=dt, N=N, K=K, M=M, us=round(us, 2),
                                      TBps=round(wbytes / us / 1e6, 2))), flush=True)
            del ws
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
