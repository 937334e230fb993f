#!/usr/bin/env python3
"""Library-GEMM reference point (torch.mm -> hipBLASLt) for the decode GEMM shapes, to price the
hand-written kernels against (weights > Infinity Cache, as in a real decode step)."""
import json
import math
import sys

import torch


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    rows = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,16,64,128").split(",")]
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gateup": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    dev = torch.device("cuda")
    for role, (n, k) in shapes.items():
        ncopy = max(1, math.ceil(600e6 / (n * k * 2)))
        ws = [torch.randn(n, k, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
        for m in rows:
            x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
            it = [0]

            def run():
                w = ws[it[0] % ncopy]
                it[0] += 1
                return x @ w.t()
            us = timeit(run)
            print(json.dumps(dict(kind="torch_mm", role=role, M=m, N=n, K=k, us=round(us, 2),
                                  TBps=round(n * k * 2 / us / 1e6, 3))), flush=True)
        del ws


if __name__ == "__main__":
    main()
