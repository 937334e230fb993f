#!/usr/bin/env python3
"""Sweep weight-streaming GEMM variants (tools/gemm_tune.hip) on the llama3.1:8b decode shapes.

Interleaved rounds in one process; each call streams a different weight copy
(> 600 MB per role) so the Infinity Cache does not serve the weights."""
import ctypes
import itertools
import json
import math
import os
import subprocess
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
SO = HERE / "gemm_tune.so"


def build():
    if not SO.exists() or SO.stat().st_mtime < (HERE / "gemm_tune.hip").stat().st_mtime:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", str(SO),
                        str(HERE / "gemm_tune.hip")], check=True)
    lib = ctypes.CDLL(str(SO))
    lib.tune_gemm.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] * 2 + [ctypes.c_void_p] + [ctypes.c_int] * 5 + [
        ctypes.c_void_p]
    return lib


VARIANTS = [(1, 4, 8, 1, 0), (1, 8, 8, 1, 0), (1, 16, 8, 1, 0), (1, 4, 16, 1, 0), (1, 8, 16, 1, 0),
            (1, 16, 16, 1, 0), (1, 8, 8, 0, 0), (1, 16, 8, 0, 0), (1, 8, 16, 0, 0), (2, 4, 8, 1, 0),
            (2, 8, 8, 1, 0), (2, 16, 8, 1, 0), (2, 8, 4, 1, 0), (2, 16, 4, 1, 0), (1, 8, 4, 1, 1), (1, 8, 8, 1, 1),
            (1, 16, 4, 1, 1), (1, 16, 8, 1, 1), (1, 4, 8, 1, 1), (2, 8, 4, 1, 1), (2, 16, 4, 1, 1)]


def main():
    lib = build()
    dev = torch.device("cuda")
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gateup": (28672, 4096), "down": (4096, 14336)}
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for role, (N, K) in shapes.items():
        ncopy = max(1, math.ceil(600e6 / (N * K * 2)))
        Ws = [torch.randn(N * K, device=dev).bfloat16() for _ in range(ncopy)]
        X = torch.randn(16, K, device=dev).bfloat16()
        Y = torch.empty(16, N, device=dev).bfloat16()
        res = {}
        for rnd in range(3):
            for v in VARIANTS:
                nt = v[0]
                if N % (16 * nt):
                    continue
                it = [0]

                def run():
                    w = Ws[it[0] % ncopy]
                    it[0] += 1
                    rc = lib.tune_gemm(ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(X.data_ptr()), K, N,
                                       ctypes.c_void_p(Y.data_ptr()), *v, st)
                    assert rc == 0, rc
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(40):
                    run()
                b.record()
                torch.cuda.synchronize()
                us = a.elapsed_time(b) / 40 * 1e3
                res.setdefault(v, []).append(us)
        for v, ts in sorted(res.items(), key=lambda kv: min(kv[1])):
            us = min(ts)
            print(json.dumps(dict(role=role, N=N, K=K, nt=v[0], waves=v[1], U=v[2], nt_load=v[3], pipe=v[4],
                                  us=round(us, 2), TBps=round(N * K * 2 / us / 1e6, 3))), flush=True)


if __name__ == "__main__":
    main()
