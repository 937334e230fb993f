"""Graph-replayed launch floor on this GPU: N dependent launches of a trivial kernel, and of kernels that touch
1 KiB / 64 KiB per workgroup, timed per launch (round-6 batch-1 analysis: is the ~3.6 us fixed cost per GEMM the
launch boundary or the first loads?)."""
import sys
import time

import torch

dev = "cuda"
N = 200


def graph_time(fn, label):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(N):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / (20 * N) * 1e6
    print(f"{label:50s} {dt:7.2f} us per launch", flush=True)


x1 = torch.zeros(1, device=dev)
graph_time(lambda: x1.add_(1), "1-element add (1 workgroup)")
x2 = torch.zeros(256 * 1024, device=dev)  # 1 MiB: 1 KiB per thread-block-ish
graph_time(lambda: x2.add_(1), "1 MiB add")
x3 = torch.zeros(8 * 1024 * 1024, device=dev)  # 32 MiB
graph_time(lambda: x3.add_(1), "32 MiB add (read + write 64 MiB)")
w = torch.zeros(4096, 4096, device=dev, dtype=torch.bfloat16)
v = torch.zeros(4096, 1, device=dev, dtype=torch.bfloat16)
graph_time(lambda: torch.mm(w, v), "hipBLASLt 4096x4096 bf16 GEMV (32 MiB)")
