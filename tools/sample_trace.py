"""Where the two-stage sampler's time goes (csrc/sample.hip sample_split_kernel): per-phase timestamps of one
launch over real logits (a random-init model's next-token logits) and over N(0, 3^2) logits.

    python tools/sample_trace.py [--model qwen2:1.5b]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cain_amd import ops  # noqa: E402
from cain_amd.engine.engine import DecodeEngine  # noqa: E402

PHASES = ["loaded", "tau", "gathered", "ranked", "ticket", "merged", "end"]


def run(logits, opts, label, hist_ids=64):
    dev = logits.device
    M, V = logits.shape
    z = lambda: torch.zeros(M, device=dev, dtype=torch.int32)  # noqa: E731
    hist = torch.randint(0, V, (M * 64,), device=dev, dtype=torch.int32)
    n_gen = torch.full((M,), hist_ids, device=dev, dtype=torch.int32)
    params = ops.sample_params_tensor([opts] * M, dev)
    tr = torch.zeros(M * 16, 8, device=dev, dtype=torch.int64)
    lib = ops.load()
    for it in range(6):
        lib.cain_sample_set_trace(tr.data_ptr() if it == 5 else None)
        tok = z()
        ops.sample(logits.clone(), tok, z() + 10, torch.zeros(M, 2048, device=dev, dtype=torch.int32), n_gen.clone(),
                   torch.full((M,), 4096, device=dev, dtype=torch.int32), z(), hist, torch.arange(M, device=dev,
                   dtype=torch.int32), params, 4096, split=True)
    torch.cuda.synchronize()
    lib.cain_sample_set_trace(None)
    t = tr.cpu()
    t0 = t[:, 0].min()
    us = (t - t0).double() * 0.01  # int64 difference first: float32 cannot hold raw ticks
    merger = int((t[:, 7] > 0).nonzero()[0, 0])
    print(f"{label}: stage-1 candidates per slice {t[:, 6][t[:, 7] == 0].tolist()}")
    for i, name in enumerate(PHASES, 1):
        if i == 6:
            print(f"  {name:9s} merger {us[merger, 6]:7.2f} us")
            continue
        if i == 7:
            print(f"  {name:9s} merger {us[merger, 7]:7.2f} us")
            continue
        col = us[:, i]
        print(f"  {name:9s} median {col.median():7.2f}  max {col.max():7.2f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen2:1.5b")
    a = ap.parse_args()
    opts = dict(temperature=0.8, top_p=0.9, repeat_penalty=1.1, top_k=40, repeat_last_n=64, eos_id=-1, seed=7)
    eng = DecodeEngine(a.model, device="cuda", max_batch=1, max_context=512, seed=1234)
    real = eng.last_logits(["In 1000 words, please give me information about India"]).float().contiguous()
    print(f"real logits: mean {real.mean():.3f} std {real.std():.3f} max {real.max():.3f}")
    run(real, opts, f"{a.model} logits")
    run(torch.randn_like(real) * 3, opts, "N(0,9) logits")
    run(real, dict(opts, temperature=0.0), f"{a.model} logits, greedy")


if __name__ == "__main__":
    main()
