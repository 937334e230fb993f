"""Where the lean chunk-maximum sampler's time goes (csrc/sample.hip sample_lean_kernel): per-phase timestamps
(s_memrealtime, 10 ns) of one launch over a random-init model's next-token logits and over N(0, 3^2) logits, with
Ollama's default options (penalty on, 64 history ids), greedy, and the penalty off.

    python tools/sample_lean_trace.py [--model qwen2:1.5b]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cain_amd import ops  # noqa: E402
from cain_amd.engine.engine import DecodeEngine  # noqa: E402

PHASES = ["maxima exact", "tau_c", "chunks gathered", "logits staged", "elements gathered", "ranked", "end"]


def run(logits, opts, label, hist_ids=64):
    dev = logits.device
    M, V = logits.shape
    z = lambda: torch.zeros(M, device=dev, dtype=torch.int32)  # noqa: E731
    hist = torch.randint(0, V, (M * 64,), device=dev, dtype=torch.int32)
    n_gen = torch.full((M,), hist_ids, device=dev, dtype=torch.int32)
    params = ops.sample_params_tensor([opts] * M, dev)
    cmax = logits.view(M, V // 16, 16).amax(-1).contiguous()
    tr = torch.zeros(M, 8, device=dev, dtype=torch.int64)
    lib = ops.load()
    rows = []
    for it in range(8):
        tr.zero_()
        lib.cain_sample_set_trace(tr.data_ptr() if it >= 3 else None)
        ops.sample(logits.clone(), z(), z() + 10, torch.zeros(M, 2048, device=dev, dtype=torch.int32), n_gen.clone(),
                   torch.full((M,), 4096, device=dev, dtype=torch.int32), z(), hist,
                   torch.arange(M, device=dev, dtype=torch.int32), params, 4096, cmax=cmax, lean=True)
        torch.cuda.synchronize()
        if it >= 3:
            t = tr[0].cpu()
            rows.append([(float(t[i] - t[0]) * 0.01) for i in range(1, 8)])
    lib.cain_sample_set_trace(None)
    med = torch.tensor(rows).median(0).values.tolist()
    print(f"{label}: " + ", ".join(f"{n} {v:.2f}" for n, v in zip(PHASES, med)) + " us", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen2:1.5b")
    a = ap.parse_args()
    opts = dict(temperature=0.8, top_p=0.9, repeat_penalty=1.1, top_k=40, repeat_last_n=64, eos_id=-1, seed=7)
    eng = DecodeEngine(a.model, device="cuda", max_batch=1, max_context=512, seed=1234)
    real = eng.last_logits(["In 1000 words, please give me information about India"]).float().contiguous()
    print(f"{a.model} real logits: V {real.shape[1]} mean {real.mean():.3f} std {real.std():.3f} max {real.max():.3f}")
    run(real, opts, "real, Ollama defaults")
    run(real, dict(opts, repeat_penalty=1.0), "real, penalty off")
    run(real, dict(opts, temperature=0.0), "real, greedy")
    run(torch.randn_like(real) * 3, opts, "N(0,9), Ollama defaults")


if __name__ == "__main__":
    main()
