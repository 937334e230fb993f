"""Where the fused layer front's time goes (csrc/front.hip): per-role timestamps of one launch, and the fused vs
three-launch time per layer on the same operands.

    python tools/front_trace.py [--model qwen2:1.5b] [--pos 700] [--iters 200]

Timestamps are s_memrealtime ticks (10 ns), relative to the first workgroup's start; per role the median and max of
start / wait begin / wait end / end over its workgroups.
"""
import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cain_amd import ops  # noqa: E402
from cain_amd.engine.engine import attention_splits  # noqa: E402
from cain_amd.models.config import get_config  # noqa: E402
from cain_amd.models.weights import pack_mfma_a  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen2:1.5b")
    ap.add_argument("--pos", type=int, default=700)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rows", type=int, default=1)
    a = ap.parse_args()
    cfg = get_config(a.model)
    d, H, Hkv, hd = cfg.d_model, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
    M, T_max, dev = a.rows, 2048, torch.device("cuda")
    ns = attention_splits(M, Hkv, T_max)
    assert ops.front_eligible(M, d, H, Hkv, hd, ns), (d, H, Hkv, hd, ns)
    qkv_dim = (H + 2 * Hkv) * hd
    Wp = pack_mfma_a((torch.randn(qkv_dim, d, device=dev) * 0.02).bfloat16())
    Wop = pack_mfma_a((torch.randn(d, H * hd, device=dev) * 0.02).bfloat16())
    bias = torch.zeros(qkv_dim, device=dev)
    kc = torch.randn(M, Hkv, T_max, hd, device=dev).bfloat16()
    vt = torch.randn(M, Hkv, hd, T_max, device=dev).bfloat16()
    x = torch.randn(M, d, device=dev).bfloat16()
    q = torch.zeros(M, H * hd, device=dev, dtype=torch.bfloat16)
    attn = torch.zeros_like(q)
    slot = torch.arange(M, device=dev, dtype=torch.int32)
    pos = torch.full((M,), a.pos, device=dev, dtype=torch.int32)
    inv = 1.0 / (10000.0 ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(T_max, dtype=torch.float64)[:, None] * inv[None]
    cos_t, sin_t = ang.cos().float().to(dev), ang.sin().float().to(dev)
    part_o = torch.empty(M * H * ns * hd, device=dev)
    part_ml = torch.empty(ops.attention_ml_floats(M, H, Hkv, ns), device=dev)
    ctr = torch.zeros(M * Hkv, device=dev, dtype=torch.int32)
    flags = torch.zeros(4096, device=dev, dtype=torch.int32)
    scale = 1.0 / math.sqrt(hd)

    def fused(trace=None):
        ops.layer_front(Wp, bias, Wop, x, q, attn, kc, vt, slot, pos, cos_t, sin_t, H, Hkv, hd, ns, scale,
                        part_o=part_o, part_ml=part_ml, counters=ctr, flags=flags, trace=trace)

    def three():
        ops.qkv_rope(Wp, x, qkv_dim, q, kc, vt, slot, pos, cos_t, sin_t, H, Hkv, hd, bias=bias, norm=True)
        ops.attention(q, kc, vt, slot, pos, H, Hkv, hd, ns, scale, out=attn, part_o=part_o, part_ml=part_ml,
                      counters=ctr)
        ops.skinny_gemm(Wop, attn, d, ops.EPI_RESID, out=x)

    def timed(fn):
        for _ in range(20):
            fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.iters):
                fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / a.iters

    t3, tf = timed(three), timed(fused)
    n_qkv, n_att, n_o = qkv_dim // 16, M * Hkv * ns, d // 16
    tr = torch.zeros(n_qkv + n_att + n_o, 4, device=dev, dtype=torch.int64)
    for _ in range(5):
        fused(tr)
    torch.cuda.synchronize()
    t = (tr - tr[:, 0].min()).float().cpu() * 0.01  # us
    print(f"{a.model} rows={M} pos={a.pos} nsplit={ns}: three launches {t3:.2f} us/layer, fused {tf:.2f} us/layer")
    for name, lo, hi in (("qkv", 0, n_qkv), ("att", n_qkv, n_qkv + n_att), ("o", n_qkv + n_att, n_qkv + n_att + n_o)):
        r = t[lo:hi]
        med, mx = r.median(0).values, r.max(0).values
        print(f"  {name:4s} n={hi - lo:4d}  start {med[0]:6.2f}/{mx[0]:6.2f}  wait-begin {med[1]:6.2f}/{mx[1]:6.2f}"
              f"  wait-end {med[2]:6.2f}/{mx[2]:6.2f}  end {med[3]:6.2f}/{mx[3]:6.2f}   (median/max us)")


if __name__ == "__main__":
    main()
