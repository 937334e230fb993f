"""Stream vs tile MXFP4 kernels on qwen2:1.5b / gemma:2b shapes (round-6 debugging): max relative difference."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from cain_amd import ops  # noqa: E402
from cain_amd.models.weights import pack_mxfp4, quantize_mxfp4, rope_pair_order  # noqa: E402

DEV = "cuda"


def run(N, K, M, epi, norm, var, bias=False):
    torch.manual_seed(N + K + M)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    c, s = quantize_mxfp4(W)
    wq, ws = pack_mxfp4(c, s)
    b = torch.randn(N, device=DEV) if bias else None
    ops.set_w4_variant(var)
    try:
        if epi == ops.EPI_RESID:
            out = torch.randn(M, N, device=DEV, generator=torch.Generator(DEV).manual_seed(3)).bfloat16()
            ops.gemm_w4(wq, ws, x, N, epi, out=out, norm=norm)
        else:
            out = ops.gemm_w4(wq, ws, x, N, epi, bias=b, norm=norm)
    finally:
        ops.set_w4_variant(-1)
    torch.cuda.synchronize()
    return out.float()


for (N, K, epi, norm, bias, tag) in [(1536, 1536, ops.EPI_RESID, False, False, "qwen O"),
                                     (17920, 1536, ops.EPI_SILU, True, False, "qwen gate/up"),
                                     (1536, 8960, ops.EPI_RESID, False, False, "qwen down"),
                                     (151936, 1536, ops.EPI_F32, True, False, "qwen LM head"),
                                     (2048, 1536, ops.EPI_BF16, True, True, "qwen QKV as bf16+bias"),
                                     (2048, 2048, ops.EPI_RESID, False, False, "gemma O"),
                                     (4096, 1536, ops.EPI_F32, False, False, "K1536 f32")]:
    for M in (1, 5, 16):
        a = run(N, K, M, epi, norm, -1, bias)
        t = run(N, K, M, epi, norm, 2 if N * 0 == 0 else 2, bias)
        d = float((a - t).norm() / (t.norm() + 1e-9))
        print(f"{tag:24s} M={M:2d} rel diff stream vs tile {d:.2e} variant {ops.load().cain_gemm_w4_variant(N, K, M, epi)}",
              flush=True)
