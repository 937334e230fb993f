#!/usr/bin/env python3
"""Operand-layout probe of the W4A8 kernel (wgemm8.hip FP4): identity weights (row n one-hot at k = n) against
identity activations (row m one-hot at k = m): Y[m][n] != 0 iff the MFMA pairs weight k-position n with activation
k-position m.  Prints, per activation row m < 256, the weight positions it met and the values."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from cain_amd import ops  # noqa: E402
from cain_amd.models.weights import dequantize_mxfp4, pack_mxfp4, quantize_mxfp4  # noqa: E402


def main():
    dev = torch.device("cuda")
    K = N = 512
    M = 256
    W = torch.eye(N, K, device=dev)
    c, s = quantize_mxfp4(W.bfloat16())
    assert torch.equal(dequantize_mxfp4(c, s), W)
    wq, ws = pack_mxfp4(c, s)
    x = torch.eye(M, K, device=dev).bfloat16()
    y = ops.gemm_w4a8(wq, ws, x, N, ops.EPI_F32).float().cpu()
    out = []
    for m in range(M):
        nz = (y[m].abs() > 1e-30).nonzero().flatten().tolist()
        out.append({"m": m, "n": nz[:8], "v": [float(y[m, n]) for n in nz[:8]]})
    for r in out:
        print(json.dumps(r))
    ok = sum(1 for r in out if r["n"] == [r["m"]] and abs(r["v"][0] - 1) < 1e-6)
    print(json.dumps({"identity_rows": ok, "of": M}))


if __name__ == "__main__":
    main()
