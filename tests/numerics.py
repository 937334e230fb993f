"""Relative numerics criterion of the full-depth GPU tests.

Random-init stacks are chaotic at depth, so an absolute threshold (cosine > 0.995, > 0.8 for W8A8) either admits
a real precision regression or fails on weight chaos.  Instead the HIP engine's error against the fp32 oracle is
compared with the error of a plain PyTorch eager model of the same precision on the same weights and prompts
(``ReferenceModel(compute_dtype=torch.bfloat16)``; for fp8 paths the same model on the fp8-rounded weights, with
the per-row e4m3 activation rounding where the kernels do it): the engine may be at most ``FACTOR`` times as far
from fp32 as that eager baseline."""
import torch

from cain_amd.models.reference import ReferenceModel

FACTOR = 1.25


def rel(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def eager_bf16(weights, **kw) -> ReferenceModel:
    """The bf16 PyTorch-eager baseline (bf16 weights are used as they are: no second copy)."""
    return ReferenceModel(weights, compute_dtype=torch.bfloat16, memo_weights=True, **kw)


def assert_within_eager(err_engine, err_eager, tag, factor: float = FACTOR, floor: float = 1e-4):
    """Summed relative errors over the checked rows: engine <= factor x eager (+ a floor for near-exact cases)."""
    e, b = float(sum(err_engine)), float(sum(err_eager))
    assert e <= factor * b + floor, f"{tag}: engine error {e:.5f} > {factor} x bf16-eager error {b:.5f}"
