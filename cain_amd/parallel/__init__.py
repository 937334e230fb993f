"""Data-parallel trial fan-out (one process per GPU, rank-0 single writer, RCCL/gloo object collectives)."""
from .fanout import launch, run_rank  # noqa: F401
