"""Statistical analysis of run tables (replaces the reference's R notebook)."""
from . import stats
from .report import analyze, load_run_table, make_subsets

__all__ = ["stats", "analyze", "load_run_table", "make_subsets"]
