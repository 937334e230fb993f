"""Statistics of the paper's R notebook, re-implemented on numpy/scipy with R's conventions.

Every function names the R routine whose numbers it reproduces and the notebook cell that calls it
(`data-analysis/analysis-visualization.ipynb`, R kernel):

* :func:`quantile7`            — ``quantile(x, p)`` (type 7), used by ``remove_outliers`` (ipynb:345-361)
* :func:`remove_outliers`      — sequential 1.5·IQR filter over METRICS, inclusive bounds (ipynb:345-361)
* :func:`describe`             — ``mean/median/sd`` (n-1) of the summary table (ipynb:425-531)
* :func:`shapiro`              — ``shapiro.test`` (Royston AS R94, same algorithm as scipy) (ipynb:1047-1067)
* :func:`skewness`             — ``e1071::skewness`` type 3 (ipynb:1110)
* :func:`wilcox_test`          — ``wilcox.test(x, y, "two.sided")``: W = rank-sum of x − n_x(n_x+1)/2;
  exact p when both n < 50 and no ties, otherwise normal approximation with tie and continuity
  correction (ipynb:1342)
* :func:`cliff_delta`          — ``effsize::cliff.delta(x, y, return.ci=TRUE)``: dominance mean, Cliff's
  consistent variance, Feng–Cliff asymmetric CI (ipynb:1345), magnitude thresholds 0.147 / 0.33 / 0.474
  (ipynb:1356)
* :func:`spearman_test`        — ``cor.test(x, y, method="spearman")``: ρ = Pearson of mid-ranks; with ties
  the t_{n-2} approximation (R warns "Cannot compute exact p-value with ties" and uses it); without ties
  exact enumeration for n ≤ 9 and the AS 89 Edgeworth series above (ipynb:1567)
* :func:`stars`                — significance stars of the H2 table (ipynb:1572)
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
from scipy import stats as _st


def _arr(x) -> np.ndarray:
    a = np.asarray(x, dtype=np.float64).ravel()
    return a[~np.isnan(a)]


def quantile7(x, p: float) -> float:
    """R ``quantile(type=7)``: linear interpolation at h = (n-1)p between order statistics."""
    a = np.sort(_arr(x))
    if a.size == 0:
        return float("nan")
    h = (a.size - 1) * p
    lo = int(math.floor(h))
    hi = min(lo + 1, a.size - 1)
    return float(a[lo] + (h - lo) * (a[hi] - a[lo]))


def iqr_bounds(x, k: float = 1.5) -> Tuple[float, float]:
    q1, q3 = quantile7(x, 0.25), quantile7(x, 0.75)
    r = q3 - q1
    return q1 - k * r, q3 + k * r


def remove_outliers(df, columns: Sequence[str], k: float = 1.5):
    """Apply the IQR filter column after column; each column's quartiles are computed on the rows that
    survived the previous columns (the notebook's ``filtered_data`` loop). NaN rows are dropped by the
    comparison, as dplyr::filter does."""
    out = df
    for c in columns:
        lo, hi = iqr_bounds(out[c].to_numpy(dtype=np.float64), k)
        v = out[c].to_numpy(dtype=np.float64)
        out = out[(v >= lo) & (v <= hi)]
    return out


@dataclass
class Describe:
    n: int
    mean: float
    median: float
    sd: float


def describe(x) -> Describe:
    a = _arr(x)
    sd = float(np.std(a, ddof=1)) if a.size > 1 else float("nan")
    return Describe(int(a.size), float(np.mean(a)) if a.size else float("nan"),
                    float(np.median(a)) if a.size else float("nan"), sd)


def skewness(x) -> float:
    """``e1071::skewness`` default (type 3): g1 · ((n-1)/n)^{3/2}."""
    a = _arr(x)
    n = a.size
    m = a - a.mean()
    m2 = np.mean(m ** 2)
    if n < 3 or m2 == 0:
        return 0.0
    g1 = np.mean(m ** 3) / m2 ** 1.5
    return float(g1 * ((n - 1) / n) ** 1.5)


def skew_label(s: float) -> str:
    return "Positively Skewed" if s > 0 else ("Negatively Skewed" if s < 0 else "Symmetric")


@dataclass
class TestResult:
    statistic: float
    p_value: float
    method: str = ""
    warning: Optional[str] = None


def shapiro(x) -> TestResult:
    a = _arr(x)
    w, p = _st.shapiro(a)
    return TestResult(float(w), float(p), "Shapiro-Wilk normality test")


def transform_towards_normality(on_device, remote) -> Tuple[str, str, List[Tuple[str, float, float]]]:
    """The notebook's ``transform_pairs_towards_normality`` (ipynb:1110): if both arms are skewed the same
    way, try sqrt/log (positive) or square/cube (negative) and report Shapiro p-values per transform."""
    a, b = _arr(on_device), _arr(remote)
    la, lb = skew_label(skewness(a)), skew_label(skewness(b))
    rows: List[Tuple[str, float, float]] = []
    if la != lb:
        return la, lb, rows
    if la == "Positively Skewed":
        tr = [("Original", lambda v: v), ("Square Root", np.sqrt), ("Logarithm", np.log)]
    else:
        tr = [("Original", lambda v: v), ("Power 2", lambda v: v ** 2), ("Power 3", lambda v: v ** 3)]
    for name, f in tr:
        rows.append((name, shapiro(f(a)).p_value, shapiro(f(b)).p_value))
    return la, lb, rows


def _midranks(v: np.ndarray) -> np.ndarray:
    return _st.rankdata(v, method="average")


def wilcox_test(x, y, correct: bool = True, exact: Optional[bool] = None) -> TestResult:
    """Two-sample two-sided Wilcoxon rank-sum test, R semantics (``stats:::wilcox.test.default``)."""
    x, y = _arr(x), _arr(y)
    nx, ny = x.size, y.size
    r = _midranks(np.concatenate([x, y]))
    w = float(r[:nx].sum() - nx * (nx + 1) / 2.0)
    ties = len(np.unique(r)) != r.size
    if exact is None:
        exact = nx < 50 and ny < 50
    if exact and not ties:
        p = float(_st.mannwhitneyu(x, y, alternative="two-sided", method="exact").pvalue)
        return TestResult(w, min(1.0, p), "Wilcoxon rank sum exact test")
    _, counts = np.unique(r, return_counts=True)
    z = w - nx * ny / 2.0
    sigma = math.sqrt((nx * ny / 12.0) * ((nx + ny + 1) - np.sum(counts ** 3 - counts) / ((nx + ny) * (nx + ny - 1))))
    corr = 0.5 * np.sign(z) if correct else 0.0
    zz = (z - corr) / sigma if sigma > 0 else 0.0
    p = 2.0 * min(_st.norm.cdf(zz), _st.norm.sf(zz))
    warn = "cannot compute exact p-value with ties" if exact and ties else None
    return TestResult(w, min(1.0, float(p)), "Wilcoxon rank sum test with continuity correction", warn)


CLIFF_THRESHOLDS = (0.147, 0.33, 0.474)


def cliff_magnitude(d: float) -> str:
    a = abs(d)
    if a < CLIFF_THRESHOLDS[0]:
        return "Negligible"
    if a < CLIFF_THRESHOLDS[1]:
        return "Small"
    if a < CLIFF_THRESHOLDS[2]:
        return "Medium"
    return "Large"


@dataclass
class CliffResult:
    estimate: float
    lower: float
    upper: float
    variance: float
    magnitude: str


def cliff_delta(x, y, conf_level: float = 0.95, use_normal: bool = False) -> CliffResult:
    """Cliff's δ = P(x>y) − P(x<y) with an asymmetric Feng & Cliff interval
    ``(δ−δ³ ∓ z·s·√((1−δ²)² + z²s²)) / (1−δ²+z²s²)``.

    The variance is Cliff's consistent dominance-matrix estimate
    ``s² = [(n_y−1)²Σ(d_i.−δ)² + (n_x−1)²Σ(d_.j−δ)² − ΣΣ(d_ij−δ)²] / [n_x n_y (n_x−1)(n_y−1)]`` and z is the
    Student-t quantile with min(n_x, n_y)−1 df (``use_normal`` → normal quantile). Of the textbook
    variants (n² vs (n−1)² weights, normal vs t(n_x+n_y−2) vs t(min n−1), with or without the z²s² term
    under the root) this is the one that reproduces all six published CI endpoints of the H1 table
    (ipynb:1307-1311; see tests/test_analysis.py). O(n_x·n_y) memory, fine for the study's cells."""
    x, y = _arr(x), _arr(y)
    n1, n2 = x.size, y.size
    dom = np.sign(x[:, None] - y[None, :])
    d = float(dom.mean())
    di = dom.mean(axis=1)
    dj = dom.mean(axis=0)
    s2 = (((n2 - 1) ** 2 * np.sum((di - d) ** 2) + (n1 - 1) ** 2 * np.sum((dj - d) ** 2) - np.sum((dom - d) ** 2))
          / (n1 * n2 * (n1 - 1) * (n2 - 1)))
    s2 = float(max(s2, 0.0))
    q = (1 + conf_level) / 2
    z = _st.norm.ppf(q) if use_normal else _st.t.ppf(q, min(n1, n2) - 1)
    s = math.sqrt(s2)
    root = math.sqrt((1 - d * d) ** 2 + z * z * s2)
    den = 1 - d * d + z * z * s2
    if den <= 0.0:  # complete separation (|δ| = 1, s² = 0): the interval degenerates to the point estimate
        return CliffResult(d, d, d, s2, cliff_magnitude(d))
    lo = (d - d ** 3 - z * s * root) / den
    hi = (d - d ** 3 + z * s * root) / den
    return CliffResult(d, float(max(-1.0, lo)), float(min(1.0, hi)), s2, cliff_magnitude(d))


# AS 89 (Best & Roberts 1975) Edgeworth series coefficients for the Spearman S statistic upper tail
_AS89 = (0.2274, 0.2531, 0.1745, 0.0758, 0.1033, 0.3932, 0.0879, 0.0151, 0.0072, 0.0831, 0.0131, 4.6e-4)


def _spearman_upper_exact(s: float, n: int) -> float:
    """P(S ≥ s) by enumerating all n! permutations (n ≤ 9)."""
    base = np.arange(1, n + 1)
    perms = np.array(list(itertools.permutations(range(1, n + 1))), dtype=np.int64)
    ss = np.sum((perms - base) ** 2, axis=1)
    return float(np.mean(ss >= s - 1e-9))


def _spearman_upper_edgeworth(s: float, n: int) -> float:
    """AS 89 upper-tail probability P(S ≥ s) for n > 9 (R's ``prho``)."""
    c1, c2, c3, c4, c5, c6, c7, c8, c9, c10, c11, c12 = _AS89
    b = 1.0 / n
    x = (6.0 * (s - 1) * b / (n * n - 1) - 1.0) * math.sqrt(1.0 / b - 1.0)
    y = x * x
    u = x * b * (c1 + b * (c2 + c3 * b) + y * (-c4 + b * (c5 + c6 * b)
                                               - y * b * (c7 + c8 * b - y * (c9 - c10 * b + y * b * (c11 - c12 * y)))))
    p = u / math.exp(y / 2.0) + _st.norm.sf(x)
    return min(1.0, max(0.0, p))


def spearman_test(x, y) -> TestResult:
    """``cor.test(x, y, method="spearman")`` two-sided: returns ρ and its p-value (R semantics)."""
    x, y = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)
    ok = ~(np.isnan(x) | np.isnan(y))
    x, y = x[ok], y[ok]
    n = x.size
    rx, ry = _midranks(x), _midranks(y)
    rho = float(np.corrcoef(rx, ry)[0, 1])
    ties = len(np.unique(rx)) < n or len(np.unique(ry)) < n
    den = n * (n * n - 1) / 6.0
    q = den * (1.0 - rho)
    warn = None
    if ties or n > 1290:
        warn = "Cannot compute exact p-value with ties" if ties else None
        t = rho / math.sqrt(max(1e-300, (1 - rho * rho) / (n - 2))) if abs(rho) < 1 else math.copysign(math.inf, rho)
        p = 2.0 * _st.t.sf(abs(t), n - 2)
    else:
        upper = _spearman_upper_exact if n <= 9 else _spearman_upper_edgeworth
        if q > den:   # negative correlation: upper tail of S
            pv = upper(round(q), n)
        else:         # P(S ≤ q) = 1 − P(S ≥ q + 2) (S takes even values)
            pv = 1.0 - upper(round(q) + 2, n)
        p = min(2.0 * pv, 1.0)
    return TestResult(rho, float(min(1.0, p)), "Spearman's rank correlation rho", warn)


def stars(p: float) -> str:
    return "***" if p < 0.001 else ("**" if p < 0.01 else ("*" if p < 0.05 else ""))
