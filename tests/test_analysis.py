"""Golden test of the analysis module against every published number of the paper's R notebook
(`data-analysis/analysis-visualization.ipynb:524-531, 1062-1067, 1307-1311, 1714-1720`),
recomputed from the reference's own run table (tests/fixtures/run_table.csv, data only)."""
import itertools
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from cain_amd.analysis import stats as S
from cain_amd.analysis.report import analyze, load_run_table, make_subsets

FIX = Path(__file__).parent / "fixtures" / "run_table.csv"

# (length, method) -> n, energy mean/median/sd, time mean/median/sd (ipynb:524-531)
SUMMARY = {
    ("short", "on_device"): (167, 52.82, 55.00, 20.94, 15.07, 15.47, 3.44),
    ("short", "remote"): (175, 15.18, 14.30, 5.86, 8.90, 8.76, 0.97),
    ("medium", "on_device"): (182, 349.34, 403.80, 179.15, 35.99, 38.77, 12.16),
    ("medium", "remote"): (160, 41.01, 47.55, 14.18, 13.17, 14.21, 2.35),
    ("long", "on_device"): (191, 431.97, 462.50, 246.92, 43.35, 43.19, 18.50),
    ("long", "remote"): (162, 48.56, 47.80, 19.86, 14.38, 14.30, 3.29),
}
H1 = {"short": ("28370", 0.941, 0.905, 0.964), "medium": ("28486", 0.956, 0.920, 0.976),
      "long": ("29587", 0.912, 0.868, 0.942)}
H2 = {  # rho time, cpu, gpu, memory (ipynb:1714-1720)
    "on_device_short": (0.991, -0.708, -0.176, 0.541), "on_device_medium": (0.928, -0.284, 0.153, 0.520),
    "on_device_long": (0.986, -0.276, 0.315, 0.536), "remote_short": (0.891, -0.785, -0.647, 0.010),
    "remote_medium": (0.963, -0.645, -0.723, -0.032), "remote_long": (0.983, -0.710, -0.640, -0.045)}
SHAPIRO_W = {"on_device_short": 0.9547488, "on_device_medium": 0.8745747, "on_device_long": 0.9290627,
             "remote_short": 0.8594111, "remote_medium": 0.9094642, "remote_long": 0.9322779}


@pytest.fixture(scope="module")
def result(tmp_path_factory):
    return analyze(FIX, tmp_path_factory.mktemp("an"), quiet=True)


def test_summary_table_matches_paper(result):
    for r in result["summary"]:
        exp = SUMMARY[(r["length"], r["method"])]
        got = (r["n"], r["energy_usage_J"]["mean"], r["energy_usage_J"]["median"], r["energy_usage_J"]["sd"],
               r["execution_time"]["mean"], r["execution_time"]["median"], r["execution_time"]["sd"])
        assert got[0] == exp[0]
        assert [f"{v:.2f}" for v in got[1:]] == [f"{v:.2f}" for v in exp[1:]]


def test_h1_wilcoxon_and_cliff(result):
    for r in result["h1"]:
        w, d, lo, hi = H1[r["length"]]
        assert f"{r['W']:.0f}" == w and r["p"] < 2.2e-16 and r["magnitude"] == "Large"
        assert (f"{r['cliffs_delta']:.3f}", f"{r['lower_ci']:.3f}", f"{r['upper_ci']:.3f}") == \
            (f"{d:.3f}", f"{lo:.3f}", f"{hi:.3f}")
    assert [r["W"] for r in result["h1"]] == [28370.0, 28485.5, 29587.0]


def test_h2_spearman(result):
    for r in result["h2"]:
        exp = H2[f"{r['method']}_{r['length']}"]
        got = tuple(round(r[k]["rho"], 3) for k in ("execution_time", "cpu_usage", "gpu_usage", "memory_usage"))
        assert got == pytest.approx(exp, abs=1e-9)
    rs = {f"{r['method']}_{r['length']}": r for r in result["h2"]}
    assert rs["on_device_short"]["gpu_usage"]["stars"] == "*"
    assert f"{rs['remote_short']['memory_usage']['p']:.3f}" == "0.893"
    assert f"{rs['remote_long']['memory_usage']['p']:.3f}" == "0.570"


def test_shapiro_and_skew(result):
    for r in result["shapiro"]:
        if "W" in r:
            assert round(r["W"], 7) == SHAPIRO_W[r["subset"]] and r["p"] <= 3.3e-5
    sk = {r["subset"]: r for r in result["shapiro"] if "skew_on_device" in r}
    assert sk["short"]["transforms"] == []  # arms skew differently -> no transformation (ipynb output)
    assert [t["name"] for t in sk["medium"]["transforms"]] == ["Original", "Power 2", "Power 3"]
    assert sk["medium"]["transforms"][0]["p_on_device"] == pytest.approx(3.521535e-11, rel=1e-4)


def test_outputs_written(result, tmp_path):
    out = Path(result["source"]).parent
    res = analyze(FIX, tmp_path, quiet=True)
    tex = (tmp_path / "h1.tex").read_text()
    assert "\\textbf{Short (100 words)} & 28370 & < 2.2e-16 & 0.941 & 0.905 & 0.964 & Large" in tex
    assert "52.82 & 55.00 & 20.94" in (tmp_path / "summary.tex").read_text()
    assert len(res["per_model"]) == 42 and (tmp_path / "results.json").exists()
    llama = [r for r in res["per_model"] if r["model"] == "llama3.1:8b" and r["method"] == "on_device"
             and r["length"] == 1000][0]
    assert round(llama["energy_J"], 1) == 764.7 and round(llama["time_s"], 2) == 69.27


def test_quantile_type7_and_iqr():
    x = [1, 2, 3, 4, 100]
    assert S.quantile7(x, 0.25) == 2 and S.quantile7(x, 0.75) == 4
    assert S.quantile7([1, 2], 0.25) == 1.25


def test_wilcox_exact_small_sample():
    x = [1.83, 0.50, 1.62, 2.48, 1.68, 1.88, 1.55, 3.06, 1.30]
    y = [0.878, 0.647, 0.598, 2.05, 1.06, 1.29, 1.07, 3.14, 1.28]
    r = S.wilcox_test(x, y)
    # W counts pairs x>y; 9 x 9 without ties -> exact distribution (R: n < 50 and no ties)
    assert r.statistic == sum(a > b for a in x for b in y) and r.warning is None and "exact" in r.method
    x2 = [1.0, 2.0, 2.0, 3.0]
    r2 = S.wilcox_test(x2, [2.0, 4.0, 5.0])
    assert r2.warning  # ties force the normal approximation, like R


def test_spearman_edgeworth_matches_enumeration():
    n = 10
    perms = np.array(list(itertools.permutations(range(1, n + 1))), dtype=np.int16)
    ss = np.sum((perms - np.arange(1, n + 1)) ** 2, axis=1)
    for s in (100, 150, 200, 260):
        assert S._spearman_upper_edgeworth(s, n) == pytest.approx(np.mean(ss >= s), abs=1e-3)
    r = S.spearman_test([1, 2, 3, 4, 5], [5, 6, 7, 8, 7.5])
    assert r.statistic == pytest.approx(0.9) and r.warning is None


def test_cli_analyze(tmp_path):
    r = subprocess.run([sys.executable, "-m", "cain_amd", "analyze", str(FIX), "--out", str(tmp_path), "--plots"],
                       capture_output=True, text=True, timeout=300, cwd=Path(__file__).parent.parent)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "28370" in r.stdout
    assert (tmp_path / "scatter_plots" / "cpu_usage_vs_energy_usage_J.pdf").exists()
    # the reference's 75 PDFs, same tree and file names (data-analysis/{violin,density,qq,scatter}_plots)
    ref = Path("/root/reference/data-analysis")
    ours = sorted(str(p.relative_to(tmp_path)) for p in tmp_path.rglob("*.pdf"))
    assert len(ours) == 75
    if ref.exists():
        theirs = sorted(str(p.relative_to(ref)) for p in ref.rglob("*.pdf"))
        assert ours == theirs


def test_cliff_delta_complete_separation_has_a_point_interval():
    """Every on-device run above every remote run (the MI355X study): δ = 1 with a degenerate [1, 1] interval,
    not the [-1, 1] a 0/0 made of it."""
    r = S.cliff_delta([10.0, 11.0, 12.0, 13.0], [1.0, 2.0, 3.0])
    assert r.estimate == 1.0 and r.lower == 1.0 and r.upper == 1.0 and r.magnitude == "Large"


def test_energy_views_and_remote_board_rederivation(tmp_path):
    """H1 and the arm ratio on gross AND idle-subtracted energy; an older run table whose
    remote rows left the client board at 0 J (server on the client's GPU) is re-charged at the recorded idle power x
    window, so gross means the same in both arms."""
    import csv as _csv

    from cain_amd.analysis.report import analyze

    rows = []
    for i in range(12):
        for length, t in ((100, 0.4), (500, 1.6), (1000, 3.2)):
            w = t * (1 + 0.01 * i)
            rows.append(dict(__run_id=f"o{i}_{length}", __done="DONE", model="m", method="on_device", length=length,
                             execution_time=w, cpu_usage=5, gpu_usage=90, memory_usage=3,
                             energy_usage_J=round(1000 * w, 3), gpu_energy_J=round(999 * w, 3),
                             idle_subtracted_J=round(740 * w, 3), idle_power_W=260.0, energy_window_s=w))
            rows.append(dict(__run_id=f"r{i}_{length}", __done="DONE", model="m", method="remote", length=length,
                             execution_time=w, cpu_usage=6, gpu_usage=0, memory_usage=3,
                             energy_usage_J=round(1 * w, 3), gpu_energy_J=0.0, idle_subtracted_J=round(1 * w, 3),
                             idle_power_W=260.0, energy_window_s=w))
    p = tmp_path / "run_table.csv"
    with open(p, "w", newline="") as fh:
        wr = _csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
        wr.writeheader()
        wr.writerows(rows)
    raw = analyze(p, tmp_path / "raw", quiet=True)
    fixed = analyze(p, tmp_path / "fixed", quiet=True, rederive=True)
    v_raw = {(r["length"], r["view"]): r for r in raw["energy_views"]}
    v_fix = {(r["length"], r["view"]): r for r in fixed["energy_views"]}
    assert set(v_fix) == {(L, v) for L in ("short", "medium", "long")
                          for v in ("gross", "idle_normalised", "idle_subtracted")}
    # one idle floor across the table: the idle-normalised view is the gross one
    assert v_fix[("long", "idle_normalised")]["ratio"] == pytest.approx(v_fix[("long", "gross")]["ratio"])
    # as written: remote gross is the client's CPU only -> a 1000x ratio; rederived: board idle included -> 1000/261
    assert v_raw[("long", "gross")]["ratio"] == pytest.approx(1000.0, rel=1e-3)
    assert v_fix[("long", "gross")]["ratio"] == pytest.approx(1000.0 / 261.0, rel=1e-3)
    # the idle-subtracted view does not change: the board's part is idle - idle = 0
    assert v_fix[("long", "idle_subtracted")]["ratio"] == pytest.approx(v_raw[("long", "idle_subtracted")]["ratio"])
    assert (tmp_path / "fixed" / "energy_views.md").read_text().count("idle_subtracted") == 3


def test_idle_normalised_view_removes_box_idle_spread():
    """sessions on boxes with different idle floors; the idle-normalised energy charges every run
    at the table's mean idle power, so two runs with the same request energy on a 240 W and a 300 W box agree."""
    import pandas as pd

    from cain_amd.analysis.report import IDLE_NORM, add_idle_normalised

    df = pd.DataFrame(dict(energy_usage_J=[240 * 2 + 100, 300 * 2 + 100], idle_power_W=[240.0, 300.0],
                           energy_window_s=[2.0, 2.0]))
    ref = add_idle_normalised(df)
    assert ref == pytest.approx(270.0)
    assert df[IDLE_NORM].tolist() == pytest.approx([640.0, 640.0])
    # a table without idle columns has no such view
    assert add_idle_normalised(pd.DataFrame(dict(energy_usage_J=[1.0]))) is None


def test_replicate_run_tables_pool(tmp_path):
    """Two replicates of one design (same run ids, different seeds) pool into one analysis: run ids are prefixed by
    the replicate, every cell's n is the sum, and a single path still behaves as before."""
    import csv as _csv

    from cain_amd.analysis.report import analyze, load_run_table

    paths = []
    for rep in range(2):
        rows = []
        for i in range(6):
            for method, e in (("on_device", 900.0), ("remote", 300.0)):
                w = 1.0 + 0.01 * i + 0.001 * rep
                rows.append(dict(__run_id=f"run_{i}_{method}", __done="DONE", model="m", method=method, length=500,
                                 execution_time=w, cpu_usage=5, gpu_usage=50, memory_usage=3,
                                 energy_usage_J=round(e * w, 3), idle_subtracted_J=round((e - 280) * w, 3)))
        p = tmp_path / f"rep{rep}" / "run_table.csv"
        p.parent.mkdir()
        with open(p, "w", newline="") as fh:
            wr = _csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
            wr.writeheader()
            wr.writerows(rows)
        paths.append(p)
    one = load_run_table(paths[0])
    both = load_run_table(paths)
    assert len(both) == 2 * len(one) and both["__run_id"].is_unique
    assert sorted(both["replicate"].unique()) == [0, 1]
    res = analyze(paths, tmp_path / "pooled", quiet=True)
    assert res["subset_sizes"]["on_device_medium"] == 12 and res["subset_sizes"]["remote_medium"] == 12
    assert "rep0" in res["source"] and "rep1" in res["source"]
