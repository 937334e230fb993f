"""Paper tables and plots from a run table — the notebook pipeline as a CLI.

``python -m cain_amd analyze <run_table.csv> [--out DIR] [--plots] [--format latex|markdown|both]``

Pipeline (``data-analysis/analysis-visualization.ipynb``):

1. read the CSV; if ``energy_usage_J`` is missing derive it from ``codecarbon__energy_consumed`` (kWh × 3.6e6,
   rounded to 3 d.p. — the study's ``after_experiment``, `experiment/RunnerConfig.py:249-259`)
2. six subsets method × length, each IQR-filtered over METRICS sequentially (ipynb:345-405)
3. summary table mean/median/SD per metric (ipynb:425-531)
4. Shapiro-Wilk per subset (ipynb:1047-1067), skew check + transformations (ipynb:1110)
5. H1: Wilcoxon rank-sum + Cliff's δ with CI per length (ipynb:1285-1393)
6. H2: Spearman ρ of energy vs time/CPU/GPU/memory with stars (ipynb:1539-1730)
7. optional PDFs: density / violin / QQ / scatter (ipynb:560-1003, 1404-1530), per-LLM energy violins
8. new: per (model, method, length) cells incl. measured J/token and tokens/s when the run table carries
   ``tokens_generated`` (this framework captures the Ollama ``eval_count`` that the reference discarded)
9. new: energy views (``energy_views.md``): the on-device / remote ratio of mean energy and H1 on both the gross
   client-device energy (``energy_usage_J``, the reference's quantity) and the idle-subtracted energy
   (``idle_subtracted_J``), per length.  ``--rederive-remote-board`` re-charges remote rows of run tables written
   before the one-definition accounting (round 4: a remote server sharing the client's GPU left the client's board
   at 0 J) with the board's recorded idle power x window, the definition ``experiments/study.py`` now records.

Outputs go to ``--out`` (default: next to the CSV, ``analysis/``): ``summary.{tex,md}``, ``h1.{tex,md}``,
``h2.{tex,md}``, ``shapiro.md``, ``per_model.md``, ``results.json``.
"""
from __future__ import annotations

import argparse
import json
import math
from dataclasses import asdict
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import stats as S

ON_DEVICE, REMOTE = "on_device", "remote"
METHODS = (ON_DEVICE, REMOTE)
LENGTH_MAP = {"short": 100, "medium": 500, "long": 1000}
ENERGY, TIME, CPU, GPU, MEMORY = "energy_usage_J", "execution_time", "cpu_usage", "gpu_usage", "memory_usage"
METRICS = (ENERGY, TIME, CPU, GPU, MEMORY)
AXIS_LABELS = {ENERGY: "Energy Usage (J)", TIME: "Execution Time (s)", CPU: "CPU Usage (%)",
               GPU: "GPU Usage (%)", MEMORY: "Memory Usage (%)"}
TABLE_HEADINGS = {ENERGY: "Energy Usage (Joule)", TIME: "Execution Time (second)", CPU: "Average CPU Usage (\\%)",
                  GPU: "Average GPU Usage (\\%)", MEMORY: "Average Memory Usage (\\%)"}
LLM_NAMES = {"Qwen 2 1.5B": "qwen2:1.5b", "Gemma 1.1 2B": "gemma:2b", "Phi 3 3B": "phi3:3.8b",
             "Qwen 2 7B": "qwen2:7b", "Gemma 1.1 7B": "gemma:7b", "Mistral 0.3 7B": "mistral:7b",
             "Llama 3.1 8B": "llama3.1:8b"}
COLOR_MAP = {ON_DEVICE: "coral", REMOTE: "lightblue"}


def _title(label: str) -> str:
    return label[:1].upper() + label[1:]


def rederive_remote_board(df):
    """Remote rows whose client board was charged 0 J because the remote server shared the client's GPU (run tables
    from before the one-definition accounting): charge the board at the row's recorded idle power x energy window,
    as ``StudyConfig.energy_sources_for`` now does ("gpu_idle"), and add it to ``energy_usage_J``.  Idle-subtracted
    energy is unchanged (the board's part is idle - idle = 0).  Returns the number of rows re-charged."""
    import pandas as pd

    need = {"method", "gpu_energy_J", "idle_power_W", "energy_window_s", ENERGY}
    if not need <= set(df.columns):
        return 0
    src = df["gpu_energy_source"].astype(str) if "gpu_energy_source" in df.columns else pd.Series("", index=df.index)
    gpu = pd.to_numeric(df["gpu_energy_J"], errors="coerce")
    idle = pd.to_numeric(df["idle_power_W"], errors="coerce")
    win = pd.to_numeric(df["energy_window_s"], errors="coerce")
    sel = (df["method"] == REMOTE) & (gpu == 0) & idle.notna() & win.notna() & ~src.isin(["measured", "idle_model"])
    add = (idle * win).where(sel, 0.0)
    df.loc[sel, "gpu_energy_J"] = add[sel].round(3)
    df.loc[sel, ENERGY] = (pd.to_numeric(df.loc[sel, ENERGY], errors="coerce") + add[sel]).round(3)
    df.loc[sel, "gpu_energy_source"] = "idle_model(rederived)"
    return int(sel.sum())


def load_run_table(path, rederive: bool = False):
    """One run table, or several replicates of one design (a list of paths): those are concatenated, each run id
    prefixed by its replicate index and a `replicate` column added, so the cells pool n = sum of repetitions."""
    import pandas as pd

    if isinstance(path, (list, tuple)):
        if len(path) == 1:
            return load_run_table(path[0], rederive)
        parts = []
        for i, p in enumerate(path):
            d = load_run_table(p, rederive)
            d = d.assign(replicate=i)
            if "__run_id" in d.columns:
                d["__run_id"] = f"r{i}_" + d["__run_id"].astype(str)
            parts.append(d)
        return pd.concat(parts, ignore_index=True)
    df = pd.read_csv(path)
    if rederive:
        rederive_remote_board(df)
    if ENERGY not in df.columns and "codecarbon__energy_consumed" in df.columns:
        df[ENERGY] = (pd.to_numeric(df["codecarbon__energy_consumed"], errors="coerce") * 3_600_000).round(3)
    if "__done" in df.columns:
        df = df[df["__done"].astype(str) == "DONE"]
    for c in METRICS:
        if c in df.columns:
            df[c] = pd.to_numeric(df[c], errors="coerce")
    df["length"] = pd.to_numeric(df["length"], errors="coerce")
    return df


def make_subsets(df, metrics: Sequence[str] = METRICS) -> Dict[str, "object"]:
    metrics = [m for m in metrics if m in df.columns]
    out = {}
    for m in METHODS:
        for label, L in LENGTH_MAP.items():
            part = df[(df["method"] == m) & (df["length"] == L)]
            if len(part):
                out[f"{m}_{label}"] = S.remove_outliers(part, metrics)
    return out


def summary_rows(subsets) -> List[dict]:
    rows = []
    for label, L in LENGTH_MAP.items():
        for m in METHODS:
            d = subsets.get(f"{m}_{label}")
            if d is None:
                continue
            row = {"length": label, "words": L, "method": m, "n": int(len(d))}
            for k in METRICS:
                if k in d.columns:
                    st = S.describe(d[k])
                    row[k] = {"mean": st.mean, "median": st.median, "sd": st.sd}
            rows.append(row)
    return rows


def h1_rows(subsets) -> List[dict]:
    rows = []
    for label, L in LENGTH_MAP.items():
        a, b = subsets.get(f"{ON_DEVICE}_{label}"), subsets.get(f"{REMOTE}_{label}")
        if a is None or b is None:
            continue
        w = S.wilcox_test(a[ENERGY], b[ENERGY])
        c = S.cliff_delta(a[ENERGY], b[ENERGY])
        rows.append({"length": label, "words": L, "W": w.statistic, "p": w.p_value, "cliffs_delta": c.estimate,
                     "lower_ci": c.lower, "upper_ci": c.upper, "magnitude": c.magnitude})
    return rows


IDLE_SUB = "idle_subtracted_J"
IDLE_NORM = "idle_normalised_J"


def add_idle_normalised(df) -> Optional[float]:
    """Per-session idle normalisation: each study session ran on a fresh box whose idle floor
    differs by ~40 W, and at short lengths the client board's idle x window is most of the gross energy, so box
    identity inflates the spread.  ``idle_normalised_J`` = gross + (idle_ref - the row's ``idle_power_W``) x its
    ``energy_window_s``: every run charged at ONE idle floor, idle_ref = the mean session idle power of the pooled
    table (returned).  Gross (the reference's quantity) and idle-subtracted stay as they are."""
    import pandas as pd

    if not {"idle_power_W", "energy_window_s", ENERGY} <= set(df.columns):
        return None
    idle = pd.to_numeric(df["idle_power_W"], errors="coerce")
    win = pd.to_numeric(df["energy_window_s"], errors="coerce")
    if not idle.notna().any():
        return None
    ref = float(idle.dropna().mean())
    df[IDLE_NORM] = df[ENERGY] + (ref - idle) * win
    return ref


def energy_view_rows(subsets) -> List[dict]:
    """Per length: mean energy per arm, the on-device / remote ratio and H1 (Wilcoxon + Cliff's delta) on the gross
    client-device energy and, where recorded, on the idle-subtracted energy (same IQR-filtered subsets)."""
    import pandas as pd

    rows = []
    for label, L in LENGTH_MAP.items():
        a, b = subsets.get(f"{ON_DEVICE}_{label}"), subsets.get(f"{REMOTE}_{label}")
        if a is None or b is None:
            continue
        for view, col in (("gross", ENERGY), ("idle_normalised", IDLE_NORM), ("idle_subtracted", IDLE_SUB)):
            if col not in a.columns or col not in b.columns:
                continue
            x = pd.to_numeric(a[col], errors="coerce").dropna()
            y = pd.to_numeric(b[col], errors="coerce").dropna()
            if not len(x) or not len(y):
                continue
            w, c = S.wilcox_test(x, y), S.cliff_delta(x, y)
            mx, my = float(x.mean()), float(y.mean())
            rows.append({"length": label, "words": L, "view": view, "n_on_device": int(len(x)),
                         "n_remote": int(len(y)), "mean_on_device": mx, "mean_remote": my,
                         "sd_on_device": float(x.std()), "sd_remote": float(y.std()),
                         "ratio": mx / my if my > 0 else float("nan"), "W": w.statistic, "p": w.p_value,
                         "cliffs_delta": c.estimate, "magnitude": c.magnitude})
    return rows


def h2_rows(subsets) -> List[dict]:
    rows = []
    for m in METHODS:
        for label, L in LENGTH_MAP.items():
            d = subsets.get(f"{m}_{label}")
            if d is None:
                continue
            row = {"method": m, "length": label, "words": L}
            for k in (TIME, CPU, GPU, MEMORY):
                if k in d.columns:
                    t = S.spearman_test(d[ENERGY], d[k])
                    row[k] = {"rho": t.statistic, "p": t.p_value, "stars": S.stars(t.p_value)}
            rows.append(row)
    return rows


def shapiro_rows(subsets) -> List[dict]:
    rows = [{"subset": k, "W": S.shapiro(d[ENERGY]).statistic, "p": S.shapiro(d[ENERGY]).p_value}
            for k, d in subsets.items()]
    for label in LENGTH_MAP:
        a, b = subsets.get(f"{ON_DEVICE}_{label}"), subsets.get(f"{REMOTE}_{label}")
        if a is None or b is None:
            continue
        la, lb, tr = S.transform_towards_normality(a[ENERGY], b[ENERGY])
        rows.append({"subset": label, "skew_on_device": la, "skew_remote": lb,
                     "transforms": [{"name": n, "p_on_device": p1, "p_remote": p2} for n, p1, p2 in tr]})
    return rows


def per_model_rows(df) -> List[dict]:
    """Raw (unfiltered) per-cell means — the BASELINE.md table — plus measured J/token and tok/s."""
    rows = []
    has_tok = "tokens_generated" in df.columns
    for (model, method, length), g in df.groupby(["model", "method", "length"], sort=True):
        r = {"model": model, "method": method, "length": int(length), "n": int(len(g)),
             "energy_J": float(g[ENERGY].mean()), "time_s": float(g[TIME].mean())}
        if has_tok:
            tok = g["tokens_generated"].astype(float)
            r["tokens"] = float(tok.mean())
            r["J_per_token"] = float((g[ENERGY] / tok).mean())
            r["tok_per_s"] = float((tok / g[TIME]).mean())
        rows.append(r)
    return rows


# ---------------------------------------------------------------------------------------------- formatting
def _p_fmt(p: float) -> str:
    return "< 2.2e-16" if p < 0.001 else f"{p:.1e}"


def summary_latex(rows) -> str:
    lines = ["\\begin{table*}[htbp]", "    \\centering",
             "    \\caption{Mean, Median, and Standard Deviation (SD) of Energy Usage and Performance Metrics for "
             "Fetching LLM Content On-Device vs. Remote Across Varying Content Lengths}",
             "    \\scalebox{0.8}{", "    \\begin{tabular}{|l|l|ccc|ccc|ccc|ccc|ccc|}", "        \\hline",
             "        \\multirow{2}{*}{\\textbf{Content Length}} & \\multirow{2}{*}{\\textbf{Treatment}} & "
             + " & ".join(f"\\multicolumn{{3}}{{c|}}{{\\textbf{{{TABLE_HEADINGS[k]}}}}}" for k in METRICS) + " \\\\ ",
             "        \\cline{3-17}",
             "        & & " + " & ".join(["\\textbf{Mean} & \\textbf{Median} & \\textbf{SD}"] * 5) + " \\\\ ",
             "        \\hline"]
    for r in rows:
        vals = " & ".join(f"{r[k]['mean']:.2f} & {r[k]['median']:.2f} & {r[k]['sd']:.2f}" for k in METRICS if k in r)
        if r["method"] == ON_DEVICE:
            head = f"\\textbf{{{_title(r['length'])} ({r['words']} words)}} & \\textbf{{On-Device}}"
        else:
            head = "& \\textbf{Remote}"
        lines.append(f"        {head} & {vals} \\\\ ")
        if r["method"] == REMOTE:
            lines.append("        \\hline")
    lines += ["    \\end{tabular}", "    }", "    \\label{table:performance_metrics}", "\\end{table*}"]
    return "\n".join(lines) + "\n"


def summary_markdown(rows) -> str:
    hdr = "| Length | Arm | n | " + " | ".join(f"{AXIS_LABELS[k]} mean / median / SD" for k in METRICS) + " |"
    out = [hdr, "|" + "---|" * (3 + len(METRICS))]
    for r in rows:
        vals = " | ".join(f"{r[k]['mean']:.2f} / {r[k]['median']:.2f} / {r[k]['sd']:.2f}" if k in r else "-"
                          for k in METRICS)
        out.append(f"| {_title(r['length'])} ({r['words']}) | {r['method']} | {r['n']} | {vals} |")
    return "\n".join(out) + "\n"


def h1_latex(rows) -> str:
    lines = ["\\begin{table}[H]", "  \\centering",
             "  \\caption{Results for Hypothesis 1 - Energy Usage Difference Between On-device and Remote LLMs "
             "Content Fetching}", "  \\resizebox{\\columnwidth}{!}{%", "    \\begin{tabular}{lcccccc}", "      \\hline",
             "      \\textbf{Content Length} & \\textbf{W-Value} & \\textbf{P-Value} & \\textbf{Cliff’s Delta} & "
             "\\textbf{Lower CI} & \\textbf{Upper CI} & \\textbf{Delta} \\\\", "      \\hline"]
    for r in rows:
        lines.append(f"      \\textbf{{{_title(r['length'])} ({r['words']} words)}} & {r['W']:.0f} & {_p_fmt(r['p'])} & "
                     f"{r['cliffs_delta']:.3f} & {r['lower_ci']:.3f} & {r['upper_ci']:.3f} & {r['magnitude']} \\\\")
        lines.append("      \\hline")
    lines += ["    \\end{tabular}%", "}", "  \\label{table:h1}", "\\end{table}"]
    return "\n".join(lines) + "\n"


def h1_markdown(rows) -> str:
    out = ["| Length | Wilcoxon W | p | Cliff's δ [95% CI] | magnitude |", "|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| {_title(r['length'])} ({r['words']}) | {r['W']:.1f} | {r['p']:.3g} | {r['cliffs_delta']:.3f} "
                   f"[{r['lower_ci']:.3f}, {r['upper_ci']:.3f}] | {r['magnitude']} |")
    return "\n".join(out) + "\n"


def _h2_cell(c, latex: bool) -> str:
    if not np.isfinite(c["rho"]):
        return "n/a (constant)"  # e.g. the remote arm's client GPU %, 0 by construction
    coef = f"{c['rho']:.3f}"
    p = "<0.001" if c["p"] < 0.001 else f"{c['p']:.3f}"
    s = f"{coef} ({p}{c['stars']})"
    if latex and c["p"] < 0.05:
        return f"\\textbf{{{s}}}"
    return s


def h2_latex(rows) -> str:
    body = ""
    for m in METHODS:
        mr = [r for r in rows if r["method"] == m]
        if not mr:
            continue
        body += f"\\multirow{{3}}{{*}}{{\\textbf{{{_title(m.replace('_', '-'))}}}}} "
        for r in mr:
            cells = " & ".join(_h2_cell(r[k], True) for k in (TIME, CPU, GPU, MEMORY) if k in r)
            body += f"& \\textbf{{{_title(r['length'])} ({r['words']})}} & {cells} \\\\ \\cline{{2-6}}\n"
        body += "\\hline\n"
    return ("\\begin{table*}[htbp]\n    \\centering\n    \\caption{Spearman Rank Correlation for Hypothesis 2: Energy "
            "Usage vs. Performance Metrics.}\n    \\begin{tabular}{|l|l|c|c|c|c|}\n    \\hline\n"
            "    \\textbf{Treatment} & \\textbf{Content Length} & \\textbf{Execution Time} & \\textbf{CPU Usage} & "
            "\\textbf{GPU Usage} & \\textbf{Memory Usage} \\\\ \\hline\n" + body +
            "    \\end{tabular}\n    \\label{table:h2}\n\\end{table*}\n")


def h2_markdown(rows) -> str:
    out = ["| Arm / length | vs exec time | vs CPU % | vs GPU % | vs memory % |", "|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| {r['method']} {r['length']} | " +
                   " | ".join(_h2_cell(r[k], False) if k in r else "-" for k in (TIME, CPU, GPU, MEMORY)) + " |")
    return "\n".join(out) + "\n"


def energy_views_markdown(rows) -> str:
    lines = ["| Length | View | On-device J (mean / SD) | Remote J (mean / SD) | On-device / remote | W | p | "
             "Cliff's delta |", "|---|---|---|---|---|---|---|---|"]
    for r in rows:
        ratio = f"{r['ratio']:.2f}x" if r["ratio"] == r["ratio"] else "n/a"
        lines.append(f"| {_title(r['length'])} ({r['words']}) | {r['view']} | {r['mean_on_device']:.2f} / "
                     f"{r.get('sd_on_device', float('nan')):.2f} | {r['mean_remote']:.2f} / "
                     f"{r.get('sd_remote', float('nan')):.2f} | {ratio} | {r['W']:.0f} | {_p_fmt(r['p'])} | "
                     f"{r['cliffs_delta']:.3f} ({r['magnitude']}) |")
    return "\n".join(lines) + "\n"


def per_model_markdown(rows) -> str:
    tok = rows and "J_per_token" in rows[0]
    out = ["| model | method | length | n | energy J | time s |" + (" tokens | J/token | tok/s |" if tok else ""),
           "|---|---|---|---|---|---|" + ("---|---|---|" if tok else "")]
    for r in rows:
        s = f"| {r['model']} | {r['method']} | {r['length']} | {r['n']} | {r['energy_J']:.1f} | {r['time_s']:.2f} |"
        if tok:
            s += f" {r['tokens']:.0f} | {r['J_per_token']:.4f} | {r['tok_per_s']:.1f} |"
        out.append(s)
    return "\n".join(out) + "\n"


# ---------------------------------------------------------------------------------------------- plots
def make_plots(df, subsets, out: Path) -> List[Path]:
    """The notebook's 75 PDFs in its directory tree (matplotlib; the notebook used ggplot2):

    * ``density_plots/<metric>/density_plot_<length>.pdf`` + ``combined_density_plots_<metric>.pdf``
      (analysis-visualization.ipynb:696, :720);
    * ``violin_plots/<metric>/violin_plot_<length>.pdf`` + ``combined_violin_plots_<metric>.pdf`` (:710, :724)
      + ``violin_plots/energy_usage_J/combined_violin_plots_llms_energy_usage_J.pdf`` (:919);
    * ``qq_plots/<method>/<metric>/qq_plot_<length>.pdf`` (:964-1007);
    * ``scatter_plots/<metric>_vs_energy_usage_J.pdf`` (:1484)."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    from scipy import stats as st

    written: List[Path] = []
    labels = list(LENGTH_MAP)

    def save(fig, p: Path) -> None:
        p.parent.mkdir(parents=True, exist_ok=True)
        fig.tight_layout()
        fig.savefig(p)
        plt.close(fig)
        written.append(p)

    def density(ax, k, label):
        for m in METHODS:
            d = subsets.get(f"{m}_{label}")
            if d is None or len(d) < 2:
                continue
            v = d[k].to_numpy(float)
            if np.ptp(v) > 0:
                xs = np.linspace(v.min(), v.max(), 200)
                ax.fill_between(xs, st.gaussian_kde(v)(xs), alpha=0.5, color=COLOR_MAP[m], label=m)
        ax.set_title(f"{_title(label)} ({LENGTH_MAP[label]})")
        ax.set_xlabel(AXIS_LABELS[k])
        ax.set_ylabel("Density")

    def violin(ax, k, label):
        data, ticks, cols = [], [], []
        for m in METHODS:
            d = subsets.get(f"{m}_{label}")
            if d is not None and len(d):
                data.append(d[k].to_numpy(float))
                ticks.append(_title(m))
                cols.append(COLOR_MAP[m])
        if data:
            parts = ax.violinplot(data, showmedians=True)
            for b, c in zip(parts["bodies"], cols):
                b.set_facecolor(c)
            ax.set_xticks(range(1, len(ticks) + 1), ticks)
        ax.set_title(f"{_title(label)} ({LENGTH_MAP[label]})")
        ax.set_ylabel(AXIS_LABELS[k])

    for k in METRICS:
        for kind, draw in (("density", density), ("violin", violin)):
            d_dir = out / f"{kind}_plots" / k
            for label in labels:
                fig, ax = plt.subplots(figsize=(4, 3.5))
                draw(ax, k, label)
                if kind == "density":
                    ax.legend()
                save(fig, d_dir / f"{kind}_plot_{label}.pdf")
            fig, axes = plt.subplots(1, len(labels), figsize=(4 * len(labels), 3.5))
            for ax, label in zip(axes, labels):
                draw(ax, k, label)
            if kind == "density":
                axes[0].legend()
            save(fig, d_dir / f"combined_{kind}_plots_{k}.pdf")
        for m in METHODS:
            for label in labels:
                d = subsets.get(f"{m}_{label}")
                fig, ax = plt.subplots(figsize=(4, 4))
                if d is not None and len(d) >= 3:
                    st.probplot(d[k].to_numpy(float), plot=ax)
                ax.set_title(f"{_title(m)} {_title(label)}: {AXIS_LABELS[k]}")
                save(fig, out / "qq_plots" / m / k / f"qq_plot_{label}.pdf")

    for k in (TIME, CPU, GPU, MEMORY):
        fig, axes = plt.subplots(2, 3, figsize=(12, 8))
        for i, m in enumerate(METHODS):
            for j, label in enumerate(labels):
                ax = axes[i][j]
                d = subsets.get(f"{m}_{label}")
                if d is None or len(d) < 2:
                    continue
                x, y = d[ENERGY].to_numpy(float), d[k].to_numpy(float)
                ax.scatter(x, y, s=2, color="black")
                if np.ptp(x) > 0:
                    a, b = np.polyfit(x, y, 1)
                    ax.plot(np.sort(x), a * np.sort(x) + b, color=COLOR_MAP[m])
                ax.set_title(f"{_title(m)} - {_title(label)} ({LENGTH_MAP[label]})")
                ax.set_xlabel(AXIS_LABELS[ENERGY] if m == REMOTE else "")
                ax.set_ylabel(AXIS_LABELS[k] if label == "short" else "")
        save(fig, out / "scatter_plots" / f"{k}_vs_{ENERGY}.pdf")

    fig, ax = plt.subplots(figsize=(12, 4))
    data, ticks = [], []
    if "model" in df.columns:
        for nice, name in LLM_NAMES.items():
            for m in METHODS:
                v = df[(df["model"] == name) & (df["method"] == m)][ENERGY].dropna().to_numpy(float)
                if v.size:
                    data.append(v)
                    ticks.append(f"{nice}\n{m}")
    if data:
        ax.violinplot(data, showmedians=True)
        ax.set_xticks(range(1, len(ticks) + 1), ticks, fontsize=6)
    ax.set_ylabel(AXIS_LABELS[ENERGY])
    save(fig, out / "violin_plots" / ENERGY / f"combined_violin_plots_llms_{ENERGY}.pdf")
    return written


# ---------------------------------------------------------------------------------------------- entry points
def analyze(path, out: Optional[Path] = None, plots: bool = False, fmt: str = "both", quiet: bool = False,
            rederive: bool = False) -> dict:
    paths = [Path(p) for p in path] if isinstance(path, (list, tuple)) else [Path(path)]
    out = Path(out) if out else paths[0].parent / "analysis"
    out.mkdir(parents=True, exist_ok=True)
    df = load_run_table(paths, rederive=rederive)
    idle_ref = add_idle_normalised(df)
    subsets = make_subsets(df)
    res = {"source": ", ".join(str(p) for p in paths), "n_rows": int(len(df)), "subset_sizes": {k: int(len(v)) for k, v in subsets.items()},
           "summary": summary_rows(subsets), "shapiro": shapiro_rows(subsets), "h1": h1_rows(subsets),
           "h2": h2_rows(subsets), "per_model": per_model_rows(df) if "model" in df.columns else [],
           "energy_views": energy_view_rows(subsets), "rederived_remote_board": bool(rederive),
           "idle_ref_W": idle_ref}
    texts = {}
    if fmt in ("latex", "both"):
        texts.update({"summary.tex": summary_latex(res["summary"]), "h1.tex": h1_latex(res["h1"]),
                      "h2.tex": h2_latex(res["h2"])})
    if fmt in ("markdown", "both"):
        sh = ["| subset | W | p |", "|---|---|---|"] + [f"| {r['subset']} | {r['W']:.7f} | {r['p']:.6e} |"
                                                        for r in res["shapiro"] if "W" in r]
        texts.update({"summary.md": summary_markdown(res["summary"]), "h1.md": h1_markdown(res["h1"]),
                      "h2.md": h2_markdown(res["h2"]), "shapiro.md": "\n".join(sh) + "\n",
                      "per_model.md": per_model_markdown(res["per_model"]),
                      "energy_views.md": energy_views_markdown(res["energy_views"])})
    for name, t in texts.items():
        (out / name).write_text(t)
    if plots:
        res["plots"] = [str(p) for p in make_plots(df, subsets, out)]
    (out / "results.json").write_text(json.dumps(res, indent=1, default=float))
    if not quiet:
        for name in ("summary.md", "h1.md", "h2.md", "energy_views.md"):
            if name in texts:
                print(texts[name])
        print(f"wrote {len(texts)} tables{' and plots' if plots else ''} to {out}")
    return res


def main(argv: Optional[List[str]] = None) -> None:
    ap = argparse.ArgumentParser(prog="python -m cain_amd analyze", description=__doc__.split("\n")[0])
    ap.add_argument("run_table", nargs="+", help="run_table.csv; several = replicates of one design, pooled")
    ap.add_argument("--out", default=None)
    ap.add_argument("--plots", action="store_true", help="also write density/violin/QQ/scatter PDFs")
    ap.add_argument("--format", choices=["latex", "markdown", "both"], default="both")
    ap.add_argument("--rederive-remote-board", action="store_true",
                    help="charge remote rows of older run tables (client board 0 J on a shared GPU) at the board's "
                         "recorded idle power x window")
    a = ap.parse_args(argv)
    analyze(a.run_table, a.out, a.plots, a.format, rederive=a.rederive_remote_board)


if __name__ == "__main__":
    main()
