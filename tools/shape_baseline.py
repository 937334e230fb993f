#!/usr/bin/env python3
"""Same-box regression baseline of the batch-1 GEMMs: a fixed per-shape µs table for A/B runs to check against
(VERDICT r5 weak 5 / item 1 -- round 5's 5-13 % MXFP4 loss went unnoticed because every A/B compared two new
builds with each other and nothing with a fixed reference).

  record:  python3 tools/shape_baseline.py record --out baselines/b1_shapes_mi355x.json
  check:   python3 tools/shape_baseline.py check baselines/b1_shapes_mi355x.json [--tol 0.08]

Both run tools/w4_bench.py (in-graph µs per call, weights rotated past the Infinity Cache: the decode step's cost) on
the seven study models' QKV / O / gate-up / down / LM-head shapes at one row, MXFP4 (the shape rule's kernel) and
GGUF Q4_K.  `check` prints one JSON line per shape with its ratio to the table and exits 1 when any shape is slower
than the table by more than --tol (a second box measured 0.94-1.06 of the table per shape, mean 0.998, so the
default 8 % flags a real loss, not noise: baselines/checks/).
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
from pathlib import Path
from typing import Dict, Iterable, List

ROOT = Path(__file__).resolve().parent.parent
MODELS = ("llama3.1:8b", "qwen2:1.5b", "gemma:2b", "phi3:3.8b", "qwen2:7b", "gemma:7b", "mistral:7b")
ROLES = "qkv,o,gateup,down,lm_head"
DTYPES = "fp4,q4_k"


def key(rec: dict, model: str) -> str:
    return f"{model}/{rec['dtype']}/{rec['role']}"


def measure(models: Iterable[str], dtypes: str = DTYPES, roles: str = ROLES) -> Dict[str, float]:
    """model/dtype/role -> µs per call, from one w4_bench.py process per model."""
    out: Dict[str, float] = {}
    for m in models:
        r = subprocess.run([sys.executable, str(ROOT / "tools" / "w4_bench.py"), "--model", m, "--dtypes", dtypes,
                            "--variants", "rule", "--roles", roles], capture_output=True, text=True, cwd=str(ROOT))
        if r.returncode != 0:
            raise RuntimeError(f"w4_bench.py --model {m} failed:\n{r.stderr[-3000:]}")
        for line in r.stdout.splitlines():
            if line.startswith("{"):
                rec = json.loads(line)
                out[key(rec, m)] = float(rec["us"])
        print(f"[shape_baseline] {m}: {sum(k.startswith(m + '/') for k in out)} shapes", file=sys.stderr, flush=True)
    return out


def compare(table: Dict[str, float], now: Dict[str, float], tol: float) -> List[dict]:
    """One record per shape of the table: its µs then and now, the ratio, and whether it regressed beyond tol."""
    rows = []
    for k, ref in sorted(table.items()):
        if k not in now:
            rows.append(dict(shape=k, ref_us=ref, us=None, ratio=None, regressed=False, missing=True))
            continue
        ratio = now[k] / ref
        rows.append(dict(shape=k, ref_us=ref, us=now[k], ratio=round(ratio, 3), regressed=ratio > 1.0 + tol))
    return rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    rec = sub.add_parser("record")
    rec.add_argument("--out", required=True)
    rec.add_argument("--models", default=",".join(MODELS))
    chk = sub.add_parser("check")
    chk.add_argument("table")
    chk.add_argument("--tol", type=float, default=0.08)
    chk.add_argument("--models", default=None, help="subset of the table's models (default: all)")
    a = ap.parse_args(argv)
    if a.cmd == "record":
        shapes = measure(a.models.split(","))
        import torch

        doc = {"what": "in-graph µs per call, one row, weights rotated past the Infinity Cache (tools/w4_bench.py)",
               "device": torch.cuda.get_device_name(0), "roles": ROLES, "dtypes": DTYPES, "shapes": shapes}
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(doc, indent=1) + "\n")
        print(f"[shape_baseline] {len(shapes)} shapes -> {a.out}", file=sys.stderr)
        return 0
    table = json.loads(Path(a.table).read_text())["shapes"]
    models = a.models.split(",") if a.models else sorted({k.split("/")[0] for k in table})
    table = {k: v for k, v in table.items() if k.split("/")[0] in models}
    rows = compare(table, measure(models), a.tol)
    for r in rows:
        print(json.dumps(r), flush=True)
    bad = [r["shape"] for r in rows if r["regressed"]]
    print(f"[shape_baseline] {len(rows)} shapes, {len(bad)} beyond +{a.tol:.0%}: {bad}", file=sys.stderr)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
