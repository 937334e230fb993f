#!/usr/bin/env python3
"""Parameterised bench sweep: one bench.py run per point of a grid of arguments and environment settings, one
JSON line per run (the bench's own line plus the point) -- replaces round 1's one-off sweep scripts.

    python tools/sweep.py --out gpurun_out/sweep.jsonl \\
        --arg model=llama3.1:8b,gemma:2b --arg words=100,500,1000 --arg batch=256 \\
        --env CAIN_W8A8=0,1 --fixed "--steps 1 --warmup 1 --no-single"

Each run has its own time limit; a run that crashes or times out (exit >= 124, 134, 139) ends the sweep, a run
that merely fails (exit 1) is recorded and the sweep goes on.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import shlex
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _axis(spec: str):
    key, _, vals = spec.partition("=")
    return key, [v for v in vals.split(",") if v != ""]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--arg", action="append", default=[], help="bench.py option axis: name=v1,v2,...")
    ap.add_argument("--env", action="append", default=[], help="environment axis: NAME=v1,v2,...")
    ap.add_argument("--fixed", default="--steps 1 --warmup 1", help="bench.py options common to every run")
    ap.add_argument("--timeout", type=int, default=400)
    ap.add_argument("--script", default=str(ROOT / "bench.py"))
    ns = ap.parse_args()
    axes = [("arg", *_axis(a)) for a in ns.arg] + [("env", *_axis(e)) for e in ns.env]
    out = Path(ns.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    points = list(itertools.product(*[v for _, _, v in axes])) if axes else [()]
    for vals in points:
        point = {k: v for (_, k, _), v in zip(axes, vals)}
        cmd = [sys.executable, ns.script] + shlex.split(ns.fixed)
        env = dict(os.environ)
        for (kind, k, _), v in zip(axes, vals):
            if kind == "arg":
                cmd += [f"--{k}", v]
            else:
                env[k] = v
        t0 = time.time()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=ns.timeout, cwd=str(ROOT))
            rc, stdout, stderr = r.returncode, r.stdout, r.stderr
        except subprocess.TimeoutExpired as exc:
            rc, stdout, stderr = 124, exc.stdout or "", exc.stderr or ""
            stdout = stdout.decode() if isinstance(stdout, bytes) else stdout
            stderr = stderr.decode() if isinstance(stderr, bytes) else stderr
        lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
        rec = {"point": point, "rc": rc, "wall_s": round(time.time() - t0, 1)}
        if lines:
            rec["result"] = json.loads(lines[-1])
        else:
            rec["stderr_tail"] = stderr[-1500:]
        with open(out, "a") as fh:
            fh.write(json.dumps(rec) + "\n")
        res = rec.get("result", {})
        print(f"[sweep] {point} rc={rc} value={res.get('value')} J/tok={res.get('J_per_token')}", flush=True)
        if rc >= 124 or rc in (134, 139) or rc < 0:
            print("[sweep] stopping after a crash / time limit", flush=True)
            return rc if rc > 0 else 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
