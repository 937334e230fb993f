"""bench.py's multi-rank contract on CPU (gloo, torch oracle backend): ``--gpus N`` without a launcher spawns N
ranks and reports the whole-job value with ``n_gpus: N``; under a launcher ``--gpus`` must match WORLD_SIZE."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
ARGS = ["--device", "cpu", "--model", "tiny-llama3.1:8b", "--words", "3", "--batch", "2", "--context", "64",
        "--steps", "1", "--warmup", "0", "--no-energy", "--no-single"]


def _run(extra, env=None, timeout=240):
    e = dict(os.environ, OMP_NUM_THREADS="1")
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + extra + ARGS, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=str(ROOT))


def _line(out):
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_bench_spawns_n_ranks(n):
    r = _run(["--gpus", str(n)])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == n and d["config"]["parallelism"] == f"dp{n}"
    assert d["config"]["global_batch"] == 2 * n
    assert d["tokens_generated"] == 2 * n * d["config"]["seq_len"]
    assert d["scaling"] == "weak" and d["value"] > 0


def test_bench_rejects_mismatched_launcher():
    r = _run(["--gpus", "2"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_bench_on_a_checkpoint(tmp_path):
    """--checkpoint: the bench model's engine loads a Hugging Face checkpoint (here a tiny one written by
    transformers) instead of random-init weights, and the JSON line says so."""
    pytest.importorskip("transformers")
    sys.path.insert(0, str(ROOT / "tests"))
    from hf_fixtures import make_checkpoint

    make_checkpoint("llama", tmp_path / "ck")
    r = _run(["--checkpoint", str(tmp_path / "ck")])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert "checkpoint weights (ck)" in d["data"] and d["tokens_generated"] == 2 * d["config"]["seq_len"]
