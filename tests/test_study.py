"""The study RunnerConfig end to end on CPU: runner → per-rank Ollama-compatible server (tiny model, torch
backend) + modelled remote server → HTTP client → energy plugin → run_table.csv with the reference's columns
first and the measured-token columns after them."""
import csv
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _env(tmp_path, **kw):
    env = dict(os.environ, PYTHONPATH=str(ROOT), CAIN_ASSUME_YES="1", NO_COLOR="1", CAIN_DIST_BACKEND="gloo",
               CAIN_STUDY_MODELS="tiny-qwen2:1.5b", CAIN_STUDY_LENGTHS="6", CAIN_STUDY_REPETITIONS="2",
               CAIN_STUDY_COOLDOWN_MS="0", CAIN_STUDY_RESULTS_DIR=str(tmp_path), CAIN_STUDY_SEED="5",
               CAIN_STUDY_REMOTE="fake", CAIN_STUDY_REMOTE_FAKE_TOK_S="500", CAIN_STUDY_CLIENT="http",
               CAIN_STUDY_PORT_BASE=str(20000 + os.getpid() % 20000), CAIN_STUDY_IDLE_SETTLE_S="0",
               CAIN_STUDY_IDLE_BASELINE_S="0.5")
    env.update(kw)
    return env


@pytest.mark.parametrize("gpus", [0, 2])
def test_study_config_runs_both_arms(tmp_path, gpus):
    cmd = [sys.executable, "-m", "cain_amd", str(ROOT / "experiments" / "study.py")]
    if gpus:
        cmd += ["--gpus", str(gpus)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=_env(tmp_path, CAIN_STUDY_PORT_BASE=str(21000 + gpus * 500 + os.getpid() % 400),
                                CAIN_STUDY_WINDOW="reference" if gpus else "request"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = list(csv.DictReader(open(tmp_path / "full_factorial" / "run_table.csv")))
    assert len(rows) == 4 and all(x["__done"] == "DONE" for x in rows)
    cols = list(rows[0].keys())
    assert cols[:11] == ["__run_id", "__done", "model", "method", "length", "topic", "execution_time", "cpu_usage",
                         "gpu_usage", "memory_usage", "codecarbon__energy_consumed"]
    assert cols[11] == "energy_usage_J" and "J_per_token" in cols and cols.index("J_per_token") > 11
    for x in rows:
        assert int(x["tokens_generated"]) == 8  # "In 6 words" -> ceil(6 * 4/3) tokens
        assert float(x["execution_time"]) > 0 and float(x["tok_per_s"]) > 0
        assert x["topic"] and x["server"].startswith("http://127.0.0.1:")
    methods = sorted(x["method"] for x in rows)
    assert methods == ["on_device", "on_device", "remote", "remote"]
    if gpus:
        assert "rank 1/2" in r.stdout
    run_dirs = [d for d in (tmp_path / "full_factorial").iterdir() if d.is_dir() and d.name.startswith("run_")]
    assert len(run_dirs) == 4
    assert all((d / "response.json").exists() for d in run_dirs)
    assert any((d / "cpu_mem_usage.csv").exists() for d in run_dirs)
    # the writer post-processed the table into the paper's tables
    assert (tmp_path / "full_factorial" / "analysis" / "results.json").exists()


def test_study_eight_ranks_share_one_remote_server(tmp_path):
    """The real StudyConfig at 8 data-parallel ranks (gloo, modelled servers): ONE remote server for the node
    (rank 0 starts it and publishes its URL on the job's store; the reference has one server every trial talks
    to), each rank's energy sampler on a core of its own, and a single writer of run_table.csv."""
    import json

    from cain_amd.energy.meter import sampler_core

    base = 23000 + os.getpid() % 1000
    r = subprocess.run([sys.executable, "-m", "cain_amd", str(ROOT / "experiments" / "study.py"), "--gpus", "8"],
                       capture_output=True, text=True, timeout=900, cwd=ROOT,
                       env=_env(tmp_path, CAIN_STUDY_PORT_BASE=str(base), CAIN_STUDY_REPETITIONS="8",
                                CAIN_STUDY_DEVICE_BACKEND="fake", CAIN_STUDY_REMOTE="local:cpu",
                                CAIN_STUDY_REMOTE_BACKEND="fake", CAIN_STUDY_REMOTE_FAKE_TOK_S="2000",
                                CAIN_STUDY_REMOTE_FAKE_PREFILL_S="0", CAIN_STUDY_IDLE_BASELINE_S="0"))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    out = tmp_path / "full_factorial"
    rows = list(csv.DictReader(open(out / "run_table.csv")))
    assert len(rows) == 16 and all(x["__done"] == "DONE" for x in rows)
    remote = [x for x in rows if x["method"] == "remote"]
    assert len({x["server"] for x in remote}) == 1, {x["server"] for x in remote}
    logs = sorted(p.name for p in (out / "servers").iterdir())
    assert "remote_node.log" in logs and not any(n.startswith("remote_rank") for n in logs), logs
    assert sum(n.startswith("on_device_rank") for n in logs) == 8
    # single writer: only rank 0 commits rows
    commits = [ln for ln in r.stdout.splitlines() if "committed" in ln]
    assert commits and all("rank 0/8" in ln for ln in commits), commits[:5]
    # distinct sampler cores: on-device rows name their rank's server port (port_base + 1 + rank)
    cores = {}
    for x in rows:
        if x["method"] != "on_device":
            continue
        rank = int(x["server"].rsplit(":", 1)[1]) - base - 1
        core = json.load(open(out / x["__run_id"] / "energy.json"))["sampler_core"]
        assert core == sampler_core(rank), (rank, core)
        cores.setdefault(rank, set()).add(core)
    assert len(cores) >= 2
    if len(os.sched_getaffinity(0)) >= 8:
        flat = [next(iter(c)) for c in cores.values()]
        assert len(set(flat)) == len(flat), cores


def test_study_dedicated_remote_server_gpu_at_eight_ranks(tmp_path):
    """``remote=local:3`` in an 8-rank job: GPU 3 is a client GPU, so its rank hosts the node's remote server and
    claims no runs (8 ranks -> 7 clients): no on-device window is ever measured on the server's board, and the
    rank starts no on-device server of its own.  Client CPU energy is process-attributed (the default)."""
    base = 25000 + os.getpid() % 1000
    r = subprocess.run([sys.executable, "-m", "cain_amd", str(ROOT / "experiments" / "study.py"), "--gpus", "8"],
                       capture_output=True, text=True, timeout=900, cwd=ROOT,
                       env=_env(tmp_path, CAIN_STUDY_PORT_BASE=str(base), CAIN_STUDY_REPETITIONS="8",
                                CAIN_STUDY_DEVICE_BACKEND="fake", CAIN_STUDY_REMOTE="local:3",
                                CAIN_STUDY_REMOTE_BACKEND="fake", CAIN_STUDY_REMOTE_FAKE_TOK_S="2000",
                                CAIN_STUDY_REMOTE_FAKE_PREFILL_S="0", CAIN_STUDY_IDLE_BASELINE_S="0"))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    out = tmp_path / "full_factorial"
    rows = list(csv.DictReader(open(out / "run_table.csv")))
    assert len(rows) == 16 and all(x["__done"] == "DONE" for x in rows)
    ranks = {int(x["dp_rank"]) for x in rows}
    assert 3 not in ranks and ranks <= set(range(8)) - {3}, ranks
    # no on-device row was served by a server on GPU 3 (rank r's on-device server listens on port_base + 1 + r)
    assert all(int(x["server"].rsplit(":", 1)[1]) != base + 1 + 3 for x in rows if x["method"] == "on_device")
    remote = [x for x in rows if x["method"] == "remote"]
    assert len({x["server"] for x in remote}) == 1 and remote[0]["server"].endswith(f":{base + 101}")
    logs = sorted(p.name for p in (out / "servers").iterdir())
    assert "remote_node.log" in logs and "on_device_rank3.log" not in logs, logs
    assert sum(n.startswith("on_device_rank") for n in logs) == 7
    assert "rank 3 hosts the node's remote server" in r.stdout
    assert all(x["cpu_energy_source"].startswith("process(") for x in rows), {x["cpu_energy_source"] for x in rows}


@pytest.mark.gpu
def test_study_on_device_arm_on_gpu_measures_energy(tmp_path):
    """On the GPU box: the per-rank server runs the HIP engine, the window reads the amd-smi accumulator."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    r = subprocess.run([sys.executable, "-m", "cain_amd", str(ROOT / "experiments" / "study.py")],
                       capture_output=True, text=True, timeout=900, cwd=ROOT,
                       env=_env(tmp_path, CAIN_STUDY_MODELS="gemma:2b", CAIN_STUDY_LENGTHS="100",
                                CAIN_STUDY_REPETITIONS="2", CAIN_STUDY_METHODS="on_device", CAIN_STUDY_CLIENT="curl"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = list(csv.DictReader(open(tmp_path / "full_factorial" / "run_table.csv")))
    assert len(rows) == 2
    for x in rows:
        assert int(x["tokens_generated"]) == 134
        assert float(x["gpu_energy_J"]) > 0 and float(x["avg_gpu_power_W"]) > 50
        assert float(x["J_per_token"]) > 0 and x["idle_subtracted_J"] != ""


@pytest.mark.gpu
def test_study_both_arms_against_real_engine_servers(tmp_path):
    """Both arms through curl against this framework's own engine: the on-device server and a remote server
    (``CAIN_STUDY_REMOTE=local:0``: a separate engine process on the box's GPU).  The remote rows decode at the
    engine's rate (not the 70 tok/s modelled server).  One client-device definition (round 5): the board the remote
    server shares is charged to the client at the session's measured idle power x the window (idle_model), the
    on-device rows' board is measured."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    r = subprocess.run([sys.executable, "-m", "cain_amd", str(ROOT / "experiments" / "study.py")],
                       capture_output=True, text=True, timeout=900, cwd=ROOT,
                       env=_env(tmp_path, CAIN_STUDY_MODELS="qwen2:1.5b", CAIN_STUDY_LENGTHS="100",
                                CAIN_STUDY_REPETITIONS="2", CAIN_STUDY_METHODS="on_device,remote",
                                CAIN_STUDY_REMOTE="local:0", CAIN_STUDY_CLIENT="curl"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = list(csv.DictReader(open(tmp_path / "full_factorial" / "run_table.csv")))
    assert len(rows) == 4 and all(x["__done"] == "DONE" for x in rows)
    for x in rows:
        assert int(x["tokens_generated"]) == 134
        # the client's process-attributed CPU energy (its CPU seconds, 10-ms ticks) can round to 0 on a short
        # request; RAM energy keeps every row's total positive
        assert float(x["cpu_energy_J"]) >= 0 and float(x["energy_usage_J"]) > 0
    remote = [x for x in rows if x["method"] == "remote"]
    local = [x for x in rows if x["method"] == "on_device"]
    assert all(float(x["tok_per_s"]) > 150 for x in remote), [x["tok_per_s"] for x in remote]
    for x in remote:
        assert x["gpu_energy_source"] == "idle_model"
        assert float(x["gpu_energy_J"]) == pytest.approx(float(x["idle_power_W"]) * float(x["energy_window_s"]),
                                                         rel=2e-2, abs=0.05)
        assert float(x["gpu_energy_J"]) > 0
    assert all(float(x["gpu_energy_J"]) > 0 and x["gpu_energy_source"] == "measured" for x in local)
    # gpu_usage keeps the reference meaning (the client's own GPU residency: none, the client never opens the
    # GPU); the shared board's activity is the server's and goes to server_gpu_usage
    assert all(float(x["gpu_usage"]) == 0.0 and float(x["server_gpu_usage"]) > 0 for x in remote)
    assert all(x["server_gpu_usage"] == "" for x in local)
    assert all(x["server"] != local[0]["server"] for x in remote)


class _IdleBoardSampler:
    """Stand-in for the native sampler of one GPU whose board idles at ``watts`` (a client GPU of a data-parallel
    job while its remote request runs on the dedicated server GPU)."""

    n, thread_id, host_energy_source = 1, 0, ""

    def __init__(self, watts):
        self.watts = watts

    def energy_between(self, i, t0, t1):
        return self.watts * (t1 - t0) * 1e-9

    def drain(self):
        return []

    def trim(self, t):
        pass

    def trace_points(self, i):
        return 0

    def close(self):
        pass


def test_remote_row_energy_has_one_definition_at_every_world_size(monkeypatch):
    """a remote-arm row means the same thing at world 1 (the remote server shares the client's
    GPU) and at world 8 (a dedicated server GPU): client board + client CPU + RAM, the board at idle.  At world 1 the
    board is charged at its measured idle power (``gpu_idle``; it runs the server's decode), at world 8 it is
    measured while it idles -- the same columns, the same composition, the same idle subtraction."""
    import time

    from cain_amd.energy.meter import EnergyMeter
    from cain_amd.experiments.study import StudyConfig
    from cain_amd.runner.models import RunnerContext

    monkeypatch.setenv("CAIN_STUDY_REMOTE", "local:0")
    cfg = StudyConfig()
    ctx = RunnerContext({"__run_id": "r", "method": "remote", "model": "m", "length": "100"}, 0, Path("/tmp"))
    ondev = RunnerContext({"__run_id": "o", "method": "on_device", "model": "m", "length": "100"}, 0, Path("/tmp"))
    idle_w, cpu_idle = 260.0, 0.05
    readings = {}
    for world, shared in ((1, True), (8, False)):
        cfg.remote_shares_gpu = shared
        cfg.dp_world = world
        srcs = cfg.energy_sources_for(ctx)
        assert cfg.energy_sources_for(ondev) == ("gpu", "cpu", "ram")
        cfg.idle_power_w = None
        assert cfg.gpu_energy_source(ctx) == ("none(no idle baseline)" if shared else "measured")
        cfg.idle_power_w = idle_w
        assert cfg.gpu_energy_source(ctx) == ("idle_model" if shared else "measured")
        m = EnergyMeter(smi_indices=[], period_ms=10, cpu_tdp_w=100.0, sources=srcs, cpu_attribution="process")
        m.sampler.close()
        m.sampler = _IdleBoardSampler(idle_w)
        m.idle_power_w, m.idle_cpu_power_w = idle_w, cpu_idle
        m.start()
        time.sleep(0.2)
        readings[world] = m.stop(settle_ms=0)
    for r in readings.values():
        # the client's board is charged at idle in both topologies, never 0 and never the server's decode power
        assert r.gpu_energy_j == pytest.approx(idle_w * r.duration_s, rel=1e-6)
        assert r.total_energy_j == pytest.approx(r.gpu_energy_j + r.cpu_energy_j + r.ram_energy_j)
        # idle-subtracted: the board's part is ~0 in both, so what is left is the client's own work
        assert r.idle_subtracted_j == pytest.approx(r.cpu_energy_j - cpu_idle * r.duration_s + r.ram_energy_j,
                                                    abs=1e-6)
    w1, w8 = readings[1], readings[8]
    assert w1.gpu_power_w == pytest.approx(w8.gpu_power_w, rel=1e-6)
