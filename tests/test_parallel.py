"""Data-parallel fan-out on CPU ranks (gloo): shard, gather to the single writer, failure, resume with
a different world size."""
import csv
import os
import subprocess
import sys
import textwrap

import pytest
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

CFG = textwrap.dedent('''
    import os
    from pathlib import Path
    from EventManager.Models.RunnerEvents import RunnerEvents
    from EventManager.EventSubscriptionController import EventSubscriptionController
    from ConfigValidator.Config.Models.RunTableModel import RunTableModel
    from ConfigValidator.Config.Models.FactorModel import FactorModel
    from ConfigValidator.Config.Models.OperationType import OperationType

    OUT = Path(os.environ["CAIN_TEST_OUT"])

    class RunnerConfig:
        name = "dp"
        results_output_path = OUT
        operation_type = OperationType.AUTO
        time_between_runs_in_ms = 0

        def __init__(self):
            EventSubscriptionController.subscribe_to_multiple_events([
                (RunnerEvents.START_RUN, self.start_run),
                (RunnerEvents.POPULATE_RUN_DATA, self.populate),
                (RunnerEvents.AFTER_EXPERIMENT, self.after)])

        def create_run_table_model(self):
            self.run_table_model = RunTableModel([FactorModel("model", ["a", "b", "c"]),
                                                  FactorModel("length", ["100", "500"])],
                                                 repetitions=2, data_columns=["rank", "pid"], shuffle=True, seed=7)
            return self.run_table_model

        def start_run(self, ctx):
            flag = OUT / "failed_once"
            if ctx.run_variation["__run_id"] == "run_3_repetition_1" and not flag.exists():
                flag.touch()
                raise RuntimeError("injected")

        def populate(self, ctx):
            return {"rank": ctx.rank, "pid": os.getpid()}

        def after(self):
            (OUT / "after_ran").write_text(str(self.dp_rank))

        experiment_path = None
''')


def _run(cfg, gpus, out):
    env = dict(os.environ, PYTHONPATH=str(ROOT), CAIN_TEST_OUT=str(out), CAIN_DIST_BACKEND="gloo",
               CAIN_ASSUME_YES="1", NO_COLOR="1")
    return subprocess.run([sys.executable, "-m", "cain_amd", str(cfg), "--gpus", str(gpus)], capture_output=True,
                          text=True, env=env, timeout=240)


def test_fanout_two_ranks_then_resume_on_one(tmp_path):
    cfg = tmp_path / "cfg.py"
    cfg.write_text(CFG)
    r = _run(cfg, 2, tmp_path)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = list(csv.DictReader(open(tmp_path / "dp" / "run_table.csv")))
    assert len(rows) == 12
    done = [x for x in rows if x["__done"] == "DONE"]
    assert len(done) == 11 and {x["rank"] for x in done} == {"0", "1"}
    assert [x["__run_id"] for x in rows if x["__done"] == "TODO"] == ["run_3_repetition_1"]
    assert (tmp_path / "after_ran").read_text() == "0"  # AFTER_EXPERIMENT on the writer only
    r = _run(cfg, 1, tmp_path)
    assert r.returncode == 0, r.stdout[-2000:]
    rows2 = list(csv.DictReader(open(tmp_path / "dp" / "run_table.csv")))
    assert all(x["__done"] == "DONE" for x in rows2)
    assert [x["__run_id"] for x in rows2] == [x["__run_id"] for x in rows]  # order preserved
    assert r.stdout.count("NEW RUN") == 1


CRASH_CFG = CFG.replace("(RunnerEvents.START_RUN, self.start_run),",
                        "(RunnerEvents.BEFORE_RUN, self.before_run), (RunnerEvents.START_RUN, self.start_run),"
                        ).replace('''    def start_run(self, ctx):''', '''    def before_run(self):
        # BEFORE_RUN runs in the rank process itself (not the per-run child): this kills the worker
        crash = OUT / "crashed_once"
        if self.dp_rank == 1 and not crash.exists():
            crash.touch()
            os._exit(9)

    def start_run(self, ctx):''')
assert CRASH_CFG != CFG


def test_dead_rank_is_detected_and_job_restarts(tmp_path):
    cfg = tmp_path / "cfg.py"
    cfg.write_text(CRASH_CFG)
    env = dict(os.environ, PYTHONPATH=str(ROOT), CAIN_TEST_OUT=str(tmp_path), CAIN_DIST_BACKEND="gloo",
               CAIN_ASSUME_YES="1", NO_COLOR="1")
    r = subprocess.run([sys.executable, "-m", "cain_amd", str(cfg), "--gpus", "2", "--max-restarts", "1",
                        "--retry-failed", "1"], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "died" in r.stdout and "elastic restart 1/1" in r.stdout
    rows = list(csv.DictReader(open(tmp_path / "dp" / "run_table.csv")))
    assert len(rows) == 12 and all(x["__done"] == "DONE" for x in rows)


QUEUE_CFG = CFG.replace('repetitions=2, data_columns=["rank", "pid"], shuffle=True, seed=7)',
                        'repetitions=4, data_columns=["rank", "pid"], shuffle=True, seed=7)')
assert QUEUE_CFG != CFG


def test_fanout_eight_ranks_work_queue_then_resume_on_three(tmp_path):
    """8 gloo ranks pull rows from the shared queue (24 runs); the injected failure stays TODO; a resume on 3
    ranks runs exactly that row (1/2/4/8 ranks, resume across world sizes)."""
    cfg = tmp_path / "cfg.py"
    cfg.write_text(QUEUE_CFG)
    r = _run(cfg, 8, tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = list(csv.DictReader(open(tmp_path / "dp" / "run_table.csv")))
    assert len(rows) == 24
    done = [x for x in rows if x["__done"] == "DONE"]
    assert len(done) == 23 and len({x["rank"] for x in done}) >= 4  # the queue spread the work
    assert (tmp_path / "after_ran").read_text() == "0"
    r = _run(cfg, 3, tmp_path)
    assert r.returncode == 0, r.stdout[-3000:]
    rows2 = list(csv.DictReader(open(tmp_path / "dp" / "run_table.csv")))
    assert all(x["__done"] == "DONE" for x in rows2)
    assert [x["__run_id"] for x in rows2] == [x["__run_id"] for x in rows]
    assert r.stdout.count("NEW RUN") == 1


def test_fanout_four_ranks(tmp_path):
    cfg = tmp_path / "cfg.py"
    cfg.write_text(CFG)
    r = _run(cfg, 4, tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = list(csv.DictReader(open(tmp_path / "dp" / "run_table.csv")))
    assert sum(x["__done"] == "DONE" for x in rows) == 11
    assert "12 TODO runs over 4 ranks" in r.stdout


@pytest.mark.gpu
def test_fanout_one_rank_over_rccl(tmp_path):
    """The same fan-out with the backend the GPU node picks by itself (nccl = RCCL on ROCm): process-group
    start-up bound to cuda:0, object broadcasts and the store work queue on a real MI355X (world 1 -- one card
    per box here; the 8-GPU node runs are the driver's)."""
    import torch
    if not torch.cuda.is_available():  # pragma: no cover
        pytest.skip("needs a GPU")
    cfg = tmp_path / "cfg.py"
    cfg.write_text(CFG)
    env = dict(os.environ, PYTHONPATH=str(ROOT), CAIN_TEST_OUT=str(tmp_path), CAIN_ASSUME_YES="1", NO_COLOR="1")
    env.pop("CAIN_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, "-m", "cain_amd", str(cfg), "--gpus", "1"], capture_output=True,
                       text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "backend nccl" in r.stdout, r.stdout[-2000:]
    rows = list(csv.DictReader(open(tmp_path / "dp" / "run_table.csv")))
    assert sum(x["__done"] == "DONE" for x in rows) == 11 and {x["rank"].strip() for x in rows if x["rank"].strip()} == {"0"}


class _DictStore:
    """In-process stand-in for the c10d store (add / set / get / check)."""

    def __init__(self):
        self.d = {}

    def add(self, k, v):
        self.d[k] = int(self.d.get(k, 0)) + int(v)
        return self.d[k]

    def set(self, k, v):
        self.d[k] = v.encode() if isinstance(v, str) else v

    def get(self, k):
        v = self.d[k]
        return v if isinstance(v, bytes) else str(v).encode()

    def check(self, keys):
        return all(k in self.d for k in keys)


def _writer_pass(monkeypatch, store, todo, claims_runs=True, **kw):
    from cain_amd.parallel import fanout
    from cain_amd.runner import store as store_mod
    from cain_amd.runner.models import OperationType

    committed = []

    class _CSV:
        def __init__(self, path):
            pass

        def update_rows(self, rows):
            committed.extend(r["__run_id"] for r in rows)

    monkeypatch.setattr(store_mod, "CSVOutputManager", _CSV)

    class _Ctrl:
        path = None

        def cooldown(self):
            pass

        def run_variation(self, v, commit):
            return dict(v)

    class _Cfg:
        operation_type = OperationType.AUTO

    _Cfg.claims_runs = claims_runs

    by_id = {t: {"__run_id": t} for t in todo}
    return fanout._work_queue(store, "cain/0/", todo, by_id, _Ctrl(), _Cfg(), True, 2, poll_s=0.01, **kw), committed


def test_writer_does_not_wait_forever_for_a_dead_claimant(monkeypatch):
    """a rank that claims a queue index and dies without publishing it no longer makes the writer spin
    forever -- once the claimant's heartbeat stops, the index is recorded as failed (row left TODO)."""
    store = _DictStore()
    store.add("cain/0/next", 1)      # rank 1 claimed index 0 ...
    store.set("cain/0/claim/0", "1")
    store.add("cain/hb/1", 1)        # ... and its heartbeat never moves again
    failed, committed = _writer_pass(monkeypatch, store, ["a", "b"], rank=0, hb_timeout_s=0.3, deadline_s=30)
    assert failed == ["a"] and committed == ["b"]


def test_writer_deadline_raises_and_names_the_claimant(monkeypatch):
    """With the claimant alive but nothing published for the deadline, the writer records the missing runs and
    raises, so the job exits non-zero instead of hanging."""
    import threading

    store = _DictStore()
    store.add("cain/0/next", 1)
    store.set("cain/0/claim/0", "1")
    stop = threading.Event()

    def beat():
        while not stop.is_set():
            store.add("cain/hb/1", 1)
            stop.wait(0.02)

    t = threading.Thread(target=beat, daemon=True)
    t.start()
    try:
        with pytest.raises(RuntimeError, match=r"a \(rank 1\)"):
            _writer_pass(monkeypatch, store, ["a", "b"], rank=0, hb_timeout_s=30, deadline_s=0.3)
    finally:
        stop.set()


def test_run_budget_leaves_unclaimed_runs_todo(monkeypatch):
    """CAIN_RUN_BUDGET_S: once the session's budget is used, ranks stop claiming and the writer waits only for
    the runs that were claimed -- the rest stay TODO for the next (resumed) session."""
    import time

    from cain_amd.parallel import fanout

    monkeypatch.setenv("CAIN_RUN_BUDGET_S", "5")
    store = _DictStore()
    monkeypatch.setattr(fanout, "_SESSION_T0", [time.monotonic()])
    failed, committed = _writer_pass(monkeypatch, store, ["a", "b", "c"], rank=0, hb_timeout_s=30, deadline_s=30)
    assert failed == [] and committed == ["a", "b", "c"]  # within the budget: everything runs
    store = _DictStore()
    monkeypatch.setattr(fanout, "_SESSION_T0", [time.monotonic() - 10])
    t0 = time.monotonic()
    failed, committed = _writer_pass(monkeypatch, store, ["a", "b", "c"], rank=0, hb_timeout_s=30, deadline_s=30)
    assert failed == [] and committed == [] and time.monotonic() - t0 < 5


def test_budget_stop_hands_back_a_late_claim(monkeypatch):
    """another rank that claims an index after the writer's budget stop publishes it back untouched
    (the writer may already have counted it as claimed): the writer neither waits for it nor records a failure,
    and the row stays TODO for the next session."""
    import pickle
    import time

    from cain_amd.parallel import fanout

    monkeypatch.setenv("CAIN_RUN_BUDGET_S", "5")
    store = _DictStore()
    store.add("cain/0/next", 1)  # rank 1 claimed index 0 before the stop ...
    store.set("cain/0/claim/0", "1")
    store.set("cain/0/res/0", pickle.dumps(fanout._SKIPPED))  # ... saw the stop key and handed it back
    monkeypatch.setattr(fanout, "_SESSION_T0", [time.monotonic() - 10])  # the writer's budget is spent
    failed, committed = _writer_pass(monkeypatch, store, ["a", "b"], rank=0, hb_timeout_s=30, deadline_s=5)
    assert failed == [] and committed == [] and store.check(["cain/0/stop"])


def _client(store, todo, rank=1, delay_s=0.02, stop=None):
    """A client rank's claim loop on the in-process store (claim, run for ``delay_s``, publish), with its heartbeat."""
    import pickle
    import threading
    import time

    from cain_amd.parallel import fanout

    def body():
        while stop is None or not stop.is_set():
            store.add(f"cain/hb/{rank}", 1)
            i = int(store.add("cain/0/next", 1)) - 1
            if i >= len(todo):
                return
            store.set(f"cain/0/claim/{i}", str(rank))
            if store.check(["cain/0/stop"]):
                store.set(f"cain/0/res/{i}", pickle.dumps(fanout._SKIPPED))
                return
            time.sleep(delay_s)
            store.set(f"cain/0/res/{i}", pickle.dumps({"__run_id": todo[i]}))

    t = threading.Thread(target=body, daemon=True)
    t.start()
    return t


def test_server_only_writer_commits_every_client_run(monkeypatch):
    """the writer (rank 0) hosting only the remote server (claims_runs False, remote=local:0) must not
    treat not-yet-claimed indices as runs of a dead rank: it commits every row the client ranks publish."""
    import time

    from cain_amd.parallel import fanout

    monkeypatch.delenv("CAIN_RUN_BUDGET_S", raising=False)
    monkeypatch.setattr(fanout, "_SESSION_T0", [time.monotonic()])
    store = _DictStore()
    todo = [f"run_{i}" for i in range(12)]
    t = _client(store, todo, delay_s=0.05)
    failed, committed = _writer_pass(monkeypatch, store, todo, claims_runs=False, rank=0, hb_timeout_s=0.1,
                                     deadline_s=30)
    t.join(5)
    assert failed == [] and sorted(committed) == sorted(todo)


def test_server_only_writer_budget_stops_claims_when_spent(monkeypatch):
    """With CAIN_RUN_BUDGET_S, a server-only writer keeps committing until its own budget runs out, then stops the
    claims: the client's runs before the stop are committed, the rest stay TODO (no failures)."""
    import time

    from cain_amd.parallel import fanout

    monkeypatch.setenv("CAIN_RUN_BUDGET_S", "0.5")
    monkeypatch.setattr(fanout, "_SESSION_T0", [time.monotonic()])
    store = _DictStore()
    todo = [f"run_{i}" for i in range(200)]
    t = _client(store, todo, delay_s=0.05)
    failed, committed = _writer_pass(monkeypatch, store, todo, claims_runs=False, rank=0, hb_timeout_s=30,
                                     deadline_s=30)
    t.join(5)
    assert failed == [] and 3 <= len(committed) < len(todo)
    assert committed == todo[:len(committed)] and store.check(["cain/0/stop"])
