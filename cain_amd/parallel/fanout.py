"""Data-parallel trial fan-out across the GPUs of one node (SURVEY §2.5 row DP, §5.8).

The reference runs its 1,260 trials strictly one after another
(experiment-runner/ExperimentOrchestrator/Experiment/ExperimentController.py:119-137)
with a 90 s cooldown each — 31.5 h of sleep.  Trials are independent, so here
they are sharded over N worker processes, one per GPU:

* every rank builds the same ``RunnerConfig`` (the config file is re-imported in
  each spawned worker — HIP state never crosses a fork);
* rank 0 owns ``run_table.csv`` / ``metadata.json`` (creation, resume, md5 check)
  and ``broadcast_object_list``s the TODO run ids; the shard of rank r is every
  world-th TODO row starting at r, recomputed from the TODO rows on every start,
  so a resume works with a different GPU count;
* BEFORE_EXPERIMENT runs on every rank (per-GPU setup such as starting that
  rank's local server); AFTER_EXPERIMENT — the reference's run-table
  post-processing — on the writer only, then ``config.teardown_rank()`` if defined;
* work is a dynamic queue, not lock-step waves: a rank takes the next TODO row
  with one atomic ``add`` on the process group's key-value store (the c10d
  TCPStore the rendezvous already created), runs it (hooks see
  ``context.rank`` / ``context.device``; the energy plugin measures that
  rank's GPU), publishes the finished row under its queue index and takes the
  next -- a slow run (a 1,000-word on-device trial of a 7B model next to a
  100-word one) no longer holds every other GPU at a wave boundary.  Rank 0
  also runs rows; between its own runs it commits every published row to
  ``run_table.csv`` in one atomic rewrite (single writer).  The
  cooldown is per rank, so it overlaps across GPUs;
* the control messages are a few hundred bytes (the store, plus RCCL over xGMI
  for the broadcast / barrier when the process group is ``nccl``; ``gloo`` on
  CPU), i.e. latency-bound: there is nothing to tune for bandwidth here.

Failure handling: an exception in a run leaves that row TODO (reference
semantics) and is logged to ``errors.jsonl``; ``retry_failed`` re-runs such rows
in extra waves.  A rank that DIES (segfault, OOM kill, GPU fault) is detected by
the launcher, which stops the surviving ranks at once (they would otherwise
block in the next collective until the process-group timeout) and — with
``max_restarts`` — starts a fresh job that resumes the TODO rows (the finished
rows were committed wave by wave, so at most one wave is redone).  Under
``torchrun`` its own ``--max-restarts`` plays that role.
"""
from __future__ import annotations

import datetime
import os
import socket
import traceback
from typing import Any, Dict, List, Optional


_SESSION_T0 = [0.0]  # monotonic start of this rank (run_rank), for CAIN_RUN_BUDGET_S
_SKIPPED = "__skipped__"  # published for a queue index claimed after the writer's budget stop (not run)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _backend() -> str:
    forced = os.environ.get("CAIN_DIST_BACKEND")
    if forced:
        return forced
    try:
        import torch
        return "nccl" if torch.cuda.is_available() and torch.cuda.device_count() > 0 else "gloo"
    except Exception:  # pragma: no cover
        return "gloo"


def run_rank(config_path: str, rank: int, world: int, isolation: Optional[str] = None,
             timeout: Optional[float] = None, assume_yes: Optional[bool] = None, retry_failed: int = 0,
             pg_timeout_s: float = 3600.0) -> int:
    """Body of one worker; the process group must already be initialisable from the environment."""
    import torch
    import torch.distributed as dist

    from ..runner.cli import build_config
    from ..runner.controller import ExperimentController
    from ..runner.events import EventSubscriptionController, RunnerEvents
    from ..runner.models import OperationType, RunProgress
    from ..runner.output import OutputProcedure as output
    from ..runner.store import CSVOutputManager
    from ..runner.validator import ConfigValidator

    import time

    _SESSION_T0[0] = time.monotonic()
    backend = _backend()
    local = int(os.environ.get("LOCAL_RANK", rank))
    device = None
    if backend == "nccl":
        torch.cuda.set_device(local)
        device = f"cuda:{local}"
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=pg_timeout_s),
                                device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=pg_timeout_s))
    output.tag = f"[rank {rank}/{world}]"
    try:
        config, metadata, source = build_config(config_path)
        config.dp_rank, config.dp_world = rank, world
        if device is not None and not hasattr(config, "energy_devices"):
            config.energy_devices = [local]
        ConfigValidator.validate_config(config, quiet=rank != 0)
        writer = rank == 0
        ctrl = None
        if writer:
            ctrl = ExperimentController(config, metadata, source=source, source_name=config_path,
                                        assume_yes=assume_yes, isolation=isolation, run_timeout_s=timeout,
                                        writer=True, rank=rank, device=device)
        dist.barrier()
        if not writer:
            ctrl = ExperimentController(config, metadata, isolation=isolation, run_timeout_s=timeout, writer=False,
                                        rank=rank, device=device)
            # adopt the writer's (possibly resumed, re-ordered) table
            ctrl.run_table = CSVOutputManager(ctrl.path).read_run_table()
        todo_ids = [[v["__run_id"] for v in ctrl.pending()] if writer else None]
        dist.broadcast_object_list(todo_ids, src=0)
        todo_ids = todo_ids[0]
        by_id = {v["__run_id"]: v for v in ctrl.run_table}
        output.console_log_OK(f"{len(todo_ids)} TODO runs over {world} ranks (backend {backend})")
        EventSubscriptionController.raise_event(RunnerEvents.BEFORE_EXPERIMENT)
        passes = 1 + max(0, int(retry_failed))
        store = dist.distributed_c10d._get_default_store()
        hb = _Heartbeat(store, rank)
        for p in range(passes):
            failed = _work_queue(store, f"cain/{p}/", todo_ids, by_id, ctrl, config, writer, world, rank=rank,
                                 deadline_s=pg_timeout_s)
            retry = [failed if writer else None]
            dist.broadcast_object_list(retry, src=0)
            todo_ids = retry[0]
            if not todo_ids or p + 1 >= passes:
                break
            output.console_log_WARNING(f"retrying {len(todo_ids)} failed runs (pass {p + 2}/{passes})")
        hb.close()
        dist.barrier()
        if writer:
            output.console_log_OK("Experiment completed...")
            EventSubscriptionController.raise_event(RunnerEvents.AFTER_EXPERIMENT)
        dist.barrier()
        # per-rank teardown (e.g. the rank's local Ollama-compatible server); AFTER_EXPERIMENT is the
        # reference's post-processing of run_table.csv and runs on the single writer only
        if hasattr(config, "teardown_rank"):
            config.teardown_rank()
        return 0
    except Exception:
        traceback.print_exc()
        return 1
    finally:
        try:
            dist.destroy_process_group()
        except Exception:
            pass


class _Heartbeat:
    """A rank's liveness counter on the job's store (``cain/hb/<rank>``), bumped by a daemon thread: the writer
    tells a rank that died (its counter stops) from one that is merely busy with a long run."""

    def __init__(self, store, rank: int, period_s: float = 2.0):
        import threading

        self.store, self.key, self.period = store, f"cain/hb/{rank}", period_s
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self) -> None:
        fails = 0
        while not self._stop.is_set():
            try:
                self.store.add(self.key, 1)
                fails = 0
            except Exception as exc:  # a transient store error must not make a live rank look dead: retry
                fails += 1
                if fails in (1, 10, 100):
                    from ..runner.output import OutputProcedure as output

                    output.console_log_WARNING(f"heartbeat: store error ({fails}x): {exc}")
            self._stop.wait(self.period)

    def close(self) -> None:
        self._stop.set()


def _work_queue(store, prefix: str, todo_ids: List[str], by_id: Dict[str, Dict[str, Any]], ctrl, config,
                writer: bool, world: int, poll_s: float = 0.2, rank: int = 0, hb_timeout_s: float = 60.0,
                deadline_s: float = 3600.0) -> List[str]:
    """One pass over ``todo_ids`` as a shared queue.  Every rank claims indices with ``store.add`` (recording
    the claim under ``<prefix>claim/<index>``) and publishes each finished row (pickled; None = the run failed)
    under ``<prefix>res/<index>``; the writer commits what is published between its own runs and, after its last
    one, until every index is in.  That final wait is bounded: an index whose claimant's heartbeat
    (``_Heartbeat``) has stopped for ``hb_timeout_s`` is recorded as failed (its row stays TODO for a resume or
    retry), and when nothing at all is published for ``deadline_s`` the writer records every missing index as
    failed, names the claimants and raises (the job exits non-zero).  Returns, on the writer, the run ids that
    failed in this pass."""
    import pickle
    import time

    from ..runner.events import EventSubscriptionController, RunnerEvents
    from ..runner.models import OperationType, RunProgress
    from ..runner.output import OutputProcedure as output
    from ..runner.store import CSVOutputManager

    n = len(todo_ids)
    pending = set(range(n))  # writer: indices not committed yet
    failed: List[str] = []

    def commit_published() -> None:
        keys = [i for i in sorted(pending) if store.check([f"{prefix}res/{i}"])]
        done = []
        for i in keys:
            row = pickle.loads(store.get(f"{prefix}res/{i}"))
            pending.discard(i)
            if row == _SKIPPED:  # claimed after the writer's stop: not run, stays TODO (not a failure)
                continue
            if row is None:
                failed.append(todo_ids[i])
            else:
                row = dict(row)
                row["__done"] = RunProgress.DONE
                done.append(row)
        if done:
            CSVOutputManager(ctrl.path).update_rows(done)
            output.console_log_WARNING(f"CSVManager: committed {len(done)} rows ({n - len(pending)}/{n})")

    ran = 0
    # CAIN_RUN_BUDGET_S > 0: stop claiming runs that long after the rank started (chunked sessions of a long study:
    # the rest stays TODO and the next session resumes it)
    budget = float(os.environ.get("CAIN_RUN_BUDGET_S", "0") or 0)
    # a rank that only hosts a shared server (the study's dedicated remote-server GPU) claims no runs; as the
    # writer it still commits every published row below
    claims = bool(getattr(config, "claims_runs", True))
    while claims:
        if budget > 0 and time.monotonic() - _SESSION_T0[0] > budget:
            output.console_log_WARNING(f"run budget of {budget:.0f} s used: the remaining runs stay TODO (resume)")
            if writer:  # every rank stops claiming too, so the writer's count of claimed runs below is final
                store.set(f"{prefix}stop", "1")
            break
        i = int(store.add(f"{prefix}next", 1)) - 1
        if i >= n:
            break
        store.set(f"{prefix}claim/{i}", str(rank))
        if budget > 0 and store.check([f"{prefix}stop"]):
            # the writer stopped (and may already have counted this index as claimed): hand it back untouched
            store.set(f"{prefix}res/{i}", pickle.dumps(_SKIPPED))
            break
        if ran:
            ctrl.cooldown()  # per rank: overlaps with the other ranks' runs
        rid = todo_ids[i]
        row = ctrl.run_variation(by_id[rid], commit=lambda r: None)
        store.set(f"{prefix}res/{i}", pickle.dumps(row))
        ran += 1
        if writer:
            commit_published()
        if config.operation_type is OperationType.SEMI:
            EventSubscriptionController.raise_event(RunnerEvents.CONTINUE)
    if writer:
        stopped = [False]

        def stop_claims() -> None:
            # indices nobody claimed stay TODO: wait for the claimed ones only.  Set the stop key (also when the
            # queue simply ran out) before counting, so an index claimed after the count is handed back
            store.set(f"{prefix}stop", "1")
            claimed = min(n, int(store.add(f"{prefix}next", 0)))
            pending.difference_update(range(claimed, n))
            stopped[0] = True

        # a claiming writer has stopped claiming by now (queue empty or its budget spent).  A server-only writer
        # (claims_runs False, e.g. remote=local:0) keeps committing while the other ranks claim, and stops the
        # claims only when its own budget runs out
        if budget > 0 and claims:
            stop_claims()
        last_progress = time.monotonic()
        beats: Dict[int, tuple] = {}  # rank -> (last counter value, when it changed, writer clock)

        def claimant(i: int) -> int:
            key = f"{prefix}claim/{i}"
            return int(store.get(key)) if store.check([key]) else -1

        def alive(r: int, now: float) -> bool:
            key = f"cain/hb/{r}"
            v = int(store.add(key, 0)) if r >= 0 else 0
            old = beats.get(r)
            if old is None or old[0] != v:
                beats[r] = (v, now)
                return True
            return now - old[1] < hb_timeout_s

        while pending:
            before = len(pending)
            commit_published()
            now = time.monotonic()
            if len(pending) < before:
                last_progress = now
            if not pending:
                break
            if budget > 0 and not stopped[0] and now - _SESSION_T0[0] > budget:
                output.console_log_WARNING(f"run budget of {budget:.0f} s used: the remaining runs stay TODO (resume)")
                stop_claims()
                if not pending:
                    break
            # an index nobody has claimed yet (claimant -1) is waiting for a client rank, not lost: only a claimed
            # index whose claimant's heartbeat stopped is recorded as failed (the deadline covers the rest)
            dead = [i for i in sorted(pending) if claimant(i) >= 0 and not alive(claimant(i), now)]
            for i in dead:
                output.console_log_FAIL(f"run {todo_ids[i]} (queue index {i}) was claimed by rank {claimant(i)}, "
                                        f"whose heartbeat stopped: left TODO")
                pending.discard(i)
                failed.append(todo_ids[i])
            if pending and now - last_progress > deadline_s:
                lost = sorted(pending)
                for i in lost:
                    failed.append(todo_ids[i])
                pending.clear()
                raise RuntimeError(f"no run published for {deadline_s:.0f} s; unpublished runs (left TODO): "
                                   + ", ".join(f"{todo_ids[i]} (rank {claimant(i)})" for i in lost))
            if pending:
                time.sleep(poll_s)
    output.console_log(f"rank ran {ran} of {n} runs in this pass ({world} ranks)")
    return failed


def _spawn_entry(rank, world, port, config_path, isolation, timeout, assume_yes, retry_failed):
    import signal
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # SIGTERM from the launcher → SystemExit, so atexit handlers (e.g. a config's local servers) still run
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))
    sys.exit(run_rank(config_path, rank, world, isolation, timeout, assume_yes, retry_failed))


def _run_job(ctx, config_path, n_gpus, isolation, timeout, assume_yes, retry_failed, poll_s: float = 0.2) -> int:
    """One job: spawn the ranks, and if any rank dies stop the others instead of letting them wait for
    the process-group timeout.  Returns 0 when every rank exited 0."""
    import time

    port = _free_port()
    procs = [ctx.Process(target=_spawn_entry, args=(r, n_gpus, port, os.path.abspath(config_path), isolation,
                                                    timeout, assume_yes, retry_failed))
             for r in range(n_gpus)]
    for p in procs:
        p.start()
    failed = None
    while any(p.is_alive() for p in procs):
        bad = [r for r, p in enumerate(procs) if p.exitcode not in (None, 0)]
        if bad:
            failed = bad
            break
        time.sleep(poll_s)
    if failed is not None:
        from ..runner.output import OutputProcedure as output

        output.console_log_FAIL(f"rank(s) {failed} died (exit {[procs[r].exitcode for r in failed]}): "
                                f"stopping the surviving ranks")
        for p in procs:
            if p.is_alive():
                p.terminate()
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
                p.join()
    for p in procs:
        p.join()
    return 0 if all(p.exitcode == 0 for p in procs) else 1


def launch(config_path: str, n_gpus: int, isolation: Optional[str] = None, timeout: Optional[float] = None,
           assume_yes: Optional[bool] = None, retry_failed: int = 0, max_restarts: int = 0) -> int:
    """Run ``config_path`` data-parallel on ``n_gpus`` ranks (spawned here, or the current torchrun job).
    ``max_restarts``: after a rank dies, start up to that many fresh jobs; each resumes the TODO rows."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return run_rank(config_path, int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), isolation, timeout,
                        assume_yes, retry_failed)
    import multiprocessing as mp

    from ..runner.output import OutputProcedure as output

    ctx = mp.get_context("spawn")
    rc = 1
    for attempt in range(1 + max(0, int(max_restarts))):
        if attempt:
            output.console_log_WARNING(f"elastic restart {attempt}/{max_restarts}: resuming the TODO rows")
            assume_yes = True  # the same config: the md5 prompt was answered by the first job
        rc = _run_job(ctx, config_path, n_gpus, isolation, timeout, assume_yes, retry_failed)
        if rc == 0:
            break
    return rc
