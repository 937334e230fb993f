"""Experiment and run controllers.

Reference call stacks:
* ``ExperimentController.__init__`` — experiment-runner/ExperimentOrchestrator/
  Experiment/ExperimentController.py:33-108 (run-table generation, fresh start
  vs resume);
* ``ExperimentController.do_experiment`` — :110-146 (BEFORE_EXPERIMENT, per
  variation BEFORE_RUN → isolated run → cooldown → CONTINUE (SEMI),
  AFTER_EXPERIMENT);
* ``RunController.do_run`` — Experiment/Run/RunController.py:9-44 (START_RUN →
  START_MEASUREMENT → INTERACT → STOP_MEASUREMENT → STOP_RUN →
  POPULATE_RUN_DATA, shallow-merge, ``__done = DONE``, row rewrite).

Design changes (all SURVEY-motivated):
* the run body returns the finished row and the *controller* commits it, so
  there is exactly one CSV writer — the same path the
  data-parallel rank-0 writer uses (``cain_amd.parallel``);
* a failed or timed-out run leaves its row ``TODO`` (reference semantics) and
  appends a JSON line to ``<experiment>/errors.jsonl`` instead of only a
  traceback on stdout;
* one isolation level instead of two forks, with a timeout (``isolation.py``);
* ``pending()`` / ``run_variation()`` are public so the fan-out can drive a
  shard of rows through the same code.
"""
from __future__ import annotations

import json
import os
import time
import traceback
from pathlib import Path
from typing import Any, Callable, Dict, List, Optional

from .errors import AllRunsCompletedOnRestartError, BaseError, RunTimeoutError
from .events import EventSubscriptionController, RunnerEvents
from .fingerprint import matches as fingerprint_matches
from .isolation import call_isolated
from .models import Metadata, OperationType, RunnerContext, RunProgress
from .output import OutputProcedure as output
from .store import CSVOutputManager, JSONOutputManager


def _cooldown_ms(config) -> int:
    env = os.environ.get("CAIN_COOLDOWN_MS")
    if env is not None:
        return int(env)
    return int(getattr(config, "time_between_runs_in_ms", 0) or 0)


class RunController:
    """Executes the per-run hook sequence for one variation."""

    def __init__(self, variation: Dict[str, Any], config: Any, current_run: int, total_runs: int,
                 rank: int = 0, device: Optional[str] = None):
        self.variation = variation
        self.config = config
        self.current_run = current_run
        self.run_dir = Path(config.experiment_path) / str(variation["__run_id"])
        self.run_dir.mkdir(parents=True, exist_ok=True)
        self.run_context = RunnerContext(self.variation, current_run, self.run_dir, rank=rank, device=device)
        print(f"\n-----------------NEW RUN [{current_run} / {total_runs}]-----------------\n", flush=True)

    def execute(self) -> Dict[str, Any]:
        ctx = self.run_context
        raise_event = EventSubscriptionController.raise_event
        output.console_log_WARNING("Calling start_run config hook")
        raise_event(RunnerEvents.START_RUN, ctx)
        output.console_log_WARNING("... Starting measurement ...")
        raise_event(RunnerEvents.START_MEASUREMENT, ctx)
        output.console_log_WARNING("Calling interaction config hook")
        raise_event(RunnerEvents.INTERACT, ctx)
        output.console_log_OK("... Run completed ...")
        output.console_log_WARNING("... Stopping measurement ...")
        raise_event(RunnerEvents.STOP_MEASUREMENT, ctx)
        output.console_log_WARNING("Calling stop_run config hook")
        raise_event(RunnerEvents.STOP_RUN, ctx)
        output.console_log_WARNING("Calling populate_run_data config hook")
        user_data = raise_event(RunnerEvents.POPULATE_RUN_DATA, ctx)
        row = dict(ctx.run_variation)
        if user_data:
            row.update(user_data)
        row["__done"] = RunProgress.DONE
        return row

    def do_run(self) -> Dict[str, Any]:
        """Reference-named entry: execute and commit the row directly."""
        row = self.execute()
        CSVOutputManager(self.config.experiment_path).update_row_data(dict(row))
        return row


class ExperimentController:
    def __init__(self, config: Any, metadata: Metadata, source: Optional[str] = None,
                 source_name: str = "<config>", assume_yes: Optional[bool] = None,
                 isolation: Optional[str] = None, run_timeout_s: Optional[float] = None,
                 writer: bool = True, rank: int = 0, device: Optional[str] = None):
        self.config = config
        self.metadata = metadata
        self.isolation = isolation if isolation is not None else getattr(config, "run_isolation", None)
        self.run_timeout_s = run_timeout_s if run_timeout_s is not None else getattr(config, "run_timeout_s", None)
        self.rank = rank
        self.device = device
        self.writer = writer
        self.path = Path(config.experiment_path)
        self.csv_data_manager = CSVOutputManager(self.path)
        self.json_data_manager = JSONOutputManager(self.path)
        self.run_table = config.create_run_table_model().generate_experiment_run_table()
        self.restarted = False
        if not writer:
            # non-writer ranks read the table rank 0 created (fan-out path)
            return
        try:
            self.path.mkdir(parents=True, exist_ok=False)
        except FileExistsError:
            if not (self.path / "run_table.csv").exists():
                output.console_log_WARNING(f"Experiment path {self.path} exists without a run table: starting fresh")
            else:
                self._resume(source, source_name, assume_yes)
        if not self.restarted:
            self.csv_data_manager.write_run_table(self.run_table)
            self.json_data_manager.write_metadata(self.metadata)
        output.console_log_WARNING("Experiment run table created...")

    # -- resume (reference ExperimentController.py:45-103) ---------------
    def _resume(self, source, source_name, assume_yes) -> None:
        output.console_log_WARNING(f"Reusing already existing experiment path: {self.path}")
        existing = self.csv_data_manager.read_run_table()
        if not any(v["__done"] != RunProgress.DONE for v in existing):
            raise AllRunsCompletedOnRestartError()
        gen_cols = set(self.run_table[0].keys())
        disk_cols = set(existing[0].keys())
        if not gen_cols <= disk_cols:
            raise BaseError("The generated run table from the config file, and the found run table in the CSV in "
                            "the experiment output path, do not define the same columns!")
        extra = disk_cols - gen_cols
        if extra:
            output.console_log_WARNING(f"run_table.csv carries extra columns {sorted(extra)}; they are preserved")
        stored = self.json_data_manager.read_metadata()
        same = (stored.md5sum == self.metadata.md5sum) or (
            source is not None and fingerprint_matches(stored, source, source_name))
        if not same:
            cont = output.query_yes_no("md5sum mismatch! This can occur if the configuration code has changed "
                                       "since the last run. Continue anyway?", default=None, assume=assume_yes)
            if not cont:
                raise BaseError("Aborting due to md5sum mismatch.")
            output.console_log_WARNING(f"Updating md5sum from {stored.md5sum.hex()} to {self.metadata.md5sum.hex()}")
            self.json_data_manager.write_metadata(self.metadata)
        if len(existing) != len(self.run_table):
            raise BaseError(f"run_table.csv has {len(existing)} rows but the config generates {len(self.run_table)}")
        by_id = {v["__run_id"]: v for v in self.run_table}
        reordered = []
        factor_names = [f.factor_name for f in self.config.run_table_model.get_factors()]
        data_cols = list(self.config.run_table_model.get_data_columns())
        for ex in existing:
            gen = by_id.get(ex["__run_id"])
            if gen is None:
                raise BaseError(f"run id {ex['__run_id']} on disk is not generated by the config")
            for k in factor_names:
                if str(gen[k]) != str(ex[k]):
                    raise BaseError(f"{ex['__run_id']}: factor {k} is {ex[k]!r} on disk but {gen[k]!r} in the config")
            for k in data_cols + ["__done"] + sorted(extra):
                gen[k] = ex[k]
            reordered.append(gen)
        self.run_table = reordered
        self.restarted = True
        output.console_log_WARNING(">> WARNING << -- Experiment is restarted!")

    # -- loop -------------------------------------------------------------
    def pending(self) -> List[Dict[str, Any]]:
        return [v for v in self.run_table if v["__done"] != RunProgress.DONE]

    def index_of(self, variation: Dict[str, Any]) -> int:
        rid = variation["__run_id"]
        for i, v in enumerate(self.run_table):
            if v["__run_id"] == rid:
                return i
        raise KeyError(rid)

    def log_error(self, run_id: str, exc: BaseException) -> None:
        rec = {"__run_id": run_id, "time": time.time(), "rank": self.rank, "type": type(exc).__name__,
               "message": str(exc)[-4000:]}
        try:
            with open(self.path / "errors.jsonl", "a") as fh:
                fh.write(json.dumps(rec) + "\n")
        except OSError:  # pragma: no cover
            pass

    def run_variation(self, variation: Dict[str, Any], commit: Optional[Callable[[Dict[str, Any]], None]] = None
                      ) -> Optional[Dict[str, Any]]:
        """BEFORE_RUN in this process, then the isolated run body.  Returns the finished row
        (already committed when this controller is the writer) or None on failure."""
        output.console_log_WARNING("Calling before_run config hook")
        EventSubscriptionController.raise_event(RunnerEvents.BEFORE_RUN)
        rc = RunController(variation, self.config, self.index_of(variation) + 1, len(self.run_table),
                           rank=self.rank, device=self.device)
        try:
            row = call_isolated(rc.execute, mode=self.isolation, timeout=self.run_timeout_s,
                                label=str(variation["__run_id"]))
        except (Exception, RunTimeoutError) as exc:  # row stays TODO (reference semantics)
            output.console_log_FAIL(f"Run {variation['__run_id']} failed: {type(exc).__name__}: {exc}")
            traceback.print_exc()
            self.log_error(str(variation["__run_id"]), exc)
            return None
        variation.update(row)
        if commit is not None:
            commit(dict(row))
        elif self.writer:
            self.csv_data_manager.update_row_data(dict(row))
        return row

    def cooldown(self) -> None:
        ms = _cooldown_ms(self.config)
        if ms > 0:
            output.console_log_bold(f"Run fully ended, waiting for: {ms}ms == {ms / 1000}s")
            time.sleep(ms / 1000)

    def do_experiment(self) -> None:
        output.console_log_OK("Experiment setup completed...")
        output.console_log_WARNING("Calling before_experiment config hook")
        try:
            EventSubscriptionController.raise_event(RunnerEvents.BEFORE_EXPERIMENT)
            todo = self.pending()
            # session budget (seconds; config `run_budget_s` or CAIN_RUN_BUDGET_S): no run starts after it, the
            # rest stays TODO for the next invocation of the same command (allocation windows shorter than a study)
            budget = float(os.environ.get("CAIN_RUN_BUDGET_S", getattr(self.config, "run_budget_s", 0) or 0))
            t_start = time.monotonic()
            for n, variation in enumerate(todo):
                if budget > 0 and n > 0 and time.monotonic() - t_start > budget:  # >= 1 run per session
                    output.console_log_WARNING(f"session budget of {budget:.0f} s reached: {len(todo) - n} runs left "
                                               "TODO; run the same command again to resume")
                    return
                self.run_variation(variation)
                if n + 1 < len(todo):
                    self.cooldown()
                if self.config.operation_type is OperationType.SEMI:
                    EventSubscriptionController.raise_event(RunnerEvents.CONTINUE)
            output.console_log_OK("Experiment completed...")
            output.console_log_WARNING("Calling after_experiment config hook")
            EventSubscriptionController.raise_event(RunnerEvents.AFTER_EXPERIMENT)
        finally:
            # per-process resources a config started in BEFORE_EXPERIMENT (e.g. its local servers); the
            # data-parallel path calls the same hook once per rank (parallel/fanout.py)
            teardown = getattr(self.config, "teardown_rank", None)
            if callable(teardown):
                teardown()
