"""Canonical user-config skeleton (``config-create`` copies this file).

Same shape as the reference template (experiment-runner/ConfigValidator/
Config/RunnerConfig.py:15-123): class attributes are the settings, the nine
methods are the lifecycle hooks, ``create_run_table_model`` declares the
design.  Extra optional attributes understood by this framework:
``run_timeout_s``, ``run_isolation`` and ``shuffle_seed``.
"""
from __future__ import annotations

from os.path import dirname, realpath
from pathlib import Path
from typing import Any, Dict, Optional

from cain_amd.runner.events import EventSubscriptionController, RunnerEvents
from cain_amd.runner.models import FactorModel, OperationType, RunnerContext, RunTableModel
from cain_amd.runner.output import OutputProcedure as output


class RunnerConfig:
    ROOT_DIR = Path(dirname(realpath(__file__)))

    # ================================ USER SPECIFIC CONFIG ================================
    """The name of the experiment."""
    name: str = "new_runner_experiment"

    """Output folder; the experiment lives in results_output_path / name."""
    results_output_path: Path = ROOT_DIR / "experiments"

    """AUTO continues after the cooldown; SEMI raises RunnerEvents.CONTINUE after each run."""
    operation_type: OperationType = OperationType.AUTO

    """Cooldown between runs (ms)."""
    time_between_runs_in_ms: int = 1000

    """Wall-clock limit per run (s); a run over it is killed and stays TODO.  None = no limit."""
    run_timeout_s: Optional[float] = None

    """'fork' (default), 'inline' or 'spawn' isolation of each run's hooks."""
    run_isolation: Optional[str] = None

    def __init__(self):
        EventSubscriptionController.subscribe_to_multiple_events([
            (RunnerEvents.BEFORE_EXPERIMENT, self.before_experiment),
            (RunnerEvents.BEFORE_RUN, self.before_run),
            (RunnerEvents.START_RUN, self.start_run),
            (RunnerEvents.START_MEASUREMENT, self.start_measurement),
            (RunnerEvents.INTERACT, self.interact),
            (RunnerEvents.STOP_MEASUREMENT, self.stop_measurement),
            (RunnerEvents.STOP_RUN, self.stop_run),
            (RunnerEvents.POPULATE_RUN_DATA, self.populate_run_data),
            (RunnerEvents.AFTER_EXPERIMENT, self.after_experiment),
        ])
        self.run_table_model = None
        output.console_log("Custom config loaded")

    def create_run_table_model(self) -> RunTableModel:
        factor1 = FactorModel("example_factor1", ["example_treatment1", "example_treatment2", "example_treatment3"])
        factor2 = FactorModel("example_factor2", [True, False])
        self.run_table_model = RunTableModel(
            factors=[factor1, factor2],
            exclude_variations=[
                {factor1: ["example_treatment1"]},
                {factor1: ["example_treatment2"], factor2: [True]},
            ],
            data_columns=["avg_cpu", "avg_mem"],
        )
        return self.run_table_model

    def before_experiment(self) -> None:
        output.console_log("Config.before_experiment() called!")

    def before_run(self) -> None:
        output.console_log("Config.before_run() called!")

    def start_run(self, context: RunnerContext) -> None:
        output.console_log("Config.start_run() called!")

    def start_measurement(self, context: RunnerContext) -> None:
        output.console_log("Config.start_measurement() called!")

    def interact(self, context: RunnerContext) -> None:
        output.console_log("Config.interact() called!")

    def stop_measurement(self, context: RunnerContext) -> None:
        output.console_log("Config.stop_measurement called!")

    def stop_run(self, context: RunnerContext) -> None:
        output.console_log("Config.stop_run() called!")

    def populate_run_data(self, context: RunnerContext) -> Optional[Dict[str, Any]]:
        output.console_log("Config.populate_run_data() called!")
        return None

    def after_experiment(self) -> None:
        output.console_log("Config.after_experiment() called!")

    # ================================ DO NOT ALTER BELOW THIS LINE ================================
    experiment_path: Path = None
