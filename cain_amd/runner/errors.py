"""User-facing error hierarchy.

Same class names and messages as the reference so ``except`` clauses in user
configs keep working (reference: experiment-runner/ConfigValidator/CustomErrors/
BaseError.py:3-6, CLIErrors.py:3-14, ConfigErrors.py:4-21,
ExperimentOutputErrors.py:4-10, ProgressErrors.py:3-9).  Added:
``RunTimeoutError`` (per-run wall-clock limit) and
``WorkerLostError`` (a data-parallel GPU worker died, its shard is re-queued).
"""
from __future__ import annotations

from .output import BashHeaders


class BaseError(Exception):
    def __init__(self, message: str):
        self.plain_message = message
        super().__init__(BashHeaders.FAIL + "[FAIL]: " + BashHeaders.ENDC
                         + "EXPERIMENT_RUNNER ENCOUNTERED AN ERROR!\n\n"
                         + BashHeaders.FAIL + message + BashHeaders.ENDC)


class CommandNotRecognisedError(BaseError):
    def __init__(self, command: str = ""):
        extra = f": {command!r}" if command else ""
        super().__init__("The command entered by the user is not recognised" + extra)


class InvalidUserSpecifiedPathError(BaseError):
    def __init__(self, path):
        super().__init__("The user specified path is invalid or the user does not have the correct "
                         f"permissions\n{path}")


class ConfigBaseError(BaseError):
    pass


class ConfigInvalidError(ConfigBaseError):
    def __init__(self):
        super().__init__("Config found to be invalid, please refer to the config attribute table.")


class ConfigInvalidClassNameError(ConfigBaseError):
    def __init__(self):
        super().__init__("The config file specified does not have a valid config class name as "
                         "expected (RunnerConfig).")


class ConfigAttributeInvalidError(ConfigBaseError):
    def __init__(self, attribute, found, expected):
        super().__init__(f"INVALID config attribute {attribute}\n"
                         + "%-*s  %s\n" % (10, "FOUND:", found)
                         + "%-*s  %s" % (10, "EXPECTED:", expected))


class ExperimentOutputFileDoesNotExistError(BaseError):
    def __init__(self):
        super().__init__("The experiment_path (experiment output folder) exists, but the run_table.csv "
                         "does not exist.\nExperiment-runner cannot restart!")


class ProgressBaseError(BaseError):
    pass


class AllRunsCompletedOnRestartError(ProgressBaseError):
    def __init__(self):
        super().__init__("The experiment was restarted, but all runs have already been completed.")


class RunTimeoutError(BaseError):
    def __init__(self, run_id: str, seconds: float):
        super().__init__(f"Run {run_id} exceeded its wall-clock limit of {seconds:.1f}s and was killed.")


class WorkerLostError(BaseError):
    def __init__(self, rank: int, detail: str = ""):
        super().__init__(f"Worker rank {rank} was lost. {detail}".strip())
