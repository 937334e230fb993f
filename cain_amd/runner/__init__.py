"""Experiment-runner core: reference-compatible orchestration API."""
from .controller import ExperimentController, RunController  # noqa: F401
from .errors import BaseError  # noqa: F401
from .events import EventSubscriptionController, RunnerEvents  # noqa: F401
from .models import (FactorModel, Metadata, OperationType, RunnerContext, RunProgress,  # noqa: F401
                     RunTableModel, SupportsStr)
from .output import OutputProcedure  # noqa: F401
from .store import CSVOutputManager, JSONOutputManager  # noqa: F401
from .validator import ConfigValidator  # noqa: F401
