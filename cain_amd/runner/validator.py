"""Config validation.

Reference: experiment-runner/ConfigValidator/Config/Validation/
ConfigValidator.py:22-65.  Sets ``config.experiment_path =
results_output_path / name`` (``~`` expanded), type-checks the core
attributes, prints the config as an RST table and raises
``ConfigInvalidError``.  Two reference checks were vacuous and are real here
(SURVEY §2.8): ``operation_type`` is ``isinstance``-checked, and the
writability check receives ``str(path)`` so it actually runs.  Added checks
cover the engine/profiler attributes this framework understands.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Dict

from tabulate import tabulate

from .errors import ConfigAttributeInvalidError, ConfigInvalidError
from .models import OperationType
from .paths import is_path_exists_or_creatable


def class_to_dict(obj: Any) -> Dict[str, Any]:
    """Public, non-callable attributes of a config instance (reference DictConversion.py:4-10)."""
    out: Dict[str, Any] = {}
    for k in dir(obj):
        if k.startswith("_"):
            continue
        try:
            v = getattr(obj, k)
        except Exception:
            continue
        if callable(v):
            continue
        out[k] = v
    return out


#: optional attributes: name -> (types, predicate, description)
_OPTIONAL = {
    "run_timeout_s": ((int, float, type(None)), lambda v: v is None or v > 0, "positive number or None"),
    "run_isolation": ((str, type(None)), lambda v: v is None or v in ("fork", "inline", "spawn"),
                      "'fork' | 'inline' | 'spawn'"),
    "shuffle_seed": ((int, type(None)), lambda v: True, "int or None"),
}


class ConfigValidator:
    @staticmethod
    def validate_config(config: Any, quiet: bool = False) -> None:
        config.experiment_path = Path(os.path.expanduser(str(config.results_output_path))) / config.name
        table = class_to_dict(config)
        errors = False

        def flag(name, value, expected):
            nonlocal errors
            errors = True
            table[name] = f"{table.get(name, value)}\n\n{ConfigAttributeInvalidError(name, value, expected).plain_message}"

        if not isinstance(getattr(config, "name", None), str) or not config.name:
            flag("name", getattr(config, "name", None), "non-empty str")
        if not isinstance(getattr(config, "operation_type", None), OperationType):
            flag("operation_type", getattr(config, "operation_type", None), OperationType)
        tbr = getattr(config, "time_between_runs_in_ms", None)
        if not isinstance(tbr, int) or isinstance(tbr, bool) or tbr < 0:
            flag("time_between_runs_in_ms", tbr, "int >= 0")
        if not isinstance(getattr(config, "results_output_path", None), Path):
            flag("results_output_path", getattr(config, "results_output_path", None), Path)
        elif not is_path_exists_or_creatable(str(config.experiment_path)):
            flag("results_output_path", config.experiment_path, "path must be valid and writable")
        for name, (types, pred, desc) in _OPTIONAL.items():
            if hasattr(config, name):
                v = getattr(config, name)
                if not isinstance(v, types) or not pred(v):
                    flag(name, v, desc)

        if not quiet:
            print(tabulate([(k, str(v)) for k, v in table.items()], ["Key", "Value"], tablefmt="rst"))
        if errors:
            raise ConfigInvalidError()
