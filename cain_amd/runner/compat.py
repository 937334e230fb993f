"""Import-name compatibility for reference ``RunnerConfig.py`` files.

A reference config starts with imports such as
``from EventManager.Models.RunnerEvents import RunnerEvents`` or
``from Plugins.Profilers import CodecarbonWrapper`` (reference
experiment/RunnerConfig.py:1-16) because the reference runs with
``experiment-runner/`` as the import root.  ``install()`` registers alias
modules for every such name, pointing at this framework's implementations,
so those files load unchanged under ``python -m cain_amd <config.py>``.
"""
from __future__ import annotations

import sys
import types
from typing import Dict


def _aliases() -> Dict[str, Dict[str, object]]:
    from . import controller, errors, events, isolation, models, output, paths, store, validator
    from ..energy import plugin as energy_plugin
    from ..energy import wattsup
    from . import template

    ob = {
        "EventManager.Models.RunnerEvents": {"RunnerEvents": events.RunnerEvents},
        "EventManager.EventSubscriptionController": {
            "EventSubscriptionController": events.EventSubscriptionController},
        "ConfigValidator.Config.Models.RunTableModel": {"RunTableModel": models.RunTableModel},
        "ConfigValidator.Config.Models.FactorModel": {"FactorModel": models.FactorModel},
        "ConfigValidator.Config.Models.RunnerContext": {"RunnerContext": models.RunnerContext},
        "ConfigValidator.Config.Models.OperationType": {"OperationType": models.OperationType},
        "ConfigValidator.Config.Models.Metadata": {"Metadata": models.Metadata},
        "ConfigValidator.Config.RunnerConfig": {"RunnerConfig": template.RunnerConfig},
        "ConfigValidator.CustomErrors.BaseError": {"BaseError": errors.BaseError},
        "ConfigValidator.CustomErrors.CLIErrors": {
            "CommandNotRecognisedError": errors.CommandNotRecognisedError,
            "InvalidUserSpecifiedPathError": errors.InvalidUserSpecifiedPathError},
        "ConfigValidator.CustomErrors.ConfigErrors": {
            "ConfigBaseError": errors.ConfigBaseError, "ConfigInvalidError": errors.ConfigInvalidError,
            "ConfigInvalidClassNameError": errors.ConfigInvalidClassNameError,
            "ConfigAttributeInvalidError": errors.ConfigAttributeInvalidError},
        "ConfigValidator.CustomErrors.ExperimentOutputErrors": {
            "ExperimentOutputFileDoesNotExistError": errors.ExperimentOutputFileDoesNotExistError},
        "ConfigValidator.CustomErrors.ProgressErrors": {
            "ProgressBaseError": errors.ProgressBaseError,
            "AllRunsCompletedOnRestartError": errors.AllRunsCompletedOnRestartError},
        "ProgressManager.Output.OutputProcedure": {"OutputProcedure": output.OutputProcedure},
        "ProgressManager.Output.CSVOutputManager": {"CSVOutputManager": store.CSVOutputManager},
        "ProgressManager.Output.JSONOutputManager": {"JSONOutputManager": store.JSONOutputManager},
        "ProgressManager.Output.BaseOutputManager": {"BaseOutputManager": store.BaseOutputManager},
        "ProgressManager.RunTable.Models.RunProgress": {"RunProgress": models.RunProgress},
        "ExtendedTyping.Typing": {"SupportsStr": models.SupportsStr},
        "ExperimentOrchestrator.Architecture.Processify": {"processify": isolation.processify},
        "ExperimentOrchestrator.Misc.BashHeaders": {"BashHeaders": output.BashHeaders},
        "ExperimentOrchestrator.Misc.PathValidation": {
            n: getattr(paths, n) for n in ("is_pathname_valid", "is_path_creatable", "is_path_exists_or_creatable",
                                           "is_path_sibling_creatable", "is_path_exists_or_creatable_portable")},
        "ExperimentOrchestrator.Misc.DictConversion": {
            "class_to_dict": validator.class_to_dict},
        "ExperimentOrchestrator.Experiment.ExperimentController": {
            "ExperimentController": controller.ExperimentController},
        "ExperimentOrchestrator.Experiment.Run.RunController": {"RunController": controller.RunController},
        "ConfigValidator.Config.Validation.ConfigValidator": {"ConfigValidator": validator.ConfigValidator},
        "Plugins.Profilers.CodecarbonWrapper": {
            "DataColumns": energy_plugin.DataColumns, "emission_tracker": energy_plugin.emission_tracker},
        "Plugins.Profilers.WattsUpPro": {"WattsUpPro": wattsup.WattsUpPro},
    }
    return ob


_installed = False


def install() -> None:
    global _installed
    if _installed:
        return
    for dotted, attrs in _aliases().items():
        parts = dotted.split(".")
        for i in range(1, len(parts) + 1):
            name = ".".join(parts[:i])
            mod = sys.modules.get(name)
            if mod is None:
                mod = types.ModuleType(name)
                mod.__path__ = []  # mark as package so submodules resolve
                mod.__cain_alias__ = True
                sys.modules[name] = mod
                if i > 1:
                    setattr(sys.modules[".".join(parts[:i - 1])], parts[i - 1], mod)
        leaf = sys.modules[dotted]
        for k, v in attrs.items():
            setattr(leaf, k, v)
    # `from Plugins.Profilers import CodecarbonWrapper` needs the attribute on the package
    sys.modules["Plugins.Profilers"].CodecarbonWrapper = sys.modules["Plugins.Profilers.CodecarbonWrapper"]
    # python-dotenv is not installed in this image; the reference config imports it
    # (experiment/RunnerConfig.py:22) — serve the same two names from cain_amd.utils.env
    try:
        import dotenv  # noqa: F401
    except ImportError:
        from ..utils import env as _env

        mod = types.ModuleType("dotenv")
        mod.load_dotenv = _env.load_dotenv
        mod.dotenv_values = _env.dotenv_values
        mod.__cain_alias__ = True
        sys.modules["dotenv"] = mod
    _installed = True
