"""Experiment-runner core: run table, persistence, resume, events, isolation, CLI."""
import csv
import json
import os
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

from cain_amd.runner import compat
from cain_amd.runner.controller import ExperimentController
from cain_amd.runner.errors import AllRunsCompletedOnRestartError, BaseError, ConfigInvalidError
from cain_amd.runner.events import EventSubscriptionController, RunnerEvents
from cain_amd.runner.fingerprint import ast_md5, fingerprint, legacy_md5, matches
from cain_amd.runner.isolation import call_isolated, processify
from cain_amd.runner.models import FactorModel, Metadata, OperationType, RunProgress, RunTableModel
from cain_amd.runner.store import CSVOutputManager, JSONOutputManager
from cain_amd.runner.validator import ConfigValidator

ROOT = Path(__file__).resolve().parent.parent
REF_CONFIG = Path("/root/reference/experiment/RunnerConfig.py")

STUDY_MODELS = ['llama3.1:8b', 'gemma:2b', 'gemma:7b', 'phi3:3.8b', 'qwen2:1.5b', 'qwen2:7b', 'mistral:7b']


# ------------------------------------------------------------------ run table
def test_factorial_ids_and_columns():
    f1, f2 = FactorModel("a", [1, 2, 3]), FactorModel("b", ["x", "y"])
    t = RunTableModel([f1, f2], repetitions=2, data_columns=["d1"]).generate_experiment_run_table()
    assert len(t) == 12
    assert list(t[0]) == ["__run_id", "__done", "a", "b", "d1"]
    assert t[0]["__run_id"] == "run_0_repetition_0" and (t[0]["a"], t[0]["b"]) == (1, "x")
    assert t[6]["__run_id"] == "run_0_repetition_1"  # repetitions are the outer loop
    assert t[5]["__run_id"] == "run_5_repetition_0" and (t[5]["a"], t[5]["b"]) == (3, "y")
    assert all(r["__done"] is RunProgress.TODO and r["d1"] == " " for r in t)


def test_exclusions_match_reference_semantics_and_remove_each_row_once():
    f1 = FactorModel("f1", ["t1", "t2", "t3"])
    f2 = FactorModel("f2", [True, False])
    m = RunTableModel([f1, f2], exclude_variations=[{f1: ["t1"]}, {f1: ["t2"], f2: [True]},
                                                     {"f1": ["t1"], "f2": [False]}])  # overlaps the first
    t = m.generate_experiment_run_table()
    assert [(r["f1"], r["f2"]) for r in t] == [("t2", False), ("t3", True), ("t3", False)]
    assert [r["__run_id"] for r in t] == ["run_0_repetition_0", "run_1_repetition_0", "run_2_repetition_0"]


def test_shuffle_seeded_and_validation():
    f = [FactorModel("a", list(range(10)))]
    a = RunTableModel(f, shuffle=True, seed=3).generate_experiment_run_table()
    b = RunTableModel(f, shuffle=True, seed=3).generate_experiment_run_table()
    assert [r["__run_id"] for r in a] == [r["__run_id"] for r in b]
    assert sorted(r["__run_id"] for r in a) == sorted(f"run_{i}_repetition_0" for i in range(10))
    with pytest.raises(BaseError):
        RunTableModel(f, repetitions=0)
    with pytest.raises(BaseError):
        RunTableModel([FactorModel("a", [1]), FactorModel("a", [2])])
    with pytest.raises(BaseError):
        RunTableModel(f, data_columns=["x", "x"])
    with pytest.raises(BaseError):
        FactorModel("a", [1, 1])


def test_golden_run_ids_of_shipped_run_table(fixtures_dir):
    """The shipped table was produced with method order ['on_device', 'remote']:
    every __run_id maps back to its (model, method, length)."""
    rows = list(csv.DictReader(open(fixtures_dir / "run_table.csv")))
    assert len(rows) == 1260
    model = RunTableModel([FactorModel("model", STUDY_MODELS), FactorModel("method", ["on_device", "remote"]),
                           FactorModel("length", ["100", "500", "1000"])], repetitions=30)
    gen = {r["__run_id"]: r for r in model.generate_experiment_run_table()}
    assert all(gen[r["__run_id"]]["model"] == r["model"] and gen[r["__run_id"]]["method"] == r["method"]
               and gen[r["__run_id"]]["length"] == r["length"] for r in rows)
    shipped_order = RunTableModel([FactorModel("model", STUDY_MODELS), FactorModel("method", ["remote", "on_device"]),
                                   FactorModel("length", ["100", "500", "1000"])], repetitions=30)
    gen2 = {r["__run_id"]: r for r in shipped_order.generate_experiment_run_table()}
    assert sum(gen2[r["__run_id"]]["method"] == r["method"] for r in rows) == 0


# ------------------------------------------------------------------ persistence
def test_csv_roundtrip_coercions_and_row_update(tmp_path):
    m = CSVOutputManager(tmp_path)
    table = [{"__run_id": "run_0_repetition_0", "__done": RunProgress.TODO, "n": 5, "e": " "},
             {"__run_id": "run_1_repetition_0", "__done": RunProgress.DONE, "n": 7, "e": "5.46E+01"}]
    m.write_run_table([dict(r) for r in table])
    back = m.read_run_table()
    assert back[0]["n"] == 5 and back[0]["__done"] is RunProgress.TODO
    assert back[1]["e"] == "5.46E+01" and back[1]["__done"] is RunProgress.DONE  # not numeric: stays str
    m.update_row_data({"__run_id": "run_0_repetition_0", "__done": RunProgress.DONE, "n": 9, "e": 1.5,
                       "extra_col": "x"})
    back = m.read_run_table()
    assert back[0]["__done"] is RunProgress.DONE and back[0]["n"] == 9 and back[0]["e"] == "1.5"
    assert back[0]["extra_col"] == "x" and back[1]["extra_col"] == ""
    assert [p.name for p in tmp_path.iterdir()] == ["run_table.csv"]  # no temp files left behind
    with pytest.raises(KeyError):
        m.update_rows([{"__run_id": "nope", "__done": RunProgress.DONE}])


def test_metadata_legacy_and_roundtrip(tmp_path, fixtures_dir):
    legacy = JSONOutputManager(fixtures_dir).read_metadata()
    assert legacy.scheme == "legacy-dill" and len(legacy.md5sum) == 16
    j = JSONOutputManager(tmp_path)
    j.write_metadata(Metadata(b"\x01" * 16))
    assert j.read_metadata().md5sum == b"\x01" * 16
    doc = json.loads((tmp_path / "metadata.json").read_text())
    assert "py/b64" in doc["_md5sum"]


def test_fingerprint_ignores_comments_docstrings_positions():
    a = 'class A:\n    """doc"""\n    x = 1  # c\n'
    b = '\n\nclass A:\n    """other doc"""\n\n    x = 1\n'
    c = 'class A:\n    x = 2\n'
    assert ast_md5(a) == ast_md5(b) != ast_md5(c)
    assert matches(fingerprint(a), b)
    assert legacy_md5(a) is not None


# ------------------------------------------------------------------ events / isolation
def test_event_registry_single_callback_and_context():
    EventSubscriptionController.clear()
    seen = []
    EventSubscriptionController.subscribe_to_single_event(RunnerEvents.START_RUN, lambda c: seen.append(("a", c)))
    EventSubscriptionController.subscribe_to_single_event(RunnerEvents.START_RUN, lambda c: seen.append(("b", c)))
    EventSubscriptionController.raise_event(RunnerEvents.START_RUN, 0)  # falsy context still passed
    assert seen == [("b", 0)]
    assert EventSubscriptionController.raise_event(RunnerEvents.STOP_RUN) is None
    EventSubscriptionController.clear()


def _boom():
    raise ValueError("xyz")


def _gen():
    yield "generator"
    yield "function"


def _big():
    return list(range(30000))


@processify
def _pid():
    return os.getpid()


def test_isolation_modes():
    assert call_isolated(_big, mode="fork") == list(range(30000))  # no pipe deadlock on large results
    assert call_isolated(_gen, mode="fork") == ["generator", "function"]
    with pytest.raises(ValueError, match="xyz"):
        call_isolated(_boom, mode="fork")
    assert _pid() != os.getpid()
    assert call_isolated(os.getpid, mode="inline") == os.getpid()


def test_isolation_timeout_kills():
    import time

    from cain_amd.runner.errors import RunTimeoutError
    with pytest.raises(RunTimeoutError):
        call_isolated(time.sleep, 30, mode="fork", timeout=0.5)


# ------------------------------------------------------------------ controller
CONFIG_SRC = textwrap.dedent('''
    import json, os, time
    from pathlib import Path
    from EventManager.Models.RunnerEvents import RunnerEvents
    from EventManager.EventSubscriptionController import EventSubscriptionController
    from ConfigValidator.Config.Models.RunTableModel import RunTableModel
    from ConfigValidator.Config.Models.FactorModel import FactorModel
    from ConfigValidator.Config.Models.OperationType import OperationType

    OUT = Path(os.environ["CAIN_TEST_OUT"])

    class RunnerConfig:
        name = "exp"
        results_output_path = OUT
        operation_type = OperationType.SEMI
        time_between_runs_in_ms = 0
        run_timeout_s = float(os.environ.get("CAIN_TEST_TIMEOUT", "30"))

        def __init__(self):
            EventSubscriptionController.subscribe_to_multiple_events([
                (RunnerEvents.BEFORE_EXPERIMENT, lambda: self.log("before_experiment")),
                (RunnerEvents.BEFORE_RUN, lambda: self.log("before_run")),
                (RunnerEvents.START_RUN, lambda c: self.step("start_run", c)),
                (RunnerEvents.START_MEASUREMENT, lambda c: self.step("start_measurement", c)),
                (RunnerEvents.INTERACT, lambda c: self.step("interact", c)),
                (RunnerEvents.STOP_MEASUREMENT, lambda c: self.step("stop_measurement", c)),
                (RunnerEvents.STOP_RUN, lambda c: self.step("stop_run", c)),
                (RunnerEvents.POPULATE_RUN_DATA, self.populate),
                (RunnerEvents.CONTINUE, lambda: self.log("continue")),
                (RunnerEvents.AFTER_EXPERIMENT, lambda: self.log("after_experiment")),
            ])

        def log(self, what):
            with open(OUT / "events.log", "a") as fh:
                fh.write(what + "\\n")

        def step(self, what, ctx):
            self.log(what)
            bad = os.environ.get("CAIN_TEST_FAIL")
            if bad and ctx.run_variation["__run_id"] == bad and what == "interact":
                raise RuntimeError("injected failure")
            hang = os.environ.get("CAIN_TEST_HANG")
            if hang and ctx.run_variation["__run_id"] == hang and what == "interact":
                time.sleep(60)

        def create_run_table_model(self):
            self.run_table_model = RunTableModel(
                factors=[FactorModel("f", ["a", "b"]), FactorModel("g", [1, 2])],
                data_columns=["value", "pid"], repetitions=1, shuffle=True)
            return self.run_table_model

        def populate(self, ctx):
            self.log("populate_run_data")
            return {"value": f"{ctx.run_variation['f']}{ctx.run_variation['g']}", "pid": os.getpid()}

        experiment_path = None
''')


@pytest.fixture
def exp_config(tmp_path, monkeypatch):
    monkeypatch.setenv("CAIN_TEST_OUT", str(tmp_path))
    p = tmp_path / "cfg.py"
    p.write_text(CONFIG_SRC)
    return p


def _run(cfg_path, assume_yes=None, isolation=None):
    from cain_amd.runner.cli import build_config

    EventSubscriptionController.clear()
    config, md, src = build_config(str(cfg_path))
    ConfigValidator.validate_config(config, quiet=True)
    ExperimentController(config, md, source=src, source_name=str(cfg_path), assume_yes=assume_yes,
                         isolation=isolation).do_experiment()
    return config


@pytest.mark.parametrize("isolation", ["fork", "inline"])
def test_experiment_hook_order_and_rows(exp_config, tmp_path, isolation):
    cfg = _run(exp_config, isolation=isolation)
    rows = CSVOutputManager(cfg.experiment_path).read_run_table()
    assert all(r["__done"] is RunProgress.DONE for r in rows)
    assert sorted(r["value"] for r in rows) == ["a1", "a2", "b1", "b2"]
    pids = {r["pid"] for r in rows}
    if isolation == "fork":
        assert os.getpid() not in pids and len(pids) == 4
    ev = (tmp_path / "events.log").read_text().split()
    per_run = ["before_run", "start_run", "start_measurement", "interact", "stop_measurement", "stop_run",
               "populate_run_data", "continue"]
    assert ev == ["before_experiment"] + per_run * 4 + ["after_experiment"]
    assert all((cfg.experiment_path / r["__run_id"]).is_dir() for r in rows)


def test_failed_run_stays_todo_then_resume(exp_config, tmp_path, monkeypatch):
    monkeypatch.setenv("CAIN_TEST_FAIL", "run_1_repetition_0")
    cfg = _run(exp_config)
    rows = {r["__run_id"]: r for r in CSVOutputManager(cfg.experiment_path).read_run_table()}
    assert rows["run_1_repetition_0"]["__done"] is RunProgress.TODO
    assert sum(r["__done"] is RunProgress.DONE for r in rows.values()) == 3
    err = [json.loads(ln) for ln in (cfg.experiment_path / "errors.jsonl").read_text().splitlines()]
    assert err[0]["__run_id"] == "run_1_repetition_0" and "injected" in err[0]["message"]
    order_before = [r["__run_id"] for r in CSVOutputManager(cfg.experiment_path).read_run_table()]
    monkeypatch.delenv("CAIN_TEST_FAIL")
    (tmp_path / "events.log").unlink()
    cfg = _run(exp_config)  # resume: only the TODO row runs, order preserved
    rows = CSVOutputManager(cfg.experiment_path).read_run_table()
    assert [r["__run_id"] for r in rows] == order_before
    assert all(r["__done"] is RunProgress.DONE for r in rows)
    assert (tmp_path / "events.log").read_text().split().count("start_run") == 1
    with pytest.raises(AllRunsCompletedOnRestartError):
        _run(exp_config)


def test_timeout_kills_run_and_continues(exp_config, monkeypatch):
    monkeypatch.setenv("CAIN_TEST_HANG", "run_0_repetition_0")
    monkeypatch.setenv("CAIN_TEST_TIMEOUT", "1.5")
    cfg = _run(exp_config)
    rows = {r["__run_id"]: r for r in CSVOutputManager(cfg.experiment_path).read_run_table()}
    assert rows["run_0_repetition_0"]["__done"] is RunProgress.TODO
    assert sum(r["__done"] is RunProgress.DONE for r in rows.values()) == 3


def test_session_budget_leaves_rest_todo_then_resumes(exp_config, tmp_path, monkeypatch):
    """CAIN_RUN_BUDGET_S: no run starts once the session budget is spent; the next invocation of the same
    command resumes the TODO rows (studies longer than one allocation window)."""
    monkeypatch.setenv("CAIN_TEST_HANG", "")  # no hang
    monkeypatch.setenv("CAIN_RUN_BUDGET_S", "1e-9")  # spent after the first run
    cfg = _run(exp_config, isolation="inline")
    rows = CSVOutputManager(cfg.experiment_path).read_run_table()
    assert sum(r["__done"] is RunProgress.DONE for r in rows) == 1
    assert "after_experiment" not in (tmp_path / "events.log").read_text().split()
    monkeypatch.delenv("CAIN_RUN_BUDGET_S")
    cfg = _run(exp_config, isolation="inline")
    assert all(r["__done"] is RunProgress.DONE for r in CSVOutputManager(cfg.experiment_path).read_run_table())
    assert (tmp_path / "events.log").read_text().split().count("after_experiment") == 1


def test_resume_md5_mismatch_requires_consent(exp_config, monkeypatch):
    monkeypatch.setenv("CAIN_TEST_FAIL", "run_2_repetition_0")
    _run(exp_config)
    exp_config.write_text(CONFIG_SRC.replace("repetitions=1", "repetitions=1 ") + "\nX = 1\n")
    with pytest.raises(BaseError, match="md5sum mismatch"):
        _run(exp_config, assume_yes=False)
    _run(exp_config, assume_yes=True)  # continue, metadata rewritten


def test_validator_rejects_bad_attributes(tmp_path):
    class C:
        name = "x"
        results_output_path = tmp_path
        operation_type = "AUTO"          # not an OperationType (the reference's check was vacuous)
        time_between_runs_in_ms = 10

    with pytest.raises(ConfigInvalidError):
        ConfigValidator.validate_config(C(), quiet=True)
    C.operation_type = OperationType.AUTO
    (tmp_path / "a_file").write_text("x")
    C.results_output_path = tmp_path / "a_file" / "sub"      # parent is a regular file: not creatable
    with pytest.raises(ConfigInvalidError):
        ConfigValidator.validate_config(C(), quiet=True)


# ------------------------------------------------------------------ CLI / compat
def _cli(*args, cwd=None):
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    return subprocess.run([sys.executable, "-m", "cain_amd", *args], capture_output=True, text=True, cwd=cwd,
                          env=env, timeout=120)


def test_cli_help_config_create_dry_run(tmp_path):
    r = _cli("help")
    assert r.returncode == 0 and "config-create" in r.stdout and "serve" in r.stdout
    r = _cli("config-create", str(tmp_path))
    assert r.returncode == 0
    created = list(tmp_path.glob("RunnerConfig-*.py"))
    assert len(created) == 1
    r = _cli(str(created[0]), "--dry-run")
    assert r.returncode == 0 and "dry run: 3 runs" in r.stdout  # 6 combos minus 3 excluded
    r = _cli("no-such-command")
    assert r.returncode == 1 and "not recognised" in r.stdout


@pytest.mark.skipif(not REF_CONFIG.exists(), reason="reference checkout not mounted")
def test_reference_config_loads_unchanged():
    from cain_amd.runner.cli import build_config

    EventSubscriptionController.clear()
    cfg, md, _ = build_config(str(REF_CONFIG))
    table = cfg.create_run_table_model().generate_experiment_run_table()
    assert len(table) == 1260
    assert list(table[0]) == ["__run_id", "__done", "model", "method", "length", "topic", "execution_time",
                              "cpu_usage", "gpu_usage", "memory_usage", "codecarbon__energy_consumed"]
    assert cfg.time_between_runs_in_ms == 90000
    EventSubscriptionController.clear()


def test_compat_modules_expose_reference_names():
    compat.install()
    from ConfigValidator.Config.Models.OperationType import OperationType as OT
    from Plugins.Profilers import CodecarbonWrapper
    from ProgressManager.Output.OutputProcedure import OutputProcedure
    import dotenv

    assert OT is OperationType
    assert CodecarbonWrapper.DataColumns.ENERGY_CONSUMED.name == "codecarbon__energy_consumed"
    assert callable(OutputProcedure.console_log) and callable(dotenv.load_dotenv)


def test_reference_utility_modules_import_by_reference_names(tmp_path):
    from cain_amd.runner import compat

    compat.install()
    from ExperimentOrchestrator.Misc.DictConversion import class_to_dict
    from ExperimentOrchestrator.Misc.PathValidation import (is_path_creatable, is_path_exists_or_creatable,
                                                             is_path_exists_or_creatable_portable,
                                                             is_path_sibling_creatable, is_pathname_valid)

    class Cfg:
        name = "x"
        repetitions = 2

    assert class_to_dict(Cfg)["repetitions"] == 2
    assert is_pathname_valid(str(tmp_path / "x")) and not is_pathname_valid("")
    assert is_path_creatable(str(tmp_path / "new" / "dir")) and is_path_sibling_creatable(str(tmp_path / "f"))
    assert is_path_exists_or_creatable(tmp_path / "p") and is_path_exists_or_creatable_portable(str(tmp_path / "q"))

    class Cfg:
        name = "n"
        x = 3

    assert class_to_dict(Cfg())["x"] == 3
