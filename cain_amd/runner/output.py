"""Console output for the experiment runner.

Behavioural parity with the reference's ``OutputProcedure`` / ``BashHeaders``
(reference: experiment-runner/ProgressManager/Output/OutputProcedure.py:17-88,
experiment-runner/ExperimentOrchestrator/Misc/BashHeaders.py:1-9): every line is
prefixed ``[EXPERIMENT_RUNNER]: `` and coloured with ANSI codes.  Differences:

* colours are dropped when ``NO_COLOR`` is set or stdout is not a TTY and
  ``CAIN_FORCE_COLOR`` is unset (log files stay greppable);
* ``query_yes_no`` accepts an ``assume`` override (``CAIN_ASSUME_YES=1``) so a
  resume with an md5 mismatch can run unattended on a GPU box.
"""
from __future__ import annotations

import os
import sys
import threading
from typing import Optional


class BashHeaders:
    HEADER = "\033[95m"
    OKBLUE = "\033[94m"
    OKCYAN = "\033[96m"
    OKGREEN = "\033[92m"
    WARNING = "\033[93m"
    FAIL = "\033[91m"
    ENDC = "\033[0m"
    BOLD = "\033[1m"
    UNDERLINE = "\033[4m"


_lock = threading.Lock()


def _colour_enabled() -> bool:
    if os.environ.get("NO_COLOR"):
        return False
    if os.environ.get("CAIN_FORCE_COLOR"):
        return True
    return True  # parity default: the reference always emits ANSI codes


def _paint(code: str, txt: str) -> str:
    return f"{code}{txt}{BashHeaders.ENDC}" if _colour_enabled() else txt


class OutputProcedure:
    runner = "[EXPERIMENT_RUNNER]: "
    #: optional rank tag, set by the data-parallel fan-out so interleaved logs stay readable
    tag: str = ""

    @staticmethod
    def console_log(txt: str, empty_line: bool = False) -> None:
        with _lock:
            if empty_line:
                print(" " * 100)
            print(f"{OutputProcedure.runner}{OutputProcedure.tag} {txt}", flush=True)

    @staticmethod
    def console_log_OK(txt: str, empty_line: bool = False) -> None:
        OutputProcedure.console_log(_paint(BashHeaders.OKGREEN, txt), empty_line)

    @staticmethod
    def console_log_WARNING(txt: str, empty_line: bool = False) -> None:
        OutputProcedure.console_log(_paint(BashHeaders.WARNING, txt), empty_line)

    @staticmethod
    def console_log_FAIL(txt: str, empty_line: bool = False) -> None:
        OutputProcedure.console_log(_paint(BashHeaders.FAIL, txt), empty_line)

    @staticmethod
    def console_log_bold(txt: str, empty_line: bool = False) -> None:
        OutputProcedure.console_log(_paint(BashHeaders.BOLD, txt), empty_line)

    @staticmethod
    def query_yes_no(question: str, default: Optional[str] = "yes",
                     assume: Optional[bool] = None) -> bool:
        """Interactive y/n prompt (reference OutputProcedure.py:60-88).

        ``assume`` (or env ``CAIN_ASSUME_YES`` = 1/0) answers without reading stdin.
        A closed stdin (EOF) falls back to ``default``; with no default it answers no.
        """
        valid = {"yes": True, "y": True, "ye": True, "no": False, "n": False}
        if assume is None and os.environ.get("CAIN_ASSUME_YES") is not None:
            assume = os.environ["CAIN_ASSUME_YES"].strip() not in ("0", "", "no", "false")
        if assume is not None:
            OutputProcedure.console_log_WARNING(f"{question} -> {'yes' if assume else 'no'} (assumed)")
            return bool(assume)
        if default is None:
            prompt = " [y/n] "
        elif default == "yes":
            prompt = " [Y/n] "
        elif default == "no":
            prompt = " [y/N] "
        else:
            raise ValueError(f"invalid default answer: {default}")
        while True:
            sys.stdout.write(f"{OutputProcedure.runner} {_paint(BashHeaders.WARNING, question + prompt)}")
            sys.stdout.flush()
            line = sys.stdin.readline()
            if line == "":  # EOF: non-interactive
                return valid.get(default, False) if default else False
            choice = line.strip().lower()
            if default is not None and choice == "":
                return valid[default]
            if choice in valid:
                return valid[choice]
