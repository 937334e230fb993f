"""Per-run process isolation.

Reference: ``@processify`` (experiment-runner/ExperimentOrchestrator/
Architecture/Processify.py:17-103) runs a function in a forked child and
ships ``(result, error)`` back over a ``multiprocessing.Queue``; the
controller wraps that in ANOTHER ``Process`` (ExperimentController.py:127-132),
so every run costs two forks and has no timeout.

Here one child per run is enough, and three modes exist:

``fork``   parity mode (default on Linux).  Refused once HIP is initialised in
           the parent — a HIP context does not survive ``fork`` (SURVEY §7.4
           item 5) — in which case ``inline`` is used and a warning printed.
``inline`` run in the calling process (GPU worker ranks, tests).
``spawn``  fresh interpreter; the callable and its arguments must pickle.

A timeout kills the child's whole process group (SIGKILL) so helper
processes it launched (curl, samplers) die with it, and raises
``RunTimeoutError``.  Exceptions re-raise in the parent with the child's
traceback text appended, like the reference.
"""
from __future__ import annotations

import functools
import inspect
import multiprocessing as mp
import os
import signal
import sys
import time
import traceback
from typing import Any, Callable, Optional

from .errors import RunTimeoutError
from .output import OutputProcedure as output


class _Sentinel:
    pass


def hip_initialised() -> bool:
    """True if this process has an initialised HIP runtime (fork-unsafe)."""
    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:  # pragma: no cover
        return False


def resolve_mode(mode: Optional[str]) -> str:
    mode = (mode or os.environ.get("CAIN_ISOLATION") or "fork").lower()
    if mode not in ("fork", "inline", "spawn"):
        raise ValueError(f"unknown isolation mode {mode!r}")
    if mode == "fork" and (hip_initialised() or "fork" not in mp.get_all_start_methods()):
        output.console_log_WARNING("HIP is initialised in this process: fork isolation is unsafe, running inline")
        return "inline"
    return mode


def _child_entry(conn, fn, args, kwargs, setpgrp: bool):
    if setpgrp:
        try:
            os.setpgrp()
        except OSError:  # pragma: no cover
            pass
    try:
        if inspect.isgeneratorfunction(fn):
            for item in fn(*args, **kwargs):
                conn.send((item, None))
            conn.send((_Sentinel, None))
        else:
            conn.send((fn(*args, **kwargs), None))
    except BaseException as exc:  # noqa: BLE001 - transported to parent
        tb = "".join(traceback.format_exception(type(exc), exc, exc.__traceback__))
        try:
            conn.send((None, (type(exc), str(exc), tb)))
        except Exception:  # unpicklable exception type
            conn.send((None, (RuntimeError, repr(exc), tb)))
    finally:
        conn.close()


def _raise_child(error) -> None:
    ex_type, msg, tb = error
    text = f"{msg} (in subprocess)\n{tb}"
    try:
        exc = ex_type(text)
    except Exception:
        exc = RuntimeError(text)
    raise exc


def _kill_group(proc) -> None:
    try:
        os.killpg(proc.pid, signal.SIGKILL)
    except (ProcessLookupError, PermissionError, OSError):
        try:
            proc.kill()
        except Exception:
            pass


def call_isolated(fn: Callable, *args, mode: Optional[str] = None, timeout: Optional[float] = None,
                  label: str = "run", **kwargs) -> Any:
    """Run ``fn(*args, **kwargs)`` under the chosen isolation and return its value."""
    mode = resolve_mode(mode)
    if mode == "inline":
        if inspect.isgeneratorfunction(fn):
            return list(fn(*args, **kwargs))
        return fn(*args, **kwargs)
    ctx = mp.get_context(mode)
    parent, child = ctx.Pipe(duplex=False)
    proc = ctx.Process(target=_child_entry, args=(child, fn, args, kwargs, True), daemon=False)
    proc.start()
    child.close()
    deadline = None if not timeout else time.monotonic() + timeout
    results = []
    try:
        while True:
            remaining = None if deadline is None else max(0.0, deadline - time.monotonic())
            if not parent.poll(remaining):
                if deadline is not None and time.monotonic() >= deadline:
                    _kill_group(proc)
                    proc.join(5)
                    raise RunTimeoutError(label, timeout)
                continue
            try:
                item, error = parent.recv()
            except EOFError:
                proc.join(5)
                raise RuntimeError(f"{label}: child process died (exit code {proc.exitcode}) without a result")
            if error is not None:
                proc.join(5)
                _raise_child(error)
            if inspect.isgeneratorfunction(fn):
                if item is _Sentinel:
                    proc.join()
                    return results
                results.append(item)
                continue
            proc.join()
            return item
    finally:
        if proc.is_alive():
            _kill_group(proc)
            proc.join(5)
        parent.close()


def processify(func: Callable) -> Callable:
    """Decorator form (reference-compatible name): always isolates in a child process."""

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        return call_isolated(func, *args, mode=kwargs.pop("_isolation", None),
                             timeout=kwargs.pop("_timeout", None), **kwargs)

    return wrapper
