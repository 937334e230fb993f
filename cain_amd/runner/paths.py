"""Path validity / writability checks (reference ExperimentOrchestrator/Misc/PathValidation.py:14-149).

Simplified to what the framework needs: a pathname is valid if every
component is ≤ NAME_MAX bytes and free of NUL, and creatable if the nearest
existing ancestor is a writable directory.
"""
from __future__ import annotations

import errno
import os
from pathlib import Path


def is_pathname_valid(pathname: str) -> bool:
    if not isinstance(pathname, (str, os.PathLike)):
        return False
    pathname = os.fspath(pathname)
    if not pathname or "\x00" in pathname:
        return False
    try:
        name_max = os.pathconf("/", "PC_NAME_MAX")
    except (OSError, ValueError, AttributeError):  # pragma: no cover
        name_max = 255
    return all(len(part.encode()) <= name_max for part in Path(pathname).parts if part not in ("/", ""))


def nearest_existing_ancestor(path: Path) -> Path:
    p = Path(os.path.abspath(path))
    while not p.exists():
        if p.parent == p:
            break
        p = p.parent
    return p


def is_path_exists_or_creatable(pathname: str) -> bool:
    if not is_pathname_valid(pathname):
        return False
    p = Path(os.path.abspath(os.path.expanduser(os.fspath(pathname))))
    if p.exists():
        return os.access(p if p.is_dir() else p.parent, os.W_OK)
    anc = nearest_existing_ancestor(p)
    return anc.is_dir() and os.access(anc, os.W_OK | os.X_OK)


def ensure_dir(path: Path) -> Path:
    try:
        Path(path).mkdir(parents=True, exist_ok=True)
    except OSError as exc:  # pragma: no cover
        if exc.errno != errno.EEXIST:
            raise
    return Path(path)
