"""Path validity / writability checks (reference ExperimentOrchestrator/Misc/PathValidation.py:14-149).

A pathname is valid if every component is ≤ NAME_MAX bytes and free of NUL, and creatable if the
nearest existing ancestor is a writable directory.  The reference's five public names exist here too
(``is_path_creatable``, ``is_path_sibling_creatable`` and the ``_portable`` variant included); unlike the
reference they accept ``Path`` objects, which is what made its writability check a no-op.
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


def is_path_creatable(pathname: str) -> bool:
    """True if the nearest existing ancestor directory of ``pathname`` is writable."""
    if not is_pathname_valid(pathname):
        return False
    anc = nearest_existing_ancestor(Path(os.path.expanduser(os.fspath(pathname))))
    return anc.is_dir() and os.access(anc, os.W_OK | os.X_OK)


def is_path_sibling_creatable(pathname: str) -> bool:
    """True if a file next to ``pathname`` could be created (its directory is writable)."""
    if not is_pathname_valid(pathname):
        return False
    parent = Path(os.path.abspath(os.path.expanduser(os.fspath(pathname)))).parent
    anc = nearest_existing_ancestor(parent)
    return anc.is_dir() and os.access(anc, os.W_OK | os.X_OK)


def is_path_exists_or_creatable_portable(pathname: str) -> bool:
    """Same answer as :func:`is_path_exists_or_creatable` by actually probing with a temporary file."""
    import tempfile

    if not is_pathname_valid(pathname):
        return False
    p = Path(os.path.abspath(os.path.expanduser(os.fspath(pathname))))
    if p.exists():
        return True
    try:
        with tempfile.TemporaryFile(dir=nearest_existing_ancestor(p)):
            return True
    except OSError:
        return False
