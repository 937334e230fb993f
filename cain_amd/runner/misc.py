"""Small utilities of the reference's ``ExperimentOrchestrator`` kept for import parity.

* ``Singleton`` / ``SingletonABCMeta`` (reference ExperimentOrchestrator/Architecture/Singleton.py:3-15) —
  per-class instance caches; unused by the reference's runner (dead code) and by ours,
  provided so user configs that import them keep working.
* ``pop_from_each_dict_in_list`` (reference Misc/DictConversion.py:12-16, also dead there).
"""
from __future__ import annotations

import threading
from abc import ABCMeta
from typing import Any, Dict, List


class Singleton(type):
    """Metaclass: the first instantiation of a class is returned by every later call."""

    _instances: Dict[type, Any] = {}
    _lock = threading.Lock()

    def __call__(cls, *args, **kwargs):
        with Singleton._lock:
            if cls not in Singleton._instances:
                Singleton._instances[cls] = super().__call__(*args, **kwargs)
            return Singleton._instances[cls]


class SingletonABCMeta(ABCMeta):
    """``Singleton`` for abstract base classes."""

    _instances: Dict[type, Any] = {}
    _lock = threading.Lock()

    def __call__(cls, *args, **kwargs):
        with SingletonABCMeta._lock:
            if cls not in SingletonABCMeta._instances:
                SingletonABCMeta._instances[cls] = super().__call__(*args, **kwargs)
            return SingletonABCMeta._instances[cls]


def pop_from_each_dict_in_list(dicts: List[Dict[str, Any]], key: str) -> List[Dict[str, Any]]:
    """Remove ``key`` (if present) from every dict; returns the same list."""
    for d in dicts:
        d.pop(key, None)
    return dicts
