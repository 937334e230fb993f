"""Lifecycle event bus.

Reference: experiment-runner/EventManager/Models/RunnerEvents.py:3-13 and
EventManager/EventSubscriptionController.py:4-34.  Same public surface: one
callback per event held in a class-level registry (a later subscription
replaces the earlier one), ``raise_event`` returns the callback's value or
``None`` when nothing is subscribed.

Differences:
* the context is passed whenever it is not ``None`` (the reference tests
  truthiness, which would drop a falsy-but-valid context);
* ``snapshot()``/``restore()`` let a spawned worker process rebuild the
  registry (the reference relied on ``fork`` inheriting module state, which is
  not HIP-safe: SURVEY §7.4 item 5);
* the registry is guarded by a lock (runs may be dispatched from threads).
"""
from __future__ import annotations

import threading
from enum import Enum
from typing import Any, Callable, Dict, List, Optional, Tuple


class RunnerEvents(Enum):
    BEFORE_EXPERIMENT = 1
    BEFORE_RUN = 2
    START_RUN = 3
    START_MEASUREMENT = 4
    INTERACT = 5
    CONTINUE = 6
    STOP_MEASUREMENT = 7
    STOP_RUN = 8
    POPULATE_RUN_DATA = 9
    AFTER_EXPERIMENT = 10


#: per-run hook order executed by ``RunController`` (reference RunController.py:13-34)
RUN_HOOK_ORDER = (
    RunnerEvents.START_RUN,
    RunnerEvents.START_MEASUREMENT,
    RunnerEvents.INTERACT,
    RunnerEvents.STOP_MEASUREMENT,
    RunnerEvents.STOP_RUN,
    RunnerEvents.POPULATE_RUN_DATA,
)


class EventSubscriptionController:
    _registry: Dict[RunnerEvents, Callable] = {}
    _lock = threading.RLock()

    @staticmethod
    def subscribe_to_single_event(event: RunnerEvents, callback: Callable) -> None:
        with EventSubscriptionController._lock:
            EventSubscriptionController._registry[event] = callback

    @staticmethod
    def subscribe_to_multiple_events(subscriptions: List[Tuple[RunnerEvents, Callable]]) -> None:
        for event, callback in subscriptions:
            EventSubscriptionController.subscribe_to_single_event(event, callback)

    @staticmethod
    def raise_event(event: RunnerEvents, runner_context: Any = None) -> Any:
        with EventSubscriptionController._lock:
            cb = EventSubscriptionController._registry.get(event)
        if cb is None:
            return None
        return cb() if runner_context is None else cb(runner_context)

    @staticmethod
    def get_event_callback(event: RunnerEvents) -> Optional[Callable]:
        return EventSubscriptionController._registry.get(event)

    @staticmethod
    def clear() -> None:
        with EventSubscriptionController._lock:
            EventSubscriptionController._registry.clear()

    @staticmethod
    def snapshot() -> Dict[RunnerEvents, Callable]:
        with EventSubscriptionController._lock:
            return dict(EventSubscriptionController._registry)

    @staticmethod
    def restore(reg: Dict[RunnerEvents, Callable]) -> None:
        with EventSubscriptionController._lock:
            EventSubscriptionController._registry = dict(reg)
