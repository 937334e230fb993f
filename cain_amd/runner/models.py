"""Experiment-design value objects.

Parity map (reference ``experiment-runner/``):

=====================  ==================================================
this module            reference
=====================  ==================================================
``RunProgress``        ProgressManager/RunTable/Models/RunProgress.py:3-5
``OperationType``      ConfigValidator/Config/Models/OperationType.py:3-10
``FactorModel``        ConfigValidator/Config/Models/FactorModel.py:7-21
``RunTableModel``      ConfigValidator/Config/Models/RunTableModel.py:12-97
``RunnerContext``      ConfigValidator/Config/Models/RunnerContext.py:4-9
``Metadata``           ConfigValidator/Config/Models/Metadata.py:3-14
``SupportsStr``        ExtendedTyping/Typing.py:5-12
=====================  ==================================================

Run-table generation keeps the reference's exact row identity: the full
factorial in factor order (``itertools.product``), exclusions removed, then
``__run_id = run_{i}_repetition_{j}`` with repetitions as the OUTER loop, so a
shipped ``run_table.csv`` maps back to its factor levels.
Changes: a row matched by several exclusion combos is removed once (the
reference deletes by duplicated index and can drop a wrong row), exclusions
may name a factor by object or by name, and ``shuffle`` takes an optional
``seed`` (the reference's shuffle is unseeded).
"""
from __future__ import annotations

import itertools
import os
import random
from dataclasses import dataclass, field
from enum import Enum
from pathlib import Path
from typing import Any, Dict, Iterable, List, Mapping, Optional, Protocol, Sequence, Union, runtime_checkable

from .errors import BaseError


@runtime_checkable
class SupportsStr(Protocol):
    def __str__(self) -> str: ...


class RunProgress(Enum):
    TODO = 1
    DONE = 2


class OperationType(Enum):
    """AUTO: continue after the cooldown.  SEMI: raise ``RunnerEvents.CONTINUE``
    after each run so a hook can block for manual continuation."""
    AUTO = 1
    SEMI = 2


class FactorModel:
    def __init__(self, factor_name: str, treatments: Sequence[SupportsStr]):
        treatments = list(treatments)
        if len(set(map(_hashable, treatments))) != len(treatments):
            raise BaseError(f"Treatment levels for factor {factor_name} are not unique!")
        self._name = factor_name
        self._treatments = treatments

    @property
    def factor_name(self) -> str:
        return self._name

    @property
    def treatments(self) -> List[SupportsStr]:
        return self._treatments

    def __repr__(self) -> str:  # pragma: no cover - debugging aid
        return f"FactorModel({self._name!r}, {self._treatments!r})"


def _hashable(x):
    try:
        hash(x)
        return x
    except TypeError:
        return repr(x)


ExclusionSpec = Mapping[Union[FactorModel, str], Sequence[SupportsStr]]


class RunTableModel:
    def __init__(self,
                 factors: List[FactorModel],
                 exclude_variations: Optional[Iterable[ExclusionSpec]] = None,
                 repetitions: int = 1,
                 data_columns: Optional[List[str]] = None,
                 shuffle: bool = False,
                 seed: Optional[int] = None):
        exclude_variations = list(exclude_variations or [])
        data_columns = [] if data_columns is None else data_columns
        if repetitions < 1:
            raise BaseError("Negative number of repetitions detected!")
        names = [f.factor_name for f in factors]
        if len(set(names)) != len(names):
            raise BaseError("Duplicate factor name detected!")
        if len(set(data_columns)) != len(data_columns):
            raise BaseError("Duplicate data column detected!")
        reserved = {"__run_id", "__done"}
        if reserved & (set(names) | set(data_columns)):
            raise BaseError("Factor/data column names may not use the reserved names __run_id/__done")
        self._factors = list(factors)
        self._exclude = exclude_variations
        self._repetitions = repetitions
        # NB: returned by reference so plugins can append columns (reference
        # CodecarbonWrapper.py:75-78 relies on this aliasing).
        self._data_columns = data_columns
        self._shuffle = shuffle
        if seed is None and os.environ.get("CAIN_SHUFFLE_SEED"):
            seed = int(os.environ["CAIN_SHUFFLE_SEED"])
        self._seed = seed

    # -- accessors (reference names) --------------------------------------
    def get_factors(self) -> List[FactorModel]:
        return self._factors

    def get_data_columns(self) -> List[str]:
        return self._data_columns

    @property
    def repetitions(self) -> int:
        return self._repetitions

    @property
    def shuffle(self) -> bool:
        return self._shuffle

    def column_names(self) -> List[str]:
        return ["__run_id", "__done"] + [f.factor_name for f in self._factors] + list(self._data_columns)

    # -- generation --------------------------------------------------------
    def _factor_index(self, key: Union[FactorModel, str]) -> int:
        for i, f in enumerate(self._factors):
            if f is key or f.factor_name == key or (isinstance(key, FactorModel) and f.factor_name == key.factor_name):
                return i
        raise BaseError(f"exclude_variations names an unknown factor: {key!r}")

    def _excluded(self, combo: tuple) -> bool:
        for exclusion in self._exclude:
            idx = [self._factor_index(k) for k in exclusion.keys()]
            allowed = [list(v) for v in exclusion.values()]
            if all(combo[i] in levels for i, levels in zip(idx, allowed)):
                return True
        return False

    def variations(self) -> List[tuple]:
        """The filtered full factorial, in reference order (index i of ``run_i``)."""
        combos = itertools.product(*[f.treatments for f in self._factors])
        return [c for c in combos if not self._excluded(c)]

    def generate_experiment_run_table(self) -> List[Dict[str, Any]]:
        cols = self.column_names()
        nf = len(self._factors)
        variations = self.variations()
        table: List[Dict[str, Any]] = []
        for j in range(self._repetitions):
            for i, combo in enumerate(variations):
                row: Dict[str, Any] = {"__run_id": f"run_{i}_repetition_{j}", "__done": RunProgress.TODO}
                for k in range(nf):
                    row[cols[2 + k]] = combo[k]
                for dc in self._data_columns:
                    row[dc] = " "
                table.append(row)
        if self._shuffle:
            rng = random.Random(self._seed) if self._seed is not None else random
            rng.shuffle(table)
        return table


@dataclass
class RunnerContext:
    run_variation: Dict[str, Any]
    run_nr: int
    run_dir: Path
    #: added: rank / device of the data-parallel worker executing this run
    rank: int = 0
    device: Optional[str] = None
    extras: Dict[str, Any] = field(default_factory=dict)


class Metadata:
    """Config fingerprint (reference Metadata.py).  ``md5sum`` is raw bytes."""

    def __init__(self, md5sum: bytes, scheme: str = "ast-v2"):
        self._md5sum = md5sum
        self.scheme = scheme

    @property
    def md5sum(self) -> bytes:
        return self._md5sum

    @md5sum.setter
    def md5sum(self, v: bytes) -> None:
        self._md5sum = v

    def __eq__(self, other) -> bool:
        return isinstance(other, Metadata) and other._md5sum == self._md5sum

    def __repr__(self) -> str:  # pragma: no cover
        return f"Metadata({self._md5sum.hex()}, scheme={self.scheme})"
