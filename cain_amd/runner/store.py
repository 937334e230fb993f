"""Persistence of experiment progress: ``run_table.csv`` + ``metadata.json``.

Reference behaviour kept (experiment-runner/ProgressManager/Output/
CSVOutputManager.py:13-65, JSONOutputManager.py:9-16):

* ``run_table.csv`` is the single source of truth for progress; ``__done`` is
  written as the enum *name* and parsed back to ``RunProgress``;
* on read, strings for which ``str.isnumeric()`` holds become ``int`` (all
  other values, including ``5.46E+01``, stay strings);
* ``update_row_data`` rewrites the row whose ``__run_id`` matches.

Fixed: the rewrite goes through a temp file in the SAME
directory followed by ``os.replace`` (atomic on POSIX; the reference moved a
``/tmp`` file across filesystems), keys a populate hook adds that are not yet
columns are appended to the header instead of producing a ragged CSV, and a
batch form ``update_rows`` lets the data-parallel rank-0 writer commit a whole
gather in one rewrite.

``metadata.json`` is written in the jsonpickle-compatible shape the reference
ships (``{"py/object": ..., "_md5sum": {"py/b64": ...}}``, see
experiment/experiments_output/new_runner_experiment/metadata.json:1-6) without
needing jsonpickle, and both the legacy and this module's object paths are
accepted on read.
"""
from __future__ import annotations

import base64
import csv
import io
import json
import os
import tempfile
import threading
from pathlib import Path
from typing import Any, Dict, Iterable, List, Optional

from .errors import ExperimentOutputFileDoesNotExistError
from .models import Metadata, RunProgress
from .output import OutputProcedure as output

RUN_TABLE = "run_table.csv"
METADATA = "metadata.json"


def _cell(v: Any) -> Any:
    if isinstance(v, RunProgress):
        return v.name
    return v


def _atomic_write_text(path: Path, text: str) -> None:
    path = Path(path)
    fd, tmp = tempfile.mkstemp(prefix=f".{path.name}.", suffix=".tmp", dir=str(path.parent))
    try:
        with os.fdopen(fd, "w", newline="") as fh:
            fh.write(text)
            fh.flush()
            os.fsync(fh.fileno())
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise


class BaseOutputManager:
    def __init__(self, experiment_path: Path):
        self._experiment_path = Path(experiment_path)

    @property
    def experiment_path(self) -> Path:
        return self._experiment_path


class CSVOutputManager(BaseOutputManager):
    _lock = threading.Lock()

    @property
    def path(self) -> Path:
        return self._experiment_path / RUN_TABLE

    # -- read ------------------------------------------------------------
    def read_run_table(self) -> List[Dict[str, Any]]:
        try:
            with open(self.path, "r", newline="") as fh:
                reader = csv.DictReader(fh)
                rows = []
                for row in reader:
                    for k, v in row.items():
                        if v is None:
                            continue
                        if k == "__done":
                            row[k] = RunProgress[v]
                        elif v.isnumeric():
                            row[k] = int(v)
                    rows.append(row)
                return rows
        except (OSError, KeyError) as exc:
            raise ExperimentOutputFileDoesNotExistError() from exc

    def read_header(self) -> List[str]:
        with open(self.path, "r", newline="") as fh:
            return next(csv.reader(fh))

    # -- write -----------------------------------------------------------
    @staticmethod
    def _render(fieldnames: List[str], rows: Iterable[Dict[str, Any]]) -> str:
        buf = io.StringIO()
        w = csv.DictWriter(buf, fieldnames=fieldnames, extrasaction="raise", lineterminator="\r\n")
        w.writeheader()
        for r in rows:
            w.writerow({k: _cell(r.get(k, "")) for k in fieldnames})
        return buf.getvalue()

    def write_run_table(self, run_table: List[Dict[str, Any]]) -> None:
        if not run_table:
            raise ExperimentOutputFileDoesNotExistError()
        fieldnames = list(run_table[0].keys())
        with self._lock:
            _atomic_write_text(self.path, self._render(fieldnames, run_table))

    def update_row_data(self, updated_row: Dict[str, Any]) -> None:
        self.update_rows([updated_row])
        output.console_log_WARNING(f"CSVManager: Updated row {updated_row['__run_id']}")

    def update_rows(self, updated_rows: List[Dict[str, Any]]) -> None:
        if not updated_rows:
            return
        by_id = {r["__run_id"]: r for r in updated_rows}
        with self._lock:
            with open(self.path, "r", newline="") as fh:
                reader = csv.DictReader(fh)
                fieldnames = list(reader.fieldnames or [])
                existing = [dict(r) for r in reader]
            for r in updated_rows:
                for k in r.keys():
                    if k not in fieldnames:
                        fieldnames.append(k)
            found = set()
            merged = []
            for row in existing:
                rid = row.get("__run_id")
                if rid in by_id:
                    found.add(rid)
                    new = dict(row)
                    new.update(by_id[rid])
                    merged.append(new)
                else:
                    merged.append(row)
            missing = set(by_id) - found
            if missing:
                raise KeyError(f"run ids not present in {self.path}: {sorted(missing)[:5]}")
            _atomic_write_text(self.path, self._render(fieldnames, merged))


class JSONOutputManager(BaseOutputManager):
    LEGACY_OBJECT = "ConfigValidator.Config.Models.Metadata.Metadata"
    OBJECT = "cain_amd.runner.models.Metadata"

    @property
    def path(self) -> Path:
        return self._experiment_path / METADATA

    def write_metadata(self, metadata: Metadata) -> None:
        doc = {
            "py/object": self.OBJECT,
            "_md5sum": {"py/b64": base64.b64encode(metadata.md5sum).decode("ascii")},
            "scheme": metadata.scheme,
        }
        _atomic_write_text(self.path, json.dumps(doc, indent=2))

    def read_metadata(self) -> Metadata:
        with open(self.path, "r") as fh:
            doc = json.load(fh)
        md5 = doc.get("_md5sum")
        if isinstance(md5, dict) and "py/b64" in md5:
            raw = base64.b64decode(md5["py/b64"])
        elif isinstance(md5, str):
            raw = bytes.fromhex(md5)
        else:
            raise ValueError(f"unrecognised metadata.json layout in {self.path}")
        scheme = doc.get("scheme") or ("legacy-dill" if doc.get("py/object") == self.LEGACY_OBJECT else "ast-v2")
        return Metadata(raw, scheme=scheme)


def read_run_table_frame(path: Path):
    """Convenience: the run table as a pandas DataFrame (analysis entry point)."""
    import pandas as pd

    p = Path(path)
    if p.is_dir():
        p = p / RUN_TABLE
    return pd.read_csv(p)
