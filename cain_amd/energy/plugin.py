"""Energy-profiler plugin: class decorator that instruments a ``RunnerConfig``.

Drop-in for the reference's ``@CodecarbonWrapper.emission_tracker(...)``
(experiment-runner/Plugins/Profilers/CodecarbonWrapper.py:31-99): the same
decorator name, the same ``DataColumns`` enum with the same
``codecarbon__<name>`` column names, the same four hook wrappers —

(a) after ``create_run_table_model`` append the requested data columns,
(b) open the energy window *before* the user's ``start_measurement`` body,
(c) close it *after* the user's ``stop_measurement`` body,
(d) after ``populate_run_data`` fill the columns from the window.

— but backed by ``EnergyMeter`` (amd-smi hardware counters on a native
sampler thread) instead of codecarbon's estimate.  Extra columns the
reference lacks are opt-in members of ``DataColumns`` (``ENERGY_USAGE_J``,
``GPU_ENERGY_J``, ``CPU_ENERGY_J``, ``IDLE_SUBTRACTED_J``, ``AVG_GPU_POWER_W``,
``WINDOW_S``); the reference's kWh → J post-processing
(experiment/RunnerConfig.py:251-259) becomes the ``ENERGY_USAGE_J`` column.

Decorator kwargs: ``devices`` (HIP ordinals of the *measured device*),
``period_ms`` (slow-sample cadence, default 100 like powermetrics),
``cpu_tdp_w``, ``ram_w_per_gb``, ``sources``, ``country_iso_code`` (carbon
intensity for the EMISSIONS columns), ``save_samples`` (write
``energy_samples.csv`` into the run dir), ``idle_baseline_s`` (measure idle
power once in the first window's process).  A config may define
``energy_sources_for(context) -> ("gpu", "cpu", ...)`` to choose the measured
sources per run.  Unknown codecarbon kwargs are
accepted and ignored so reference configs load unchanged.
"""
from __future__ import annotations

import functools
import json
import math
import re
from enum import Enum
from typing import Any, Dict, Iterable, Optional

from .meter import EnergyMeter, EnergyReading, write_samples_csv

#: grid carbon intensity, kg CO2-eq per kWh (coarse public averages; override with carbon_intensity=)
CARBON_INTENSITY = {"NLD": 0.328, "DEU": 0.381, "FRA": 0.056, "USA": 0.369, "GBR": 0.207, "WORLD": 0.475}


class DataColumns(Enum):
    EMISSIONS = "codecarbon__emissions"
    EMISSIONS_RATE = "codecarbon__emissions_rate"
    CPU_ENERGY = "codecarbon__cpu_energy"
    GPU_ENERGY = "codecarbon__gpu_energy"
    RAM_ENERGY = "codecarbon__ram_energy"
    ENERGY_CONSUMED = "codecarbon__energy_consumed"
    # additions (new columns go after the reference ones)
    ENERGY_USAGE_J = "energy_usage_J"
    GPU_ENERGY_J = "gpu_energy_J"
    CPU_ENERGY_J = "cpu_energy_J"
    RAM_ENERGY_J = "ram_energy_J"
    CPU_ENERGY_SOURCE = "cpu_energy_source"
    IDLE_SUBTRACTED_J = "idle_subtracted_J"
    AVG_GPU_POWER_W = "avg_gpu_power_W"
    WINDOW_S = "energy_window_s"

    @property
    def name(self) -> str:  # reference: DataColumns.name is the column name
        return self.value

    @property
    def column(self) -> str:
        return self.value


_PATTERN = re.compile(r"(codecarbon__)(.+)")
_KWH = 1.0 / 3.6e6


def column_values(reading: EnergyReading, cols: Iterable[DataColumns], country: str = "WORLD",
                  carbon_intensity: Optional[float] = None) -> Dict[str, Any]:
    ci = carbon_intensity if carbon_intensity is not None else CARBON_INTENSITY.get(country, CARBON_INTENSITY["WORLD"])
    kwh = reading.total_energy_j * _KWH
    vals = {
        DataColumns.ENERGY_CONSUMED: kwh,
        DataColumns.CPU_ENERGY: reading.cpu_energy_j * _KWH,
        DataColumns.GPU_ENERGY: reading.gpu_energy_j * _KWH,
        DataColumns.RAM_ENERGY: reading.ram_energy_j * _KWH,
        DataColumns.EMISSIONS: kwh * ci,
        DataColumns.EMISSIONS_RATE: kwh * ci / reading.duration_s,
        DataColumns.ENERGY_USAGE_J: round(reading.total_energy_j, 3),
        DataColumns.GPU_ENERGY_J: round(reading.gpu_energy_j, 3),
        DataColumns.CPU_ENERGY_J: round(reading.cpu_energy_j, 3),
        DataColumns.RAM_ENERGY_J: round(reading.ram_energy_j, 3),
        DataColumns.CPU_ENERGY_SOURCE: reading.cpu_energy_source,
        DataColumns.IDLE_SUBTRACTED_J: (round(reading.idle_subtracted_j, 3)
                                        if not math.isnan(reading.idle_subtracted_j) else ""),
        DataColumns.AVG_GPU_POWER_W: (round(reading.gpu_power_w, 3) if not math.isnan(reading.gpu_power_w) else ""),
        DataColumns.WINDOW_S: round(reading.duration_s, 6),
    }
    return {c.value: vals[c] for c in cols}


def emission_tracker(online: bool = False, *decargs, **deckwargs):
    """Class decorator (reference signature ``emission_tracker(online=False, *args, **kwargs)``)."""
    data_columns = list(deckwargs.pop("data_columns", [DataColumns.EMISSIONS]))
    meter_kwargs = {k: deckwargs.pop(k) for k in ("devices", "smi_indices", "period_ms", "fast_period_ms",
                                                    "cpu_core", "cpu_tdp_w", "ram_w_per_gb", "sources", "host_share",
                                                    "cpu_attribution")
                    if k in deckwargs}
    country = deckwargs.pop("country_iso_code", "WORLD")
    carbon = deckwargs.pop("carbon_intensity", None)
    save_samples = deckwargs.pop("save_samples", True)
    idle_s = deckwargs.pop("idle_baseline_s", 0.0)
    # remaining codecarbon kwargs (project_name, output_dir, log_level, ...) are accepted and ignored

    def decorate(cls):
        cls.create_run_table_model = _add_columns(data_columns)(cls.create_run_table_model)
        cls.start_measurement = _start(meter_kwargs, idle_s)(cls.start_measurement)
        cls.stop_measurement = _stop(cls.stop_measurement)
        cls.populate_run_data = _populate(data_columns, country, carbon, save_samples)(cls.populate_run_data)
        cls.__energy_columns__ = [c.value for c in data_columns]
        cls.__energy_meter_kwargs__ = dict(meter_kwargs)
        cls.__energy_idle_s__ = idle_s
        return cls

    return decorate


def _add_columns(cols):
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(self, *a, **kw):
            fn(self, *a, **kw)
            dc = self.run_table_model.get_data_columns()
            for c in cols:
                if c.value not in dc:
                    dc.append(c.value)
            return self.run_table_model
        return wrapper
    return deco


def _meter_for(self, meter_kwargs, idle_s) -> EnergyMeter:
    meter = getattr(self, "__energy_meter__", None)
    if meter is None:
        kw = dict(getattr(self, "__energy_meter_kwargs__", None) or meter_kwargs)
        kw.setdefault("devices", getattr(self, "energy_devices", None))
        # the host's CPU energy is shared by the data-parallel ranks of the node
        kw.setdefault("host_share", 1.0 / max(1, int(getattr(self, "dp_world", 1) or 1)))
        kw.setdefault("cpu_attribution", getattr(self, "cpu_attribution", "system"))
        meter = EnergyMeter(**kw)
        if getattr(self, "idle_power_w", None) is not None:
            meter.idle_power_w = float(self.idle_power_w)
            meter.idle_cpu_power_w = float(getattr(self, "idle_cpu_power_w", float("nan")))
        elif idle_s:
            meter.measure_idle(idle_s)
            self.idle_power_w = meter.idle_power_w
            self.idle_cpu_power_w = meter.idle_cpu_power_w
        self.__energy_meter__ = meter
    return meter


def ensure_meter(config) -> EnergyMeter:
    """Create the decorated config's meter now (e.g. at START_RUN, so its start-up is not inside a window)."""
    return _meter_for(config, {}, getattr(config, "__energy_idle_s__", 0.0))


def measure_idle_baseline(config, seconds: float = 2.0) -> float:
    """Idle board power of the config's measured GPUs (W) and idle host CPU power (W, this rank's share),
    measured with a short-lived meter and stored as ``config.idle_power_w`` / ``config.idle_cpu_power_w`` —
    call it from BEFORE_EXPERIMENT, before any run and without leaving a sampler thread behind (forked run
    children could not use it)."""
    kw = dict(getattr(config, "__energy_meter_kwargs__", None) or {})
    kw.setdefault("devices", getattr(config, "energy_devices", None))
    kw.setdefault("host_share", 1.0 / max(1, int(getattr(config, "dp_world", 1) or 1)))
    kw.setdefault("cpu_attribution", getattr(config, "cpu_attribution", "system"))
    with EnergyMeter(**kw) as m:
        config.idle_power_w = m.measure_idle(seconds)
        config.idle_cpu_power_w = m.idle_cpu_power_w
    return config.idle_power_w


def _start(meter_kwargs, idle_s):
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(self, context, *a, **kw):
            meter = _meter_for(self, meter_kwargs, idle_s)
            pick = getattr(self, "energy_sources_for", None)
            if callable(pick):  # per-run measured sources (e.g. the remote arm: client CPU only)
                meter.sources = tuple(pick(context))
            procs = getattr(self, "cpu_processes_for", None)
            if callable(procs):  # process attribution: the client's process tree of this run
                meter.cpu_roots, meter.cpu_exclude = (list(x) for x in procs(context))
            meter.start()
            return fn(self, context, *a, **kw)
        return wrapper
    return deco


def _stop(fn):
    @functools.wraps(fn)
    def wrapper(self, context, *a, **kw):
        ret = fn(self, context, *a, **kw)
        self.__energy_reading__ = self.__energy_meter__.stop()
        return ret
    return wrapper


def _populate(cols, country, carbon, save_samples):
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(self, context, *a, **kw):
            ret = fn(self, context, *a, **kw) or {}
            reading: EnergyReading = self.__energy_reading__
            ret.update(column_values(reading, cols, country, carbon))
            try:
                with open(context.run_dir / "energy.json", "w") as fh:
                    json.dump(reading.as_dict(), fh, indent=1, default=str)
                if save_samples and reading.samples:
                    write_samples_csv(context.run_dir / "energy_samples.csv", reading.samples)
            except OSError:  # pragma: no cover
                pass
            return ret
        return wrapper
    return deco
