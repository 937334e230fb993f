"""Energy measurement windows.

``EnergyMeter`` is the object a run hook opens and closes around the
measured work.  It replaces three reference mechanisms at once:
codecarbon's whole-machine kWh estimate, the powermetrics GPU residency file
and the psutil cpu%/mem% loop.

Energy sources, per window:

* ``gpu``  — amd-smi energy accumulator of the tracked GPUs, integrated on the
  native sampler's piecewise-linear trace (exact counter deltas, interpolated
  at the window edges);
* ``cpu``  — RAPL package energy when ``/sys/class/powercap`` exposes it,
  otherwise a model ``cpu_tdp_w × mean CPU utilisation × duration``
  (codecarbon's fallback strategy; labelled ``cpu_energy_source = model``);
* ``ram``  — optional model ``ram_w_per_gb × GB × duration`` (codecarbon's
  3 W / 8 GB rule), off by default.

The window also reports the reference's utilisation columns: mean CPU %
(``cpu_usage``), mean GPU gfx activity % (``gpu_usage``, mean like the
reference — experiment/RunnerConfig.py:224-226), mean system memory %
(``memory_usage``) and idle-subtracted energy when an idle baseline was taken.
"""
from __future__ import annotations

import math
import os
import threading
import time
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Sequence

from . import native


def _env_float(name: str, default: float) -> float:
    try:
        return float(os.environ.get(name, default))
    except ValueError:
        return default


@dataclass
class EnergyReading:
    t_start_ns: int
    t_end_ns: int
    duration_s: float
    gpu_energy_j: float
    cpu_energy_j: float
    ram_energy_j: float
    total_energy_j: float
    cpu_energy_source: str
    gpu_usage: float          # mean gfx activity % of tracked GPUs
    cpu_usage: float          # mean host CPU %
    memory_usage: float       # mean host memory %
    gpu_power_w: float        # mean board power over the window (energy / time)
    vram_usage: float
    idle_power_w: float = float("nan")
    idle_subtracted_j: float = float("nan")
    gpu_counter_updates: int = 0
    per_gpu_energy_j: List[float] = field(default_factory=list)
    samples: List[dict] = field(default_factory=list)

    @property
    def kwh(self) -> float:
        return self.total_energy_j / 3.6e6

    def as_dict(self, with_samples: bool = False) -> Dict:
        d = asdict(self)
        if not with_samples:
            d.pop("samples")
        return d


def resolve_smi_indices(devices: Optional[Sequence[int]] = None) -> List[int]:
    """Map HIP device ordinals of this process to amd-smi GPU indices (by PCI BDF when torch
    already initialised HIP; otherwise by the visible-devices env, else identity)."""
    n = native.init()
    if n == 0:
        return []
    if devices is None:
        devices = [0]
    bdfs = native.gpu_bdfs()
    torch = None
    try:
        import sys
        torch = sys.modules.get("torch")
        if torch is not None and not torch.cuda.is_initialized():
            torch = None
    except Exception:
        torch = None
    out = []
    for d in devices:
        idx = None
        if torch is not None:
            p = torch.cuda.get_device_properties(d)
            want = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
            for i, b in enumerate(bdfs):
                if b.startswith(want):
                    idx = i
                    break
        if idx is None:
            vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") \
                or os.environ.get("CUDA_VISIBLE_DEVICES")
            if vis:
                ids = [int(x) for x in vis.split(",") if x.strip().isdigit()]
                idx = ids[d] if d < len(ids) else d
            else:
                idx = d
        if 0 <= idx < n:
            out.append(idx)
    return out


class EnergyMeter:
    """Sampler + window bookkeeping.  Use as ``with meter.window() as w: ...; w.reading``
    or explicitly ``start()`` / ``stop() -> EnergyReading``."""

    def __init__(self, devices: Optional[Sequence[int]] = None, smi_indices: Optional[Sequence[int]] = None,
                 period_ms: float = 100.0, fast_period_ms: float = 1.0, cpu_core: int = -1,
                 cpu_tdp_w: Optional[float] = None, ram_w_per_gb: float = 0.0,
                 sources: Sequence[str] = ("gpu", "cpu"), keep_samples: bool = True):
        self.smi = list(smi_indices) if smi_indices is not None else resolve_smi_indices(devices)
        self.sources = tuple(sources)
        self.cpu_tdp_w = cpu_tdp_w if cpu_tdp_w is not None else _env_float("CAIN_CPU_TDP_W", 0.0)
        self.ram_w_per_gb = ram_w_per_gb
        self.keep_samples = keep_samples
        self.sampler = native.NativeSampler(self.smi, period_ms=period_ms, fast_period_ms=fast_period_ms,
                                            cpu_core=cpu_core)
        self.sampler.start()
        self._t0: Optional[int] = None
        self.idle_power_w: float = float("nan")
        self._lock = threading.Lock()
        self._pending: List[dict] = []

    # -- lifecycle --------------------------------------------------------
    def close(self) -> None:
        self.sampler.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def n_gpus(self) -> int:
        return self.sampler.n

    def _collect(self) -> List[dict]:
        with self._lock:
            self._pending.extend(self.sampler.drain())
            return self._pending

    # -- idle baseline ----------------------------------------------------
    def measure_idle(self, seconds: float = 2.0) -> float:
        """Mean board power of the tracked GPUs while idle (W, summed over GPUs)."""
        if self.n_gpus == 0:
            self.idle_power_w = 0.0
            return 0.0
        t0 = native.now_ns()
        time.sleep(seconds)
        t1 = native.now_ns()
        time.sleep(0.05)  # let the counter tick past t1
        e = sum(self.sampler.energy_between(i, t0, t1) for i in range(self.n_gpus))
        self.idle_power_w = e / ((t1 - t0) * 1e-9)
        return self.idle_power_w

    # -- windows ----------------------------------------------------------
    def start(self) -> int:
        with self._lock:
            self._pending = []
        self.sampler.drain()  # discard samples before the window
        self._t0 = native.now_ns()
        return self._t0

    def stop(self, settle_ms: float = 25.0) -> EnergyReading:
        if self._t0 is None:
            raise RuntimeError("EnergyMeter.stop() without start()")
        t1 = native.now_ns()
        t0 = self._t0
        self._t0 = None
        # the accumulator updates every ~10-20 ms: wait for the update that covers t1
        if settle_ms > 0 and self.n_gpus:
            time.sleep(settle_ms / 1000.0)
        return self._reading(t0, t1)

    def reading_between(self, t0_ns: int, t1_ns: int) -> EnergyReading:
        return self._reading(t0_ns, t1_ns)

    def _reading(self, t0: int, t1: int) -> EnergyReading:
        dur = max(1e-9, (t1 - t0) * 1e-9)
        samples = [s for s in self._collect() if t0 <= s["t_ns"] <= t1 + 5_000_000]
        with self._lock:
            self._pending = [s for s in self._pending if s["t_ns"] > t1]
        per_gpu = [self.sampler.energy_between(i, t0, t1) for i in range(self.n_gpus)] if "gpu" in self.sources else []
        gpu_j = float(sum(x for x in per_gpu if not math.isnan(x))) if per_gpu else 0.0

        def mean(key, gpu_only=False):
            vals = [s[key] for s in samples if not math.isnan(s[key]) and (not gpu_only or s["gpu"] >= 0)]
            return float(sum(vals) / len(vals)) if vals else float("nan")

        cpu_pct = mean("cpu_pct")
        mem_pct = mean("mem_pct")
        if math.isnan(cpu_pct):
            cpu_pct = _instant_cpu_pct()
        if math.isnan(mem_pct):
            mem_pct = _instant_mem_pct()
        gfx = mean("gfx_pct", True)
        vram = mean("vram_pct", True)
        cpu_j, cpu_src = 0.0, "none"
        if "cpu" in self.sources:
            rapl = [s["cpu_energy_j"] for s in samples if not math.isnan(s["cpu_energy_j"])]
            if len(rapl) >= 2:
                cpu_j = (rapl[-1] - rapl[0]) * dur / max(1e-9, (samples[-1]["t_ns"] - samples[0]["t_ns"]) * 1e-9)
                cpu_src = "rapl"
            elif self.cpu_tdp_w > 0:
                cpu_j = self.cpu_tdp_w * (cpu_pct / 100.0 if not math.isnan(cpu_pct) else 0.0) * dur
                cpu_src = "model"
        ram_j = 0.0
        if "ram" in self.sources and self.ram_w_per_gb > 0:
            ram_j = self.ram_w_per_gb * _total_mem_gb() * dur
        total = gpu_j + cpu_j + ram_j
        idle_sub = float("nan")
        if not math.isnan(self.idle_power_w):
            idle_sub = total - self.idle_power_w * dur
        updates = 0
        if self.n_gpus:
            updates = self.sampler.trace_points(0)
        return EnergyReading(
            t_start_ns=t0, t_end_ns=t1, duration_s=dur, gpu_energy_j=gpu_j, cpu_energy_j=cpu_j, ram_energy_j=ram_j,
            total_energy_j=total, cpu_energy_source=cpu_src, gpu_usage=gfx, cpu_usage=cpu_pct, memory_usage=mem_pct,
            gpu_power_w=gpu_j / dur if self.n_gpus else float("nan"), vram_usage=vram,
            idle_power_w=self.idle_power_w, idle_subtracted_j=idle_sub, gpu_counter_updates=updates,
            per_gpu_energy_j=per_gpu, samples=samples if self.keep_samples else [])


def _instant_cpu_pct() -> float:
    try:
        import psutil
        return float(psutil.cpu_percent(interval=0.05))
    except Exception:  # pragma: no cover
        return float("nan")


def _instant_mem_pct() -> float:
    try:
        import psutil
        return float(psutil.virtual_memory().percent)
    except Exception:  # pragma: no cover
        return float("nan")


def _total_mem_gb() -> float:
    try:
        import psutil
        return psutil.virtual_memory().total / 2**30
    except Exception:  # pragma: no cover
        return 0.0


def write_samples_csv(path, samples: List[dict]) -> None:
    """Per-run raw samples (the reference kept ``cpu_mem_usage.csv`` per run,
    experiment/RunnerConfig.py:146-150)."""
    import csv

    cols = native.SAMPLE_FIELDS
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=cols)
        w.writeheader()
        for s in samples:
            w.writerow({k: s.get(k) for k in cols})
