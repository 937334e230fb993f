"""Energy measurement windows.

``EnergyMeter`` is the object a run hook opens and closes around the
measured work.  It replaces three reference mechanisms at once:
codecarbon's whole-machine kWh estimate, the powermetrics GPU residency file
and the psutil cpu%/mem% loop.

Energy sources, per window:

* ``gpu``  — amd-smi energy accumulator of the tracked GPUs, integrated on the
  native sampler's piecewise-linear trace (exact counter deltas, interpolated
  at the window edges);
* ``gpu_idle`` — the tracked GPUs charged at their measured idle board power x the window
  (``measure_idle``): the client device's board while another process -- a remote server
  co-located on the client's GPU -- runs on it, i.e. what the client's idle board costs;
* ``cpu``  — the host CPU energy counter the native sampler can read (amd-smi
  CPU sockets through HSMP, RAPL package zones, hwmon ``amd_energy``; wrap-aware),
  otherwise codecarbon's CPU-load model ``TDP × mean CPU utilisation × duration``
  with the TDP of this host's CPU model × sockets (``cpu_tdp_w`` / ``CAIN_CPU_TDP_W``
  override; labelled ``cpu_energy_source = model(...)``).  On by default;
* ``ram``  — codecarbon's 3 W per 8 GB rule applied to this process's resident
  memory (the client's share of the DIMMs, not the whole 3 TB host).

The host is shared by every rank of a node.  ``cpu_attribution="system"`` charges a
window ``host_share`` (1 / ranks per node) of the host-wide CPU energy;
``cpu_attribution="process"`` (the study's default) charges only the client's own
work: the CPU seconds the client process tree spent in the window (``cpu_roots``
and their descendants, minus ``cpu_exclude`` subtrees and the meter's own sampling
thread; from ``/proc/<pid>/stat`` utime + stime + the reaped children's cutime +
cstime) times the per-CPU share of the socket TDP -- codecarbon's CPU-load model
applied to the client's CPU time instead of the whole host's, so neither a
co-located server nor another rank's work is charged to the window (the
reference's client laptop ran none of the server, README.md:15-16).  Idle subtraction is per
source: a window charged with GPU and CPU energy subtracts the idle GPU and the
idle CPU power measured by ``measure_idle`` (never the GPU's idle power from a
CPU-only window).  Reference: codecarbon measured CPU + GPU + RAM of the client
(experiment-runner/Plugins/Profilers/CodecarbonWrapper.py:43-68).

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


#: TDP (W per socket) by CPU model substring, codecarbon-style (its cpu_power.csv); first match wins
CPU_TDP_TABLE = [("EPYC 9965", 500.0), ("EPYC 9755", 500.0), ("EPYC 9575F", 400.0), ("EPYC 9655", 400.0),
                 ("EPYC 9555", 360.0), ("EPYC 9654", 360.0), ("EPYC 9754", 360.0), ("EPYC 9474F", 360.0),
                 ("EPYC 9534", 280.0), ("EPYC 7763", 280.0), ("EPYC 7713", 225.0), ("Xeon(R) Platinum 8592", 350.0),
                 ("Xeon(R) Platinum 8480", 350.0), ("Xeon(R) Platinum 8380", 270.0), ("Apple M2", 20.0)]
DEFAULT_TDP_PER_SOCKET_W = 250.0
RAM_W_PER_GB = 3.0 / 8.0  # codecarbon's RAM rule


def host_cpu_tdp_w() -> tuple:
    """(total TDP in W, description) of this host's CPU sockets from /proc/cpuinfo."""
    model, sockets = "", set()
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name") and not model:
                    model = line.split(":", 1)[1].strip()
                elif line.startswith("physical id"):
                    sockets.add(line.split(":", 1)[1].strip())
    except OSError:
        pass
    n = max(1, len(sockets))
    per = next((w for key, w in CPU_TDP_TABLE if key in model), DEFAULT_TDP_PER_SOCKET_W)
    return per * n, f"{n}x {model or 'unknown CPU'} @ {per:.0f} W"


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
    host_share: float = 1.0
    idle_cpu_power_w: float = float("nan")
    sampler_core: int = -1    # CPU core the native sampler thread was pinned to
    client_cpu_s: float = float("nan")  # cpu_attribution="process": CPU seconds of the client process tree
    samples: List[dict] = field(default_factory=list)

    @property
    def kwh(self) -> float:
        return self.total_energy_j / 3.6e6

    def as_dict(self, with_samples: bool = False) -> Dict:
        d = asdict(self)
        if not with_samples:
            d.pop("samples")
        return d


def sampler_core(local_rank: Optional[int] = None, cpus: Optional[Sequence[int]] = None) -> int:
    """CPU core for this process's sampler thread: the ``local_rank``-th highest core of the affinity mask
    (``LOCAL_RANK`` by default), so the samplers of the ranks of one node each get a core of their own instead
    of all polling amd-smi on the mask's last core (the native default).  Wraps when there are more ranks than
    allowed cores; -1 when the mask is unknown (the native sampler then picks)."""
    if local_rank is None:
        try:
            local_rank = int(os.environ.get("LOCAL_RANK", "0") or 0)
        except ValueError:
            local_rank = 0
    if cpus is None:
        try:
            cpus = sorted(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            return -1
    cpus = sorted(int(c) for c in cpus)
    if not cpus:
        return -1
    return cpus[-1 - (max(0, int(local_rank)) % len(cpus))]


_CLK_TCK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100


def _stat_fields(path: str) -> Optional[List[str]]:
    """Fields after the ``(comm)`` of a /proc stat file (index 0 = state, 1 = ppid, 11 = utime, 12 = stime,
    13 = cutime, 14 = cstime), or None if it vanished."""
    try:
        with open(path, "rb") as fh:
            raw = fh.read().decode(errors="replace")
    except OSError:
        return None
    i = raw.rfind(")")
    return raw[i + 2:].split() if i >= 0 else None


def process_tree(roots: Sequence[int], exclude: Sequence[int] = ()) -> List[int]:
    """``roots`` and all their live descendants (one /proc scan), without the ``exclude`` pids' subtrees."""
    children: Dict[int, List[int]] = {}
    try:
        entries = os.listdir("/proc")
    except OSError:  # pragma: no cover
        return list(roots)
    for e in entries:
        if not e.isdigit():
            continue
        f = _stat_fields(f"/proc/{e}/stat")
        if f is not None and len(f) > 1:
            children.setdefault(int(f[1]), []).append(int(e))
    skip, out, todo = set(int(x) for x in exclude), [], [int(r) for r in roots]
    seen = set()
    while todo:
        p = todo.pop()
        if p in skip or p in seen:
            continue
        seen.add(p)
        out.append(p)
        todo.extend(children.get(p, ()))
    return out


def tree_cpu_seconds(roots: Sequence[int], exclude: Sequence[int] = (), skip_threads: Sequence[tuple] = ()) -> float:
    """CPU seconds (user + system, including reaped children) of the process tree of ``roots``, minus the
    ``(pid, tid)`` threads in ``skip_threads`` (e.g. the measurement's own sampler thread)."""
    ticks = 0
    for p in process_tree(roots, exclude):
        f = _stat_fields(f"/proc/{p}/stat")
        if f is not None and len(f) > 14:
            ticks += int(f[11]) + int(f[12]) + int(f[13]) + int(f[14])
    for pid, tid in skip_threads:
        if tid > 0:
            f = _stat_fields(f"/proc/{pid}/task/{tid}/stat")
            if f is not None and len(f) > 12:
                ticks -= int(f[11]) + int(f[12])
    return ticks / float(_CLK_TCK)


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
                 cpu_tdp_w: Optional[float] = None, ram_w_per_gb: float = RAM_W_PER_GB,
                 sources: Sequence[str] = ("gpu", "cpu", "ram"), keep_samples: bool = True,
                 host_share: float = 1.0, cpu_attribution: str = "system"):
        if cpu_attribution not in ("system", "process"):
            raise ValueError(f"cpu_attribution must be 'system' or 'process', got {cpu_attribution!r}")
        self.smi = list(smi_indices) if smi_indices is not None else resolve_smi_indices(devices)
        self.sources = tuple(sources)
        tdp, desc = host_cpu_tdp_w()
        env_tdp = _env_float("CAIN_CPU_TDP_W", 0.0)
        if cpu_tdp_w is not None or env_tdp > 0:
            tdp = float(cpu_tdp_w if cpu_tdp_w is not None else env_tdp)
            desc = f"configured {tdp:.0f} W"
        self.cpu_tdp_w, self.cpu_tdp_desc = tdp, desc
        self.ram_w_per_gb = ram_w_per_gb
        self.host_share = float(host_share)
        self.cpu_attribution = cpu_attribution
        # process attribution: the client's process tree (default: this process) and subtrees left out of it
        self.cpu_roots: Optional[List[int]] = None
        self.cpu_exclude: List[int] = []
        self.n_cpus = max(1, os.cpu_count() or 1)
        self._cpu0 = 0.0
        self.keep_samples = keep_samples
        if cpu_core is None or cpu_core < 0:
            cpu_core = sampler_core()
        self.cpu_core = int(cpu_core)
        self.sampler = native.NativeSampler(self.smi, period_ms=period_ms, fast_period_ms=fast_period_ms,
                                            cpu_core=cpu_core)
        self.sampler.start()
        self.host_source = self.sampler.host_energy_source
        self._t0: Optional[int] = None
        self._rss0 = 0.0
        self.idle_power_w: float = float("nan")      # idle GPU board power (W, summed over tracked GPUs)
        self.idle_cpu_power_w: float = float("nan")  # idle host CPU power charged to this meter (W, shared)
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
        """Idle baselines over one quiet window: GPU board power of the tracked GPUs (W, summed; the return value)
        and host CPU power as charged by ``_cpu_energy`` (W, this meter's share), each subtracted from its own
        source only."""
        self.start()
        time.sleep(seconds)
        r = self.stop(settle_ms=50.0)
        self.idle_power_w = r.gpu_energy_j / r.duration_s if self.n_gpus else 0.0
        self.idle_cpu_power_w = r.cpu_energy_j / r.duration_s
        return self.idle_power_w

    # -- windows ----------------------------------------------------------
    def start(self) -> int:
        with self._lock:
            self._pending = []
        self.sampler.drain()  # discard samples before the window
        self._t0 = native.now_ns()
        # bound the counter trace of a long-lived meter (a study keeps one for ~1,260 runs): keep 2 s of history
        # before the window for the interpolation at its left edge
        self.sampler.trim(max(0, self._t0 - 2_000_000_000))
        self._rss0 = _rss_gb()
        if self.cpu_attribution == "process":
            self._cpu0 = self._client_cpu_s()
        return self._t0

    def _client_cpu_s(self) -> float:
        roots = self.cpu_roots or [os.getpid()]
        return tree_cpu_seconds(roots, self.cpu_exclude, [(os.getpid(), self.sampler.thread_id)])

    def stop(self, settle_ms: float = 25.0) -> EnergyReading:
        if self._t0 is None:
            raise RuntimeError("EnergyMeter.stop() without start()")
        t1 = native.now_ns()
        cpu_s = self._client_cpu_s() - self._cpu0 if self.cpu_attribution == "process" else None
        t0 = self._t0
        self._t0 = None
        # the accumulator updates every ~10-20 ms: wait for the update that covers t1
        if settle_ms > 0 and self.n_gpus:
            time.sleep(settle_ms / 1000.0)
        return self._reading(t0, t1, cpu_s)

    def reading_between(self, t0_ns: int, t1_ns: int) -> EnergyReading:
        return self._reading(t0_ns, t1_ns)

    def _reading(self, t0: int, t1: int, client_cpu_s: Optional[float] = None) -> EnergyReading:
        dur = max(1e-9, (t1 - t0) * 1e-9)
        samples = [s for s in self._collect() if t0 <= s["t_ns"] <= t1 + 5_000_000]
        with self._lock:
            self._pending = [s for s in self._pending if s["t_ns"] > t1]
        per_gpu = [self.sampler.energy_between(i, t0, t1) for i in range(self.n_gpus)] if "gpu" in self.sources else []
        gpu_j = float(sum(x for x in per_gpu if not math.isnan(x))) if per_gpu else 0.0
        if "gpu_idle" in self.sources and self.n_gpus and not math.isnan(self.idle_power_w):
            # the client's board while another process (a co-located remote server) runs on it: charged at the
            # board's measured idle power, what the client device would have drawn waiting on a remote server
            gpu_j = self.idle_power_w * dur
            per_gpu = [gpu_j / self.n_gpus] * self.n_gpus

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
            cpu_j, cpu_src = self._cpu_energy(samples, dur, cpu_pct, client_cpu_s)
        ram_j = 0.0
        if "ram" in self.sources and self.ram_w_per_gb > 0:
            ram_j = self.ram_w_per_gb * 0.5 * (self._rss0 + _rss_gb()) * dur
        total = gpu_j + cpu_j + ram_j
        # idle subtraction per source: GPU idle only from GPU energy, CPU idle only from CPU energy; the RAM model
        # is the client's working set, charged as is
        idle_sub = float("nan")
        parts = []
        if ("gpu" in self.sources or "gpu_idle" in self.sources) and self.n_gpus:
            parts.append(gpu_j - self.idle_power_w * dur)
        if "cpu" in self.sources:
            parts.append(cpu_j - self.idle_cpu_power_w * dur)
        if parts and not any(math.isnan(x) for x in parts):
            idle_sub = float(sum(parts)) + ram_j
        updates = 0
        if self.n_gpus:
            updates = self.sampler.trace_points(0)
        return EnergyReading(
            t_start_ns=t0, t_end_ns=t1, duration_s=dur, gpu_energy_j=gpu_j, cpu_energy_j=cpu_j, ram_energy_j=ram_j,
            total_energy_j=total, cpu_energy_source=cpu_src, gpu_usage=gfx, cpu_usage=cpu_pct, memory_usage=mem_pct,
            gpu_power_w=gpu_j / dur if self.n_gpus else float("nan"), vram_usage=vram,
            idle_power_w=self.idle_power_w, idle_subtracted_j=idle_sub, gpu_counter_updates=updates,
            per_gpu_energy_j=per_gpu, host_share=self.host_share, idle_cpu_power_w=self.idle_cpu_power_w,
            sampler_core=self.cpu_core, client_cpu_s=float("nan") if client_cpu_s is None else client_cpu_s,
            samples=samples if self.keep_samples else [])

    def _cpu_energy(self, samples: List[dict], dur: float, cpu_pct: float, client_cpu_s: Optional[float] = None):
        """(joules, source) of CPU energy charged to a window of ``dur`` s.  Process attribution: the client tree's
        CPU seconds x (socket TDP / logical CPUs).  System attribution: the readable host counter's increase
        (rescaled from the sample span to the window), else the CPU-load model; times ``host_share``."""
        if client_cpu_s is not None:
            return (self.cpu_tdp_w / self.n_cpus * max(0.0, client_cpu_s),
                    f"process(client cpu-s x tdp {self.cpu_tdp_w:.0f} W / {self.n_cpus} cpus; {self.cpu_tdp_desc})")
        ctr = [s for s in samples if not math.isnan(s["cpu_energy_j"])]
        # one host sample per slow period (the per-GPU rows repeat it)
        seen, pts = set(), []
        for s in ctr:
            if s["t_ns"] not in seen:
                seen.add(s["t_ns"])
                pts.append((s["t_ns"], s["cpu_energy_j"]))
        if self.host_source and len(pts) >= 2 and pts[-1][0] > pts[0][0]:
            span = (pts[-1][0] - pts[0][0]) * 1e-9
            return (pts[-1][1] - pts[0][1]) * dur / span * self.host_share, self.host_source
        util = (cpu_pct / 100.0) if not math.isnan(cpu_pct) else 0.0
        return (self.cpu_tdp_w * util * dur * self.host_share,
                f"model(tdp {self.cpu_tdp_w:.0f} W x util; {self.cpu_tdp_desc})")


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


def _rss_gb() -> float:
    """Resident memory of this process (GB): the RAM model's working set."""
    try:
        with open("/proc/self/statm") as fh:
            return int(fh.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 1e9
    except (OSError, ValueError, IndexError):  # pragma: no cover
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
