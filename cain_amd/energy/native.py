"""ctypes binding of the native sampler (``csrc/sampler.cpp`` → ``libcain_energy.so``).

The library is built in-tree by ``cain_amd.build`` (``python -m cain_amd.build``
or ``__graft_entry__.build()``); ``load()`` builds it on first use when a C++
compiler is present, so a fresh checkout works without an explicit step.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from pathlib import Path
from typing import List, Optional

HERE = Path(__file__).resolve().parent
LIB = HERE / "libcain_energy.so"
SRC = HERE / "csrc" / "sampler.cpp"


class ESample(ctypes.Structure):
    _fields_ = [
        ("t_ns", ctypes.c_uint64),
        ("gpu", ctypes.c_int32),
        ("pad", ctypes.c_int32),
        ("energy_j", ctypes.c_double),
        ("power_w", ctypes.c_double),
        ("gfx_pct", ctypes.c_double),
        ("umc_pct", ctypes.c_double),
        ("vram_pct", ctypes.c_double),
        ("cpu_pct", ctypes.c_double),
        ("mem_pct", ctypes.c_double),
        ("cpu_energy_j", ctypes.c_double),
    ]


SAMPLE_FIELDS = [f for f, _ in ESample._fields_ if f != "pad"]

_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None


def build(force: bool = False, verbose: bool = False) -> Path:
    if LIB.exists() and not force and LIB.stat().st_mtime >= SRC.stat().st_mtime:
        return LIB
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", f"-I{rocm}/include", "-o", str(LIB) + ".tmp",
           str(SRC), "-ldl", "-lpthread"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(str(LIB) + ".tmp", LIB)
    return LIB


def load() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB.exists() or LIB.stat().st_mtime < SRC.stat().st_mtime:
            build()
        lib = ctypes.CDLL(str(LIB))
        lib.es_init.restype = ctypes.c_int
        lib.es_last_error.restype = ctypes.c_char_p
        lib.es_gpu_count.restype = ctypes.c_int
        lib.es_gpu_bdf.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_uint32)] * 4
        lib.es_read_energy.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_float),
                                       ctypes.POINTER(ctypes.c_uint64)]
        lib.es_now_ns.restype = ctypes.c_uint64
        lib.es_create.restype = ctypes.c_void_p
        lib.es_create.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int]
        for fn in ("es_start", "es_stop", "es_num_tracked"):
            getattr(lib, fn).argtypes = [ctypes.c_void_p]
            getattr(lib, fn).restype = ctypes.c_int
        lib.es_destroy.argtypes = [ctypes.c_void_p]
        lib.es_energy_between.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        lib.es_energy_between.restype = ctypes.c_double
        lib.es_trace_points.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.es_trace_points.restype = ctypes.c_int64
        lib.es_trace.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        lib.es_trim.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        lib.es_drain.argtypes = [ctypes.c_void_p, ctypes.POINTER(ESample), ctypes.c_int]
        lib.es_dropped.argtypes = [ctypes.c_void_p]
        lib.es_dropped.restype = ctypes.c_uint64
        lib.es_sampler_tid.argtypes = [ctypes.c_void_p]
        lib.es_sampler_tid.restype = ctypes.c_long
        lib.es_host_energy_source.argtypes = [ctypes.c_void_p]
        lib.es_host_energy_source.restype = ctypes.c_char_p
        lib.es_test_wrap_accumulate.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_uint64]
        lib.es_test_wrap_accumulate.restype = ctypes.c_double
        if lib.es_sample_size() != ctypes.sizeof(ESample):
            raise RuntimeError("libcain_energy.so ABI mismatch (rebuild with python -m cain_amd.build)")
        _lib = lib
        return lib


def init() -> int:
    """Initialise amd-smi; returns the GPU count (0 if no GPU / library)."""
    lib = load()
    n = lib.es_init()
    return max(n, 0)


def gpu_bdfs() -> List[str]:
    lib = load()
    out = []
    for i in range(lib.es_gpu_count()):
        d, b, dv, f = (ctypes.c_uint32() for _ in range(4))
        if lib.es_gpu_bdf(i, ctypes.byref(d), ctypes.byref(b), ctypes.byref(dv), ctypes.byref(f)) == 0:
            out.append(f"{d.value:04x}:{b.value:02x}:{dv.value:02x}.{f.value:x}")
        else:
            out.append("")
    return out


def now_ns() -> int:
    return int(load().es_now_ns())


class NativeSampler:
    """Owns one native sampler thread tracking a set of amd-smi GPU indices."""

    def __init__(self, smi_indices: List[int], period_ms: float = 100.0, fast_period_ms: float = 1.0,
                 cpu_core: int = -1, ring_capacity: int = 1 << 16):
        self.lib = load()
        self.lib.es_init()
        arr = (ctypes.c_int * max(1, len(smi_indices)))(*smi_indices)
        self.h = self.lib.es_create(arr, len(smi_indices), int(period_ms * 1000), int(fast_period_ms * 1000),
                                    int(cpu_core), int(ring_capacity))
        if not self.h:
            raise RuntimeError("es_create failed")
        self.n = self.lib.es_num_tracked(self.h)
        self.running = False

    def start(self) -> None:
        if self.lib.es_start(self.h) != 0:
            raise RuntimeError("sampler already running")
        self.running = True

    def stop(self) -> None:
        if self.running:
            self.lib.es_stop(self.h)
            self.running = False

    def energy_between(self, slot: int, t0_ns: int, t1_ns: int) -> float:
        return float(self.lib.es_energy_between(self.h, slot, ctypes.c_uint64(t0_ns), ctypes.c_uint64(t1_ns)))

    def trace_points(self, slot: int) -> int:
        return int(self.lib.es_trace_points(self.h, slot))

    def trace(self, slot: int, max_points: int = 100000):
        ts = (ctypes.c_uint64 * max_points)()
        js = (ctypes.c_double * max_points)()
        n = self.lib.es_trace(self.h, slot, ts, js, max_points)
        return [(int(ts[i]), float(js[i])) for i in range(max(n, 0))]

    def trim(self, before_ns: int) -> None:
        self.lib.es_trim(self.h, ctypes.c_uint64(before_ns))

    @property
    def thread_id(self) -> int:
        """Kernel tid of the sampling thread (0 until it runs)."""
        return int(self.lib.es_sampler_tid(self.h))

    @property
    def host_energy_source(self) -> str:
        """Readable host CPU energy counter: "amdsmi-cpu", "rapl", "hwmon" or "" (none)."""
        return self.lib.es_host_energy_source(self.h).decode()

    def drain(self, max_samples: int = 65536) -> List[dict]:
        buf = (ESample * max_samples)()
        n = self.lib.es_drain(self.h, buf, max_samples)
        return [{f: getattr(buf[i], f) for f in SAMPLE_FIELDS} for i in range(max(n, 0))]

    def close(self) -> None:
        if self.h:
            self.stop()
            self.lib.es_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def wrap_accumulate(raw: List[int], modulus: int) -> float:
    """Joules the native wrap-aware accumulator makes of a raw microjoule counter sequence (tests)."""
    arr = (ctypes.c_uint64 * len(raw))(*raw)
    return float(load().es_test_wrap_accumulate(arr, len(raw), ctypes.c_uint64(modulus)))
