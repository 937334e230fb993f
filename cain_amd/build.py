"""In-tree build of the native libraries.

* ``cain_amd/ops/libcain_kernels.so`` — every HIP kernel + the decode runtime,
  compiled by ``hipcc --offload-arch=gfx950`` (cross-compiles without a GPU); no vendor
  GEMM library is linked;
* ``cain_amd/ops/libcain_blas.so`` — OPT-IN (``--blas`` / ``CAIN_BUILD_BLAS=1``): the hipBLASLt
  A/B path (``ops/csrc_blas/blas.hip``), registered with the runtime by ``ops.enable_lt()``;
* ``cain_amd/energy/libcain_energy.so`` — the amd-smi sampler (g++).

Both are plain C ABIs loaded with ctypes, so the build needs no torch headers
(fast, seconds per file) and the same ``.so`` is what tests and the bench load.
Usage: ``python -m cain_amd.build [--force] [--blas] [-v]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path
from typing import List

ROOT = Path(__file__).resolve().parent
OPS = ROOT / "ops"
CSRC = OPS / "csrc"
KLIB = OPS / "libcain_kernels.so"
BLAS_SRC = OPS / "csrc_blas" / "blas.hip"
BLAS_LIB = OPS / "libcain_blas.so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def hipcc() -> str:
    for c in (os.path.join(ROCM, "bin", "hipcc"), shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the HIP kernels)")


def _sources() -> List[Path]:
    return sorted(CSRC.glob("*.hip"))


def _headers() -> List[Path]:
    return sorted(CSRC.glob("*.h"))


def _stale(target: Path, deps: List[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_kernels(force: bool = False, verbose: bool = False, jobs: int = 0) -> Path:
    srcs = _sources()
    hdrs = _headers()
    objdir = OPS / "build"
    objdir.mkdir(exist_ok=True)
    cc = hipcc()
    flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
             "-munsafe-fp-atomics", f"-I{CSRC}"]

    def compile_one(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        if force or _stale(obj, [src] + hdrs):
            cmd = [cc] + flags + ["-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
            if verbose and r.stderr.strip():
                print(r.stderr[-3000:])
        return obj

    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, srcs))
    if force or _stale(KLIB, objs):
        tmp = str(KLIB) + ".tmp"
        cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + [str(o) for o in objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(tmp, KLIB)
    return KLIB


def build_blas(force: bool = False, verbose: bool = False) -> Path:
    """The opt-in hipBLASLt A/B library (not part of the default build or the headline path)."""
    if not (force or _stale(BLAS_LIB, [BLAS_SRC] + _headers())):
        return BLAS_LIB
    tmp = str(BLAS_LIB) + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-shared", f"-I{CSRC}", str(BLAS_SRC),
           "-o", tmp, f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib", "-lhipblaslt"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {BLAS_SRC.name}:\n{r.stderr[-6000:]}")
    os.replace(tmp, BLAS_LIB)
    return BLAS_LIB


def build_all(force: bool = False, verbose: bool = False, blas: bool = False) -> None:
    from .energy import native as energy_native

    energy_native.build(force=force, verbose=verbose)
    build_kernels(force=force, verbose=verbose)
    if blas or os.environ.get("CAIN_BUILD_BLAS", "0") == "1":
        build_blas(force=force, verbose=verbose)
    if verbose:
        print(f"built {KLIB} and {energy_native.LIB}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--blas", action="store_true", help="also build the opt-in hipBLASLt A/B library")
    ns = ap.parse_args(argv)
    build_all(force=ns.force, verbose=ns.verbose, blas=ns.blas)
    return 0


if __name__ == "__main__":
    sys.exit(main())
