"""In-tree build of the native libraries.

* ``cain_amd/ops/libcain_kernels.so`` — every HIP kernel + the decode runtime,
  compiled by ``hipcc --offload-arch=gfx950`` (cross-compiles without a GPU); no vendor
  GEMM library is linked;
* ``cain_amd/energy/libcain_energy.so`` — the amd-smi sampler (g++).

Both are plain C ABIs loaded with ctypes, so the build needs no torch headers
(fast, seconds per file) and the same ``.so`` is what tests and the bench load.
Usage: ``python -m cain_amd.build [--force] [-v]``.
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


def build_all(force: bool = False, verbose: bool = False) -> None:
    from .energy import native as energy_native

    energy_native.build(force=force, verbose=verbose)
    build_kernels(force=force, verbose=verbose)
    if verbose:
        print(f"built {KLIB} and {energy_native.LIB}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ns = ap.parse_args(argv)
    build_all(force=ns.force, verbose=ns.verbose)
    return 0


if __name__ == "__main__":
    sys.exit(main())
