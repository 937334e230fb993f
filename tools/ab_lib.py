#!/usr/bin/env python3
"""Build an A/B variant of the kernel library: the current objects with some sources taken from another git ref.

    python3 tools/ab_lib.py <name> <git-ref> <csrc file> [<csrc file> ...]
    -> ab/libcain_kernels_<name>.so, loaded in a GPU run with CAIN_KERNELS_LIB=ab/libcain_kernels_<name>.so

so that a kernel change and its predecessor run interleaved on one box (boxes differ by 1-3 %, profiles/r4)."""
from __future__ import annotations

import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from cain_amd import build as B  # noqa: E402


def main(argv) -> int:
    if len(argv) < 3:
        print(__doc__)
        return 2
    name, ref, files = argv[0], argv[1], argv[2:]
    B.build_kernels()
    objdir = B.OPS / "build"
    objs = {p.stem: p for p in objdir.glob("*.o")}
    cc = B.hipcc()
    flags = [f"--offload-arch={B.ARCH}", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", f"-I{B.CSRC}"]
    with tempfile.TemporaryDirectory() as td:
        for f in files:
            src = Path(td) / Path(f).name
            src.write_text(subprocess.run(["git", "show", f"{ref}:cain_amd/ops/csrc/{Path(f).name}"], cwd=ROOT,
                                          check=True, capture_output=True, text=True).stdout)
            obj = Path(td) / (src.stem + ".o")
            subprocess.run([cc] + flags + ["-c", str(src), "-o", str(obj)], check=True)
            objs[src.stem] = obj
        out = ROOT / "ab" / f"libcain_kernels_{name}.so"
        out.parent.mkdir(exist_ok=True)
        subprocess.run([cc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out)] +
                       [str(p) for p in objs.values()], check=True)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
