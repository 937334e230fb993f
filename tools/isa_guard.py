#!/usr/bin/env python3
"""Counted-wait guard for the weight-streaming kernels, read from the BUILT library's code objects.

The few-row stream kernels (gemm_w4.hip w4_stream_kernel) keep U weight loads in flight in a register ring and rely
on hipcc's counted ``s_waitcnt vmcnt(N)`` waits: when a change makes the compiler drain the ring (``vmcnt(0)``) at
every item, decode slows 5-13 % with every numerics test still green (round 5: a runtime split-K branch compiled
into every instance).  This tool pulls the gfx950 code objects out of ``libcain_kernels.so`` (the
``.hip_fatbin`` section: one clang offload bundle per translation unit), disassembles them with llvm-objdump, and
counts, per kernel, the ``vmcnt(0)`` waits inside loops (address ranges closed by a backward branch).

usage: python3 tools/isa_guard.py [--lib cain_amd/ops/libcain_kernels.so] [--filter w4_stream_kernel]
"""
from __future__ import annotations

import argparse
import os
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path
from typing import Dict, List, Tuple

ROOT = Path(__file__).resolve().parent.parent
LLVM = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib" / "llvm" / "bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib: Path, arch: str = "gfx950") -> List[bytes]:
    """Every device ELF for ``arch`` in the library's fat binary (offload bundles are 4 KiB-aligned in the section)."""
    with tempfile.TemporaryDirectory() as td:
        fat = Path(td) / "fat.bin"
        subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(lib),
                        str(Path(td) / "stripped")], check=True, capture_output=True)
        blob = fat.read_bytes()
    out = []
    at = blob.find(MAGIC)
    while at >= 0:
        n = struct.unpack_from("<Q", blob, at + len(MAGIC))[0]
        p = at + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith(arch) and size:
                out.append(blob[at + off:at + off + size])
        at = blob.find(MAGIC, at + len(MAGIC))
    return out


def disassemble(elf: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(elf)
        f.flush()
        return subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", f.name], check=True,
                              capture_output=True, text=True).stdout


_FUNC = re.compile(r"^([0-9a-f]+) <(\S+)>:$")
_INST = re.compile(r"^\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):(.*)$")
_TARGET = re.compile(r"<(\S+?)(?:\+0x([0-9a-f]+))?>")


def kernel_loop_waits(text: str, name_filter: str = "") -> Dict[str, Tuple[int, int]]:
    """name -> (instructions inside loops, vmcnt(0) waits inside loops)."""
    funcs: Dict[str, List[Tuple[int, str, str]]] = {}
    cur = None
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = m.group(2) if name_filter in m.group(2) else None
            if cur:
                funcs[cur] = []
            continue
        if cur is None:
            continue
        m = _INST.match(line)
        if m:
            funcs[cur].append((int(m.group(2), 16), m.group(1), m.group(3)))
    res = {}
    for name, insts in funcs.items():
        if not insts:
            continue
        base = insts[0][0]
        ranges = []
        for addr, ins, rest in insts:
            b = _TARGET.search(rest) if re.match(r"s_(c)?branch", ins) else None
            if b:
                tgt = base + int(b.group(2) or "0", 16)
                if b.group(1) == name and tgt <= addr:
                    ranges.append((tgt, addr))
        inside = [ins for addr, ins, _ in insts if any(lo <= addr <= hi for lo, hi in ranges)]
        res[name] = (len(inside), sum("vmcnt(0)" in i for i in inside))
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=str(ROOT / "cain_amd" / "ops" / "libcain_kernels.so"))
    ap.add_argument("--filter", default="w4_stream_kernel")
    ns = ap.parse_args(argv)
    for co in code_objects(Path(ns.lib)):
        for name, (n, w) in sorted(kernel_loop_waits(disassemble(co), ns.filter).items()):
            print(f"{name}  loop_insts={n}  loop_vmcnt0={w}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
