"""Host-code sanitizers: the native energy sampler's producer thread and its concurrent
consumers under ThreadSanitizer, and the same stress under AddressSanitizer + UBSan.  GPU sanitizers are
not available on this pool; the HIP kernels are covered by the numerics tests instead."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "cain_amd" / "energy" / "csrc" / "sampler.cpp"
DRIVER = ROOT / "tests" / "csrc" / "sampler_stress.cpp"


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_energy_sampler_under_sanitizer(tmp_path, san):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = tmp_path / "stress"
    build = subprocess.run([cxx, "-O1", "-g", "-std=c++17", f"-fsanitize={san}", "-fno-omit-frame-pointer",
                            "-I/opt/rocm/include", str(DRIVER), str(SRC), "-o", str(exe), "-ldl", "-lpthread"],
                           capture_output=True, text=True, timeout=300)
    if build.returncode != 0 and "cannot find" in build.stderr and "san" in build.stderr:
        pytest.skip(f"sanitizer runtime for {san} not installed")
    assert build.returncode == 0, build.stderr[-3000:]
    env = {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1", "ASAN_OPTIONS": "detect_leaks=1",
           "UBSAN_OPTIONS": "halt_on_error=1 print_stacktrace=1", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    report = r.stdout + r.stderr
    assert r.returncode == 0, report[-4000:]
    assert "ThreadSanitizer" not in report and "AddressSanitizer" not in report and "runtime error" not in report
    assert "drained" in r.stdout
