"""Energy sampler / meter / plugin on hosts without a GPU (the amd-smi path runs in the GPU tests)."""
import math
import time
from pathlib import Path

import pytest

from cain_amd.energy import DataColumns, EnergyMeter, emission_tracker, native
from cain_amd.energy.meter import EnergyReading
from cain_amd.energy.plugin import column_values
from cain_amd.energy.wattsup import WattsUpPro, parse_frame
from cain_amd.runner.models import FactorModel, RunnerContext, RunTableModel


def test_native_sampler_host_metrics():
    s = native.NativeSampler([], period_ms=10, fast_period_ms=1)
    s.start()
    x = 0
    t_end = time.time() + 0.15
    while time.time() < t_end:  # keep one core busy so cpu% > 0
        x += 1
    s.stop()
    smp = s.drain()
    s.close()
    assert len(smp) >= 5
    assert all(sm["gpu"] == -1 for sm in smp)
    mem = [sm["mem_pct"] for sm in smp]
    assert all(0 < m < 100 for m in mem)
    assert any(sm["cpu_pct"] > 0 for sm in smp if not math.isnan(sm["cpu_pct"]))


def test_meter_window_cpu_model_without_gpu():
    m = EnergyMeter(smi_indices=[], period_ms=10, cpu_tdp_w=100.0, sources=("gpu", "cpu"))
    m.start()
    time.sleep(0.2)
    r = m.stop(settle_ms=0)
    m.close()
    assert 0.19 < r.duration_s < 0.5
    assert r.gpu_energy_j == 0.0 and r.cpu_energy_source.split("(")[0] in ("model", "rapl", "hwmon", "amdsmi-cpu")
    assert r.total_energy_j == pytest.approx(r.gpu_energy_j + r.cpu_energy_j + r.ram_energy_j)
    assert 0 < r.memory_usage < 100


def test_cpu_energy_on_by_default_with_host_tdp(monkeypatch):
    """No readable counter (this container): the CPU-load model with this host's TDP is ON by default, so the
    client's CPU energy is never silently 0 (codecarbon's fallback)."""
    monkeypatch.delenv("CAIN_CPU_TDP_W", raising=False)
    m = EnergyMeter(smi_indices=[], period_ms=10)
    assert m.cpu_tdp_w > 0 and "ram" in m.sources and "cpu" in m.sources
    m.start()
    x, t_end = 0, time.time() + 0.3
    while time.time() < t_end:  # one busy core
        x += 1
    r = m.stop(settle_ms=0)
    m.close()
    if not m.host_source:
        assert r.cpu_energy_source.startswith("model")
    assert r.cpu_energy_j > 0 and r.ram_energy_j > 0
    assert r.total_energy_j == pytest.approx(r.gpu_energy_j + r.cpu_energy_j + r.ram_energy_j)


def test_host_share_scales_cpu_energy():
    full = EnergyMeter(smi_indices=[], period_ms=10, cpu_tdp_w=400.0, sources=("cpu",))
    half = EnergyMeter(smi_indices=[], period_ms=10, cpu_tdp_w=400.0, sources=("cpu",), host_share=0.5)
    samples = [{"t_ns": 0, "cpu_energy_j": float("nan")}]
    jf, _ = full._cpu_energy(samples, 2.0, 50.0)
    jh, _ = half._cpu_energy(samples, 2.0, 50.0)
    full.close(), half.close()
    assert jf == pytest.approx(400.0) and jh == pytest.approx(200.0)


def test_idle_subtraction_is_per_source():
    """A CPU-only window (the remote arm's client) must not subtract the GPU's idle board power
    (~300 W of GPU idle taken off CPU-only energy gave large negative idle_subtracted_J)."""
    m = EnergyMeter(smi_indices=[], period_ms=10, cpu_tdp_w=100.0, sources=("cpu",))
    m.idle_power_w = 300.0     # GPU idle board power of a GPU rank
    m.idle_cpu_power_w = 1.0   # CPU idle share
    m.start()
    time.sleep(0.2)
    r = m.stop(settle_ms=0)
    m.close()
    assert r.gpu_energy_j == 0.0
    assert r.idle_subtracted_j == pytest.approx(r.cpu_energy_j - 1.0 * r.duration_s)
    assert r.idle_subtracted_j > -1.0  # no GPU idle term


def test_native_wrap_accumulation():
    """RAPL energy_uj wraps at max_energy_range_uj: deltas accumulate modulo the range."""
    rng = 262143328850  # a typical package zone max_energy_range_uj
    raw = [rng - 3_000_000, rng - 1_000_000, 1_000_000, 4_000_000]
    assert native.wrap_accumulate(raw, rng) == pytest.approx(7.0)
    # unknown modulus: a backwards step is dropped, never turned into a huge positive delta
    assert native.wrap_accumulate([5_000_000, 1_000_000, 2_000_000], 0) == pytest.approx(1.0)


def test_meter_trims_the_counter_trace():
    m = EnergyMeter(smi_indices=[], period_ms=10, sources=("cpu",))
    calls = []
    m.sampler.trim = lambda t: calls.append(t)
    t0 = m.start()
    m.stop(settle_ms=0)
    m.close()
    assert calls and calls[0] <= t0


def test_column_values_units():
    r = EnergyReading(0, int(2e9), 2.0, gpu_energy_j=360.0, cpu_energy_j=36.0, ram_energy_j=0.0,
                      total_energy_j=396.0, cpu_energy_source="model", gpu_usage=50.0, cpu_usage=5.0,
                      memory_usage=40.0, gpu_power_w=180.0, vram_usage=1.0, idle_power_w=100.0,
                      idle_subtracted_j=196.0)
    v = column_values(r, [DataColumns.ENERGY_CONSUMED, DataColumns.ENERGY_USAGE_J, DataColumns.GPU_ENERGY,
                          DataColumns.IDLE_SUBTRACTED_J, DataColumns.EMISSIONS], country="NLD")
    assert v["codecarbon__energy_consumed"] == pytest.approx(396.0 / 3.6e6)
    assert v["energy_usage_J"] == 396.0 and v["idle_subtracted_J"] == 196.0
    assert v["codecarbon__gpu_energy"] == pytest.approx(1e-4)
    assert v["codecarbon__emissions"] == pytest.approx(396.0 / 3.6e6 * 0.328)


def test_plugin_decorator_adds_and_fills_columns(tmp_path):
    @emission_tracker(data_columns=[DataColumns.ENERGY_CONSUMED, DataColumns.ENERGY_USAGE_J],
                      country_iso_code="NLD", smi_indices=[], period_ms=10, cpu_tdp_w=50.0)
    class Cfg:
        name = "x"

        def create_run_table_model(self):
            self.run_table_model = RunTableModel([FactorModel("f", [1])], data_columns=["topic"])
            return self.run_table_model

        def start_measurement(self, ctx):
            self.started = True

        def stop_measurement(self, ctx):
            self.stopped = True

        def populate_run_data(self, ctx):
            return {"topic": "t"}

    c = Cfg()
    m = c.create_run_table_model()
    assert m.get_data_columns() == ["topic", "codecarbon__energy_consumed", "energy_usage_J"]
    ctx = RunnerContext({"__run_id": "r"}, 1, tmp_path)
    c.start_measurement(ctx)
    time.sleep(0.05)
    c.stop_measurement(ctx)
    d = c.populate_run_data(ctx)
    assert d["topic"] == "t" and d["energy_usage_J"] >= 0 and "codecarbon__energy_consumed" in d
    assert (Path(tmp_path) / "energy.json").exists()
    c.__energy_meter__.close()


class _FakeSerial:
    def __init__(self, lines):
        self.lines = list(lines)
        self.written = []

    def write(self, b):
        self.written.append(b)

    def readline(self):
        return self.lines.pop(0) if self.lines else b""


def test_wattsup_parsing_and_integration():
    assert parse_frame(b"#d,-,18,1234,2301,567,x;\n").watts == pytest.approx(123.4)
    assert parse_frame(b"garbage") is None
    frames = [b"#d,-,18,1000,2300,500;\n", b"#d,-,18,1000,2300,500;\n"]
    w = WattsUpPro(serial_port=_FakeSerial(frames), interval=1.0)
    s = w.log(timeout=0.05)
    assert len(s) == 2 and w.energy_j() >= 0.0
    assert w.s.written[0].startswith(b"#L,W,3,E")


def _burn(seconds: float) -> None:
    t = time.process_time()
    while time.process_time() - t < seconds:
        pass


def test_process_attribution_charges_the_client_tree_only():
    """cpu_attribution="process": a busy process outside the client's tree (reparented away by a double fork, like
    a co-located server or another rank) does not change the window's CPU energy; the client's own CPU time and
    that of a child it reaps inside the window do, at TDP / logical CPUs per CPU second."""
    import os
    import subprocess
    import sys

    tdp = 640.0
    m = EnergyMeter(smi_indices=[], sources=("cpu",), cpu_attribution="process", keep_samples=False, cpu_tdp_w=tdp)
    per_cpu_s = tdp / m.n_cpus
    try:
        m.start()
        time.sleep(0.6)
        quiet = m.stop()
        out = subprocess.run(["sh", "-c", f"{sys.executable} -c 'import time\nt=time.time()\n"
                                          f"while time.time()-t<4: pass' >/dev/null 2>&1 & echo $!"],
                             capture_output=True, text=True, check=True)
        busy_pid = int(out.stdout.strip())
        try:
            time.sleep(0.2)
            m.start()
            time.sleep(0.6)
            unrelated = m.stop()
        finally:
            os.kill(busy_pid, 9)
        assert quiet.cpu_energy_source.startswith("process(")
        assert quiet.client_cpu_s < 0.1 and unrelated.client_cpu_s < 0.1, (quiet.client_cpu_s, unrelated.client_cpu_s)
        assert unrelated.cpu_energy_j < 0.1 * per_cpu_s
        # the client's own work and a reaped child's
        m.start()
        _burn(0.4)
        subprocess.run([sys.executable, "-c", "import time\nt=time.process_time()\n"
                                              "while time.process_time()-t<0.4: pass"], check=True)
        own = m.stop()
        assert 0.7 < own.client_cpu_s < 2.5, own.client_cpu_s  # 0.8 s of work (+ the child's interpreter start)
        assert abs(own.cpu_energy_j - own.client_cpu_s * per_cpu_s) < 1e-6
    finally:
        m.close()


def test_process_attribution_excludes_subtrees():
    from cain_amd.energy.meter import process_tree

    import os
    import subprocess
    import sys

    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(5)"])
    try:
        tree = process_tree([os.getpid()])
        assert os.getpid() in tree and p.pid in tree
        assert p.pid not in process_tree([os.getpid()], exclude=[p.pid])
    finally:
        p.kill()
        p.wait()
