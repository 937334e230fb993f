"""The CAIN'25 study as a native RunnerConfig: on-device vs remote LLM content fetching.

Behaviour of the reference study (`experiment/RunnerConfig.py`):

* factors ``model`` (7 Ollama tags) × ``method`` ∈ {remote, on_device} × ``length`` ∈ {'100','500','1000'},
  30 repetitions, shuffled (:66-87);
* a run picks a topic from ``experiment/topics.csv`` and asks ``"In {length} words, please give me
  information about {topic}"`` over ``POST /api/generate`` with ``stream: false`` — to localhost for the
  on-device arm, to ``SERVER_IP`` (from ``.env``) for the remote arm (:106-131);
* the measurement window is the request (:133-175); ``execution_time`` runs from BEFORE_RUN to STOP_RUN
  (:98-103, :189-193, :224); CPU % / memory % are sampled while it runs, GPU % from powermetrics (:195-221);
* energy comes from the emission-tracker plugin (:28-31), converted to Joules (:239-259).

MI355X-native differences:

* the on-device arm is this framework's own decode engine behind an Ollama-compatible server started per
  data-parallel rank on that rank's GPU (``python -m cain_amd serve``, port ``port_base + 1 + rank``);
* a ``local:<device>`` remote arm is ONE engine server per node (port ``port_base + 101``), as the reference
  has one server every trial talks to (README.md:15-16).  In a data-parallel job its GPU is a dedicated
  server GPU: when ``<device>`` is also a client GPU, the rank that owns it hosts the server and measures
  nothing (N ranks -> N-1 clients), so no on-device window ever integrates the board energy of remote
  decodes; otherwise rank 0 starts it on the spare GPU.  The host publishes the URL on the job's store and
  every client rank reuses it.  A single-rank study may share its one GPU with the server (runs are strictly
  sequential); the remote arm's ``gpu_usage`` then stays the client's own residency (0) and the board's
  activity goes to ``server_gpu_usage``;
* energy is the CLIENT DEVICE's, with one definition in both arms and at every world size (the reference's
  codecarbon charged its one laptop whole, idle included, in both arms): the device's GPU board (amd-smi
  hardware accumulator; for the remote arm on a GPU shared with the server, the board's measured idle power x
  the window, ``gpu_energy_source = idle_model``) plus the client's CPU energy -- by default attributed to the
  client process tree (the rank's run process, its curl child and, for the on-device arm, its own local
  server: the reference's client laptop ran Ollama itself), CPU seconds x the per-CPU share of the socket TDP,
  so neither the remote server nor another rank's work is charged (``cpu_attribution``) -- and the client's
  RAM, on a native sampler thread (``cain_amd.energy``).  ``idle_subtracted_J`` subtracts the same idle
  baselines in both arms (a remote row's board part is then ~0);
* the response JSON is captured (the reference's curl printed it and dropped it), so the run table gains
  ``tokens_generated``, ``J_per_token``, ``tok_per_s``, ``ttft_s`` ... after the reference's columns;
* topics are drawn with a per-run seeded RNG (reproducible), prompts/lengths are the reference's.

Every setting can be overridden with ``CAIN_STUDY_<FIELD>`` environment variables (lists comma-separated),
e.g. ``CAIN_STUDY_MODELS=gemma:2b CAIN_STUDY_REPETITIONS=3 python -m cain_amd experiments/study.py``.
"""
from __future__ import annotations

import atexit
import csv
import dataclasses
import json
import math
import os
import random
import shutil
import signal
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional

from ..client import CurlRequest, OllamaClient, OllamaError
from ..energy import DataColumns, emission_tracker
from ..energy.plugin import ensure_meter, measure_idle_baseline
from ..models import STUDY_ORDER
from ..runner.events import EventSubscriptionController, RunnerEvents
from ..runner.models import FactorModel, OperationType, RunnerContext, RunTableModel
from ..runner.output import OutputProcedure as output
from ..utils.env import server_url

REPO_ROOT = Path(__file__).resolve().parents[2]
DEFAULT_TOPICS = REPO_ROOT / "experiments" / "topics.csv"

REFERENCE_COLUMNS = ["topic", "execution_time", "cpu_usage", "gpu_usage", "memory_usage"]
EXTRA_COLUMNS = ["tokens_generated", "prompt_tokens", "J_per_token", "tok_per_s", "ttft_s", "gen_time_s",
                 "server_total_s", "server_eval_s", "client_wall_s", "device", "server", "server_gpu_usage",
                 "idle_power_W", "dp_rank", "gpu_energy_source"]

#: c10d store key under which rank 0 publishes the node's one remote server URL ("error:<msg>" on failure)
REMOTE_URL_KEY = "cain/remote_url/{name}"
#: HBM of one MI355X: the budget of the co-located servers' memory-fit check
GPU_MEM_BYTES = 288 * 10**9


def server_footprint_bytes(models: List[str], max_batch: int, max_context: int, weights: str = "bf16",
                           kv: str = "bf16") -> int:
    """Device memory of one ``cain_amd serve --preload`` process: every model's weights (bf16 = 2 B / param; fp8 =
    1 B and MXFP4 = 0.53 B (e2m1 + one e8m0 scale per 32) per projection parameter, plus bf16 embeddings) and KV
    cache for max_batch x max_context, plus ~2 GB of workspaces and allocator slack per model."""
    from ..models.config import get_config

    per_param = {"bf16": 2.0, "fp8": 1.0, "fp4": 0.5 + 1.0 / 32}[weights]
    total = 0
    for m in models:
        cfg = get_config(m)
        wb = cfg.weight_bytes(2)
        if weights != "bf16":
            embed = cfg.vocab * cfg.d_model
            # the projections at per_param bytes beside the bf16 embedding
            wb = int((cfg.weight_bytes(1) - embed) * per_param) + 2 * embed
        if cfg.tie_embeddings:
            wb += cfg.vocab * cfg.d_model * 2  # the engine packs its own LM-head copy of a tied embedding
        total += wb + cfg.kv_bytes_per_token(1 if kv == "fp8" else 2) * max_batch * max_context + (2 << 30)
    return total


def _dist_store():
    """The c10d key-value store of the data-parallel job (None outside one)."""
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.distributed_c10d._get_default_store()
    except Exception:  # pragma: no cover
        pass
    return None


ENERGY_COLUMNS = [DataColumns.ENERGY_CONSUMED, DataColumns.ENERGY_USAGE_J, DataColumns.GPU_ENERGY_J,
                  DataColumns.CPU_ENERGY_J, DataColumns.RAM_ENERGY_J, DataColumns.IDLE_SUBTRACTED_J,
                  DataColumns.AVG_GPU_POWER_W, DataColumns.WINDOW_S, DataColumns.CPU_ENERGY_SOURCE]


@dataclass
class StudySettings:
    name: str = "new_runner_experiment"
    models: List[str] = field(default_factory=lambda: list(STUDY_ORDER))
    methods: List[str] = field(default_factory=lambda: ["remote", "on_device"])
    lengths: List[str] = field(default_factory=lambda: ["100", "500", "1000"])
    repetitions: int = 30
    shuffle: bool = True
    seed: Optional[int] = None
    cooldown_ms: int = 90000
    results_dir: str = str(REPO_ROOT / "experiments" / "experiments_output")
    topics_csv: str = str(DEFAULT_TOPICS)
    # on-device arm: a local server per rank
    device_backend: str = "auto"          # auto (hip on GPU, torch on CPU) | hip | torch | fake
    port_base: int = 11434
    max_batch: int = 4
    max_context: int = 2048
    preload: bool = True
    # remote arm: "" -> SERVER_IP from .env, else "fake" (modelled remote GPU server on this host's CPU),
    # "local:<device>" (an engine server on another device of this host) or an explicit URL
    remote: str = ""
    # backend of a "local:<device>" remote server ("" = the server's default for its device: hip on a GPU);
    # "fake" serves modelled generations (tests of the multi-rank plumbing)
    remote_backend: str = ""
    remote_fake_tok_s: float = 70.0       # RTX 4070-class llama-8B decode rate for the modelled server
    remote_fake_prefill_s: float = 0.15
    client: str = "curl"                  # curl (reference parity) | http (in-process client)
    # measurement window: "request" opens the energy window, then issues the request;
    # "reference" issues it in START_RUN first and opens the window afterwards, like the reference
    window: str = "request"
    # remote-arm trials on a shared host take a host-wide lock while measured, so concurrent ranks do
    # not load the CPU whose energy they are charged
    remote_exclusive: bool = True
    stream: bool = False
    request_timeout_s: float = 900.0
    server_start_timeout_s: float = 900.0
    # energy: idle board power measured once per rank after the servers are up and have settled (0 disables)
    idle_baseline_s: float = 3.0
    idle_settle_s: float = 5.0
    # tracing: the on-device server records each generation with torch.profiler and the
    # Chrome trace is filed as run_dir/kernel_trace.json (adds profiler overhead to the measured window)
    trace: bool = False
    # on-device weight storage: bf16, fp8 (e4m3 per-row scaled weights; W8A8 above 16 rows, W8A16 below) or fp4
    # (OCP MXFP4, the reference's 4-bit class: W4A16 up to 64 rows, W4A8 above)
    weights: str = "bf16"
    # on-device KV-cache storage: bf16, or fp8 (e4m3)
    kv: str = "bf16"
    # weight storage of a "local:<device>" remote server ("" = the on-device arm's ``weights``: the reference's
    # Ollama served the same 4-bit builds in both arms)
    remote_weights: str = ""
    # client CPU energy: "process" (the client process tree's CPU seconds x TDP per CPU) or "system" (this
    # rank's share of the whole host's CPU energy, the round-3 model)
    cpu_attribution: str = "process"

    @classmethod
    def from_env(cls, base: Optional["StudySettings"] = None) -> "StudySettings":
        s = dataclasses.replace(base) if base is not None else cls()
        for f in dataclasses.fields(cls):
            raw = os.environ.get(f"CAIN_STUDY_{f.name.upper()}")
            if raw is None:
                continue
            cur = getattr(s, f.name)
            if isinstance(cur, list):
                val: Any = [x.strip() for x in raw.split(",") if x.strip()]
            elif isinstance(cur, bool):
                val = raw.lower() in ("1", "true", "yes", "on")
            elif isinstance(cur, int) and f.name != "seed":
                val = int(raw)
            elif isinstance(cur, float):
                val = float(raw)
            elif f.name == "seed":
                val = int(raw) if raw else None
            else:
                val = raw
            setattr(s, f.name, val)
        return s


def load_topics(path) -> List[str]:
    with open(path, newline="", encoding="utf-8") as fh:
        return [row["Topic"] for row in csv.DictReader(fh) if row.get("Topic")]


def prompt_for(length: str, topic: str) -> str:
    return f"In {length} words, please give me information about " + topic


def _wait_alive(url: str, timeout_s: float, proc: Optional[subprocess.Popen] = None,
                models: Optional[List[str]] = None) -> None:
    """Wait until OUR server answers: the child must still run (a stale server of an earlier experiment on
    the same port answers too, and its bind failure kills ours) and it must list the expected models."""
    client = OllamaClient(url, timeout=5.0)
    t_end = time.time() + timeout_s
    while time.time() < t_end:
        if proc is not None and proc.poll() is not None:
            raise RuntimeError(f"server for {url} exited with {proc.returncode} (port in use? see its log)")
        if client.alive():
            if models and not set(models) <= set(client.tags()):
                raise RuntimeError(f"{url} serves {client.tags()}, expected {models}: another server owns the port")
            return
        time.sleep(0.5)
    raise RuntimeError(f"server {url} not up after {timeout_s:.0f} s")


class _ServerProc:
    """``python -m cain_amd serve ...`` as a child process in its own process group."""

    def __init__(self, args: List[str], log_path: Path, env: Optional[Dict[str, str]] = None, role: str = ""):
        self.role = role
        log_path.parent.mkdir(parents=True, exist_ok=True)
        self.log = open(log_path, "ab")
        e = dict(os.environ)
        e.setdefault("PYTHONPATH", str(REPO_ROOT))
        if env:
            e.update(env)
        self.proc = subprocess.Popen([sys.executable, "-m", "cain_amd", "serve", *args], stdout=self.log,
                                     stderr=subprocess.STDOUT, cwd=str(REPO_ROOT), env=e, start_new_session=True)

    def stop(self) -> None:
        if self.log.closed:
            return
        if self.proc.poll() is None:
            try:
                os.killpg(self.proc.pid, signal.SIGTERM)
                self.proc.wait(timeout=20)
            except (ProcessLookupError, subprocess.TimeoutExpired):
                try:
                    os.killpg(self.proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                self.proc.wait()
        self.log.close()


class _HttpRequest:
    """In-process client request on a thread (when curl is unavailable or client='http')."""

    def __init__(self, url: str, model: str, prompt: str, stream: bool, timeout_s: float):
        self.client = OllamaClient(url, timeout=timeout_s)
        self.args = (model, prompt, stream)
        self.result = None
        self.error: Optional[BaseException] = None
        self.thread = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        try:
            m, p, st = self.args
            self.result = self.client.generate(m, p, stream=st)
        except BaseException as exc:  # noqa: BLE001
            self.error = exc

    def start(self):
        self.thread.start()
        return self

    def running(self) -> bool:
        return self.thread.is_alive()

    def wait(self, timeout=None):
        self.thread.join(timeout)
        if self.thread.is_alive():
            raise OllamaError("request timed out")
        if self.error is not None:
            raise self.error
        return self.result

    def kill(self):
        pass


class _StudyBase:
    """Reference columns only; the energy plugin decorates this layer so its columns follow them."""

    SETTINGS = StudySettings()

    def __init__(self):
        self.settings = StudySettings.from_env(type(self).SETTINGS)
        s = self.settings
        self.name = s.name
        self.results_output_path = Path(s.results_dir)
        self.operation_type = OperationType.AUTO
        self.time_between_runs_in_ms = int(s.cooldown_ms)
        self.idle_power_w = None
        self.cpu_attribution = s.cpu_attribution
        # False on a rank that only hosts the node's remote server (parallel/fanout.py: it claims no runs)
        self.claims_runs = True
        # weights provenance, printed with the config at start: tag -> checkpoint (CAIN_CHECKPOINTS, models/hf.py);
        # tags not listed run random-init weights of their architecture
        from ..models.hf import registered_checkpoints
        self.checkpoints = registered_checkpoints()
        EventSubscriptionController.subscribe_to_multiple_events([
            (RunnerEvents.BEFORE_EXPERIMENT, self.before_experiment),
            (RunnerEvents.BEFORE_RUN, self.before_run),
            (RunnerEvents.START_RUN, self.start_run),
            (RunnerEvents.START_MEASUREMENT, self.start_measurement),
            (RunnerEvents.INTERACT, self.interact),
            (RunnerEvents.STOP_MEASUREMENT, self.stop_measurement),
            (RunnerEvents.STOP_RUN, self.stop_run),
            (RunnerEvents.POPULATE_RUN_DATA, self.populate_run_data),
            (RunnerEvents.AFTER_EXPERIMENT, self.after_experiment),
        ])
        self.run_table_model = None
        self._servers: List[_ServerProc] = []
        self._threads = []
        self.local_url: Optional[str] = None
        self.remote_url: Optional[str] = None
        self.remote_shares_gpu = False
        self.topics = load_topics(s.topics_csv)
        self.request = None
        self.response = None
        self.error: Optional[str] = None

    # ------------------------------------------------------------------ table
    def create_run_table_model(self) -> RunTableModel:
        s = self.settings
        self.run_table_model = RunTableModel(
            factors=[FactorModel("model", list(s.models)), FactorModel("method", list(s.methods)),
                     FactorModel("length", list(s.lengths))],
            data_columns=list(REFERENCE_COLUMNS), repetitions=int(s.repetitions), shuffle=s.shuffle, seed=s.seed)
        return self.run_table_model

    # ------------------------------------------------------------------ rank setup / teardown
    @property
    def rank(self) -> int:
        return int(getattr(self, "dp_rank", 0))

    def _gpu_index(self) -> Optional[int]:
        devs = getattr(self, "energy_devices", None)
        if devs:
            return int(devs[0])
        try:
            import torch

            return 0 if torch.cuda.device_count() > 0 else None  # device_count does not initialise HIP
        except Exception:  # pragma: no cover
            return None

    def _device_ordinal(self) -> Optional[int]:
        """This rank's GPU ordinal on the node: its measured device, else LOCAL_RANK in a data-parallel job
        (also on CPU, where the ordinal is the rank's slot), else the GPU of a single-rank study."""
        devs = getattr(self, "energy_devices", None)
        if devs:
            return int(devs[0])
        if int(getattr(self, "dp_world", 1) or 1) > 1:
            return int(os.environ.get("LOCAL_RANK", self.rank) or self.rank)
        return self._gpu_index()

    def _remote_host_dev(self) -> Optional[str]:
        """The ``local:<dev>`` remote server's device, when it is a GPU ordinal (else None)."""
        spec = self.settings.remote or ""
        if spec.startswith("local:") and spec.split(":", 1)[1].isdigit() and "remote" in self.settings.methods:
            return spec.split(":", 1)[1]
        return None

    def serves_remote_only(self) -> bool:
        """True on the rank of a data-parallel job whose GPU is the remote server's: it hosts the server and
        measures nothing, so no measured window shares a board with the server."""
        dev = self._remote_host_dev()
        world = int(getattr(self, "dp_world", 1) or 1)
        return dev is not None and world > 1 and self._device_ordinal() == int(dev)

    def before_experiment(self) -> None:
        s = self.settings
        log_dir = self.results_output_path / s.name / "servers"
        gpu = self._gpu_index()
        if self.serves_remote_only():
            self.claims_runs = False
            self.remote_url = self._node_remote_server(self._remote_host_dev(), log_dir)
            output.console_log_OK(f"rank {self.rank} hosts the node's remote server {self.remote_url} on its GPU "
                                  f"and claims no runs (dedicated server GPU)")
            return
        if "on_device" in s.methods:
            port = s.port_base + 1 + self.rank
            backend = s.device_backend
            device = f"cuda:{gpu}" if gpu is not None else "cpu"
            if backend == "auto":
                backend = "hip" if gpu is not None else "torch"
            args = ["--host", "127.0.0.1", "--port", str(port), "--models", ",".join(s.models),
                    "--device", device, "--max-batch", str(s.max_batch), "--max-context", str(s.max_context),
                    "--backend", backend]
            if s.preload and backend != "fake":
                args.append("--preload")
            if s.weights != "bf16":
                args += ["--weights", s.weights]
            if s.kv != "bf16":
                args += ["--kv", s.kv]
            if s.trace:
                args += ["--trace-dir", str(self.results_output_path / s.name / "traces" / f"rank{self.rank}")]
            env = {}
            if gpu is not None:
                # the server sees only this rank's GPU; the rank keeps addressing it by its own ordinal
                env = {"HIP_VISIBLE_DEVICES": str(gpu)}
                args[args.index("--device") + 1] = "cuda:0"
            srv = _ServerProc(args, log_dir / f"on_device_rank{self.rank}.log", env, role="on_device")
            self._servers.append(srv)
            atexit.register(srv.stop)  # never leave a server behind, even if the experiment dies
            self.local_url = f"http://127.0.0.1:{port}"
            output.console_log(f"starting on-device server {self.local_url} on {device} ({backend})")
            _wait_alive(self.local_url, s.server_start_timeout_s, srv.proc, list(s.models))
        if "remote" in s.methods:
            self.remote_url = self._start_remote(log_dir)
        output.console_log_OK(f"servers up: on_device={self.local_url} remote={self.remote_url}")
        if s.idle_baseline_s > 0 and self.idle_power_w is None:
            # models resident, nothing running: the idle_subtracted_J baseline of every later window (after
            # a settle period: right after loading, board power is still ~15 % above its idle floor)
            time.sleep(s.idle_settle_s)
            w = measure_idle_baseline(self, s.idle_baseline_s)
            output.console_log(f"idle baseline {w:.1f} W over {s.idle_baseline_s:.1f} s")

    def _start_remote(self, log_dir: Path) -> str:
        s = self.settings
        spec = s.remote or ""
        if not spec:
            try:
                return server_url("remote")  # SERVER_IP from the environment / .env, as the reference
            except RuntimeError:
                output.console_log_WARNING("SERVER_IP not set: the remote arm uses a modelled server on this host")
                spec = "fake"
        if spec == "fake":
            from ..serve import FakeBackend, ServerThread

            th = ServerThread(FakeBackend(list(s.models), tokens_per_s=s.remote_fake_tok_s,
                                          prefill_s=s.remote_fake_prefill_s), port=0).__enter__()
            self._threads.append(th)
            return th.url
        if spec.startswith("local:"):
            return self._node_remote_server(spec.split(":", 1)[1], log_dir)
        return spec if "://" in spec else f"http://{spec}"

    def _node_remote_server(self, dev: str, log_dir: Path) -> str:
        """ONE remote server per node, as the reference has one server every trial talks to
        (README.md:15-16, experiment/RunnerConfig.py:122-131): its host starts it on device ``dev`` and publishes
        its URL on the job's c10d store; the other ranks wait for that URL and reuse the server.  The host is the
        rank whose own GPU is ``dev`` (that rank then runs nothing else: ``serves_remote_only``), else rank 0
        (``dev`` is a spare GPU or not a GPU).  Before preloading, the footprint is checked against the card's
        HBM (plus the co-located on-device server's in a single-rank study sharing its GPU)."""
        s = self.settings
        world = int(getattr(self, "dp_world", 1) or 1)
        self.remote_shares_gpu = world == 1 and dev.isdigit() and self._gpu_index() == int(dev)
        store = _dist_store() if world > 1 else None
        key = REMOTE_URL_KEY.format(name=s.name)
        host_rank = int(dev) if (world > 1 and dev.isdigit() and int(dev) < world) else 0
        if self.rank != host_rank:
            if store is None:
                raise RuntimeError("a data-parallel rank > 0 needs the job's store to find the remote server")
            val = store.get(key).decode()  # blocks until rank 0 publishes (bounded by the store timeout)
            if val.startswith("error:"):
                raise RuntimeError(f"rank 0 could not start the remote server: {val[6:]}")
            _wait_alive(val, s.server_start_timeout_s, None, list(s.models))
            return val
        try:
            backend = s.remote_backend or ""
            rweights = s.remote_weights or s.weights
            if backend != "fake" and dev.isdigit():
                need = server_footprint_bytes(list(s.models), s.max_batch, s.max_context, rweights)
                # a data-parallel job never co-locates (the GPU's rank serves only); a single-rank study may
                co_located = "on_device" in s.methods and self.remote_shares_gpu
                if co_located:
                    need += server_footprint_bytes(list(s.models), s.max_batch, s.max_context, s.weights, s.kv)
                if need > GPU_MEM_BYTES:
                    raise RuntimeError(f"remote server on GPU {dev} needs {need / 1e9:.0f} GB"
                                       f"{' with the co-located on-device server' if co_located else ''}"
                                       f" > {GPU_MEM_BYTES / 1e9:.0f} GB of HBM")
            port = s.port_base + 101
            env = {"HIP_VISIBLE_DEVICES": dev} if dev.isdigit() else {}
            device = "cuda:0" if dev.isdigit() else dev
            args = ["--host", "127.0.0.1", "--port", str(port), "--models", ",".join(s.models), "--device", device,
                    "--max-batch", str(s.max_batch), "--max-context", str(s.max_context)]
            if backend:
                args += ["--backend", backend]
            if backend == "fake":
                args += ["--fake-tok-s", str(s.remote_fake_tok_s), "--fake-prefill-s", str(s.remote_fake_prefill_s)]
            else:
                args.append("--preload")
                if rweights != "bf16":
                    args += ["--weights", rweights]
            srv = _ServerProc(args, log_dir / "remote_node.log", env, role="remote")
            self._servers.append(srv)
            atexit.register(srv.stop)
            url = f"http://127.0.0.1:{port}"
            _wait_alive(url, s.server_start_timeout_s, srv.proc, list(s.models))
        except Exception as exc:
            if store is not None:
                store.set(key, f"error:{exc}")
            raise
        if store is not None:
            store.set(key, url)
        output.console_log(f"remote server {url} on device {dev} (one per node, shared by {getattr(self, 'dp_world', 1)} ranks)")
        return url

    def cpu_processes_for(self, context: RunnerContext):
        """(roots, excluded) of the client process tree whose CPU time a window is charged with: this run's process
        (curl / the in-process client are its descendants or threads) and, for the on-device arm, the rank's own
        local server -- the device's LLM runtime, as Ollama ran on the reference's laptop; every remote server
        subtree is excluded."""
        roots = [os.getpid()]
        local = [srv.proc.pid for srv in self._servers if getattr(srv, "role", "") == "on_device"]
        others = [srv.proc.pid for srv in self._servers if getattr(srv, "role", "") != "on_device"]
        if context.run_variation.get("method") == "on_device":
            roots += local
            return roots, others
        return roots, others + local

    def teardown_rank(self) -> None:
        for srv in self._servers:
            srv.stop()
        for th in self._threads:
            th.__exit__(None, None, None)
        self._servers, self._threads = [], []

    # ------------------------------------------------------------------ per-run hooks
    def before_run(self) -> None:
        self.timestamp_start = datetime.now()

    def start_run(self, context: RunnerContext) -> None:
        ensure_meter(self)  # sampler start-up stays outside the measurement window
        v = context.run_variation
        rng = random.Random(f"{self.settings.seed}:{v['__run_id']}")
        self.topic = rng.choice(self.topics)
        self.prompt = prompt_for(str(v["length"]), self.topic)
        url = self.local_url if v["method"] == "on_device" else self.remote_url
        if url is None:
            raise RuntimeError(f"no server for method {v['method']} (before_experiment not run?)")
        self.url = url
        self.response, self.error = None, None
        self.request = None
        self._model = v["model"]
        self._lock_window(context)
        if self.settings.window == "reference":
            self._issue()

    def _issue(self) -> None:
        s = self.settings
        if s.client == "curl" and shutil.which("curl"):
            self.request = CurlRequest(self.url, self._model, self.prompt, stream=s.stream,
                                       timeout_s=s.request_timeout_s).start()
        else:
            self.request = _HttpRequest(self.url, self._model, self.prompt, s.stream, s.request_timeout_s).start()

    def _lock_window(self, context: RunnerContext) -> None:
        """Host-wide exclusive lock for measured remote-arm windows when several ranks share the host
        (taken at the end of START_RUN, i.e. before the plugin opens the window; released in STOP_RUN)."""
        self._unlock_window()
        if not (self.settings.remote_exclusive and context.run_variation.get("method") == "remote"
                and int(getattr(self, "dp_world", 1)) > 1):
            return
        import fcntl

        path = self.results_output_path / self.settings.name / ".remote_window.lock"
        fh = open(path, "a")
        fcntl.flock(fh, fcntl.LOCK_EX)
        self._lock_fh = fh

    def _unlock_window(self) -> None:
        fh = getattr(self, "_lock_fh", None)
        if fh is not None:
            import fcntl

            fcntl.flock(fh, fcntl.LOCK_UN)
            fh.close()
            self._lock_fh = None

    def energy_sources_for(self, context: RunnerContext):
        """The client device's energy, ONE definition in both arms and at every world size, as codecarbon counted
        the reference's one laptop whole, idle included (CodecarbonWrapper.py:53-67): the device's GPU board +
        the client's CPU + RAM.  The board is measured, except for the remote arm when the remote server shares
        the client's GPU (a single-GPU study): the board then runs the server's decode, so the client's board is
        charged at its measured idle power over the window ("gpu_idle") -- the same quantity a data-parallel
        job measures on a client GPU that idles while its request runs on the dedicated server GPU."""
        if self._shared_remote(context):
            return ("gpu_idle", "cpu", "ram")
        return ("gpu", "cpu", "ram")

    def _shared_remote(self, context: RunnerContext) -> bool:
        return context.run_variation.get("method") == "remote" and self.remote_shares_gpu

    def gpu_energy_source(self, context: RunnerContext) -> str:
        """Provenance of the row's gpu_energy_J: "measured" (amd-smi accumulator) or "idle_model" (idle board
        power x window, the remote arm on a GPU shared with the server; "none(no idle baseline)" when that idle power
        was not measured, and the row then carries no board energy)."""
        if not self._shared_remote(context):
            return "measured"
        idle = self.idle_power_w
        if idle is None or math.isnan(float(idle)):
            return "none(no idle baseline)"
        return "idle_model"

    def start_measurement(self, context: RunnerContext) -> None:
        # the energy window (opened by the plugin just before this body) covers the request; with
        # window="request" the request is issued only now, so none of it runs outside the window
        if self.request is None:
            self._issue()
        try:
            self.response = self.request.wait(self.settings.request_timeout_s + 30)
        except OllamaError as exc:
            self.error = str(exc)

    def interact(self, context: RunnerContext) -> None:
        pass

    def stop_measurement(self, context: RunnerContext) -> None:
        if self.request is not None and self.request.running():
            self.request.kill()

    def stop_run(self, context: RunnerContext) -> None:
        self.timestamp_end = datetime.now()
        self._unlock_window()
        if self.error is not None:
            raise RuntimeError(f"request failed: {self.error}")

    def populate_run_data(self, context: RunnerContext) -> Optional[Dict[str, Any]]:
        r = getattr(self, "__energy_reading__", None)
        gpu = round(r.gpu_usage, 3) if r is not None and r.gpu_usage == r.gpu_usage else 0.0
        # gpu_usage is the CLIENT device's GPU residency (reference experiment/RunnerConfig.py:207-226: the M2's
        # own GPU while curl waited on the remote server).  When the remote server shares this rank's GPU the
        # board's activity is the server's: the client process never opens the GPU, so its own residency is 0 and
        # the measured activity goes to server_gpu_usage instead.
        shared = context.run_variation.get("method") == "remote" and self.remote_shares_gpu
        self._server_gpu_usage = gpu if shared else ""
        data: Dict[str, Any] = {
            "topic": self.topic,
            "execution_time": (self.timestamp_end - self.timestamp_start).total_seconds(),
            "cpu_usage": round(r.cpu_usage, 3) if r is not None else "",
            "gpu_usage": 0.0 if shared else gpu,
            "memory_usage": round(r.memory_usage, 3) if r is not None else "",
        }
        self._last_stats = self.response.stats() if self.response is not None else {}
        if r is not None and r.samples:  # reference run_dir/cpu_mem_usage.csv (RunnerConfig.py:146-168)
            try:
                with open(context.run_dir / "cpu_mem_usage.csv", "w") as fh:
                    fh.write("timestamp,cpu_usage,memory_usage\n")
                    for smp in r.samples:
                        if smp.get("gpu", -1) <= 0:  # one row per sampler tick (host-only or first GPU)
                            fh.write(f"{smp['t_ns'] / 1e9:.6f},{smp['cpu_pct']:.3f},{smp['mem_pct']:.3f}\n")
            except OSError:  # pragma: no cover
                pass
        try:
            (context.run_dir / "response.json").write_text(json.dumps(self.response.data if self.response else {},
                                                                      indent=1))
        except OSError:  # pragma: no cover
            pass
        trace = self._last_stats.get("trace_file")
        if trace and os.path.exists(trace):  # server-side profiler trace of this request (settings.trace)
            shutil.move(trace, context.run_dir / "kernel_trace.json")
        return data

    def after_experiment(self) -> None:
        """Writer only: derive ``energy_usage_J`` where missing (reference :239-259) and write the paper
        tables next to the run table (cain_amd.analysis)."""
        from ..analysis import analyze

        path = self.results_output_path / self.settings.name / "run_table.csv"
        try:
            analyze(path, path.parent / "analysis", quiet=True)
            output.console_log_OK(f"analysis tables written to {path.parent / 'analysis'}")
        except Exception as exc:  # noqa: BLE001 - analysis needs both arms / enough rows
            output.console_log_WARNING(f"analysis skipped: {exc}")


@emission_tracker(data_columns=ENERGY_COLUMNS, country_iso_code="NLD")
class _MeasuredStudy(_StudyBase):
    pass


class StudyConfig(_MeasuredStudy):
    """Reference columns, then the energy columns, then the measured-token columns."""

    def create_run_table_model(self) -> RunTableModel:
        m = super().create_run_table_model()
        dc = m.get_data_columns()
        for c in EXTRA_COLUMNS:
            if c not in dc:
                dc.append(c)
        return m

    def populate_run_data(self, context: RunnerContext) -> Optional[Dict[str, Any]]:
        data = super().populate_run_data(context)  # + energy columns (plugin)
        st = getattr(self, "_last_stats", {}) or {}
        tok = int(st.get("tokens_generated") or 0)
        e = data.get(DataColumns.ENERGY_USAGE_J.value)
        wall = st.get("client_wall_s") or 0.0
        data.update({
            "tokens_generated": tok,
            "prompt_tokens": int(st.get("prompt_tokens") or 0),
            "J_per_token": round(float(e) / tok, 6) if tok and e not in (None, "") else "",
            "tok_per_s": round(tok / wall, 3) if tok and wall else "",
            "ttft_s": round(st["ttft_s"], 6) if st.get("ttft_s") is not None else "",
            "server_total_s": round(st.get("server_total_s", 0.0), 6),
            "server_eval_s": round(st.get("server_eval_s", 0.0), 6),
            "client_wall_s": round(wall, 6),
            "gen_time_s": round(st.get("server_eval_s", 0.0) + st.get("server_prompt_eval_s", 0.0), 6),
            "device": str(getattr(self, "energy_devices", [""])[0]) if getattr(self, "energy_devices", None) else "",
            "server": self.url,
            "server_gpu_usage": getattr(self, "_server_gpu_usage", ""),
            "idle_power_W": round(float(self.idle_power_w), 2) if self.idle_power_w is not None else "",
            "dp_rank": self.rank,
            "gpu_energy_source": self.gpu_energy_source(context),
        })
        return data
