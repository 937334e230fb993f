"""Ollama-compatible HTTP server over the decode engine.

The reference's both arms talk to an Ollama server on port 11434
(experiment/RunnerConfig.py:122-131; ``POST /api/generate`` with
``{"model", "prompt", "stream": false}``).  This module is that server, backed
by ``cain_amd.engine.DecodeEngine`` (HIP kernels on the GPU this process owns),
so the on-device arm (localhost) and the remote arm (another GPU / host) speak
the same protocol as the reference.  SURVEY §2.3 row 1, §5.8.

Endpoints: ``POST /api/generate`` (stream NDJSON or one JSON), ``POST /api/chat``,
``GET /api/tags``, ``POST /api/show``, ``GET /api/ps``, ``GET /api/version``,
``POST /api/pull`` (no-op: weights are random-init, nothing is downloaded),
``GET /`` ("Ollama is running").  Response statistics use Ollama's field names
and units (ns): ``total_duration``, ``load_duration``, ``prompt_eval_count``,
``prompt_eval_duration``, ``eval_count``, ``eval_duration``.

Concurrency: one worker thread per model owns the GPU work; HTTP handler
threads only enqueue and stream results back.  On the HIP backend the worker
runs **continuous batching** (``EngineBackend.serve_queue`` over
``engine.ContinuousBatch``): a request joins the running decode batch at the
next graph boundary (every ``steps_per_graph`` decode steps) and leaves it as
soon as it finishes, so a late request waits one chunk plus its own prefill
rather than the whole earlier batch.  Other backends (torch oracle, fake) and
``--static-batching`` collect the requests that arrive within
``batch_window_ms`` into one batch and run it to completion (trial batching on
the server side).

Tracing: started with ``--trace-dir DIR``, the engine backend records every decode batch
with ``torch.profiler`` (host ops + GPU kernels) and writes a Chrome trace to DIR; the response JSON
names it in ``cain_trace`` so the client can file it with its run (the study moves it into run_dir).

Length policy: random weights rarely emit EOS, so when a request does not set
``options.num_predict`` the server derives it from the prompt: "In N words ..."
(the study's prompt template, experiment/RunnerConfig.py:120) maps to
⌈4/3·N⌉ tokens; anything else gets 128 tokens.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import queue
import re
import sys
import threading
import time
from dataclasses import dataclass, field
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Callable, Dict, List, Optional

from ..models.tokenizer import StreamDecoder, tokens_for_words

VERSION = "0.5.0-cain-amd"
_WORDS = re.compile(r"\bin\s+(\d+)\s+words\b", re.IGNORECASE)
DEFAULT_NUM_PREDICT = 128


def default_num_predict(prompt: str) -> int:
    m = _WORDS.search(prompt or "")
    return tokens_for_words(int(m.group(1))) if m else DEFAULT_NUM_PREDICT


def _now() -> str:
    return datetime.datetime.now(datetime.timezone.utc).isoformat().replace("+00:00", "Z")


@dataclass
class Job:
    model: str
    prompt: Any                      # str or token ids
    num_predict: int
    options: Dict[str, Any]
    stream: Optional[Callable[[str], None]] = None   # receives text pieces
    done: threading.Event = field(default_factory=threading.Event)
    result: Any = None
    error: Optional[BaseException] = None
    t_submit: float = field(default_factory=time.perf_counter)
    trace_file: Optional[str] = None  # Chrome trace of the batch that decoded this job (--trace-dir)


class Backend:
    """Interface: decode a batch of jobs for one model."""

    def models(self) -> List[str]:
        raise NotImplementedError

    def run(self, model: str, jobs: List[Job]) -> None:
        raise NotImplementedError

    def prompt_for(self, model: str, body: Dict[str, Any], chat: bool) -> Any:
        """The decoder input of a request: Ollama's prompt handling.  A model without a chat template (every
        random-init tag) gets the text as given (a chat's turns as "role: content" lines); ``EngineBackend`` renders
        a checkpoint's template."""
        if chat:
            return "\n".join(f"{m.get('role', 'user')}: {m.get('content', '')}" for m in body.get("messages") or [])
        prompt = body.get("prompt", "")
        return f"{body['system']}\n{prompt}" if body.get("system") else prompt

    def max_batch(self, model: str) -> int:
        return 1

    def model_info(self, model: str) -> Dict[str, Any]:
        return {}


# Ollama's quantization_level names for the engine's weight storage
QUANT_LEVEL = {"bf16": "BF16", "fp8": "F8_E4M3", "fp4": "MXFP4"}


def register_checkpoints(specs: Optional[List[str]]) -> List[str]:
    """``--checkpoint TAG=PATH`` options: added to ``CAIN_CHECKPOINTS`` (so engines, and processes started from
    here, load the checkpoint for TAG; models/hf.py); returns the tags."""
    from ..models.hf import registered_checkpoints

    if not specs:
        return []
    os.environ["CAIN_CHECKPOINTS"] = ",".join(filter(None, [os.environ.get("CAIN_CHECKPOINTS", "")] + list(specs)))
    from ..models.hf import checkpoint_for

    registered_checkpoints()  # validates the syntax
    tags = [s.partition("=")[0].strip() for s in specs]
    for t in tags:
        try:
            path = checkpoint_for(t)  # resolves "ollama" entries to the local store's blob
        except (OSError, ValueError) as exc:
            raise SystemExit(f"--checkpoint {t}: {exc}")
        if not (os.path.isdir(path) or os.path.isfile(path)):
            raise SystemExit(f"--checkpoint {t}: {path} is neither a checkpoint directory nor a GGUF file")
    return tags


class EngineBackend(Backend):
    """Backed by one DecodeEngine per model on ``device`` (created on first use, then resident)."""

    def __init__(self, models: List[str], device: str = "cuda:0", max_batch: int = 16, max_context: int = 2048,
                 backend: Optional[str] = None, seed: int = 0, preload: bool = False, steps_per_graph: int = 8,
                 trace_dir: Optional[str] = None, weight_dtype: str = "bf16", continuous: bool = True,
                 kv_dtype: str = "bf16"):
        self._models = list(models)
        self.kv_dtype = kv_dtype
        # continuous batching needs the HIP engine; tracing records whole static batches
        self.continuous = continuous and not trace_dir
        self.weight_dtype = weight_dtype
        self.trace_dir = trace_dir
        self._trace_seq = 0
        self.device = device
        self._max_batch = max_batch
        self.max_context = max_context
        self.backend = backend
        self.seed = seed
        self.steps_per_graph = steps_per_graph
        self.engines: Dict[str, Any] = {}
        self._lock = threading.Lock()
        if preload:
            for m in self._models:
                self.engine(m)

    def models(self) -> List[str]:
        return list(self._models)

    def max_batch(self, model: str) -> int:
        return self._max_batch

    def engine(self, model: str):
        from ..engine import DecodeEngine

        with self._lock:
            eng = self.engines.get(model)
            if eng is None:
                if model not in self._models:
                    raise KeyError(f"model '{model}' not found, try pulling it first")
                eng = DecodeEngine(model, device=self.device, max_batch=self._max_batch,
                                   max_context=self.max_context, backend=self.backend, seed=self.seed,
                                   steps_per_graph=self.steps_per_graph, weight_dtype=self.weight_dtype,
                                   kv_dtype=self.kv_dtype)
                self.engines[model] = eng
            return eng

    def prompt_for(self, model: str, body: Dict[str, Any], chat: bool) -> Any:
        """As Ollama: a model with a chat template (a checkpoint's) gets ``/api/generate``'s prompt as one user turn
        (after ``system``) and ``/api/chat``'s messages through the template, with the generation prompt; ``raw``
        skips it.  The rendered text is tokenized without a second BOS (the template writes its own)."""
        from ..models.hf import checkpoint_for

        # only a checkpoint brings a template: random-init tags keep the lazy engine load in the scheduler thread
        tok = (getattr(self.engine(model), "tokenizer", None)
               if model in self._models and checkpoint_for(model) else None)
        if tok is None or not getattr(tok, "chat_template", None) or body.get("raw"):
            return super().prompt_for(model, body, chat)
        if chat:
            msgs = [{"role": m.get("role", "user"), "content": m.get("content", "")} for m in body.get("messages") or []]
        else:
            msgs = ([{"role": "system", "content": body["system"]}] if body.get("system") else []) + \
                   [{"role": "user", "content": body.get("prompt", "")}]
        return tok.encode(tok.render_chat(msgs), add_bos=False)

    def model_info(self, model: str) -> Dict[str, Any]:
        from ..models import get_config
        from ..models.hf import checkpoint_for

        cfg = get_config(model)
        ckpt = checkpoint_for(model)
        info = cfg.as_dict() | ({"checkpoint": ckpt} if ckpt else {"weights": "random-init"})
        out = {"details": {"family": cfg.family or cfg.name.split(":")[0],
                           "parameter_size": f"{cfg.n_params() / 1e9:.1f}B",
                           "quantization_level": QUANT_LEVEL[self.weight_dtype], "format": "cain-packed"},
               "model_info": info}
        if ckpt:  # as Ollama's show: the prompt template and the stop tokens (a checkpoint's)
            from ..models.hf import load_tokenizer

            tok = load_tokenizer(ckpt, cfg)
            if tok is not None:
                out["template"] = tok.chat_template or ""
                stops = [i for i in (cfg.eos_id, *cfg.stop_ids) if i >= 0]
                out["parameters"] = "\n".join(f"stop {json.dumps(tok.tok.id_to_token(i))}" for i in stops
                                               if tok.tok.id_to_token(i) is not None)
        return out

    def run(self, model: str, jobs: List[Job]) -> None:
        eng = self.engine(model)
        tok = eng.tokenizer
        streams = [j.stream for j in jobs]
        decs = [StreamDecoder(tok) for _ in jobs]

        def on_tokens(new_per_row: List[List[int]]) -> None:
            for j, d, ids in zip(jobs, decs, new_per_row):
                if j.stream is not None and ids:
                    piece = d.push(ids)
                    if piece:
                        j.stream(piece)

        def gen():
            return eng.generate([j.prompt for j in jobs], [j.num_predict for j in jobs], [j.options for j in jobs],
                                on_tokens=on_tokens if any(streams) else None)

        if self.trace_dir:
            res, path = self._traced(model, gen)
            for j in jobs:
                j.trace_file = path
        else:
            res = gen()
        ttft = getattr(eng, "last_ttft_ns", 0)
        for j, d, r in zip(jobs, decs, res):
            if j.stream is not None:
                tail = d.flush()  # text held back at a length cutoff inside a character
                if tail:
                    j.stream(tail)
            j.result = r
            j.ttft_ns = ttft


    def serve_queue(self, model: str, q: "queue.Queue[Job]") -> bool:
        """Continuous batching loop of one model (never returns on the HIP engine; False: not supported here,
        the scheduler falls back to static batches)."""
        eng = self.engine(model)
        if eng.backend != "hip":
            return False
        cb = eng.continuous()
        tok = eng.tokenizer
        # row -> {job, t0 (admission start), t_pre (prefill done), t_first (first token on the host)}
        live: Dict[int, Dict[str, Any]] = {}
        while True:
            pending: List[Job] = []
            if cb.n == 0:
                pending.append(q.get())  # idle: block for the next request
            while len(pending) < cb.capacity:
                try:
                    pending.append(q.get_nowait())
                except queue.Empty:
                    break
            try:
                self._cb_iteration(model, eng, cb, tok, live, pending)
            except Exception as exc:  # noqa: BLE001 - fail every request in flight, start a fresh batch
                for st in live.values():
                    st["job"].error = exc
                    st["job"].done.set()
                for j in pending:
                    if not j.done.is_set():
                        j.error = exc
                        j.done.set()
                live.clear()
                cb = eng.continuous()

    @staticmethod
    def _cb_iteration(model: str, eng, cb, tok, live: Dict[int, Dict[str, Any]], pending: List[Job]) -> None:
        """One continuous-batching iteration: admit ``pending`` (each request validated on its own: a prompt over
        the context fails that request only), then one graph chunk over every live row, then hand out tokens and
        finish the rows that are done.  Timing matches the static path (engine._generate_hip): the newly admitted
        rows' first token is decoded by a one-step graph and synchronised, so ``t_first`` is exact;
        ``eval_duration`` runs from the end of admission (first token included), ``ttft`` from its start."""
        from ..engine.engine import GenResult, _stopped

        ok: List[Job] = []
        ids: List[List[int]] = []
        for j in pending:
            try:
                p = eng.encode(j.prompt) or [eng.cfg.bos_id]
                if len(p) >= eng.T_max:
                    raise ValueError(f"prompt of {len(p)} tokens exceeds the context ({eng.T_max})")
            except Exception as exc:  # noqa: BLE001 - reported to this request only
                j.error = exc
                j.done.set()
                continue
            ok.append(j)
            ids.append(p)
        if ok:
            t0 = time.perf_counter_ns()
            rows = cb.admit(ids, [j.num_predict for j in ok], [j.options for j in ok])
            eng.stream.synchronize()
            t_pre = time.perf_counter_ns()
            cb.step(1)  # the new rows' first token on its own (the live rows advance one step with them)
            eng.stream.synchronize()
            t_first = time.perf_counter_ns()
            for r, j in zip(rows, ok):
                live[r] = {"job": j, "t0": t0, "t_pre": t_pre, "t_first": t_first, "dec": StreamDecoder(tok)}
        cb.step()
        new, fin = cb.poll()
        now = time.perf_counter_ns()
        for r, new_ids in enumerate(new):
            if new_ids and live[r]["job"].stream is not None:
                piece = live[r]["dec"].push(new_ids)
                if piece:
                    live[r]["job"].stream(piece)
        done_rows = [r for r, f in enumerate(fin) if f]
        for r in done_rows:
            st, j = live[r], live[r]["job"]
            toks = cb.tokens(r)
            if j.stream is not None:
                tail = st["dec"].flush()
                if tail:
                    j.stream(tail)
            reason = "stop" if _stopped(toks, cb.options[r]) else "length"
            j.result = GenResult(model, list(cb.prompt_tokens[r]), toks, tok.decode(toks), reason,
                                 load_duration_ns=0, prompt_eval_duration_ns=int(st["t_pre"] - st["t0"]),
                                 eval_duration_ns=int(now - st["t_pre"]),
                                 total_duration_ns=int(now - j.t_submit * 1e9))
            j.ttft_ns = int(st["t_first"] - st["t0"])
            j.done.set()
        if done_rows:
            moves = cb.retire(done_rows)
            kept = {moves.get(r, r): st for r, st in live.items() if r not in set(done_rows)}
            live.clear()
            live.update(kept)

    def _traced(self, model: str, fn):
        """Run ``fn`` under torch.profiler (CPU + GPU activity) and export a Chrome trace."""
        import os
        from pathlib import Path

        import torch
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(ProfilerActivity.CUDA)
        with profile(activities=acts) as prof:
            res = fn()
        self._trace_seq += 1
        out = Path(self.trace_dir)
        out.mkdir(parents=True, exist_ok=True)
        path = out / f"trace_{os.getpid()}_{self._trace_seq:05d}_{model.replace(':', '_').replace('/', '_')}.json"
        prof.export_chrome_trace(str(path))
        return res, str(path)


class FakeBackend(Backend):
    """Canned generations with controllable latency (tests / plumbing runs without a GPU).
    ``fail`` makes every request raise; ``hang_s`` sleeps before answering (timeout tests)."""

    def __init__(self, models=("qwen2:1.5b",), tokens_per_s: float = 2000.0, prefill_s: float = 0.0,
                 fail: bool = False, hang_s: float = 0.0):
        self._models = list(models)
        self.tokens_per_s = tokens_per_s
        self.prefill_s = prefill_s
        self.fail = fail
        self.hang_s = hang_s
        self.calls: List[Dict[str, Any]] = []

    def models(self) -> List[str]:
        return list(self._models)

    def max_batch(self, model: str) -> int:
        return 8

    def run(self, model: str, jobs: List[Job]) -> None:
        from ..engine.engine import GenResult
        from ..models.tokenizer import SyntheticTokenizer

        if self.hang_s:
            time.sleep(self.hang_s)
        if self.fail:
            raise RuntimeError("fake backend failure")
        tok = SyntheticTokenizer(32000)
        t0 = time.perf_counter_ns()
        time.sleep(self.prefill_s)
        n = max(j.num_predict for j in jobs)
        time.sleep(n / self.tokens_per_s)
        dt = time.perf_counter_ns() - t0
        for i, j in enumerate(jobs):
            ids = [16 + (i * 131 + k * 7919) % 31000 for k in range(j.num_predict)]
            text = tok.decode(ids)
            if j.stream:
                j.stream(text)
            prompt_ids = tok.encode(j.prompt) if isinstance(j.prompt, str) else list(j.prompt)
            j.result = GenResult(model, prompt_ids, ids, text, "length", 0, int(self.prefill_s * 1e9), dt, dt)
            j.ttft_ns = int(self.prefill_s * 1e9)
            self.calls.append({"model": model, "prompt": j.prompt, "num_predict": j.num_predict})


class Scheduler:
    """Per-model job queues; a worker thread per model batches jobs that arrive together."""

    def __init__(self, backend: Backend, batch_window_ms: float = 5.0):
        self.backend = backend
        self.window = batch_window_ms / 1000.0
        self.queues: Dict[str, "queue.Queue[Job]"] = {}
        self.threads: Dict[str, threading.Thread] = {}
        self.lock = threading.Lock()
        self.loaded_at: Dict[str, float] = {}

    def submit(self, job: Job) -> Job:
        if job.model not in self.backend.models():
            raise KeyError(f"model '{job.model}' not found, try pulling it first")
        with self.lock:
            q = self.queues.get(job.model)
            if q is None:
                q = self.queues[job.model] = queue.Queue()
                t = threading.Thread(target=self._worker, args=(job.model, q), daemon=True,
                                     name=f"cain-sched-{job.model}")
                self.threads[job.model] = t
                self.loaded_at[job.model] = time.time()
                t.start()
        q.put(job)
        return job

    def _worker(self, model: str, q: "queue.Queue[Job]") -> None:
        if getattr(self.backend, "continuous", False):
            try:
                if self.backend.serve_queue(model, q) is not False:
                    return
            except BaseException as exc:  # noqa: BLE001 - e.g. the model failed to load
                while True:  # fail every request of this model rather than hang it
                    j = q.get()
                    j.error = exc
                    j.done.set()
        while True:
            first = q.get()
            batch = [first]
            deadline = time.perf_counter() + self.window
            cap = self.backend.max_batch(model)
            while len(batch) < cap:
                rem = deadline - time.perf_counter()
                if rem <= 0:
                    break
                try:
                    batch.append(q.get(timeout=rem))
                except queue.Empty:
                    break
            try:
                self.backend.run(model, batch)
            except BaseException as exc:  # noqa: BLE001 - reported per job
                for j in batch:
                    j.error = exc
            for j in batch:
                j.done.set()


def _result_json(job: Job, created: Optional[str] = None) -> Dict[str, Any]:
    r = job.result
    d = r.ollama_json(created or _now())
    d["cain_ttft_ns"] = int(getattr(job, "ttft_ns", 0))
    if job.trace_file:
        d["cain_trace"] = job.trace_file
    return d


class OllamaHandler(BaseHTTPRequestHandler):
    server_version = "cain-amd-ollama/" + VERSION
    protocol_version = "HTTP/1.1"
    scheduler: Scheduler = None  # set by make_server

    def log_message(self, fmt, *args):  # keep stdout for the experiment logs
        if getattr(self.server, "verbose", False):
            sys.stderr.write("[serve] " + (fmt % args) + "\n")

    # -- helpers -------------------------------------------------------------
    def _send_json(self, code: int, obj: Any) -> None:
        body = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json; charset=utf-8")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _body(self) -> Dict[str, Any]:
        n = int(self.headers.get("Content-Length") or 0)
        raw = self.rfile.read(n) if n else b""
        if not raw:
            return {}
        return json.loads(raw.decode("utf-8"))

    # -- routes ----------------------------------------------------------------
    def do_GET(self):  # noqa: N802
        if self.path in ("/", ""):
            body = b"Ollama is running"
            self.send_response(200)
            self.send_header("Content-Type", "text/plain")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)
        elif self.path == "/api/version":
            self._send_json(200, {"version": VERSION})
        elif self.path == "/api/tags":
            be = self.scheduler.backend
            self._send_json(200, {"models": [{"name": m, "model": m, "modified_at": _now(), "size": 0,
                                              "details": be.model_info(m).get("details", {})} for m in be.models()]})
        elif self.path == "/api/ps":
            self._send_json(200, {"models": [{"name": m, "model": m,
                                              "expires_at": "2999-01-01T00:00:00Z"}
                                             for m in self.scheduler.queues]})
        else:
            self._send_json(404, {"error": "not found"})

    def do_POST(self):  # noqa: N802
        try:
            body = self._body()
        except (ValueError, UnicodeDecodeError) as exc:
            return self._send_json(400, {"error": f"invalid JSON: {exc}"})
        if self.path == "/api/generate":
            return self._generate(body, chat=False)
        if self.path == "/api/chat":
            return self._generate(body, chat=True)
        if self.path == "/api/show":
            m = body.get("model") or body.get("name")
            if m not in self.scheduler.backend.models():
                return self._send_json(404, {"error": f"model '{m}' not found"})
            return self._send_json(200, self.scheduler.backend.model_info(m))
        if self.path == "/api/pull":
            m = body.get("model") or body.get("name")
            ok = m in self.scheduler.backend.models()
            return self._send_json(200 if ok else 404, {"status": "success"} if ok else {"error": "unknown model"})
        return self._send_json(404, {"error": "not found"})

    def _generate(self, body: Dict[str, Any], chat: bool) -> None:
        model = body.get("model")
        if not model:
            return self._send_json(400, {"error": "model is required"})
        if chat:
            msgs = body.get("messages") or []
            text = msgs[-1].get("content", "") if msgs else ""
        else:
            text = body.get("prompt", "")
        try:
            prompt = self.scheduler.backend.prompt_for(model, body, chat)
        except KeyError as exc:
            return self._send_json(404, {"error": str(exc).strip("'\"")})
        except Exception as exc:  # noqa: BLE001 - a template that fails to render, a model that fails to load
            return self._send_json(400, {"error": f"{type(exc).__name__}: {exc}"})
        opts = dict(body.get("options") or {})
        n = opts.get("num_predict")
        # the length policy reads the user's words ("In N words ..."), not the template around them
        num_predict = int(n) if n is not None and int(n) > 0 else default_num_predict(text)
        stream = body.get("stream", True)
        created = _now()
        chunks: "queue.Queue[str]" = queue.Queue()
        job = Job(model, prompt, num_predict, opts, stream=chunks.put if stream else None)
        try:
            self.scheduler.submit(job)
        except KeyError as exc:
            return self._send_json(404, {"error": str(exc).strip("'\"")})
        if not stream:
            job.done.wait()
            if job.error is not None:
                return self._send_json(500, {"error": str(job.error)})
            d = _result_json(job, created)
            if chat:
                d["message"] = {"role": "assistant", "content": d.pop("response")}
            return self._send_json(200, d)
        # NDJSON streaming (chunked transfer encoding)
        self.send_response(200)
        self.send_header("Content-Type", "application/x-ndjson")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()

        def emit(obj) -> None:
            data = (json.dumps(obj) + "\n").encode()
            self.wfile.write(f"{len(data):x}\r\n".encode() + data + b"\r\n")
            self.wfile.flush()

        while not (job.done.is_set() and chunks.empty()):
            try:
                piece = chunks.get(timeout=0.05)
            except queue.Empty:
                continue
            part = {"model": model, "created_at": _now(), "done": False}
            if chat:
                part["message"] = {"role": "assistant", "content": piece}
            else:
                part["response"] = piece
            emit(part)
        if job.error is not None:
            emit({"error": str(job.error)})
        else:
            d = _result_json(job, created)
            d["response"] = ""
            if chat:
                d.pop("response")
                d["message"] = {"role": "assistant", "content": ""}
            emit(d)
        self.wfile.write(b"0\r\n\r\n")
        self.wfile.flush()


def make_server(backend: Backend, host: str = "127.0.0.1", port: int = 11434, batch_window_ms: float = 5.0,
                verbose: bool = False) -> ThreadingHTTPServer:
    sched = Scheduler(backend, batch_window_ms)
    handler = type("BoundOllamaHandler", (OllamaHandler,), {"scheduler": sched})
    srv = ThreadingHTTPServer((host, port), handler)
    srv.daemon_threads = True
    srv.verbose = verbose
    srv.scheduler = sched
    return srv


class ServerThread:
    """Run a server in a background thread (tests, in-process remote arm)."""

    def __init__(self, backend: Backend, host: str = "127.0.0.1", port: int = 0, **kw):
        self.server = make_server(backend, host, port, **kw)
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True, name="cain-ollama")

    @property
    def url(self) -> str:
        h, p = self.server.server_address[:2]
        return f"http://{h}:{p}"

    def __enter__(self):
        self.thread.start()
        return self

    def __exit__(self, *exc):
        self.server.shutdown()
        self.server.server_close()


def main(argv: Optional[List[str]] = None) -> None:
    from ..models import MODELS, TINY

    ap = argparse.ArgumentParser(prog="python -m cain_amd serve")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=11434)
    ap.add_argument("--models", default=",".join(MODELS), help="comma-separated model tags to serve")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--max-batch", type=int, default=16)
    ap.add_argument("--max-context", type=int, default=2048)
    ap.add_argument("--batch-window-ms", type=float, default=5.0)
    ap.add_argument("--backend", choices=["hip", "torch", "fake"], default=None)
    ap.add_argument("--preload", action="store_true", help="load every model at startup (all stay resident)")
    ap.add_argument("--fake-tok-s", type=float, default=2000.0, help="fake backend: modelled decode rate")
    ap.add_argument("--fake-prefill-s", type=float, default=0.0, help="fake backend: modelled time to first token")
    ap.add_argument("--trace-dir", default=None, help="write a torch.profiler Chrome trace of every decode batch here")
    ap.add_argument("--weights", choices=["bf16", "fp8", "fp4"], default="bf16",
                    help="GEMM weight storage (fp8: e4m3 per-row scaled; W8A8 above 16 rows, W8A16 below)")
    ap.add_argument("--kv", choices=["bf16", "fp8"], default="bf16", help="KV-cache storage (fp8: e4m3)")
    ap.add_argument("--static-batching", action="store_true",
                    help="batch requests that arrive within --batch-window-ms and run each batch to completion "
                         "(default on the HIP engine: continuous batching)")
    ap.add_argument("--checkpoint", action="append", metavar="TAG=PATH",
                    help="serve a Hugging Face checkpoint directory or GGUF file under TAG (repeatable; models/hf.py); "
                         "PATH 'ollama' takes the blob a local Ollama store keeps for TAG")
    ap.add_argument("-v", "--verbose", action="store_true")
    ns = ap.parse_args(argv)
    ck_tags = register_checkpoints(ns.checkpoint)
    models = [m for m in ns.models.split(",") if m]
    models += [t for t in ck_tags if t not in models]
    for m in models:
        if m not in MODELS and m not in TINY and m not in ck_tags:
            raise SystemExit(f"unknown model {m}")
    if ns.backend == "fake":
        be: Backend = FakeBackend(models, tokens_per_s=ns.fake_tok_s, prefill_s=ns.fake_prefill_s)
    else:
        be = EngineBackend(models, device=ns.device, max_batch=ns.max_batch, max_context=ns.max_context,
                           backend=ns.backend, preload=ns.preload, trace_dir=ns.trace_dir, weight_dtype=ns.weights,
                           continuous=not ns.static_batching, kv_dtype=ns.kv)
    srv = make_server(be, ns.host, ns.port, ns.batch_window_ms, ns.verbose)
    print(f"[serve] Ollama-compatible API on http://{ns.host}:{srv.server_address[1]} models={models}", flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:  # pragma: no cover
        pass


def generate_main(argv: Optional[List[str]] = None) -> None:
    """``python -m cain_amd generate --model M --prompt P``: one local generation, Ollama JSON on stdout."""
    ap = argparse.ArgumentParser(prog="python -m cain_amd generate")
    ap.add_argument("--model", required=True)
    ap.add_argument("--prompt", required=True)
    ap.add_argument("--num-predict", type=int, default=None)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--temperature", type=float, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--weights", choices=["bf16", "fp8", "fp4"], default="bf16")
    ap.add_argument("--kv", choices=["bf16", "fp8"], default="bf16")
    ap.add_argument("--checkpoint", metavar="PATH", help="a Hugging Face checkpoint directory, served as --model")
    ns = ap.parse_args(argv)
    if ns.checkpoint:
        register_checkpoints([f"{ns.model}={ns.checkpoint}"])
    be = EngineBackend([ns.model], device=ns.device, max_batch=1, weight_dtype=ns.weights, kv_dtype=ns.kv)
    opts = {k: v for k, v in (("temperature", ns.temperature), ("seed", ns.seed)) if v is not None}
    job = Job(ns.model, ns.prompt, ns.num_predict or default_num_predict(ns.prompt), opts)
    be.run(ns.model, [job])
    print(json.dumps(_result_json(job)))
