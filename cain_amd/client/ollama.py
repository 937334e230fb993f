"""Ollama-compatible HTTP client.

The reference issues its request with ``curl`` in a subprocess and never
captures the response (experiment/RunnerConfig.py:128-131), so token counts
are lost.  Two clients here, both capturing the JSON:

* ``OllamaClient`` — in-process ``http.client``; measures client-side wall time
  and, for streamed requests, time to first token; JSON bodies built with
  ``json.dumps`` (the reference's shell-quoted JSON breaks on quotes in topics,
  SURVEY §2.8).
* ``CurlRequest`` — the reference's mechanism (a ``curl`` child process the
  measurement loop can watch), but with stdout captured and parsed, a timeout,
  and ``Popen.poll()`` for liveness instead of ``psutil.pid_exists`` (which
  spins forever on a zombie on Linux).
"""
from __future__ import annotations

import http.client
import json
import shutil
import subprocess
import tempfile
import time
import urllib.parse
from dataclasses import dataclass, field
from typing import Any, Dict, Iterator, List, Optional


@dataclass
class GenerateResponse:
    data: Dict[str, Any]
    wall_s: float
    ttft_s: Optional[float] = None
    chunks: int = 1
    status: int = 200

    @property
    def text(self) -> str:
        return self.data.get("response", "") or self.data.get("message", {}).get("content", "")

    @property
    def eval_count(self) -> int:
        return int(self.data.get("eval_count", 0) or 0)

    @property
    def prompt_eval_count(self) -> int:
        return int(self.data.get("prompt_eval_count", 0) or 0)

    def stats(self) -> Dict[str, Any]:
        d = self.data
        ns = 1e-9
        out = {
            "tokens_generated": self.eval_count,
            "prompt_tokens": self.prompt_eval_count,
            "server_total_s": (d.get("total_duration") or 0) * ns,
            "server_eval_s": (d.get("eval_duration") or 0) * ns,
            "server_prompt_eval_s": (d.get("prompt_eval_duration") or 0) * ns,
            "client_wall_s": self.wall_s,
        }
        if self.ttft_s is not None:
            out["ttft_s"] = self.ttft_s
        elif d.get("cain_ttft_ns"):
            out["ttft_s"] = d["cain_ttft_ns"] * ns
        if out["server_eval_s"] > 0:
            out["server_tok_per_s"] = self.eval_count / out["server_eval_s"]
        if d.get("cain_trace"):
            out["trace_file"] = d["cain_trace"]
        return out


class OllamaError(RuntimeError):
    pass


def _split(url: str):
    u = urllib.parse.urlparse(url if "://" in url else f"http://{url}")
    return u.hostname or "127.0.0.1", u.port or 11434


class OllamaClient:
    def __init__(self, base_url: str = "http://127.0.0.1:11434", timeout: float = 600.0):
        self.host, self.port = _split(base_url)
        self.timeout = timeout

    @property
    def base_url(self) -> str:
        return f"http://{self.host}:{self.port}"

    def _conn(self) -> http.client.HTTPConnection:
        return http.client.HTTPConnection(self.host, self.port, timeout=self.timeout)

    def _request(self, method: str, path: str, body: Optional[Dict] = None):
        c = self._conn()
        data = None if body is None else json.dumps(body).encode()
        c.request(method, path, body=data, headers={"Content-Type": "application/json"} if data else {})
        return c, c.getresponse()

    def get(self, path: str) -> Any:
        c, r = self._request("GET", path)
        try:
            raw = r.read()
            if r.status != 200:
                raise OllamaError(f"GET {path}: HTTP {r.status}: {raw[:200]!r}")
            ct = r.getheader("Content-Type", "")
            return json.loads(raw) if "json" in ct else raw.decode()
        finally:
            c.close()

    def tags(self) -> List[str]:
        return [m["name"] for m in self.get("/api/tags").get("models", [])]

    def alive(self) -> bool:
        try:
            return "running" in str(self.get("/"))
        except OSError:
            return False

    def generate(self, model: str, prompt: str, stream: bool = False, options: Optional[Dict] = None,
                 on_chunk=None, system: Optional[str] = None, raw: bool = False) -> GenerateResponse:
        """``POST /api/generate``; ``system`` / ``raw`` as Ollama's fields (raw: no prompt template)."""
        body: Dict[str, Any] = {"model": model, "prompt": prompt, "stream": stream}
        if options:
            body["options"] = options
        if system is not None:
            body["system"] = system
        if raw:
            body["raw"] = True
        return self._post_gen("/api/generate", body, stream, on_chunk)

    def chat(self, model: str, messages: List[Dict[str, str]], stream: bool = False,
             options: Optional[Dict] = None) -> GenerateResponse:
        body: Dict[str, Any] = {"model": model, "messages": messages, "stream": stream}
        if options:
            body["options"] = options
        return self._post_gen("/api/chat", body, stream, None)

    def _post_gen(self, path: str, body: Dict, stream: bool, on_chunk) -> GenerateResponse:
        t0 = time.perf_counter()
        c, r = self._request("POST", path, body)
        try:
            if r.status != 200:
                raw = r.read()
                raise OllamaError(f"POST {path}: HTTP {r.status}: {raw[:300]!r}")
            if not stream:
                data = json.loads(r.read())
                return GenerateResponse(data, time.perf_counter() - t0)
            ttft = None
            pieces: List[str] = []
            last: Dict[str, Any] = {}
            n = 0
            for line in _iter_lines(r):
                obj = json.loads(line)
                n += 1
                if "error" in obj:
                    raise OllamaError(obj["error"])
                piece = obj.get("response", obj.get("message", {}).get("content", ""))
                if piece and ttft is None:
                    ttft = time.perf_counter() - t0
                if piece:
                    pieces.append(piece)
                    if on_chunk:
                        on_chunk(piece)
                last = obj
            final = dict(last)
            if "message" in final:
                final["message"] = {"role": "assistant", "content": "".join(pieces)}
            else:
                final["response"] = "".join(pieces)
            return GenerateResponse(final, time.perf_counter() - t0, ttft, n)
        finally:
            c.close()


def _iter_lines(resp) -> Iterator[str]:
    buf = b""
    while True:
        chunk = resp.read1(65536) if hasattr(resp, "read1") else resp.read(65536)
        if not chunk:
            break
        buf += chunk
        while b"\n" in buf:
            line, buf = buf.split(b"\n", 1)
            if line.strip():
                yield line.decode("utf-8")
    if buf.strip():
        yield buf.decode("utf-8")


@dataclass
class CurlRequest:
    """``curl http://HOST:PORT/api/generate -d '{...}'`` as a watched child process."""
    url: str
    model: str
    prompt: str
    stream: bool = False
    options: Optional[Dict] = None
    timeout_s: float = 600.0
    proc: Optional[subprocess.Popen] = None
    t_start: float = 0.0
    t_end: Optional[float] = None
    _out: Any = field(default=None, repr=False)

    def start(self) -> "CurlRequest":
        curl = shutil.which("curl")
        if curl is None:
            raise OllamaError("curl not found (use OllamaClient instead)")
        body: Dict[str, Any] = {"model": self.model, "prompt": self.prompt, "stream": self.stream}
        if self.options:
            body["options"] = self.options
        base = self.url if "://" in self.url else f"http://{self.url}"
        self._out = tempfile.TemporaryFile()
        self.t_start = time.perf_counter()
        self.proc = subprocess.Popen([curl, "-sS", "--max-time", str(self.timeout_s), f"{base}/api/generate",
                                      "-d", json.dumps(body)], stdout=self._out, stderr=subprocess.PIPE)
        return self

    @property
    def pid(self) -> int:
        return self.proc.pid

    def running(self) -> bool:
        return self.proc is not None and self.proc.poll() is None

    def wait(self, timeout: Optional[float] = None) -> GenerateResponse:
        try:
            self.proc.wait(timeout=timeout if timeout is not None else self.timeout_s + 5)
        except subprocess.TimeoutExpired:
            self.kill()
            raise OllamaError("curl request timed out")
        self.t_end = time.perf_counter()
        err = self.proc.stderr.read().decode() if self.proc.stderr else ""
        self._out.seek(0)
        raw = self._out.read().decode("utf-8", "replace")
        if self.proc.returncode != 0:
            raise OllamaError(f"curl exited {self.proc.returncode}: {err.strip()}")
        lines = [ln for ln in raw.splitlines() if ln.strip()]
        if not lines:
            raise OllamaError("empty response")
        objs = [json.loads(ln) for ln in lines]
        if "error" in objs[-1]:
            raise OllamaError(objs[-1]["error"])
        final = dict(objs[-1])
        if self.stream:
            final["response"] = "".join(o.get("response", "") for o in objs)
        return GenerateResponse(final, self.t_end - self.t_start, chunks=len(objs))

    def kill(self) -> None:
        if self.running():
            self.proc.kill()
            self.proc.wait()
