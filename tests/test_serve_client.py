"""Ollama-compatible server + clients (fake backend and the torch engine on CPU) — SURVEY §4 item 3."""
import threading

import pytest

from cain_amd.client import CurlRequest, OllamaClient, OllamaError
from cain_amd.serve import EngineBackend, FakeBackend, ServerThread, default_num_predict


def test_length_policy():
    assert default_num_predict("In 100 words, please give me information about India") == 134
    assert default_num_predict("in 1000 words tell me") == 1334
    assert default_num_predict("hello") == 128


def test_fake_backend_generate_show_tags_errors():
    be = FakeBackend(["qwen2:1.5b", "gemma:2b"])
    with ServerThread(be) as s:
        c = OllamaClient(s.url)
        assert c.alive() and sorted(c.tags()) == ["gemma:2b", "qwen2:1.5b"]
        r = c.generate("qwen2:1.5b", "In 100 words, please give me information about Elvis Presley")
        assert r.eval_count == 134 and r.data["done"] is True and r.data["prompt_eval_count"] > 5
        assert {"total_duration", "load_duration", "eval_duration", "prompt_eval_duration"} <= set(r.data)
        st = c.generate("gemma:2b", "x", stream=True, options={"num_predict": 7})
        assert st.eval_count == 7 and st.ttft_s is not None and st.chunks >= 2
        with pytest.raises(OllamaError, match="not found"):
            c.generate("nope:1b", "x")
        assert c.get("/api/version")["version"]
        ch = c.chat("qwen2:1.5b", [{"role": "user", "content": "hi"}], options={"num_predict": 3})
        assert ch.data["message"]["role"] == "assistant" and ch.eval_count == 3


def test_backend_failure_is_http_500():
    with ServerThread(FakeBackend(["m:1b"], fail=True)) as s:
        with pytest.raises(OllamaError, match="500"):
            OllamaClient(s.url).generate("m:1b", "x", options={"num_predict": 2})


def test_concurrent_requests_are_batched():
    be = FakeBackend(["m:1b"], tokens_per_s=200.0)
    with ServerThread(be, batch_window_ms=50) as s:
        c = OllamaClient(s.url)
        out = []
        ts = [threading.Thread(target=lambda i=i: out.append(c.generate("m:1b", f"p{i}",
                                                                         options={"num_predict": 4 + i}).eval_count))
              for i in range(4)]
        [t.start() for t in ts]
        [t.join() for t in ts]
    assert sorted(out) == [4, 5, 6, 7]
    assert len(be.calls) == 4


def test_curl_client_captures_json_and_quotes():
    import shutil

    if not shutil.which("curl"):
        pytest.skip("curl missing")
    with ServerThread(FakeBackend(["m:1b"])) as s:
        req = CurlRequest(s.url, "m:1b", 'topic with "quotes" and \'apostrophes\'', options={"num_predict": 5}).start()
        r = req.wait()
        assert r.eval_count == 5 and not req.running()


def test_engine_backend_torch_cpu_end_to_end():
    be = EngineBackend(["tiny-qwen2:1.5b"], device="cpu", max_batch=4)
    with ServerThread(be) as s:
        c = OllamaClient(s.url)
        r = c.generate("tiny-qwen2:1.5b", "In 6 words, please give me information about India",
                       options={"temperature": 0, "seed": 1})
        assert r.eval_count == 8 and r.text
        r2 = c.generate("tiny-qwen2:1.5b", "In 6 words, please give me information about India",
                        options={"temperature": 0, "seed": 1})
        assert r2.text == r.text  # greedy is deterministic
        st = c.generate("tiny-qwen2:1.5b", "hello", stream=True, options={"num_predict": 5})
        assert st.eval_count == 5


def test_engine_backend_trace_dir_writes_chrome_trace(tmp_path):
    """--trace-dir: each decode batch is profiled and the response names its trace."""
    import json

    be = EngineBackend(["tiny-qwen2:1.5b"], device="cpu", max_batch=2, trace_dir=str(tmp_path / "traces"))
    with ServerThread(be) as s:
        r = OllamaClient(s.url).generate("tiny-qwen2:1.5b", "hello", options={"num_predict": 3})
    path = r.stats()["trace_file"]
    assert path.startswith(str(tmp_path)) and r.eval_count == 3
    events = json.load(open(path))["traceEvents"]
    assert any("aten::" in e.get("name", "") for e in events)
