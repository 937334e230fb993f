"""Continuous batching (engine.ContinuousBatch + the server's HIP worker): requests join a running decode batch at
the next graph boundary and leave when done; a late request's time to first token is bounded by one chunk plus
its prefill, not by the earlier requests' generations."""
import json
import threading
import time
import urllib.request

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd.engine import DecodeEngine  # noqa: E402
from cain_amd.models.reference import ReferenceModel  # noqa: E402
from cain_amd.serve import ServerThread  # noqa: E402
from cain_amd.serve.server import EngineBackend  # noqa: E402

GREEDY = dict(temperature=0.0, repeat_penalty=1.0, eos_id=-1)


def test_rows_join_and_leave_between_chunks():
    eng = DecodeEngine("tiny-llama3.1:8b", device="cuda", max_batch=4, max_context=256, keep_natural=True, seed=4,
                       steps_per_graph=4)
    ref = ReferenceModel(eng.weights)
    cb = eng.continuous()
    a = cb.admit(["In 100 words, please give me information about India", "hello there"], [40, 9],
                 [GREEDY, GREEDY])
    assert a == [0, 1] and cb.n == 2
    got = {0: [], 1: []}
    owner = {0: "A", 1: "B"}
    out = {"A": [], "B": [], "C": []}
    late_admitted = False
    for _ in range(40):
        cb.step()
        new, fin = cb.poll()
        for r, ids in enumerate(new):
            out[owner[r]] += ids
        if not late_admitted:  # a third request joins while A is still decoding
            (c,) = cb.admit(["abc def ghi"], [12], [GREEDY])
            owner[c] = "C"
            late_admitted = True
        dead = [r for r, f in enumerate(fin) if f]
        if dead:
            moves = cb.retire(dead)
            owner = {moves.get(r, r): o for r, o in owner.items() if r not in dead}
        if cb.n == 0:
            break
    assert [len(out[k]) for k in "ABC"] == [40, 9, 12]
    assert cb.n == 0 and cb.capacity == 4
    for k, p in (("A", "In 100 words, please give me information about India"), ("B", "hello there"),
                 ("C", "abc def ghi")):
        lg = ref.forward(torch.tensor([eng.encode(p)], device="cuda"))[0, -1]
        top2 = lg.topk(2)
        if float(top2.values[0] - top2.values[1]) > 1e-2:
            assert out[k][0] == int(top2.indices[0]), k
    eng.close()


def _post(url, body, out, key):
    t0 = time.perf_counter()
    req = urllib.request.Request(url + "/api/generate", data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=300) as r:
        out[key] = (json.loads(r.read()), time.perf_counter() - t0)


def test_server_late_request_is_not_held_behind_the_running_batch():
    be = EngineBackend(["tiny-llama3.1:8b"], device="cuda:0", max_batch=4, max_context=2048, preload=True,
                       steps_per_graph=8)
    with ServerThread(be, port=0) as srv:
        _post(srv.url, {"model": "tiny-llama3.1:8b", "prompt": "warm up", "stream": False,
                        "options": {"num_predict": 16}}, {}, "w")
        out = {}
        long_t = threading.Thread(target=_post, args=(srv.url, {"model": "tiny-llama3.1:8b", "prompt": "long one",
                                                                "stream": False,
                                                                "options": {"num_predict": 900, "eos_id": -1}}, out, "long"))
        long_t.start()
        time.sleep(0.3)
        _post(srv.url, {"model": "tiny-llama3.1:8b", "prompt": "late short one", "stream": False,
                        "options": {"num_predict": 8, "eos_id": -1}}, out, "short")
        long_t.join()
    short, t_short = out["short"]
    long_, t_long = out["long"]
    assert short["eval_count"] == 8 and long_["eval_count"] == 900
    # the short request finished while the long one was still decoding
    assert t_short < 0.5 * t_long, (t_short, t_long)
    assert short["cain_ttft_ns"] < 0.25 * long_["total_duration"], (short["cain_ttft_ns"], long_["total_duration"])


def test_moved_row_keeps_its_sequence():
    """A request that retire() moves into a hole left by a finished row continues the same token stream: its
    full sequence (sampled, fixed seed) equals a static engine.generate of the same prompt and options, because
    the sampler keys its random stream by the request's seed, not by the row (sample.hip)."""
    eng = DecodeEngine("tiny-llama3.1:8b", device="cuda", max_batch=4, max_context=256, seed=4, steps_per_graph=4)
    opts = dict(temperature=0.8, top_k=40, top_p=0.9, repeat_penalty=1.1, eos_id=-1, seed=1234)
    want = eng.generate(["the mover"], 30, [opts])[0].tokens
    cb = eng.continuous()
    rows = cb.admit(["short a", "short b", "the mover"], [4, 4, 30], [GREEDY, GREEDY, opts])
    assert rows == [0, 1, 2]
    owner = {0: "a", 1: "b", 2: "m"}
    got = []
    moved = False
    for _ in range(40):
        cb.step()
        new, fin = cb.poll()
        got += new[[r for r, o in owner.items() if o == "m"][0]]
        dead = [r for r, f in enumerate(fin) if f]
        if dead:
            moves = cb.retire(dead)
            moved |= any(owner[j] == "m" for j in moves)
            owner = {moves.get(r, r): o for r, o in owner.items() if r not in dead}
        if cb.n == 0:
            break
    assert moved, "the long request was expected to move into a freed row"
    assert got == want
    eng.close()


def test_continuous_timing_matches_static_path():
    """ttft / eval_duration of one request under continuous batching are taken like the static path's: the first
    token decoded on its own (exact t_first), eval_duration from the end of admission, covering every token."""
    be = EngineBackend(["tiny-llama3.1:8b"], device="cuda:0", max_batch=4, max_context=1024, preload=True,
                       steps_per_graph=8)
    body = {"model": "tiny-llama3.1:8b", "prompt": "timing probe", "stream": False,
            "options": {"num_predict": 200, "eos_id": -1}}
    with ServerThread(be, port=0) as srv:
        _post(srv.url, body, {}, "w")
        out = {}
        _post(srv.url, body, out, "c")
    cont = out["c"][0]
    st = EngineBackend(["tiny-llama3.1:8b"], device="cuda:0", max_batch=4, max_context=1024, preload=True,
                       steps_per_graph=8, continuous=False)
    with ServerThread(st, port=0) as srv:
        _post(srv.url, body, {}, "w")
        out = {}
        _post(srv.url, body, out, "s")
    stat = out["s"][0]
    assert cont["eval_count"] == stat["eval_count"] == 200
    # the first token is not stamped a whole chunk late, and eval_duration covers all 200 tokens
    assert cont["cain_ttft_ns"] < 3 * stat["cain_ttft_ns"] + 2_000_000, (cont["cain_ttft_ns"], stat["cain_ttft_ns"])
    assert 0.5 * stat["eval_duration"] < cont["eval_duration"] < 2.0 * stat["eval_duration"] + 5_000_000, \
        (cont["eval_duration"], stat["eval_duration"])
    assert cont["eval_duration"] <= cont["total_duration"]
