"""The lean chunk-maximum sampler (csrc/sample.hip sample_lean_kernel) and the chunk maxima the few-row fp8 / MXFP4 /
GGUF Q4 LM heads now write for it (gemm_epi.h epi_cmax).

The sampler must draw exactly the token of the one-workgroup kernel (the reference sampler) for the same logits,
options, seed and history -- greedy, Ollama defaults with a repeat history (penalty > 1 and < 1), top_k 1..256,
top_p, ties, masked (-inf) vocabulary, vocabularies of 64 to 256,000 -- and advance the decode state the same way.
The chunk maxima must equal the fp32 logits' own 16-column maxima bit for bit.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.models.q4 import quant_pack_q4  # noqa: E402
from cain_amd.models.weights import pack_mfma_a_fp8, pack_mxfp4, quantize_mxfp4  # noqa: E402

DEV = torch.device("cuda")
KINDS = [  # (temperature, top_k, top_p, repeat_penalty)
    (0.0, 40, 1.0, 1.1), (0.8, 40, 0.9, 1.1), (0.8, 40, 0.9, 0.8), (1.0, 256, 1.0, 1.0), (1.2, 10, 0.5, 1.3),
    (1.0, 1, 1.0, 1.0), (0.7, 100, 0.95, 1.1), (1.0, 64, 1.0, 1.1), (0.9, 33, 0.8, 1.0), (1.0, 0, 1.0, 1.1)]


def _state(M, V, n_hist, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    hist = torch.randint(0, V, (M, 64), generator=g, dtype=torch.int32)
    return dict(tok=torch.zeros(M, device=DEV, dtype=torch.int32),
                pos=torch.full((M,), 50, device=DEV, dtype=torch.int32),
                gen=torch.zeros(M, 96, device=DEV, dtype=torch.int32),
                n_gen=torch.full((M,), n_hist, device=DEV, dtype=torch.int32),
                max_new=torch.full((M,), 90, device=DEV, dtype=torch.int32),
                done=torch.zeros(M, device=DEV, dtype=torch.int32),
                hist=hist.to(DEV).view(-1).contiguous(),
                slot=torch.arange(M, device=DEV, dtype=torch.int32))


def _run(logits, params, st, mode):
    M, V = logits.shape
    lg = logits.clone()
    cmax = logits.view(M, V // 16, 16).amax(-1).contiguous() if mode in ("cm", "lean") else None
    ops.sample(lg, st["tok"], st["pos"], st["gen"], st["n_gen"], st["max_new"], st["done"], st["hist"], st["slot"],
               params, 2048, split=(mode == "split"), cmax=cmax, lean=(mode == "lean"))
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in st.items()}


def _rows(M, seed):
    rows = []
    for i in range(M):
        t, k, p, rp = KINDS[(i + seed) % len(KINDS)]
        rows.append(dict(temperature=t, top_k=k, top_p=p, repeat_penalty=rp, repeat_last_n=64 if i % 3 else 20,
                         eos_id=-1, seed=seed * 7919 + i))
    return rows


@pytest.mark.parametrize("V", [128256, 151936, 32064, 256000, 4096, 64])
@pytest.mark.parametrize("M", [1, 5, 64])
def test_lean_sampler_draws_the_reference_token(V, M):
    torch.manual_seed(V + M)
    for rep in range(4):
        logits = torch.randn(M, V, device=DEV) * (0.5 + rep)
        logits[:, :3] += 4.0
        if rep == 1:
            logits[:, 7] = logits[:, 1]  # a tie among the top
        if rep == 2 and V >= 64:
            logits[:, V // 2:] = float("-inf")  # a masked half of the vocabulary
        params = ops.sample_params_tensor(_rows(M, rep), DEV)
        n_hist = [0, 20, 64, 5][rep]
        # plant the rows' top logits in the history so the penalty changes the winners
        st0 = _state(M, V, n_hist, rep)
        top = logits.topk(min(6, V), dim=-1).indices.to(torch.int32)
        st0["hist"].view(M, 64)[:, 1:1 + top.shape[1]] = top
        outs = {}
        for mode in ("one", "lean"):
            st = {k: v.clone() for k, v in st0.items()}
            outs[mode] = _run(logits, params, st, mode)
        for k in ("tok", "pos", "gen", "n_gen", "done", "hist"):
            assert torch.equal(outs["one"][k], outs["lean"][k]), (rep, k, outs["one"]["tok"], outs["lean"]["tok"])


def _topk_set(row, hist_ids, rp, K):
    """The top-K ids (value desc, index asc) of a row after the repeat penalty (each distinct history id once)."""
    v = row.double().cpu().clone()
    for h in set(int(x) for x in hist_ids):
        v[h] = v[h] / rp if v[h] > 0 else v[h] * rp
    order = sorted(range(v.numel()), key=lambda i: (-float(v[i]), i))
    return set(order[:K]), order[0]


@pytest.mark.parametrize("V", [151936, 4096])
def test_lean_sampler_ties_everywhere(V):
    """Rows whose logits tie massively (a constant row; blocks of equal values; one equal maximum per chunk; rounded
    values): the threshold admits far more chunks or elements than fit and is tightened to the exact (value, index)
    pair, so the draw is among the exact top-K (lowest indices first among equals) and repeatable.  (The
    one-workgroup kernel tightens on values only, so on such rows its candidates depend on arrival order: the
    reference here is the exact top-K computed on the host.)"""
    M = 6
    logits = torch.zeros(M, V, device=DEV)
    logits[3] = torch.arange(V, device=DEV).div(97, rounding_mode="floor").float().remainder(5)
    logits[4, ::16] = 1.0  # one maximum per chunk, all equal
    logits[5] = torch.randn(V, device=DEV).round()  # many ties at a few values
    kinds = [(0.0, 40, 1.0, 1.0), (1.0, 40, 1.0, 1.0), (1.0, 256, 0.9, 1.1), (0.9, 40, 0.9, 1.1), (0.9, 100, 0.9, 1.0),
             (0.9, 40, 0.9, 1.1)]
    rows = [dict(temperature=t, top_k=k, top_p=p, repeat_penalty=rp, repeat_last_n=64, eos_id=-1, seed=i + 1)
            for i, (t, k, p, rp) in enumerate(kinds)]
    params = ops.sample_params_tensor(rows, DEV)
    st0 = _state(M, V, 30, 9)
    runs = [_run(logits, params, {k: v.clone() for k, v in st0.items()}, "lean") for _ in range(2)]
    assert torch.equal(runs[0]["tok"], runs[1]["tok"])
    hist = st0["hist"].view(M, 64).cpu()
    for i, (t, k, p, rp) in enumerate(kinds):
        recent = hist[i, 0:30].tolist()  # n_gen 30: slots (29 - j) & 63 for j < 30, i.e. slots 0..29
        top, first = _topk_set(logits[i], recent if rp != 1.0 else [], rp, 1 if t == 0.0 else k)
        tok = int(runs[0]["tok"][i])
        assert tok in top, (i, tok)
        if t == 0.0:
            assert tok == first


def test_lean_sampler_stop_ids_and_idle_rows():
    V, M = 32064, 5
    logits = torch.randn(M, V, device=DEV)
    win = [101, 202, 303, 404, 505]
    for i, w in enumerate(win):
        logits[i, w] = 50.0
    rows = [dict(temperature=0.0, top_p=1.0, repeat_penalty=1.0, top_k=40, repeat_last_n=0, eos_id=-1, seed=1,
                 stop=s) for s in ([101], [7, 202], [1, 2, 303], [1, 2, 3], [])]
    st = _state(M, V, 0, 1)
    st["slot"][4] = -1  # an idle row: nothing sampled, nothing advanced
    out = _run(logits, ops.sample_params_tensor(rows, DEV), st, "lean")
    assert out["tok"].tolist()[:4] == win[:4] and int(out["tok"][4]) == 0
    assert out["done"].tolist() == [1, 1, 1, 0, 0]
    assert out["pos"].tolist() == [50, 50, 50, 51, 50]
    assert out["n_gen"].tolist() == [1, 1, 1, 1, 0]


def test_lean_sampler_distribution():
    """Frequencies over many seeds follow softmax over the top-k (top_p off)."""
    V, M = 5056, 64
    base = torch.randn(V) * 0.1
    base[:4] = torch.tensor([3.0, 2.5, 2.0, 1.0])
    logits = base.to(DEV).repeat(M, 1)
    counts = torch.zeros(4)
    for rep in range(16):
        rows = [dict(temperature=1.0, top_p=1.0, repeat_penalty=1.0, top_k=3, repeat_last_n=0, eos_id=-1,
                     seed=rep * 1000 + i) for i in range(M)]
        out = _run(logits, ops.sample_params_tensor(rows, DEV), _state(M, V, 0, rep), "lean")
        for t in out["tok"].tolist():
            assert t < 3
            counts[t] += 1
    p = torch.softmax(torch.tensor([3.0, 2.5, 2.0]), 0)
    assert torch.allclose(counts[:3] / counts.sum(), p, atol=0.06)


# ---- chunk maxima written by the few-row LM heads of the other weight formats

def _check_cmax(y, cmax):
    M, N = y.shape
    assert torch.equal(cmax, y.view(M, N // 16, 16).amax(-1))


@pytest.mark.parametrize("M,N,K", [(1, 128256, 4096), (4, 128256, 4096), (1, 32064, 3072), (7, 32064, 3072),
                                   (16, 2048, 1536), (1, 151936, 1536), (1, 256000, 2048)])
def test_w4_lm_head_writes_chunk_maxima(M, N, K):
    """(Row counts whose activations fit the stream kernel's LDS copy; the tile kernel beyond them writes none, and the
    engine's sampler then takes the two-stage kernel.)"""
    torch.manual_seed(M + N)
    W = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    c, s = quantize_mxfp4(W)
    wq, ws = pack_mxfp4(c, s)
    x = torch.randn(M, K, device=DEV).bfloat16()
    cmax = torch.full((M, N // 16), float("nan"), device=DEV)
    y = ops.gemm_w4(wq, ws, x, N, ops.EPI_F32, cmax=cmax)
    _check_cmax(y, cmax)
    # split-K LM-head shapes (narrow N, long K) finish in the last arriver: it writes them as well
    ops.set_w4_split(2)
    try:
        cm2 = torch.full_like(cmax, float("nan"))
        y2 = ops.gemm_w4(wq, ws, x, N, ops.EPI_F32, cmax=cm2)
        _check_cmax(y2, cm2)
    finally:
        ops.set_w4_split(0)


@pytest.mark.parametrize("M", [1, 16, 40])
def test_w8_lm_head_writes_chunk_maxima(M):
    torch.manual_seed(M)
    N, K = 32064, 3072
    W = torch.randn(N, K, device=DEV) * 0.02
    scale = W.abs().amax(-1) / 448.0
    q = (W / scale[:, None]).to(torch.float8_e4m3fn)
    x = torch.randn(M, K, device=DEV).bfloat16()
    cmax = torch.full((M, N // 16), float("nan"), device=DEV)
    y = ops.gemm_w8(pack_mfma_a_fp8(q.view(torch.uint8)), scale.float().contiguous(), x, N, ops.EPI_F32, cmax=cmax)
    _check_cmax(y, cmax)


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("M", [1, 20])
def test_q4_lm_head_writes_chunk_maxima(fmt, M):
    torch.manual_seed(fmt + M)
    N, K = 32064, 3072
    W = torch.randn(N, K, device=DEV) * 0.02
    wq, sbuf = quant_pack_q4(W, fmt)
    x = torch.randn(M, K, device=DEV).bfloat16()
    cmax = torch.full((M, N // 16), float("nan"), device=DEV)
    y = ops.gemm_q4(fmt, wq, sbuf, x, N, ops.EPI_F32, cmax=cmax)
    _check_cmax(y, cmax)
