"""Wide-batch library path (ops/csrc/blas.hip): hipBLASLt GEMM + fused RMSNorm-scale/activation kernel
vs plain PyTorch fp32, and the engine with the path forced on for every architecture family."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.engine import DecodeEngine  # noqa: E402
from cain_amd.models import TINY  # noqa: E402
from cain_amd.models.reference import ReferenceModel  # noqa: E402
from cain_amd.models.weights import interleave_tiles  # noqa: E402


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (256, 6144, 4096), (200, 1024, 14336), (3, 512, 256)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_lt_gemm_matches_fp32(M, N, K, accumulate):
    g = torch.Generator(device="cuda").manual_seed(M + N)
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    y0 = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    y = y0.clone()
    ops.lt_gemm(w, x, out=y, accumulate=accumulate)
    want = x.float() @ w.float().t() + (y0.float() if accumulate else 0)
    torch.cuda.synchronize()
    assert _rel(y, want) < 1e-2


def test_lt_gemm_strided_rows():
    """Row strides wider than the GEMM (the engine's activation buffers are Mpad x width)."""
    w = (torch.randn(256, 512, device="cuda") / 16).bfloat16()
    xb = torch.randn(64, 768, device="cuda").bfloat16()
    yb = torch.zeros(64, 384, device="cuda", dtype=torch.bfloat16)
    x, y = xb[:, :512], yb[:, :256]
    ops.lt_gemm(w, x, out=y)
    assert _rel(y, x.float() @ w.float().t()) < 1e-2
    assert float(yb[:, 256:].abs().max()) == 0.0


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("M,d,ffn", [(256, 4096, 14336), (130, 3072, 24576), (7, 256, 512)])
def test_rownorm_act_matches_fp32(kind, M, d, ffn):
    x = torch.randn(M, d, device="cuda").bfloat16() * 3
    gate = torch.randn(M, ffn, device="cuda")
    up = torch.randn(M, ffn, device="cuda")
    gu = interleave_tiles(gate.t(), up.t(), tile=8).t().contiguous().bfloat16()  # columns interleaved by 8
    got = ops.rownorm_act(x, gu, 1e-5, kind=kind)
    s = torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5)
    g, u = gu.float()[:, :].view(M, ffn // 8, 2, 8).unbind(2)
    g, u = (s * g.reshape(M, ffn)), (s * u.reshape(M, ffn))
    act = torch.nn.functional.silu(g) if kind == 0 else torch.nn.functional.gelu(g, approximate="tanh")
    torch.cuda.synchronize()
    assert _rel(got, act * u) < 1e-2


@pytest.mark.parametrize("name", sorted(TINY))
def test_engine_lt_path_matches_oracle(name, monkeypatch):
    """Every family with the O, gate/up and LM head projections on hipBLASLt from 2 rows up (decode and
    prefill); the LM head runs rownorm + an fp32-output library GEMM."""
    monkeypatch.setenv("CAIN_LT_MIN_ROWS", "2")
    monkeypatch.delenv("CAIN_LT_LM_HEAD", raising=False)
    prompts = ["In 100 words, please give me information about India", "hi", "Elizabeth II, Queen"]
    eng = DecodeEngine(name, device="cuda", max_batch=4, max_context=256, keep_natural=True, seed=3)
    assert eng._desc.lt_min_rows == 2 and eng._layers[0].wo_lt and eng._desc.lm_head_lt and eng._desc.xn
    got = eng.last_logits(prompts)
    ref = ReferenceModel(eng.weights)
    for i, p in enumerate(prompts):
        want = ref.forward(torch.tensor([eng.encode(p)], device="cuda"))[0, -1]
        cos = torch.nn.functional.cosine_similarity(got[i].float(), want.float(), dim=0)
        assert cos > 0.995, (name, i, float(cos))
    r = eng.generate(prompts, 6, [dict(temperature=0.0, eos_id=-1)] * 3)
    assert all(x.eval_count == 6 for x in r)
    eng.close()


def test_engine_lt_default_off(monkeypatch):
    """The library path is opt-in: the hand-written wide-batch kernel (csrc/wgemm.hip) is the default."""
    monkeypatch.delenv("CAIN_LT_MIN_ROWS", raising=False)
    from cain_amd.engine.engine import lt_min_rows
    assert lt_min_rows(256) == 0 and lt_min_rows(64) == 0
    monkeypatch.setenv("CAIN_LT_MIN_ROWS", "128")
    assert lt_min_rows(256) == 128 and lt_min_rows(64) == 0 and lt_min_rows(256, "fp8") == 0


def test_engine_lt_lm_head_matches_hand_gemm(monkeypatch):
    """The library LM head (rownorm + fp32-output hipBLASLt) against the fused hand GEMM on the same weights."""
    monkeypatch.setenv("CAIN_LT_MIN_ROWS", "2")
    prompts = ["In 100 words, please give me information about India", "hi"]
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("CAIN_LT_LM_HEAD", flag)
        eng = DecodeEngine("tiny-llama3.1:8b", device="cuda", max_batch=2, max_context=128, seed=5)
        assert bool(eng._desc.lm_head_lt) == (flag == "1")
        out[flag] = eng.last_logits(prompts).float()
        eng.close()
    assert _rel(out["1"], out["0"]) < 1e-2
