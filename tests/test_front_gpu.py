"""The fused layer front (csrc/front.hip: QKV -> attention -> O of one layer in one launch, <= 4 rows) against the
three launches it replaces (qkv_rope -> attention -> skinny_gemm EPI_RESID) and a plain PyTorch fp32 layer.

Cases: decode rows on distinct cache slots with long random contexts (the prefetch of past KV blocks before the
in-launch wait), prefill rows of ONE sequence whose positions cross a 32-position block boundary (blocks written
by the same launch must not be prefetched), attention splits 1 / 8, repeated launches (the hand-off counters
must come back to zero).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from cain_amd import ops  # noqa: E402
from cain_amd.models.weights import fold_gain, pack_mfma_a, rope_pair_order  # noqa: E402

DEV = torch.device("cuda")


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _rope_tables(hd, T_max, theta=10000.0):
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(T_max, dtype=torch.float64)[:, None] * inv[None]
    return ang.cos().float().to(DEV), ang.sin().float().to(DEV)


def _rot(x, c, s_):
    half = x.shape[-1] // 2
    return torch.cat([x[..., :half] * c - x[..., half:] * s_, x[..., half:] * c + x[..., :half] * s_], -1)


def _layer(d, H, Hkv, hd, T_max, S, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    qkv_dim = (H + 2 * Hkv) * hd
    W = (torch.randn(qkv_dim, d, generator=g) * 0.03).bfloat16().to(DEV)
    Wo = (torch.randn(d, H * hd, generator=g) * 0.03).bfloat16().to(DEV)
    bias = torch.randn(qkv_dim, generator=g).to(DEV) * 0.1
    gain = (1 + 0.2 * torch.randn(d, generator=g)).bfloat16().to(DEV)
    per = rope_pair_order(hd).to(DEV)
    perm = torch.cat([h * hd + per for h in range(H + Hkv)] + [torch.arange((H + Hkv) * hd, qkv_dim, device=DEV)])
    k_nat = (torch.randn(S, Hkv, T_max, hd, generator=g)).bfloat16().to(DEV)
    v_nat = (torch.randn(S, Hkv, T_max, hd, generator=g)).bfloat16().to(DEV)
    return dict(W=W, Wo=Wo, bias=bias, gain=gain, perm=perm, Wp=pack_mfma_a(fold_gain(W[perm], gain)),
                Wop=pack_mfma_a(Wo), bp=bias[perm].contiguous(), k_nat=k_nat, v_nat=v_nat)


def _fp32_layer(L, x, slot, pos, H, Hkv, hd, cos_t, sin_t, eps):
    """fp32 reference of the layer front over the natural caches; returns the new residual rows."""
    xf = x.float()
    xn = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * L["gain"].float()
    y = (xn @ L["W"].float().t() + L["bias"]).bfloat16().float()
    K = L["k_nat"].float().clone()
    V = L["v_nat"].float().clone()
    M = x.shape[0]
    qs = []
    for m in range(M):
        p, s = int(pos[m]), int(slot[m])
        c, sn = cos_t[p], sin_t[p]
        qs.append(_rot(y[m, : H * hd].view(H, hd), c, sn))
        K[s, :, p] = _rot(y[m, H * hd:(H + Hkv) * hd].view(Hkv, hd), c, sn)
        V[s, :, p] = y[m, (H + Hkv) * hd:].view(Hkv, hd)
    G = H // Hkv
    out = torch.empty(M, H * hd, device=DEV)
    for m in range(M):
        p, s = int(pos[m]), int(slot[m])
        for h in range(H):
            sc = (qs[m][h] @ K[s, h // G, : p + 1].t()) / math.sqrt(hd)
            out[m, h * hd:(h + 1) * hd] = sc.softmax(-1) @ V[s, h // G, : p + 1]
    return xf + out.bfloat16().float() @ L["Wo"].float().t()


CONFIGS = [  # (d, H, Hkv, hd): qwen2:1.5b, llama3.1:8b, phi3-like (hd 96, no GQA), a small hd-64 shape
    (1536, 12, 2, 128),
    (4096, 32, 8, 128),
    (3072, 32, 32, 96),
    (1024, 16, 8, 64),
]


@pytest.mark.parametrize("d,H,Hkv,hd", CONFIGS)
@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("mode", ["decode", "prefill"])
def test_front_matches_three_launches_and_fp32(d, H, Hkv, hd, M, mode):
    T_max, S, eps = 1536, 6, 1e-6
    nsplits = [ns for ns in (1, 8, 2) if ops.front_eligible(M, d, H, Hkv, hd, ns)]
    if not nsplits:
        pytest.skip("shape not eligible for the fused front at this row count")
    torch.manual_seed(3)
    L = _layer(d, H, Hkv, hd, T_max, S, seed=d + M)
    cos_t, sin_t = _rope_tables(hd, T_max)
    if mode == "decode":  # distinct slots, long random contexts
        slot = torch.tensor([5, 0, 3, 1][:M], device=DEV, dtype=torch.int32)
        pos = torch.tensor([1400, 37, 640, 1][:M], device=DEV, dtype=torch.int32)
    else:  # rows of ONE sequence, positions across the 32-position block boundary
        slot = torch.full((M,), 2, device=DEV, dtype=torch.int32)
        pos = torch.arange(32 - M // 2 - 1, 32 - M // 2 - 1 + M, device=DEV, dtype=torch.int32)
    x0 = torch.randn(M, d, device=DEV).bfloat16()
    ref = _fp32_layer(L, x0, slot, pos, H, Hkv, hd, cos_t, sin_t, eps)
    scale = 1.0 / math.sqrt(hd)
    for ns in nsplits:
        outs = {}
        for fused in (False, True, True):  # the second fused launch reuses the (self-resetting) counters
            kc = ops.pack_kcache(L["k_nat"])
            vt = ops.pack_vcache(L["v_nat"])
            x = x0.clone()
            q = torch.zeros(M, H * hd, device=DEV, dtype=torch.bfloat16)
            attn = torch.zeros(M, H * hd, device=DEV, dtype=torch.bfloat16)
            if fused:
                if "flags" not in outs:
                    outs["flags"] = torch.zeros(4096, device=DEV, dtype=torch.int32)
                    outs["ctr"] = torch.zeros(M * Hkv, device=DEV, dtype=torch.int32)
                ops.layer_front(L["Wp"], L["bp"], L["Wop"], x, q, attn, kc, vt, slot, pos, cos_t, sin_t, H, Hkv,
                                hd, ns, scale, eps=eps, counters=outs["ctr"], flags=outs["flags"])
                torch.cuda.synchronize()
                assert int(outs["flags"].abs().sum()) == 0 and int(outs["ctr"].abs().sum()) == 0
                key = "fused"
            else:
                n = (H + 2 * Hkv) * hd
                ops.qkv_rope(L["Wp"], x, n, q, kc, vt, slot, pos, cos_t, sin_t, H, Hkv, hd, bias=L["bp"], norm=True,
                             eps=eps)
                ops.attention(q, kc, vt, slot, pos, H, Hkv, hd, ns, scale, out=attn)
                ops.skinny_gemm(L["Wop"], attn, d, ops.EPI_RESID, out=x)
                key = "three"
            if key in outs:
                assert torch.equal(outs[key][0], x), "fused launches must be deterministic"
            outs[key] = (x, q, attn, ops.unpack_kcache(kc), ops.unpack_vcache(vt))
        xf, qf, af, kf, vf = outs["fused"]
        x3, q3, a3, k3, v3 = outs["three"]
        assert rel_err(qf, q3) < 1e-2, ns
        assert rel_err(kf, k3) < 1e-2 and rel_err(vf, v3) < 1e-2, ns
        assert rel_err(af, a3) < 1e-2, ns
        assert rel_err(xf - x0.float(), x3.float() - x0.float()) < 2e-2, ns
        # against fp32: within the three-launch path's own distance (the residual is rounded to bf16 either way)
        e3 = rel_err(x3.float() - x0.float(), ref - x0.float())
        assert rel_err(xf - x0.float(), ref - x0.float()) <= 1.25 * e3 + 1e-3, (ns, e3)
