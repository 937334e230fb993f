"""Fragment-major KV-cache layout (attention.hip header): the torch pack/unpack helpers are exact
inverses and place every (position, head dim) element where the kernels' offset formulas (common.h
kfrag_off / vfrag_off, mirrored in cain_amd.ops) put it.  CPU only."""
import pytest
import torch

from cain_amd import ops


@pytest.mark.parametrize("hd", [64, 96, 128, 256])
def test_kcache_pack_roundtrip_and_offsets(hd):
    T = 64
    k = torch.arange(2 * T * hd, dtype=torch.float32).reshape(2, T, hd)
    p = ops.pack_kcache(k)
    assert p.shape == k.shape
    assert torch.equal(ops.unpack_kcache(p), k)
    flat = p[1].reshape(-1)
    for t in (0, 5, 16, 31, 47, 63):
        for d in (0, 7, 8, 31, 32, hd - 1):
            assert flat[ops.kfrag_off(t, d, hd)] == k[1, t, d], (t, d)
    # one 16 x 32 tile = one MFMA A fragment: lane l holds row l & 15, k-group l >> 4
    frag = p[0].reshape(-1)[:512].reshape(64, 8)
    for lane in (0, 17, 63):
        assert torch.equal(frag[lane], k[0, lane & 15, 8 * (lane >> 4): 8 * (lane >> 4) + 8])


@pytest.mark.parametrize("hd", [64, 96, 128, 256])
def test_vcache_pack_roundtrip_and_offsets(hd):
    T = 96
    v = torch.randn(3, T, hd)
    p = ops.pack_vcache(v)
    assert p.shape == (3, hd, T)
    assert torch.equal(ops.unpack_vcache(p), v)
    flat = p[2].reshape(-1)
    for t in (0, 3, 4, 15, 16, 20, 31, 32, 95):
        for d in (0, 1, 15, 16, hd - 1):
            assert flat[ops.vfrag_off(t, d, hd)] == v[2, t, d], (t, d)
    # lane (d, hq) of a fragment holds positions 4hq..4hq+3 then 16+4hq..16+4hq+3 (P's k order)
    frag = p[0].reshape(-1)[:512].reshape(64, 8)
    for lane in (0, 21, 63):
        d, hq = lane & 15, lane >> 4
        want = torch.cat([v[0, 4 * hq: 4 * hq + 4, d], v[0, 16 + 4 * hq: 16 + 4 * hq + 4, d]])
        assert torch.equal(frag[lane], want)


def test_pack_mfma_a_fp8_k128_layout():
    """W8A8 packing: lane g*16 + r of block (t, p) holds W[16t + r][64p + 16g .. +15]."""
    from cain_amd.models.weights import pack_mfma_a_fp8_k128
    torch.manual_seed(0)
    q = torch.randn(32, 256).to(torch.float8_e4m3fn)
    p = pack_mfma_a_fp8_k128(q)
    assert p.shape == (2, 4, 64, 16) and p.dtype == torch.uint8
    u = q.view(torch.uint8)
    for t, pp, g, r in [(0, 0, 0, 0), (1, 3, 2, 5), (0, 2, 3, 15), (1, 1, 1, 9)]:
        assert torch.equal(p[t, pp, g * 16 + r], u[16 * t + r, 64 * pp + 16 * g: 64 * pp + 16 * g + 16])
