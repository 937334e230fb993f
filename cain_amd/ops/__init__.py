"""Python bindings of the hand-written gfx950 kernels (``libcain_kernels.so``).

Every op takes torch tensors living on the GPU and launches on the current
torch stream.  There is no silent eager fallback: if the native library is
missing or fails to load, the ops raise ``NativeOpsUnavailable`` (the engine's
torch-eager path is a separate, explicitly selected backend used on CPU).

Kernel inventory:

=====================  ==========================  =============================
op                     source                      replaces (Ollama/llama.cpp)
=====================  ==========================  =============================
``skinny_gemm``        csrc/gemm.hip               O / gate-up(+act) / down / LM head GEMV,
                       csrc/wgemm.hip              fused RMSNorm, residual epilogue (wgemm: the
                                                   LDS-DMA ring kernel for 64 < M <= 256 rows)
``qkv_rope``           csrc/gemm.hip               QKV GEMV + bias + RoPE + KV-cache append
``gemm_w8``            csrc/gemm_w8.hip            the same GEMMs on fp8 (e4m3) weights, <= 64 rows
``gemm_w8a8``          csrc/wgemm8.hip             fp8 weights x per-row fp8 activations, 16 < M <= 256
``gemm_w4``            csrc/gemm_w4.hip            the same GEMMs on MXFP4 (e2m1 + e8m0) weights, <= 64 rows
``gemm_q4``            csrc/gemm_q4.hip            the same GEMMs on GGUF Q4_0 / Q4_K blocks (exact values), any M
``rmsnorm``            csrc/norm.hip               RMSNorm (standalone; the engine fuses it)
``embed``              csrc/norm.hip               embedding gather (+Gemma scale)
``attention``          csrc/attention.hip          decode / prefill attention (split-K, in-kernel combine)
``sample``             csrc/sample.hip             repeat-penalty/temperature/top-k/top-p
``Plan``               csrc/runtime.hip            per-step schedule + hipGraph replay
=====================  ==========================  =============================
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path
from typing import Optional

import torch

HERE = Path(__file__).resolve().parent
# CAIN_KERNELS_LIB: another build of the library (A/B runs of a kernel change on one box)
LIB_PATH = Path(os.environ.get("CAIN_KERNELS_LIB") or HERE / "libcain_kernels.so")

EPI_BF16, EPI_RESID, EPI_F32, EPI_SILU, EPI_GELU, EPI_QKV_ROPE = 0, 1, 2, 3, 4, 5
EPI_KV_FP8 = 0x100  # or-ed into EPI_QKV_ROPE: the KV cache is fp8 e4m3 (csrc/gemm_epi.h)


class NativeOpsUnavailable(RuntimeError):
    pass


_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()

vp = ctypes.c_void_p
ci = ctypes.c_int
cf = ctypes.c_float


def load() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            if os.environ.get("CAIN_AUTOBUILD", "1") != "0":
                from .. import build
                build.build_kernels()
            if not LIB_PATH.exists():
                raise NativeOpsUnavailable(f"{LIB_PATH} missing: run `python -m cain_amd.build`")
        try:
            real = ctypes.CDLL(str(LIB_PATH))
        except OSError as exc:
            raise NativeOpsUnavailable(f"cannot load {LIB_PATH}: {exc}") from exc
        # an older build loaded for an A/B run (CAIN_KERNELS_LIB) may lack newer entry points: their signatures
        # are skipped (a call to one then fails by name)
        lib = _Lenient(real) if os.environ.get("CAIN_KERNELS_LIB") else real
        if int(real.cain_sample_params_size()) != SAMPLE_BYTES:  # also an A/B build from an older source
            raise NativeOpsUnavailable(f"{LIB_PATH} packs {int(real.cain_sample_params_size())}-byte sampling "
                                       f"options, this package {SAMPLE_BYTES}: rebuild (python -m cain_amd.build)")
        lib.cain_skinny_gemm_ex.argtypes = ([vp, vp, ci, ci, ci, ci, vp, ci, vp, ci, cf, vp, vp, vp, vp, vp, vp]
                                            + [ci] * 6 + [vp])
        lib.cain_gemm.argtypes = ([vp, vp, ci, ci, ci, ci, vp, ci, vp, ci, cf, vp, vp, vp, vp, vp, vp]
                                  + [ci] * 4 + [vp, ctypes.c_longlong, ci, ci, vp])
        lib.cain_gemm_w8.argtypes = ([vp, vp, vp, ci, ci, ci, ci, vp, ci, vp, ci, cf, vp, vp, vp, vp, vp, vp]
                                     + [ci] * 5 + [vp])
        lib.cain_gemm_w4.argtypes = ([vp, vp, vp, ci, ci, ci, ci, vp, ci, vp, ci, cf, vp, vp, vp, vp, vp, vp]
                                     + [ci] * 5 + [vp])
        lib.cain_gemm_w4_ex.argtypes = ([vp, vp, vp, ci, ci, ci, ci, vp, ci, vp, ci, cf, vp, vp, vp, vp, vp, vp]
                                        + [ci] * 4 + [vp, ctypes.c_longlong, ci, vp])
        lib.cain_gemm_w4_ws_bytes.restype = ctypes.c_longlong
        lib.cain_gemm_w4_ws_bytes.argtypes = [ci, ci, ci]
        lib.cain_gemm_w4_split.argtypes = [ci, ci, ci, ci, ctypes.c_longlong]
        lib.cain_gemm_w4_set_split.argtypes = [ci]
        lib.cain_gemm_w4_set_split_cap.argtypes = [ci]
        lib.cain_gemm_w4_set_split_min_quads.argtypes = [ci]
        lib.cain_gemm_w4_set_variant.argtypes = [ci]
        lib.cain_wgemm_set_inline.argtypes = [ci]
        lib.cain_gemm_q4.argtypes = ([ci, vp, vp, vp, vp, vp, ci, ci, ci, ci, vp, ci, vp, ci, cf, vp, vp, vp, vp, vp,
                                      vp] + [ci] * 5 + [vp])
        lib.cain_gemm_q4_rows.argtypes = [ci, ci]
        lib.cain_wgemm_inline.argtypes = [ci, ci, ci]
        lib.cain_wgemm_get_inline.argtypes = []
        lib.cain_gemm_w4_variant.argtypes = [ci, ci, ci, ci]
        lib.cain_gemm_w4_set_occupancy.argtypes = [ci]
        lib.cain_gemm_w8a8.argtypes = ([vp, vp, vp, ci, vp, ci, ci, ci, vp, ci, vp, vp, vp, vp, vp, vp, vp]
                                       + [ci] * 4 + [vp, ctypes.c_longlong, ci, vp])
        lib.cain_quant_rows.argtypes = [vp, ci, ci, ci, vp, ci, vp, ci, cf, vp]
        lib.cain_gemm_w4a8.argtypes = lib.cain_gemm_w8a8.argtypes
        lib.cain_w4a8_set_min_rows.argtypes = [ci]
        lib.cain_w8a8_eligible.argtypes = [ci, ci, ci]
        lib.cain_w8a8_ws_bytes.restype = ctypes.c_longlong
        lib.cain_w8a8_ws_bytes.argtypes = [ci, ci, ci]
        lib.cain_gemm_ws_bytes.restype = ctypes.c_longlong
        lib.cain_gemm_ws_bytes.argtypes = [ci, ci, ci]
        lib.cain_wgemm_set_min_m.argtypes = [ci]
        lib.cain_wgemm_eligible.argtypes = [ci, ci, ci]
        lib.cain_wgemm_set_shape.argtypes = [ci, ci, ci, ci, ci]
        lib.cain_wgemm_plan.argtypes = [ci, ci, ci]
        lib.cain_rmsnorm.argtypes = [vp, ci, vp, vp, ci, ci, ci, cf, vp]
        lib.cain_embed.argtypes = [vp, vp, vp, ci, ci, ci, cf, vp]
        lib.cain_attention.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, ci, ci, ci, cf, vp]
        lib.cain_attention_ex.argtypes = ([vp, vp, vp, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, ci, ci, ci, cf, ci, cf, cf]
                                          + [vp])
        lib.cain_attention_set_ring.argtypes = [ci]
        lib.cain_sample.argtypes = [vp, ci, ci, vp, vp, vp, ci, vp, vp, vp, vp, vp, ci, ci, vp, vp]
        lib.cain_sample_cm.argtypes = [vp, ci, ci, vp, vp, vp, vp, ci, vp, vp, vp, vp, vp, ci, ci, vp, vp]
        lib.cain_sample_lean.argtypes = [vp, ci, ci, vp, vp, vp, vp, ci, vp, vp, vp, vp, vp, ci, ci, vp, vp]
        lib.cain_gemm_set_cmax.argtypes = [vp]
        lib.cain_gemm_set_cmax.restype = None
        lib.cain_gemm_cmax_take.argtypes = []
        lib.cain_sample_set_cm.argtypes = [ci]
        lib.cain_gemm_set_skinny_split.argtypes = [ci]
        lib.cain_sample_ex.argtypes = [vp, ci, ci, vp, vp, vp, ci, vp, vp, vp, vp, vp, ci, ci, vp, vp,
                                       ctypes.c_longlong, vp]
        lib.cain_sample_set_trace.argtypes = [vp]
        lib.cain_sample_ws_bytes.restype = ctypes.c_longlong
        lib.cain_sample_ws_bytes.argtypes = [ci]
        lib.cain_plan_create.restype = vp
        lib.cain_plan_create.argtypes = [vp]
        lib.cain_plan_destroy.argtypes = [vp]
        lib.cain_plan_forward.argtypes = [vp, ci, vp, ci, ci, vp]
        lib.cain_plan_last_failure.restype = ctypes.c_char_p
        lib.cain_plan_capture.restype = vp
        lib.cain_plan_capture.argtypes = [vp, ci, vp, ci, vp, ctypes.POINTER(ci)]
        lib.cain_graph_launch.argtypes = [vp, vp]
        lib.cain_graph_destroy.argtypes = [vp]
        lib.cain_set_cu_budget.argtypes = [ci]
        lib.cain_cu_mask.argtypes = [ci, ci, ctypes.POINTER(ctypes.c_uint32), ci]
        lib.cain_stream_create_cu_limited.restype = vp
        lib.cain_stream_create_cu_limited.argtypes = [ci]
        lib.cain_stream_destroy.argtypes = [vp]
        if os.environ.get("CAIN_WGEMM_INLINE") and hasattr(real, "cain_wgemm_set_inline"):  # A/B runs
            real.cain_wgemm_set_inline(int(os.environ["CAIN_WGEMM_INLINE"]))
        if os.environ.get("CAIN_SAMPLE_CM"):  # A/B runs (set_sample_cm)
            real.cain_sample_set_cm(int(os.environ["CAIN_SAMPLE_CM"]))
        _lib = real
        return real


class _Lenient:
    """Signature setter over a CDLL that ignores symbols the library does not export."""

    class _Sink:
        def __setattr__(self, k, v):
            pass

    def __init__(self, lib):
        object.__setattr__(self, "_lib", lib)

    def __getattr__(self, name):
        try:
            return getattr(self._lib, name)
        except AttributeError:
            return _Lenient._Sink()


def available() -> bool:
    try:
        load()
        return True
    except NativeOpsUnavailable:
        return False


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


def _gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("cain_amd.ops kernels need GPU tensors")


# ---------------------------------------------------------------- ops
_ws_cache: dict = {}


def gemm_ws_bytes(n: int, k: int, m: int) -> int:
    """Workspace the batched GEMM path needs for this shape (0: the skinny kernel runs it)."""
    return int(load().cain_gemm_ws_bytes(n, k, m))


def set_wide_gemm_min_m(m: int) -> None:
    """Rows from which GEMMs run on the wide-batch kernel (csrc/wgemm.hip; default 64, 0 disables): A/B switch
    for tests and tuning, read at every launch and graph capture."""
    load().cain_wgemm_set_min_m(int(m))


def wide_gemm_eligible(n: int, k: int, m: int) -> bool:
    return bool(load().cain_wgemm_eligible(n, k, m))


def set_wide_gemm_plan(n: int, k: int, bm: int, ks: int, variant: int = -1) -> None:
    """Per-shape wide-GEMM plan (csrc/wgemm.hip): split count ``ks`` (<= 0: the default rule) and ring
    ``variant`` (< 0: the global one) for N = n, K = k with the bm-row tile (128 or 256)."""
    if load().cain_wgemm_set_shape(int(n), int(k), int(bm), int(ks), int(variant)) != 0:
        raise RuntimeError("wide-GEMM plan table full")


def set_wide_gemm_variant(v: int) -> None:
    """Global wide-GEMM ring variant (csrc/wgemm.hip; per-shape plans override it): 0 default, 4 fp32 slabs;
    7 / 8 / 9 the timestamped / DMA-only / MFMA-only diagnostic builds of tools/wgemm_trace.py / wgemm_bench.py."""
    load().cain_wgemm_set_variant(int(v))


def set_wide_gemm_inline(mode: int) -> None:
    """Split-K combine of the wide GEMM (csrc/wgemm.hip wg_inline_combine): 1 inside the GEMM launch (default),
    0 a separate wgemm_reduce_kernel launch, 2 inside the launch with partners that never wait (tests)."""
    load().cain_wgemm_set_inline(int(mode))


def wide_gemm_inline_mode() -> int:
    return int(load().cain_wgemm_get_inline())


def wide_gemm_inline(n: int, k: int, m: int) -> bool:
    """Whether the next wide-GEMM launch of this shape combines its split-K slabs in-launch."""
    return bool(load().cain_wgemm_inline(int(n), int(k), int(m)))


def clear_wide_gemm_plans() -> None:
    load().cain_wgemm_clear_shapes()


def wide_gemm_plan(n: int, k: int, m: int) -> Optional[tuple]:
    """(split count, ring variant) the next wide-GEMM launch of this shape uses; None if not eligible."""
    v = int(load().cain_wgemm_plan(n, k, m))
    return None if v < 0 else (v // 64, v % 64)


def _workspace(device, nbytes: int) -> Optional[torch.Tensor]:
    """Per-device zero-initialised GEMM workspace, grown on demand (its counters self-reset)."""
    if nbytes <= 0:
        return None
    key = torch.device(device)
    ws = _ws_cache.get(key)
    if ws is None or ws.numel() * 4 < nbytes:
        ws = torch.zeros(nbytes // 4 + 1, device=key, dtype=torch.int32)
        _ws_cache[key] = ws
    return ws


def _gemm_call(lib, wp, x, K, n, M, out, bias, norm, eps, slot, pos, cos_t, sin_t, kc, vtc, H, Hkv, hd, T_max, epi,
               waves, batched: bool):
    nbytes = gemm_ws_bytes(n, K, M) if batched else 0
    ws = _workspace(x.device, nbytes)
    return lib.cain_gemm(_p(wp), _p(x), x.stride(0), K, n, M, _p(out), out.stride(0), _p(bias), int(bool(norm)), eps,
                         _p(slot), _p(pos), _p(cos_t), _p(sin_t), _p(kc), _p(vtc), H, Hkv, hd, T_max, _p(ws),
                         nbytes, epi, waves, _stream())


def skinny_gemm(wp: torch.Tensor, x: torch.Tensor, n: int, epi: int = EPI_BF16, bias=None,
                out: Optional[torch.Tensor] = None, waves: int = 0, norm: bool = False, eps: float = 1e-6,
                batched: bool = True) -> torch.Tensor:
    """y[M, n] = epi(B(x)[M, K] @ W^T) with W packed by ``pack_mfma_a`` (gate/up interleaved for act epis).

    ``norm``: fused RMSNorm of x, y = rsqrt(mean(x^2) + eps) * (x @ W^T) where the norm gain must already
    be folded into W (``models.weights.fold_gain``).
    ``EPI_RESID``: ``out`` is the residual stream, updated in place.
    ``batched``: 16 < M <= 64 runs the LDS-staged split-K kernel (False forces the skinny kernel).
    """
    lib = load()
    _gpu(wp, x)
    M, K = x.shape
    assert x.dtype == torch.bfloat16 and x.stride(1) == 1
    assert wp.shape[1] * 32 == K and wp.shape[0] * 16 == n, (tuple(wp.shape), K, n)
    n_out = n // 2 if epi in (EPI_SILU, EPI_GELU) else n
    if epi == EPI_RESID:
        assert out is not None and out.shape == (M, n_out), "EPI_RESID updates `out` (the residual) in place"
    if out is None:
        out = torch.empty(M, n_out, device=x.device, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16)
    rc = _gemm_call(lib, wp, x, K, n, M, out, bias, norm, eps, None, None, None, None, None, None, 0, 0, 0, 0, epi,
                    waves, batched)
    _check(rc, "skinny_gemm")
    return out


def is_fp8_cache(t: torch.Tensor) -> bool:
    """An fp8 (e4m3) KV cache: uint8 storage (the engine's) or torch.float8_e4m3fn."""
    return t.dtype in (torch.uint8, torch.float8_e4m3fn)


def qkv_rope(wp, x, n, q_out, kc, vtc, slot, pos, cos_t, sin_t, H, Hkv, hd, bias=None, norm: bool = False,
             eps: float = 1e-6, waves: int = 0, batched: bool = True) -> None:
    """Fused QKV projection (+RMSNorm, +bias) -> RoPE -> Q buffer / K cache / V^T cache.  8-bit caches
    (``is_fp8_cache``) receive e4m3 elements (EPI_KV_FP8)."""
    lib = load()
    M, K = x.shape
    T_max = kc.shape[-2]
    epi = EPI_QKV_ROPE | (EPI_KV_FP8 if is_fp8_cache(kc) else 0)
    rc = _gemm_call(lib, wp, x, K, n, M, q_out, bias, norm, eps, slot, pos, cos_t, sin_t, kc, vtc, H, Hkv, hd,
                    T_max, epi, waves, batched)
    _check(rc, "qkv_rope")


def gemm_w8(wq: torch.Tensor, scale: torch.Tensor, x: torch.Tensor, n: int, epi: int = EPI_BF16, bias=None,
            out: Optional[torch.Tensor] = None, norm: bool = False, eps: float = 1e-6, rope=None,
            cmax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp8-weight GEMM (``csrc/gemm_w8.hip``, M <= 64): y = epi(B(x) @ (q * scale)^T) with q packed by
    ``models.weights.pack_mfma_a_fp8`` and ``scale`` the per-row fp32 scales.  Same epilogues and RMSNorm
    fusion as ``skinny_gemm``; ``rope`` = dict(kc, vtc, slot, pos, cos_t, sin_t, H, Hkv, hd) for
    ``EPI_QKV_ROPE`` (``out`` is then the Q buffer)."""
    lib = load()
    _gpu(wq, scale, x)
    M, K = x.shape
    assert x.dtype == torch.bfloat16 and x.stride(1) == 1 and 1 <= M <= 64
    assert wq.dtype == torch.uint8 and wq.shape[0] * 16 == n and wq.shape[1] * 64 == K, (tuple(wq.shape), K, n)
    assert scale.dtype == torch.float32 and scale.numel() == n
    n_out = n // 2 if epi in (EPI_SILU, EPI_GELU) else n
    if epi == EPI_RESID:
        assert out is not None and out.shape == (M, n_out), "EPI_RESID updates `out` (the residual) in place"
    if out is None:
        out = torch.empty(M, n_out, device=x.device, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16)
    r = rope or {}
    if epi == EPI_QKV_ROPE:
        assert rope is not None, "EPI_QKV_ROPE needs the rope/cache arguments"
    T_max = r["kc"].shape[-2] if rope else 0
    if rope and is_fp8_cache(r["kc"]):
        epi |= EPI_KV_FP8
    _cmax_set(lib, cmax, epi)
    rc = lib.cain_gemm_w8(_p(wq), _p(scale), _p(x), x.stride(0), K, n, M, _p(out), out.stride(0), _p(bias),
                          int(bool(norm)), eps, _p(r.get("slot")), _p(r.get("pos")), _p(r.get("cos_t")),
                          _p(r.get("sin_t")), _p(r.get("kc")), _p(r.get("vtc")), r.get("H", 0), r.get("Hkv", 0),
                          r.get("hd", 0), T_max, epi, _stream())
    _check(rc, "gemm_w8")
    _cmax_check(lib, cmax)
    return out


def gemm_w4(wq: torch.Tensor, wsc: torch.Tensor, x: torch.Tensor, n: int, epi: int = EPI_BF16, bias=None,
            out: Optional[torch.Tensor] = None, norm: bool = False, eps: float = 1e-6, rope=None,
            cmax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """MXFP4-weight GEMM (``csrc/gemm_w4.hip``, M <= 64): y = epi(B(x) @ dequant(codes, scales)^T) with
    (``wq``, ``wsc``) = ``models.weights.pack_mxfp4(...)``.  Same epilogues, RMSNorm fusion and ``rope`` arguments
    as ``gemm_w8``."""
    lib = load()
    _gpu(wq, wsc, x)
    M, K = x.shape
    assert x.dtype == torch.bfloat16 and x.stride(1) == 1 and 1 <= M <= 64
    assert wq.dtype == torch.uint8 and wq.shape[0] * 16 == n and wq.shape[1] * 128 == K, (tuple(wq.shape), K, n)
    assert wsc.dtype == torch.uint8 and wsc.numel() * 32 == n * K
    n_out = n // 2 if epi in (EPI_SILU, EPI_GELU) else n
    if epi == EPI_RESID:
        assert out is not None and out.shape == (M, n_out), "EPI_RESID updates `out` (the residual) in place"
    if out is None:
        out = torch.empty(M, n_out, device=x.device, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16)
    r = rope or {}
    if epi == EPI_QKV_ROPE:
        assert rope is not None, "EPI_QKV_ROPE needs the rope/cache arguments"
    T_max = r["kc"].shape[-2] if rope else 0
    if rope and is_fp8_cache(r["kc"]):
        epi |= EPI_KV_FP8
    nb = int(lib.cain_gemm_w4_ws_bytes(n, K, M))
    ws = _w4_ws(x.device, nb)
    _cmax_set(lib, cmax, epi)
    rc = lib.cain_gemm_w4_ex(_p(wq), _p(wsc), _p(x), x.stride(0), K, n, M, _p(out), out.stride(0), _p(bias),
                             int(bool(norm)), eps, _p(r.get("slot")), _p(r.get("pos")), _p(r.get("cos_t")),
                             _p(r.get("sin_t")), _p(r.get("kc")), _p(r.get("vtc")), r.get("H", 0), r.get("Hkv", 0),
                             r.get("hd", 0), T_max, _p(ws), nb, epi, _stream())
    _check(rc, "gemm_w4")
    _cmax_check(lib, cmax)
    return out


_W4_WS: dict = {}


def _cmax_set(lib, cmax, epi: int) -> None:
    """``cmax`` ([M][N / 16] fp32): the few-row fp32-logits GEMM also writes each row's 16-column chunk maxima (the
    chunk-maximum samplers' input, gemm_epi.h epi_cmax)."""
    if cmax is not None:
        assert epi == EPI_F32 and cmax.dtype == torch.float32 and cmax.is_contiguous()
        lib.cain_gemm_set_cmax(_p(cmax))


def _cmax_check(lib, cmax) -> None:
    if cmax is not None and int(lib.cain_gemm_cmax_take()) != 1:
        raise RuntimeError("this GEMM shape does not write chunk maxima (few-row stream kernels only)")


def gemm_q4(fmt: int, wq: torch.Tensor, sbuf: torch.Tensor, x: torch.Tensor, n: int, epi: int = EPI_BF16,
            bias=None, out: Optional[torch.Tensor] = None, norm: bool = False, eps: float = 1e-6, rope=None,
            gain: bool = False, cmax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """GGUF Q4_0 (``fmt`` 0) / Q4_K (1) weight GEMM (``csrc/gemm_q4.hip``; any M, 16-row launches): y = epi(B(x) @
    W^T) with W the blocks' exact values and (``wq``, ``sbuf``) = ``models.q4.pack_q4(...)``; ``gain``: the scale
    buffer ends with the fp32 RMSNorm gain, applied to the activations (``norm`` must be set).  Same epilogues,
    RMSNorm fusion and ``rope`` arguments as ``gemm_w8``."""
    lib = load()
    _gpu(wq, sbuf, x)
    M, K = x.shape
    assert x.dtype == torch.bfloat16 and x.stride(1) == 1 and M >= 1
    assert wq.dtype == torch.uint8 and wq.shape[0] * 16 == n and wq.shape[1] * 128 == K, (tuple(wq.shape), K, n)
    sc_bytes, dd_bytes = n * K // 16, (n * K // 64 if fmt == 1 else 0)
    assert sbuf.dtype == torch.uint8 and sbuf.numel() == sc_bytes + dd_bytes + (4 * K if gain else 0)
    n_out = n // 2 if epi in (EPI_SILU, EPI_GELU) else n
    if epi == EPI_RESID:
        assert out is not None and out.shape == (M, n_out), "EPI_RESID updates `out` (the residual) in place"
    if out is None:
        out = torch.empty(M, n_out, device=x.device, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16)
    r = rope or {}
    if epi == EPI_QKV_ROPE:
        assert rope is not None, "EPI_QKV_ROPE needs the rope/cache arguments"
    T_max = r["kc"].shape[-2] if rope else 0
    if rope and is_fp8_cache(r["kc"]):
        epi |= EPI_KV_FP8
    base = sbuf.data_ptr()
    _cmax_set(lib, cmax, epi)
    rc = lib.cain_gemm_q4(int(fmt), _p(wq), base, base + sc_bytes, (base + sc_bytes + dd_bytes) if gain else None,
                          _p(x), x.stride(0), K, n, M, _p(out), out.stride(0), _p(bias), int(bool(norm)), eps,
                          _p(r.get("slot")), _p(r.get("pos")), _p(r.get("cos_t")), _p(r.get("sin_t")),
                          _p(r.get("kc")), _p(r.get("vtc")), r.get("H", 0), r.get("Hkv", 0), r.get("hd", 0), T_max,
                          epi, _stream())
    _check(rc, "gemm_q4")
    _cmax_check(lib, cmax)
    return out


def _w4_ws(device, nbytes: int) -> torch.Tensor:
    """Zeroed split-K workspace of the W4 GEMMs (its tickets are left zero by every launch), grown as needed."""
    t = _W4_WS.get(device)
    if t is None or t.numel() < nbytes:
        t = _W4_WS[device] = torch.zeros(max(nbytes, 1 << 16), device=device, dtype=torch.uint8)
    return t


def set_w4_split(ks: int) -> None:
    """Split-K of the few-row MXFP4 stream kernel (csrc/gemm_w4.hip w4_split): 0 = the rule (narrow outputs over
    fewer tiles than CUs get up to 4 k ranges of >= 32 quads), 1 = off, k > 1 = k ranges wherever the shape allows."""
    load().cain_gemm_w4_set_split(int(ks))


def set_w4_split_cap(cap: int) -> None:
    """A/B of the split rule's budget: tiles x k ranges <= ``cap`` x CUs (1: the rule)."""
    load().cain_gemm_w4_set_split_cap(int(cap))


def set_w4_split_min_quads(q: int) -> None:
    """A/B of the split rule's shortest k range, in 128-wide quads (32: the rule)."""
    load().cain_gemm_w4_set_split_min_quads(int(q))


def w4_split(n: int, k: int, m: int, epi: int, ws_bytes: int = 1 << 30) -> int:
    """k ranges the W4 GEMM of this shape runs with (given a workspace of ``ws_bytes``)."""
    return int(load().cain_gemm_w4_split(n, k, m, epi, ws_bytes))


def set_w4_variant(v: int) -> None:
    """Force the few-row MXFP4 kernel shape (gemm_w4.hip W4Var index; -1: the shape rule; a stream shape whose LDS
    copy cannot hold the rows falls back to the rule).  Tests / tuning."""
    load().cain_gemm_w4_set_variant(int(v))


def set_w4_occupancy(wgs_per_cu: int) -> None:
    """Workgroups per CU of the persistent single-stream MXFP4 grid (0: 2 of 8 waves / 4 of 4 waves).  Tuning."""
    load().cain_gemm_w4_set_occupancy(int(wgs_per_cu))


def w4_variant(n: int, k: int, m: int, epi: int = EPI_BF16) -> int:
    """The W4Var index the shape rule picks for an (N, K, M) problem with epilogue ``epi``."""
    return int(load().cain_gemm_w4_variant(int(n), int(k), int(m), int(epi)))


def quant_rows(x: torch.Tensor, norm: bool = False, eps: float = 1e-6):
    """Per-row e4m3 quantisation of bf16 activations (csrc/wgemm8.hip quant_rows_kernel): returns (x8 uint8
    [M, K], xs fp32 [M]) with x ~= e4m3(x8) * amax/448 and xs = amax/448 * (rsqrt(mean(x^2) + eps) if norm)."""
    lib = load()
    _gpu(x)
    M, K = x.shape
    assert x.dtype == torch.bfloat16 and x.stride(1) == 1
    x8 = torch.empty(M, K, device=x.device, dtype=torch.uint8)
    xs = torch.empty(M, device=x.device, dtype=torch.float32)
    _check(lib.cain_quant_rows(_p(x), x.stride(0), K, M, _p(x8), K, _p(xs), int(bool(norm)), eps, _stream()),
           "quant_rows")
    return x8, xs


def w8a8_eligible(n: int, k: int, m: int) -> bool:
    return bool(load().cain_w8a8_eligible(n, k, m))


def gemm_w8a8(wq8: torch.Tensor, scale: torch.Tensor, x: torch.Tensor, n: int, epi: int = EPI_BF16, bias=None,
              out: Optional[torch.Tensor] = None, norm: bool = False, eps: float = 1e-6, rope=None) -> torch.Tensor:
    """W8A8 wide GEMM (csrc/wgemm8.hip, 16 < M <= 256): the bf16 rows of ``x`` are quantised per row to e4m3
    (``quant_rows``, the RMSNorm folded into the row scale when ``norm``), then y = epi(xs * scale * x8 . q^T)
    with q packed by ``models.weights.pack_mfma_a_fp8_k128``.  Epilogues and ``rope`` as ``gemm_w8``."""
    lib = load()
    _gpu(wq8, scale, x)
    M, K = x.shape
    assert wq8.dtype == torch.uint8 and wq8.shape[0] * 16 == n and wq8.shape[1] * 64 == K, (tuple(wq8.shape), K, n)
    assert w8a8_eligible(n, K, M), (n, K, M)
    n_out = n // 2 if epi in (EPI_SILU, EPI_GELU) else n
    if epi == EPI_RESID:
        assert out is not None and out.shape == (M, n_out), "EPI_RESID updates `out` (the residual) in place"
    if out is None:
        out = torch.empty(M, n_out, device=x.device, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16)
    x8, xs = quant_rows(x, norm, eps)
    r = rope or {}
    if epi == EPI_QKV_ROPE:
        assert rope is not None, "EPI_QKV_ROPE needs the rope/cache arguments"
        if is_fp8_cache(r["kc"]):
            epi |= EPI_KV_FP8
    T_max = r["kc"].shape[-2] if rope else 0
    nbytes = int(lib.cain_w8a8_ws_bytes(n, K, M))
    ws = _workspace(x.device, nbytes)
    rc = lib.cain_gemm_w8a8(_p(wq8), _p(scale), _p(x8), K, _p(xs), K, n, M, _p(out), out.stride(0), _p(bias),
                            _p(r.get("slot")), _p(r.get("pos")), _p(r.get("cos_t")), _p(r.get("sin_t")),
                            _p(r.get("kc")), _p(r.get("vtc")), r.get("H", 0), r.get("Hkv", 0), r.get("hd", 0), T_max,
                            _p(ws), nbytes, epi, _stream())
    _check(rc, "gemm_w8a8")
    return out


def gemm_w4a8(wq: torch.Tensor, wsc: torch.Tensor, x: torch.Tensor, n: int, epi: int = EPI_BF16, bias=None,
              out: Optional[torch.Tensor] = None, norm: bool = False, eps: float = 1e-6, rope=None) -> torch.Tensor:
    """W4A8 wide GEMM (csrc/wgemm8.hip FP4, 16 < M <= 256): MXFP4 weights in the few-row kernel's packing
    (``models.weights.pack_mxfp4``: wq uint8 [N/16, K/128, 64, 16], wsc e8m0 bytes [N/16, K/128, 64]) on the
    block-scaled f8f6f4 MFMA against the per-row e4m3 quantisation of ``x`` (``quant_rows``); y = epi(xs * x8 . W^T).
    Epilogues and ``rope`` as ``gemm_w8a8``."""
    lib = load()
    _gpu(wq, wsc, x)
    M, K = x.shape
    assert wq.dtype == torch.uint8 and tuple(wq.shape) == (n // 16, K // 128, 64, 16), (tuple(wq.shape), K, n)
    assert wsc.dtype == torch.uint8 and wsc.numel() * 32 == n * K, (tuple(wsc.shape), K, n)
    assert w8a8_eligible(n, K, M), (n, K, M)
    n_out = n // 2 if epi in (EPI_SILU, EPI_GELU) else n
    if epi == EPI_RESID:
        assert out is not None and out.shape == (M, n_out), "EPI_RESID updates `out` (the residual) in place"
    if out is None:
        out = torch.empty(M, n_out, device=x.device, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16)
    x8, xs = quant_rows(x, norm, eps)
    r = rope or {}
    if epi == EPI_QKV_ROPE:
        assert rope is not None, "EPI_QKV_ROPE needs the rope/cache arguments"
        if is_fp8_cache(r["kc"]):
            epi |= EPI_KV_FP8
    T_max = r["kc"].shape[-2] if rope else 0
    nbytes = int(lib.cain_w8a8_ws_bytes(n, K, M))
    ws = _workspace(x.device, nbytes)
    rc = lib.cain_gemm_w4a8(_p(wq), _p(wsc), _p(x8), K, _p(xs), K, n, M, _p(out), out.stride(0), _p(bias),
                            _p(r.get("slot")), _p(r.get("pos")), _p(r.get("cos_t")), _p(r.get("sin_t")),
                            _p(r.get("kc")), _p(r.get("vtc")), r.get("H", 0), r.get("Hkv", 0), r.get("hd", 0), T_max,
                            _p(ws), nbytes, epi, _stream())
    _check(rc, "gemm_w4a8")
    return out


def set_w4a8_min_rows(m: int) -> None:
    """Rows above which an MXFP4 engine's forwards run the W4A8 wide kernel instead of the W4A16 few-row one
    (runtime.hip; default 16, the W4A8 minimum: W4A8 is 1.5-2.7x faster at 24-64 rows,
    profiles/r4/ab/w4a8_crossover.txt).  Read at every forward / graph capture."""
    load().cain_w4a8_set_min_rows(int(m))


def rmsnorm(x: torch.Tensor, g: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    lib = load()
    _gpu(x, g)
    M, d = x.shape
    out = torch.empty_like(x) if out is None else out
    _check(lib.cain_rmsnorm(_p(x), x.stride(0), _p(g), _p(out), out.stride(0), M, d, eps, _stream()), "rmsnorm")
    return out


def embed(tok: torch.Tensor, table: torch.Tensor, scale: float = 1.0, out=None) -> torch.Tensor:
    lib = load()
    M = tok.shape[0]
    d = table.shape[1]
    out = torch.empty(M, d, device=table.device, dtype=table.dtype) if out is None else out
    _check(lib.cain_embed(_p(tok), _p(table), _p(out), out.stride(0), M, d, scale, _stream()), "embed")
    return out


# ---------------------------------------------------------------- KV-cache layout (attention.hip header)
def pack_kcache(k: torch.Tensor) -> torch.Tensor:
    """Natural K ``[..., T, hd]`` -> the fragment-major K cache layout (same shape and element count):
    per 16 positions x 32 head dims one 1-KiB MFMA A fragment, lane = (t & 15) + 16 * ((d & 31) >> 3)."""
    *lead, T, hd = k.shape
    n = len(lead)
    t = k.reshape(*lead, T // 16, 16, hd // 32, 4, 8)                 # [u, r, s, q, e]
    t = t.permute(*range(n), n, n + 2, n + 3, n + 1, n + 4)           # [u, s, q, r, e]
    return t.contiguous().reshape(*lead, T, hd)


def unpack_kcache(p: torch.Tensor) -> torch.Tensor:
    *lead, T, hd = p.shape
    n = len(lead)
    t = p.reshape(*lead, T // 16, hd // 32, 4, 16, 8)                 # [u, s, q, r, e]
    t = t.permute(*range(n), n, n + 3, n + 1, n + 2, n + 4)           # [u, r, s, q, e]
    return t.contiguous().reshape(*lead, T, hd)


def pack_vcache(v: torch.Tensor) -> torch.Tensor:
    """Natural V ``[..., T, hd]`` -> the fragment-major V^T cache layout, returned as ``[..., hd, T]`` (the
    engine's buffer shape): per 16 head dims x 32 positions one 1-KiB PV A fragment in the permuted k order
    of P, lane = (d & 15) + 16 * ((t & 15) >> 2), element 4 * ((t >> 4) & 1) + (t & 3)."""
    *lead, T, hd = v.shape
    n = len(lead)
    t = v.reshape(*lead, T // 32, 2, 4, 4, hd // 16, 16)              # [b, h, hq, j, c, dr]
    t = t.permute(*range(n), n, n + 4, n + 2, n + 5, n + 1, n + 3)    # [b, c, hq, dr, h, j]
    return t.contiguous().reshape(*lead, hd, T)


def unpack_vcache(p: torch.Tensor) -> torch.Tensor:
    """Inverse of ``pack_vcache``: ``[..., hd, T]`` buffer -> natural V ``[..., T, hd]``."""
    *lead, hd, T = p.shape
    n = len(lead)
    t = p.reshape(*lead, T // 32, hd // 16, 4, 16, 2, 4)              # [b, c, hq, dr, h, j]
    t = t.permute(*range(n), n, n + 4, n + 2, n + 5, n + 1, n + 3)    # [b, h, hq, j, c, dr]
    return t.contiguous().reshape(*lead, T, hd)


def kfrag_off(t: int, d: int, hd: int) -> int:
    """Host mirror of common.h kfrag_off (element offset inside one (slot, kv head) block)."""
    return ((t >> 4) * (hd >> 5) + (d >> 5)) * 512 + ((t & 15) + 16 * ((d & 31) >> 3)) * 8 + (d & 7)


def vfrag_off(t: int, d: int, hd: int) -> int:
    """Host mirror of common.h vfrag_off."""
    return ((t >> 5) * (hd >> 4) + (d >> 4)) * 512 + ((d & 15) + 16 * ((t & 15) >> 2)) * 8 + 4 * ((t >> 4) & 1) + (t & 3)


def attention_ml_floats(M: int, H: int, Hkv: int, nsplit: int) -> int:
    """Size of the (max, sum) partial workspace: one 128-B-aligned region per (row, kv head)."""
    G = H // Hkv
    return M * Hkv * ((G * nsplit * 2 + 31) // 32) * 32


def attention(q, kc, vtc, slot, pos, H, Hkv, hd, nsplit, scale, out=None, part_o=None, part_ml=None,
              counters=None, kscale: float = 1.0, vscale: float = 1.0):
    """Decode attention over the fragment-major caches (csrc/attention.hip); 8-bit caches (``is_fp8_cache``)
    hold e4m3 elements whose values are element * kscale / vscale."""
    lib = load()
    M = q.shape[0]
    T_max = kc.shape[-2]
    if part_o is None:
        part_o = torch.empty(M * H * nsplit * hd, device=q.device, dtype=torch.float32)
        part_ml = torch.empty(attention_ml_floats(M, H, Hkv, nsplit), device=q.device, dtype=torch.float32)
    if counters is None:
        counters = torch.zeros(M * Hkv, device=q.device, dtype=torch.int32)
    out = torch.empty(M, H * hd, device=q.device, dtype=torch.bfloat16) if out is None else out
    kv8 = is_fp8_cache(kc)
    assert kv8 == is_fp8_cache(vtc)
    _check(lib.cain_attention_ex(_p(q), _p(kc), _p(vtc), _p(slot), _p(pos), _p(part_o), _p(part_ml), _p(counters),
                                 _p(out), out.stride(0), M, H, Hkv, hd, T_max, nsplit, scale, int(kv8), kscale,
                                 vscale, _stream()),
           "attention")
    return out


def set_sample_cm(mode: int) -> None:
    """Chunk-maximum sampler (the LM head writes 16-column chunk maxima, the sampler reads only the chunks above a
    provable threshold; same tokens).  mode 0 off, 1 the round-3 chunk-maximum kernel on every decode forward, 2
    that kernel on forwards of more than 64 rows (42 vs 62 us at 256 rows; the two-stage kernel below), 3 the lean
    chunk-maximum kernel (sample.hip sample_lean_kernel) on every forward whose LM head wrote the maxima (the
    default: 10.3 vs 30.0 us in-graph at batch 1, profiles/r6/sampler/).  A/B switch for tests and profiles, read at
    every forward / graph capture (env CAIN_SAMPLE_CM at load)."""
    load().cain_sample_set_cm(int(mode))


def set_skinny_split(mode: int) -> None:
    """Split-K rule of the few-row (<= 16) skinny GEMM (gemm.hip skinny_split): 0 never, 1 narrow long-K grids
    (default).  Takes effect at the next launch; an
    engine's workspace is sized at construction, so switch before building one."""
    load().cain_gemm_set_skinny_split(int(mode))


def cu_mask(n_cu: int, total: int = 256) -> list:
    """The 32-bit words of the CU mask a CU-limited stream uses (runtime.hip cain_cu_mask): n_cu of ``total`` CUs
    as evenly spaced whole groups of 8 consecutive bits (balanced over the XCDs under either CU numbering)."""
    words = (total + 31) // 32
    arr = (ctypes.c_uint32 * words)()
    if load().cain_cu_mask(int(n_cu), int(total), arr, words) != 0:
        raise ValueError(f"no CU mask of {n_cu} of {total} CUs (multiples of 8 only)")
    return list(arr)


def set_cu_budget(n_cu: int) -> None:
    """CUs the launch sizing of persistent / CU-proportional grids assumes (0: the device's).  The engine sets it
    around every forward and graph capture of a CU-limited engine (``DecodeEngine(cu_limit=...)``)."""
    load().cain_set_cu_budget(int(n_cu))


def cu_budget() -> int:
    return int(load().cain_get_cu_budget())


def sample_cm_mode() -> int:
    """The chunk-maximum sampler mode in effect (see set_sample_cm)."""
    return int(load().cain_sample_cm_enabled())


def set_attention_ring(variant: int) -> None:
    """LDS-DMA ring body of the wide decode attention (csrc/attention.hip attn_ring_kernel; hd 128, bf16 cache,
    one split, 2 to 64 (row, kv head) pairs per CU): 0 off (the register kernel), 1 on (the default).  A/B switch
    for tests and profiles, read at every launch and graph capture."""
    load().cain_attention_set_ring(int(variant))


SAMPLE_DTYPE = [("temperature", "f4"), ("top_p", "f4"), ("repeat_penalty", "f4"), ("top_k", "i4"),
                ("repeat_last_n", "i4"), ("eos_id", "i4"), ("stop", "i4", (3,)), ("seed", "u8")]
SAMPLE_BYTES = 48  # sizeof(SampleParams), csrc/sample.hip (cain_sample_params_size)


def sample_params_tensor(rows, device) -> torch.Tensor:
    """Pack per-row sampling options (list of dicts; ``stop``: up to 3 further stop ids, default none) into the
    kernel's 48-byte struct array."""
    import numpy as np

    arr = np.zeros(len(rows), dtype=np.dtype(SAMPLE_DTYPE, align=True))
    for i, r in enumerate(rows):
        for f in SAMPLE_DTYPE:
            k = f[0]
            if k == "stop":
                st = [int(x) for x in r.get("stop", ())][:3]
                arr[i][k] = st + [-1] * (3 - len(st))
            else:
                arr[i][k] = r[k]
    assert arr.dtype.itemsize == SAMPLE_BYTES
    return torch.from_numpy(arr.view(np.uint8).copy()).to(device)


def sample(logits, tok, pos, gen, n_gen, max_new, done, hist, slot, params, T_max, split: bool = False,
           cmax=None, lean: bool = False) -> None:
    """On-device sampling + decode-state update (csrc/sample.hip).  ``split``: the two-stage kernel (vocabulary
    slices on 16 workgroups per row, last-arriver merge) that decode forwards of <= 64 rows use; ``cmax`` ([M][V/16]
    fp32 maxima of the logits' 16-column chunks, as the few-row LM head writes them): the chunk-maximum kernel that
    single-stream decode uses (``lean``: the lean chunk-maximum kernel); otherwise the one-workgroup-per-row
    kernel."""
    lib = load()
    M, V = logits.shape[0], logits.shape[1]
    if cmax is not None and lean:
        _check(lib.cain_sample_lean(_p(logits), logits.stride(0), V, _p(cmax), _p(tok), _p(pos), _p(gen),
                                    gen.stride(0), _p(n_gen), _p(max_new), _p(done), _p(hist), _p(slot), T_max, M,
                                    _p(params), _stream()), "sample_lean")
        return
    if cmax is not None:
        _check(lib.cain_sample_cm(_p(logits), logits.stride(0), V, _p(cmax), _p(tok), _p(pos), _p(gen), gen.stride(0),
                                  _p(n_gen), _p(max_new), _p(done), _p(hist), _p(slot), T_max, M, _p(params),
                                  _stream()), "sample_cm")
        return
    if split:
        nb = int(lib.cain_sample_ws_bytes(M))
        ws = _sample_ws(logits.device, nb)
        _check(lib.cain_sample_ex(_p(logits), logits.stride(0), V, _p(tok), _p(pos), _p(gen), gen.stride(0),
                                  _p(n_gen), _p(max_new), _p(done), _p(hist), _p(slot), T_max, M, _p(params), _p(ws),
                                  nb, _stream()), "sample")
        return
    _check(lib.cain_sample(_p(logits), logits.stride(0), V, _p(tok), _p(pos), _p(gen), gen.stride(0), _p(n_gen),
                           _p(max_new), _p(done), _p(hist), _p(slot), T_max, M, _p(params), _stream()), "sample")


_SAMPLE_WS: dict = {}


def _sample_ws(device, nbytes: int) -> torch.Tensor:
    """Zeroed sampler workspace per device (its tickets self-reset), grown on demand."""
    t = _SAMPLE_WS.get(device)
    if t is None or t.numel() * 4 < nbytes:
        t = _SAMPLE_WS[device] = torch.zeros((nbytes + 3) // 4, device=device, dtype=torch.int32)
    return t
