"""Autoregressive decode engine (the on-device arm's LLM; replaces Ollama/llama.cpp).

Reference: the reference never runs a model itself — it POSTs to an external
Ollama server (experiment/RunnerConfig.py:122-131).  SURVEY §2.3 row 1 and
§3.4 specify what replaces it: tokenize, prefill, autoregressive decode with a
KV cache and Ollama's sampling, returning Ollama's statistics
(``prompt_eval_count``, ``eval_count``, ``*_duration`` in ns).

Backends
--------
``hip``    the MI355X path: packed bf16 weights resident in HBM, the hand-written
           gfx950 kernels of ``cain_amd.ops`` sequenced by the native runtime
           (``csrc/runtime.hip``) and replayed from hipGraphs — ``steps_per_graph``
           decode steps per graph launch, the sampler advancing tok/pos on the
           device, one host sync per generation.
``torch``  torch-eager oracle (``models/reference.py``): CPU tests / debugging.

Batching: up to ``max_batch`` (≤ 256) sequences decode together ("trial
batching") — each row has its own cache slot, position, budget
and sampling options; rows that finish early idle until the batch ends.
Prefill: every prompt token but the last goes through the same forward as
≤128-row chunks (rows carry their own slot/position, so the decode attention
kernel doubles as causal prefill attention); the last prompt token is the
first decode step's input, so no separate prefill LM-head path exists.
"""
from __future__ import annotations

import ctypes
import math
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from ..models.config import ModelConfig, get_config, rope_inv_freq
from ..models.hf import checkpoint_for, load_hf_weights, load_pretrained, load_tokenizer
from ..models.tokenizer import get_tokenizer
from ..models.weights import WEIGHT_DTYPES, ModelWeights, pack_for_engine, random_weights, roundtrip_weights

#: Ollama's default sampling options (SURVEY §2.4 "Sampling" row)
OLLAMA_DEFAULTS = dict(temperature=0.8, top_k=40, top_p=0.9, repeat_penalty=1.1, repeat_last_n=64, seed=None)

MAX_ROWS = 256  # rows per forward: decode batch (runtime.hip CAIN_MAX_ROWS)
PREFILL_ROWS = 128  # prompt tokens per prefill forward
W8_MAX_ROWS = 64  # few-row fp8 / MXFP4 weight kernels (gemm_w8.hip / gemm_w4.hip): rows per forward without W8A8
W8A8_MIN_ROWS = 16  # fp8 engines run forwards of more rows on the W8A8 wide kernel (csrc/wgemm8.hip)


@dataclass
class GenResult:
    model: str
    prompt_tokens: List[int]
    tokens: List[int]
    text: str
    done_reason: str
    load_duration_ns: int = 0
    prompt_eval_duration_ns: int = 0
    eval_duration_ns: int = 0
    total_duration_ns: int = 0

    @property
    def prompt_eval_count(self) -> int:
        return len(self.prompt_tokens)

    @property
    def eval_count(self) -> int:
        return len(self.tokens)

    def ollama_json(self, created_at: Optional[str] = None) -> Dict:
        import datetime

        return {
            "model": self.model,
            "created_at": created_at or datetime.datetime.utcnow().isoformat() + "Z",
            "response": self.text,
            "done": True,
            "done_reason": self.done_reason,
            "context": [],
            "total_duration": self.total_duration_ns,
            "load_duration": self.load_duration_ns,
            "prompt_eval_count": self.prompt_eval_count,
            "prompt_eval_duration": self.prompt_eval_duration_ns,
            "eval_count": self.eval_count,
            "eval_duration": self.eval_duration_ns,
        }


def _row_options(opts: Optional[Dict], cfg: ModelConfig, index: int, base_seed: int) -> Dict:
    o = dict(OLLAMA_DEFAULTS)
    if opts:
        o.update({k: v for k, v in opts.items() if v is not None and k in OLLAMA_DEFAULTS})
    seed = o.get("seed")
    if seed is None:
        seed = (base_seed * 1000003 + index * 7919 + time.monotonic_ns()) & 0xFFFFFFFFFFFF
    return dict(temperature=float(o["temperature"]), top_p=float(o["top_p"]),
                repeat_penalty=float(o["repeat_penalty"]), top_k=int(o["top_k"]),
                repeat_last_n=int(o["repeat_last_n"]),
                eos_id=int(opts.get("eos_id", cfg.eos_id)) if opts and "eos_id" in opts else int(cfg.eos_id),
                # further stop ids: the caller's, else the model's unless the caller set eos_id (forced lengths:
                # eos_id -1 disables every stop)
                stop=tuple(int(x) for x in (opts["stop_ids"] if opts and "stop_ids" in opts else
                                            () if opts and "eos_id" in opts else cfg.stop_ids))[:3],
                seed=int(seed) & 0xFFFFFFFFFFFFFFFF)


def _stopped(toks: List[int], o: Dict) -> bool:
    """A generation that ended on one of its row's stop ids (done_reason "stop")."""
    return bool(toks) and ((o["eos_id"] >= 0 and toks[-1] == o["eos_id"]) or toks[-1] in o.get("stop", ()))


# ============================================================== ctypes structs
LAYER_FIELDS = ("wqkv", "bqkv", "wo", "wgu", "wdown", "sqkv", "so", "sgu", "sdown", "wqkv8", "wo8", "wgu8", "wdown8")
WFMT = {"bf16": 0, "fp8": 1, "fp4": 2, "q4_0": 3, "q4_k": 4}  # runtime.hip WFMT_*


class _CainLayer(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in LAYER_FIELDS]


class _CainPlanDesc(ctypes.Structure):
    _fields_ = ([(n, ctypes.c_int) for n in ("n_layers", "d", "H", "Hkv", "hd", "ffn", "V", "act_kind", "T_max",
                                            "Mpad", "nsplit", "waves")]
                + [(n, ctypes.c_float) for n in ("eps", "embed_scale", "attn_scale")]
                + [(n, ctypes.c_void_p) for n in ("embed", "lm_head", "layers", "kcache", "vtcache")]
                + [("kv_layer_elems", ctypes.c_longlong)]
                + [(n, ctypes.c_void_p) for n in ("cos_t", "sin_t", "x", "q", "attn", "act", "logits",
                                                 "part_o", "part_ml", "counters", "gemm_ws")]
                + [("gemm_ws_bytes", ctypes.c_longlong), ("wfmt", ctypes.c_int), ("lm_head_scale", ctypes.c_void_p)]
                + [("kv8", ctypes.c_int), ("lm_head8", ctypes.c_void_p), ("x8", ctypes.c_void_p),
                   ("xs", ctypes.c_void_p), ("x8_ld", ctypes.c_int), ("q4_gain", ctypes.c_int)])


class _CainRows(ctypes.Structure):
    _fields_ = ([(n, ctypes.c_void_p) for n in ("tok", "pos", "slot", "n_gen", "max_new", "done", "hist", "gen")]
                + [("ldg", ctypes.c_int), ("sample_params", ctypes.c_void_p)])


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _set_cu_budget(lib, n: int) -> None:
    if n or hasattr(lib, "cain_set_cu_budget"):  # (older A/B builds have no CU budget; they never run cu_limit)
        lib.cain_set_cu_budget(n)


def attention_splits(M: int, Hkv: int, T_max: int) -> int:
    """Position splits per (row, kv head): ~256 workgroups in flight, >= 4 blocks of 32 per split at
    full context, <= 64 splits (measured: 1024-WG targets lose more to the split combine than they
    gain in parallelism, profiles/kernels.md).  (Round 1-3's per-split block cap and forced split count were tuning
    switches; their measurements are in profiles/r2/attn_occupancy.md.)"""
    if M * Hkv <= 64:
        # few (row, kv head) pairs run 8-wave workgroups (attention.hip): position splits up to ~64 workgroups
        # (<= 8 splits, >= 4 blocks of 32 positions per split at full context), and at most 64 blocks per split.
        # Measured in the graph-replayed batch-1 decode (rocprof, profiles/r2/attn_occupancy.md): llama3.1:8b
        # 10.9 -> 7.7 us per call at 8 splits (4: 9.1, 16: 8.5), qwen2:1.5b 11.2 -> 8.2, gemma:2b 18.9 -> 13.2,
        # phi3 (32 pairs, 2 splits) 9.7 -> 9.2, llama at 2 rows (4 splits) 11.2 -> 9.4 -- the in-kernel combine's
        # round trips cost less than one workgroup per pair walking the whole context.
        # Round 6, with the one-round-trip split combine (profiles/r6/attn_combine/splits_ab.jsonl, one box,
        # interleaved): a single (row, kv head) pair -- gemma:2b's MQA at batch 1 -- takes 16 splits of >= 3 blocks
        # (1,235 -> 1,256 tok/s); qwen2:1.5b (2 pairs) lost 0.6 % at 12 or 16 and llama3.1:8b (8 pairs) gained 0.5 %
        # at 12, so the others keep 8.  CAIN_ATTN_FEW_SPLITS / CAIN_ATTN_MIN_BLOCKS override both for A/B runs.
        one = M * Hkv == 1
        cap = int(os.environ.get("CAIN_ATTN_FEW_SPLITS", "0") or 0) or (16 if one else 8)
        min_blocks = int(os.environ.get("CAIN_ATTN_MIN_BLOCKS", "0") or 0) or (3 if one else 4)
        few = min(cap, T_max // (32 * min_blocks), 64 // (M * Hkv))
        return int(max(1, min(64, max(few, math.ceil((T_max // 32) / 64)))))
    ns = max(1, min(T_max // 128, math.ceil(256 / (M * Hkv))))
    return int(max(1, min(64, ns)))


def _load_ckpt(ckpt, cfg: ModelConfig, device, weight_dtype: str) -> ModelWeights:
    w = load_hf_weights(ckpt, cfg, device=device)
    _attach_native(w, ckpt, cfg, weight_dtype, device)
    return w


def _attach_native(weights: ModelWeights, path, cfg: ModelConfig, weight_dtype: str, device) -> None:
    """A GGUF checkpoint run on a GGUF block format (weight_dtype q4_0 / q4_k): keep its blocks as stored
    (models/q4.py gguf_q4_native) for pack_for_engine, instead of re-quantising the decoded values."""
    from ..models.gguf import GGUFFile, is_gguf

    if weight_dtype in ("q4_0", "q4_k") and path and is_gguf(path):
        from ..models.q4 import Q4_FORMATS, gguf_q4_native

        weights.native = gguf_q4_native(GGUFFile(path), cfg, Q4_FORMATS[weight_dtype], device=device)


class DecodeEngine:
    @classmethod
    def from_pretrained(cls, path: str, device: Union[str, torch.device] = "cuda", name: Optional[str] = None,
                        **kw) -> "DecodeEngine":
        """An engine on a Hugging Face checkpoint directory (``config.json`` + safetensors + ``tokenizer.json``;
        ``models/hf.py``): the same kernels and options as a tag's engine (``weight_dtype="fp4"`` quantises the
        checkpoint's bf16 weights to MXFP4 at load, as the packing of random weights does)."""
        cfg, weights, tok = load_pretrained(path, name=name, device=torch.device(device))
        _attach_native(weights, path, cfg, kw.get("weight_dtype", "bf16"), torch.device(device))
        return cls(cfg, device=device, weights=weights, tokenizer=tok, **kw)

    def __init__(self, model: Union[str, ModelConfig], device: Union[str, torch.device] = "cuda",
                 max_batch: int = 16, max_context: int = 2048, seed: int = 0, backend: Optional[str] = None,
                 steps_per_graph: int = 8, weights: Optional[ModelWeights] = None, tokenizer=None,
                 keep_natural: bool = False, weight_dtype: str = "bf16", kv_dtype: str = "bf16", cu_limit: int = 0):
        """``weight_dtype="fp8"``: GEMM weights quantised per row to e4m3 (half the weight bytes per decode step):
        forwards of up to 16 rows run W8A16 (gemm_w8.hip, bf16 activations), wider ones W8A8 (wgemm8.hip: the
        activations quantised per row to e4m3, fp8 MFMA) up to 256 rows; CAIN_W8A8=0 keeps W8A16 only (<= 64
        rows).
        ``weight_dtype="fp4"``: OCP MXFP4 GEMM weights (e2m1, one e8m0 scale per 32 k; 0.53 bytes per parameter),
        the reference's 4-bit precision class: W4A16 few-row kernels (gemm_w4.hip) up to 16 rows per forward, W4A8
        above (wgemm8.hip FP4: the same bytes on the block-scaled fp4 x fp8 MFMA, activations per row to e4m3) up to
        256; every GEMM K (d_model, q_dim, ffn) must be a multiple of 128 (>= 512 for W4A8).
        ``weight_dtype="q4_0" / "q4_k"``: llama.cpp's GGUF 4-bit blocks (Ollama's default builds) run natively
        (gemm_q4.hip: the block values as stored, scales applied per block; 16-row launches) up to 64 rows per
        forward; every GEMM K must be a multiple of 256.
        ``kv_dtype="fp8"``: the KV cache holds e4m3 elements (half the attention bytes per decode step and half
        the cache memory; csrc/attention.hip KV8).
        ``cu_limit``: run every kernel on a stream whose hardware queue may use only that many CUs (a multiple of
        8; runtime.hip cain_stream_create_cu_limited) and size the grids for them -- the batch-1 energy lever
        measured by tools/cu_sweep.py.  0: the whole device."""
        self.cfg = get_config(model) if isinstance(model, str) else model
        if weight_dtype not in WEIGHT_DTYPES:
            raise ValueError(f"weight_dtype must be one of {WEIGHT_DTYPES}, got {weight_dtype!r}")
        if weight_dtype == "fp4" and any(k % 128 for k in (self.cfg.d_model, self.cfg.q_dim, self.cfg.ffn)):
            raise ValueError(f"weight_dtype='fp4' needs d_model, q_dim and ffn to be multiples of 128 ({self.cfg.name})")
        if weight_dtype in ("q4_0", "q4_k") and any(k % 256 for k in (self.cfg.d_model, self.cfg.q_dim, self.cfg.ffn)):
            raise ValueError(f"weight_dtype={weight_dtype!r} needs d_model, q_dim and ffn to be multiples of 256 "
                             f"({self.cfg.name})")
        if kv_dtype not in ("bf16", "fp8"):
            raise ValueError(f"kv_dtype must be 'bf16' or 'fp8', got {kv_dtype!r}")
        self.weight_dtype = weight_dtype
        self.kv_dtype = kv_dtype
        self.cu_limit = int(cu_limit)
        if self.cu_limit and (self.cu_limit < 0 or self.cu_limit % 8):
            raise ValueError(f"cu_limit must be a positive multiple of 8 (or 0), got {cu_limit}")
        # W8A8 needs whole 128-deep stages, >= 4 of them, on every GEMM's K (all real configs; not the tiny ones)
        self.w8a8 = (weight_dtype == "fp8" and os.environ.get("CAIN_W8A8", "1") != "0"
                     and all(k % 128 == 0 and k >= 512 for k in (self.cfg.d_model, self.cfg.q_dim, self.cfg.ffn)))
        # MXFP4 above 16 rows: W4A8 on the same packed bytes (csrc/wgemm8.hip FP4), same shape rule as W8A8
        self.w4a8 = (weight_dtype == "fp4"
                     and all(k % 128 == 0 and k >= 512 for k in (self.cfg.d_model, self.cfg.q_dim, self.cfg.ffn)))
        row_cap = W8_MAX_ROWS if (weight_dtype == "fp4" and not self.w4a8) or (weight_dtype == "fp8" and not self.w8a8) \
            or weight_dtype in ("q4_0", "q4_k") else MAX_ROWS
        self.device = torch.device(device)
        if backend is None:
            backend = "hip" if self.device.type == "cuda" else "torch"
        self.backend = backend
        self.max_batch = int(min(max_batch, row_cap))
        # prompt tokens per prefill forward: the engine's own row count when that is wider (a 256-row engine
        # prefills 256 tokens per forward on the wide GEMM: half the launches of 128-row chunks)
        self.prefill_chunk = int(min(int(os.environ.get("CAIN_PREFILL_ROWS", "0") or 0)
                                     or max(PREFILL_ROWS, self.max_batch), row_cap))
        self.T_max = int(math.ceil(min(max_context, self.cfg.max_context) / 32) * 32)
        self.seed = seed
        self.steps_per_graph = max(1, int(steps_per_graph))
        # a checkpoint registered under the tag (CAIN_CHECKPOINTS, models/hf.py): its weights and tokenizer
        ckpt = checkpoint_for(model) if isinstance(model, str) and weights is None else None
        if tokenizer is None and ckpt:
            tokenizer = load_tokenizer(ckpt, self.cfg)
        self.tokenizer = tokenizer or get_tokenizer(self.cfg)
        self.keep_natural = keep_natural
        t0 = time.perf_counter_ns()
        if weights is None:
            weights = (_load_ckpt(ckpt, self.cfg, self.device, weight_dtype) if ckpt
                       else random_weights(self.cfg, device=self.device, seed=seed))
        self.weights = weights
        if backend == "hip":
            self._init_hip()
        elif backend == "torch":
            from ..models.reference import ReferenceModel
            # fp8 / fp4: the oracle runs on the dequantised weights the kernels multiply by
            ref_w = roundtrip_weights(weights, weight_dtype)
            self.ref = ReferenceModel(ref_w, memo_weights=self.device.type == "cpu", kv_dtype=kv_dtype)
        else:
            raise ValueError(f"unknown backend {backend!r}")
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.load_duration_ns = time.perf_counter_ns() - t0
        self._first_call = True
        self.last_ttft_ns = 0

    # ---------------------------------------------------------------- hip setup
    def _init_hip(self) -> None:
        from .. import ops

        self.lib = ops.load()
        cfg, dev = self.cfg, self.device
        if self.device.type != "cuda":
            raise ValueError("hip backend needs a GPU device")
        w8a8 = self.w8a8 and max(self.max_batch, self.prefill_chunk) > W8A8_MIN_ROWS
        w4a8 = self.w4a8 and max(self.max_batch, self.prefill_chunk) > W8A8_MIN_ROWS
        packed = pack_for_engine(self.weights, free_natural=not self.keep_natural, weight_dtype=self.weight_dtype,
                                 w8a8=w8a8)
        torch.cuda.synchronize(dev)
        S, T, L = self.max_batch, self.T_max, cfg.n_layers
        bf = torch.bfloat16
        kv_layer = S * cfg.n_kv_heads * T * cfg.head_dim
        # zero-init: positions past a row's length must hold finite values (masked P = 0 multiplies them)
        kv_t = torch.uint8 if self.kv_dtype == "fp8" else bf
        self.kcache = torch.zeros(L * kv_layer, device=dev, dtype=kv_t)
        self.vtcache = torch.zeros(L * kv_layer, device=dev, dtype=kv_t)
        inv = rope_inv_freq(cfg)
        ang = np.arange(T, dtype=np.float64)[:, None] * inv[None, :]
        self.cos_t = torch.tensor(np.cos(ang), dtype=torch.float32, device=dev).contiguous()
        self.sin_t = torch.tensor(np.sin(ang), dtype=torch.float32, device=dev).contiguous()
        R = max(self.max_batch, self.prefill_chunk)  # rows any forward of this engine can have
        z = lambda *s, dt=bf: torch.zeros(*s, device=dev, dtype=dt)  # noqa: E731
        self.buf = dict(x=z(R, cfg.d_model), q=z(R, cfg.q_dim), attn=z(R, cfg.q_dim), act=z(R, cfg.ffn),
                        logits=z(R, cfg.vocab, dt=torch.float32), counters=z(R * cfg.n_kv_heads, dt=torch.int32))
        max_ms = max(m * attention_splits(m, cfg.n_kv_heads, T) for m in range(1, R + 1))
        self.part_o = z(max_ms * cfg.n_heads * cfg.head_dim, dt=torch.float32)
        self.part_ml = z(max(ops.attention_ml_floats(m, cfg.n_heads, cfg.n_kv_heads,
                                                     attention_splits(m, cfg.n_kv_heads, T))
                             for m in range(1, R + 1)), dt=torch.float32)
        i32 = torch.int32
        self.rows = dict(tok=z(R, dt=i32), pos=z(R, dt=i32), slot=torch.full((R,), -1, device=dev, dtype=i32),
                         n_gen=z(R, dt=i32), max_new=z(R, dt=i32), done=z(R, dt=i32), hist=z(R * 64, dt=i32))
        self.gen = z(R, self.T_max, dt=i32)
        self.prefill_rows = dict(tok=z(R, dt=i32), pos=z(R, dt=i32), slot=torch.full((R,), -1, device=dev, dtype=i32))
        from .. import ops as _ops
        self.sample_params = _ops.sample_params_tensor(
            [dict(temperature=0.0, top_p=1.0, repeat_penalty=1.0, top_k=1, repeat_last_n=0, eos_id=-1, seed=0)] * R,
            dev)
        self._layers = (_CainLayer * L)()
        for i, lp in enumerate(packed["layers"]):
            self._layers[i] = _CainLayer(*(_ptr(lp.get(k)) for k in LAYER_FIELDS))
        self._packed = packed
        d = _CainPlanDesc()
        d.n_layers, d.d, d.H, d.Hkv, d.hd = L, cfg.d_model, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
        d.ffn, d.V, d.act_kind, d.T_max, d.Mpad = cfg.ffn, cfg.vocab, 1 if cfg.act == "gelu_tanh" else 0, T, R
        d.nsplit, d.waves = 1, 0
        d.eps = cfg.norm_eps
        d.embed_scale = float(torch.tensor(math.sqrt(cfg.d_model), dtype=bf).float()) if cfg.embed_scale else 1.0
        d.attn_scale = 1.0 / math.sqrt(cfg.head_dim)
        d.embed, d.lm_head = _ptr(self.weights.embed), _ptr(packed["lm_head"])
        d.layers = ctypes.cast(self._layers, ctypes.c_void_p).value
        d.kcache, d.vtcache, d.kv_layer_elems = _ptr(self.kcache), _ptr(self.vtcache), kv_layer
        d.kv8 = int(self.kv_dtype == "fp8")
        d.cos_t, d.sin_t = _ptr(self.cos_t), _ptr(self.sin_t)
        for k in ("x", "q", "attn", "act", "logits", "counters"):
            setattr(d, k, _ptr(self.buf[k]))
        d.part_o, d.part_ml = _ptr(self.part_o), _ptr(self.part_ml)
        self.wgemm_plans = self._wide_gemm_plans(R)
        # split-K workspace of the batched / wide GEMMs and of the skinny kernel's split grids (M <= 16 on narrow
        # outputs): largest need over this model's GEMM shapes at every row count (after any
        # CAIN_WGEMM_PLANS override, which may pick larger split counts than the default rule)
        shapes = [(cfg.qkv_dim, cfg.d_model), (cfg.d_model, cfg.q_dim), (2 * cfg.ffn, cfg.d_model),
                  (cfg.d_model, cfg.ffn), (cfg.vocab, cfg.d_model)]
        ws = max([ops.gemm_ws_bytes(n, k, m) for n, k in shapes for m in range(1, R + 1)] + [0])
        if self.weight_dtype == "fp4":  # split-K tickets + partials of the few-row MXFP4 stream kernel
            ws = max([ws] + [int(self.lib.cain_gemm_w4_ws_bytes(n, k, 1)) for n, k in shapes])
        if w8a8 or w4a8:
            ws = max([ws] + [int(self.lib.cain_w8a8_ws_bytes(n, k, m)) for n, k in shapes for m in range(17, R + 1)])
            kmax = max(cfg.d_model, cfg.q_dim, cfg.ffn)
            self.x8 = torch.zeros(R, kmax, device=dev, dtype=torch.uint8)
            self.xs = torch.zeros(R, device=dev, dtype=torch.float32)
            d.lm_head8, d.x8, d.xs, d.x8_ld = _ptr(packed.get("lm_head8")), _ptr(self.x8), _ptr(self.xs), kmax
        self.gemm_ws = torch.zeros(max(ws, 16) // 4 + 1, device=dev, dtype=torch.int32)
        d.gemm_ws, d.gemm_ws_bytes = _ptr(self.gemm_ws), ws
        d.wfmt, d.lm_head_scale = WFMT[self.weight_dtype], _ptr(packed.get("lm_head_scale"))
        d.q4_gain = int(bool(packed.get("q4_gain")))  # GGUF blocks as stored: gains applied to the activations
        self._desc = d
        self._plans: Dict[int, int] = {}
        self._graphs: Dict[tuple, int] = {}
        self._cu_stream = None
        if self.cu_limit and self.cu_limit < torch.cuda.get_device_properties(dev).multi_processor_count:
            with torch.cuda.device(dev):
                h = self.lib.cain_stream_create_cu_limited(self.cu_limit)
            if not h:
                raise RuntimeError(f"hipExtStreamCreateWithCUMask failed for {self.cu_limit} CUs")
            self._cu_stream = h
            self.stream = torch.cuda.ExternalStream(h, device=dev)
        else:
            self.cu_limit = 0
            self.stream = torch.cuda.Stream(device=dev)

    def _wide_gemm_plans(self, R: int) -> list:
        """Split plans of the wide-batch GEMM (csrc/wgemm.hip) this engine runs, per projection shape at its
        widest forward: the default rule, or ``CAIN_WGEMM_PLANS="N:K:BM:KS[:VARIANT],..."`` (explicit per-shape
        plans for in-graph A/B runs; measured in the graph-replayed decode, never by isolated timings -- an
        isolated autotune's winners did not move the headline, profiles/wgemm_r2.md)."""
        from .. import ops
        for spec in filter(None, os.environ.get("CAIN_WGEMM_PLANS", "").split(",")):
            f = [int(x) for x in spec.split(":")]
            ops.set_wide_gemm_plan(f[0], f[1], f[2], f[3], f[4] if len(f) > 4 else -1)
        cfg = self.cfg
        shapes = [(cfg.qkv_dim, cfg.d_model), (cfg.d_model, cfg.q_dim), (2 * cfg.ffn, cfg.d_model),
                  (cfg.d_model, cfg.ffn), (cfg.vocab, cfg.d_model)]
        out = []
        if self.weight_dtype == "bf16" and R > 64:
            for n, k in shapes:
                if ops.wide_gemm_eligible(n, k, R):
                    ks, v = ops.wide_gemm_plan(n, k, R)
                    out.append(dict(n=n, k=k, m=R, ks=ks, variant=v))
        return out

    def _plan(self, M: int) -> int:
        """One native plan per attention split count (nsplit depends on the row count)."""
        ns = attention_splits(M, self.cfg.n_kv_heads, self.T_max)
        if ns not in self._plans:
            self._desc.nsplit = ns
            self._plans[ns] = self.lib.cain_plan_create(ctypes.byref(self._desc))
        return self._plans[ns]

    def _rows_struct(self, rows: Dict[str, torch.Tensor], with_sampling: bool) -> _CainRows:
        r = _CainRows()
        r.tok, r.pos, r.slot = _ptr(rows["tok"]), _ptr(rows["pos"]), _ptr(rows["slot"])
        if with_sampling:
            r.n_gen, r.max_new, r.done = _ptr(rows["n_gen"]), _ptr(rows["max_new"]), _ptr(rows["done"])
            r.hist, r.gen, r.ldg = _ptr(rows["hist"]), _ptr(self.gen), self.gen.stride(0)
            r.sample_params = _ptr(self.sample_params)
        return r

    def _forward(self, M: int, rows, want_logits: bool, want_sample: bool) -> None:
        rs = self._rows_struct(rows, want_sample)
        plan = self._plan(M)
        _set_cu_budget(self.lib, self.cu_limit)  # launch sizing for this engine's stream (0: whole device)
        try:
            rc = self.lib.cain_plan_forward(ctypes.c_void_p(plan), M, ctypes.byref(rs), int(want_logits),
                                            int(want_sample), ctypes.c_void_p(self.stream.cuda_stream))
        finally:
            _set_cu_budget(self.lib, 0)
        if rc != 0:
            where = self.lib.cain_plan_last_failure()
            raise RuntimeError(f"cain_plan_forward failed rc={rc}" + (f" at {where.decode()}" if where else ""))

    def _graph(self, M: int, steps: int) -> int:
        key = (M, steps)
        g = self._graphs.get(key)
        if g is None:
            rs = self._rows_struct(self.rows, True)
            err = ctypes.c_int(0)
            plan = self._plan(M)
            _set_cu_budget(self.lib, self.cu_limit)
            try:
                g = self.lib.cain_plan_capture(ctypes.c_void_p(plan), M, ctypes.byref(rs), steps,
                                               ctypes.c_void_p(self.stream.cuda_stream), ctypes.byref(err))
            finally:
                _set_cu_budget(self.lib, 0)
            if not g:
                raise RuntimeError(f"hipGraph capture failed (err={err.value})")
            self._graphs[key] = g
        return g

    def close(self) -> None:
        lib = getattr(self, "lib", None)
        if lib is None:
            return
        for g in self._graphs.values():
            lib.cain_graph_destroy(ctypes.c_void_p(g))
        for p in self._plans.values():
            lib.cain_plan_destroy(ctypes.c_void_p(p))
        self._graphs, self._plans = {}, {}
        if getattr(self, "_cu_stream", None):
            self.stream.synchronize()
            lib.cain_stream_destroy(ctypes.c_void_p(self._cu_stream))
            self._cu_stream = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- generation
    def encode(self, prompt: Union[str, Sequence[int]]) -> List[int]:
        if isinstance(prompt, str):
            return self.tokenizer.encode(prompt)
        return [int(t) for t in prompt]

    def generate(self, prompts: Sequence[Union[str, Sequence[int]]], num_predict: Union[int, Sequence[int]] = 128,
                 options: Union[None, Dict, Sequence[Optional[Dict]]] = None, use_graph: bool = True,
                 on_tokens=None) -> List[GenResult]:
        """Generate for a batch of prompts (ids or text).  ``on_tokens(list_per_row)`` streams newly
        generated ids every ``steps_per_graph`` decode steps (and stops early once every row is done)."""
        prompts = list(prompts)
        B = len(prompts)
        if B == 0:
            return []
        if B > self.max_batch:
            out = []
            for i in range(0, B, self.max_batch):
                sl = slice(i, i + self.max_batch)
                nps = num_predict[sl] if not isinstance(num_predict, int) else num_predict
                ops_ = options[sl] if isinstance(options, (list, tuple)) else options
                out += self.generate(prompts[sl], nps, ops_, use_graph, on_tokens)
            return out
        ids = [self.encode(p) or [self.cfg.bos_id] for p in prompts]
        nps = [int(num_predict)] * B if isinstance(num_predict, int) else [int(x) for x in num_predict]
        opts = list(options) if isinstance(options, (list, tuple)) else [options] * B
        row_opts = [_row_options(o, self.cfg, i, self.seed) for i, o in enumerate(opts)]
        for i in range(B):
            budget = self.T_max - len(ids[i])
            if budget < 1:
                raise ValueError(f"prompt of {len(ids[i])} tokens exceeds the context ({self.T_max})")
            nps[i] = max(1, min(nps[i], budget))
        t0 = time.perf_counter_ns()
        if self.backend == "torch":
            gen, t_pref, t_dec = self._generate_torch(ids, nps, row_opts)
            if on_tokens is not None:
                on_tokens(gen)
        else:
            gen, t_pref, t_dec = self._generate_hip(ids, nps, row_opts, use_graph, on_tokens)
        total = time.perf_counter_ns() - t0
        load = self.load_duration_ns if self._first_call else 0
        self._first_call = False
        steps = max(nps)
        self.last_prefill_ns, self.last_decode_ns = t_pref, t_dec
        out = []
        for i in range(B):
            toks = gen[i]
            reason = "stop" if _stopped(toks, row_opts[i]) else "length"
            out.append(GenResult(self.cfg.name, ids[i], toks, self.tokenizer.decode(toks), reason,
                                 load_duration_ns=load, prompt_eval_duration_ns=t_pref,
                                 eval_duration_ns=int(t_dec * len(toks) / max(1, steps)),
                                 total_duration_ns=total + load))
        return out

    def _generate_hip(self, ids, nps, row_opts, use_graph, on_tokens=None, check_every: int = 1):
        from .. import ops

        dev = self.device
        B = len(ids)
        with torch.cuda.stream(self.stream):
            # ---- prefill: all prompt tokens except the last, in <=prefill_chunk-row chunks
            t0 = time.perf_counter_ns()
            self._prefill(ids)
            # ---- decode rows
            r = self.rows
            r["tok"][:B].copy_(torch.tensor([p[-1] for p in ids], dtype=torch.int32))
            r["pos"][:B].copy_(torch.tensor([len(p) - 1 for p in ids], dtype=torch.int32))
            r["slot"][:B].copy_(torch.arange(B, dtype=torch.int32))
            r["n_gen"][:B].zero_()
            r["done"][:B].zero_()
            r["max_new"][:B].copy_(torch.tensor(nps, dtype=torch.int32))
            self.sample_params[: ops.SAMPLE_BYTES * B].copy_(ops.sample_params_tensor(row_opts, "cpu").to(dev))
            self.stream.synchronize()
            t1 = time.perf_counter_ns()
            steps = max(nps)
            stream_h = ctypes.c_void_p(self.stream.cuda_stream)

            def launch(nsteps: int) -> None:
                if not use_graph:
                    for _ in range(nsteps):
                        self._forward(B, r, want_logits=True, want_sample=True)
                    return
                k = self.steps_per_graph
                g = self._graph(B, k) if nsteps >= k else None
                for _ in range(nsteps // k):
                    rc = self.lib.cain_graph_launch(ctypes.c_void_p(g), stream_h)
                    if rc != 0:
                        raise RuntimeError(f"hipGraphLaunch failed rc={rc}")
                if nsteps % k:
                    g1 = self._graph(B, 1)
                    for _ in range(nsteps % k):
                        if self.lib.cain_graph_launch(ctypes.c_void_p(g1), stream_h) != 0:
                            raise RuntimeError("hipGraphLaunch failed")

            # first token on its own so time-to-first-token is measured exactly
            launch(1)
            self.stream.synchronize()
            t_first = time.perf_counter_ns()
            done_steps = 1
            emitted = [0] * B
            watch = on_tokens is not None or any(o["eos_id"] >= 0 or o["stop"] for o in row_opts)
            chunk = self.steps_per_graph * max(1, int(check_every))

            def poll() -> bool:
                ng = r["n_gen"][:B].cpu().tolist()
                if on_tokens is not None:
                    new = [self.gen[i, emitted[i]: ng[i]].cpu().tolist() if ng[i] > emitted[i] else []
                           for i in range(B)]
                    for i in range(B):
                        emitted[i] = ng[i]
                    on_tokens(new)
                return bool(r["done"][:B].all())

            if watch and poll():
                done_steps = steps
            while done_steps < steps:
                n = min(chunk if watch else steps, steps - done_steps)
                launch(n)
                done_steps += n
                if watch and done_steps < steps and poll():
                    break
            n_gen = r["n_gen"][:B].cpu().tolist()
            gen = self.gen[:B].cpu()
            if on_tokens is not None:
                on_tokens([gen[i, emitted[i]: n_gen[i]].tolist() for i in range(B)])
            t2 = time.perf_counter_ns()
        self.last_ttft_ns = t_first - t0
        return [gen[i, : n_gen[i]].tolist() for i in range(B)], t1 - t0, t2 - t1

    @torch.no_grad()
    def last_logits(self, prompts: Sequence[Union[str, Sequence[int]]]) -> torch.Tensor:
        """fp32 logits [B, V] of the next token after each prompt (numerics tests / debugging)."""
        ids = [self.encode(p) for p in prompts]
        B = len(ids)
        if self.backend == "torch":
            return torch.stack([self.ref.forward(torch.tensor([p], device=self.device))[0, -1] for p in ids])
        assert B <= self.max_batch
        with torch.cuda.stream(self.stream):
            self._prefill(ids)
            r = self.rows
            r["tok"][:B].copy_(torch.tensor([p[-1] for p in ids], dtype=torch.int32))
            r["pos"][:B].copy_(torch.tensor([len(p) - 1 for p in ids], dtype=torch.int32))
            r["slot"][:B].copy_(torch.arange(B, dtype=torch.int32))
            self._forward(B, r, want_logits=True, want_sample=False)
            out = self.buf["logits"][:B].clone()
            self.stream.synchronize()
        return out

    def _prefill(self, ids, slots: Optional[Sequence[int]] = None) -> None:
        """All prompt tokens but the last through the forward, into KV-cache slot ``slots[b]`` (default b)."""
        flat_tok, flat_pos, flat_slot = [], [], []
        for b, p in enumerate(ids):
            for j, t in enumerate(p[:-1]):
                flat_tok.append(t)
                flat_pos.append(j)
                flat_slot.append(b if slots is None else int(slots[b]))
        pr = self.prefill_rows
        for c in range(0, len(flat_tok), self.prefill_chunk):
            n = min(self.prefill_chunk, len(flat_tok) - c)
            pr["tok"][:n].copy_(torch.tensor(flat_tok[c:c + n], dtype=torch.int32))
            pr["pos"][:n].copy_(torch.tensor(flat_pos[c:c + n], dtype=torch.int32))
            pr["slot"][:n].copy_(torch.tensor(flat_slot[c:c + n], dtype=torch.int32))
            self._forward(n, pr, want_logits=False, want_sample=False)

    # ------------------------------------------------------------ continuous batching
    def continuous(self) -> "ContinuousBatch":
        """A persistent decode batch that requests join and leave between graph chunks (the server's
        continuous batching, serve/server.py); HIP backend only."""
        if self.backend != "hip":
            raise RuntimeError("continuous batching needs the hip backend")
        return ContinuousBatch(self)

    def _generate_torch(self, ids, nps, row_opts):
        """Oracle backend with a KV cache (one token of compute per step), sampled on the host."""
        t0 = time.perf_counter_ns()
        gens = []
        for i, p in enumerate(ids):
            o = row_opts[i]
            rng = np.random.default_rng(o["seed"])
            out = []
            cache: list = []
            step = torch.tensor([list(p)], device=self.device)
            for _ in range(nps[i]):
                logits = self.ref.forward(step, cache=cache, last_only=True)[0, -1].float().cpu()
                nxt = sample_host(logits, out, o, rng)
                out.append(nxt)
                step = torch.tensor([[nxt]], device=self.device)
                if _stopped(out, o):
                    break
            gens.append(out)
        t1 = time.perf_counter_ns()
        return gens, 0, t1 - t0


def sample_host(logits: torch.Tensor, history: List[int], o: Dict, rng) -> int:
    """Host mirror of csrc/sample.hip (same pipeline; RNG differs)."""
    lg = logits.clone()
    if o["repeat_penalty"] != 1.0 and o["repeat_last_n"] > 0:
        for t in set(history[-min(o["repeat_last_n"], 64):]):
            v = lg[t]
            lg[t] = v / o["repeat_penalty"] if v > 0 else v * o["repeat_penalty"]
    if o["temperature"] <= 0:
        return int(torch.argmax(lg))
    k = o["top_k"] if 0 < o["top_k"] <= 1024 else 1024
    vals, idx = torch.topk(lg / o["temperature"], min(k, lg.numel()))
    p = torch.softmax(vals.double(), 0)
    if 0 < o["top_p"] < 1:
        c = torch.cumsum(p, 0)
        cut = int(torch.searchsorted(c, torch.tensor(o["top_p"], dtype=c.dtype))) + 1
        p = p[:cut] / p[:cut].sum()
        idx = idx[:cut]
    return int(idx[int(rng.choice(len(p), p=p.numpy()))])


class ContinuousBatch:
    """Rows ``[0, n)`` of the engine's decode state are the live requests; each owns a KV-cache slot for its
    lifetime (``slot`` column), so rows can be compacted when requests leave while their caches stay put.

    * ``admit(prompts, num_predict, options)`` prefills new requests into free slots and appends them as rows
      ``n .. n+k-1`` (between graph chunks only);
    * ``step(steps)`` runs ``steps`` decode steps over the ``n`` live rows (hipGraphs per row count, cached);
    * ``poll()`` returns, per live row, the tokens generated since the previous poll and whether it finished;
    * ``retire(rows)`` drops finished rows, moving the last live rows into the holes (device-side copies of the
      row state, generated ids and sampling parameters) and freeing their slots.

    A request that arrives while others decode waits at most one chunk (``steps_per_graph`` steps) plus its own
    prefill, instead of the whole earlier batch (static batching)."""

    def __init__(self, eng: DecodeEngine):
        self.eng = eng
        self.n = 0
        self.free_slots = list(range(eng.max_batch))[::-1]
        self.row_slot: List[int] = []
        self.emitted: List[int] = []
        self.prompt_tokens: List[List[int]] = []
        self.options: List[Dict] = []

    @property
    def capacity(self) -> int:
        return len(self.free_slots)

    def admit(self, prompts: Sequence[Union[str, Sequence[int]]], num_predict: Sequence[int],
              options: Sequence[Optional[Dict]]) -> List[int]:
        from .. import ops

        eng = self.eng
        k = len(prompts)
        if k == 0:
            return []
        if k > len(self.free_slots):
            raise ValueError(f"{k} requests but only {len(self.free_slots)} free rows")
        ids = [eng.encode(p) or [eng.cfg.bos_id] for p in prompts]
        nps, row_opts = [], []
        for i, (p, n, o) in enumerate(zip(ids, num_predict, options)):
            budget = eng.T_max - len(p)
            if budget < 1:
                raise ValueError(f"prompt of {len(p)} tokens exceeds the context ({eng.T_max})")
            nps.append(max(1, min(int(n), budget)))
            row_opts.append(_row_options(o, eng.cfg, self.n + i, eng.seed))
        slots = [self.free_slots.pop() for _ in range(k)]
        rows = list(range(self.n, self.n + k))
        r = eng.rows
        with torch.cuda.stream(eng.stream):
            eng._prefill(ids, slots)
            sl = slice(self.n, self.n + k)
            r["tok"][sl].copy_(torch.tensor([p[-1] for p in ids], dtype=torch.int32))
            r["pos"][sl].copy_(torch.tensor([len(p) - 1 for p in ids], dtype=torch.int32))
            r["slot"][sl].copy_(torch.tensor(slots, dtype=torch.int32))
            r["n_gen"][sl].zero_()
            r["done"][sl].zero_()
            r["max_new"][sl].copy_(torch.tensor(nps, dtype=torch.int32))
            eng.sample_params[ops.SAMPLE_BYTES * self.n: ops.SAMPLE_BYTES * (self.n + k)].copy_(ops.sample_params_tensor(row_opts, "cpu").to(eng.device))
        self.n += k
        self.row_slot += slots
        self.emitted += [0] * k
        self.prompt_tokens += ids
        self.options += row_opts
        return rows

    def step(self, steps: Optional[int] = None) -> None:
        eng = self.eng
        if self.n == 0:
            return
        steps = steps or eng.steps_per_graph
        stream_h = ctypes.c_void_p(eng.stream.cuda_stream)
        with torch.cuda.stream(eng.stream):
            k = eng.steps_per_graph
            if steps >= k:
                g = eng._graph(self.n, k)
                for _ in range(steps // k):
                    if eng.lib.cain_graph_launch(ctypes.c_void_p(g), stream_h) != 0:
                        raise RuntimeError("hipGraphLaunch failed")
            if steps % k:
                g1 = eng._graph(self.n, 1)
                for _ in range(steps % k):
                    if eng.lib.cain_graph_launch(ctypes.c_void_p(g1), stream_h) != 0:
                        raise RuntimeError("hipGraphLaunch failed")

    def poll(self):
        """([new token ids per live row], [finished flag per live row])."""
        eng = self.eng
        if self.n == 0:
            return [], []
        with torch.cuda.stream(eng.stream):
            ng = eng.rows["n_gen"][: self.n].cpu().tolist()
            done = eng.rows["done"][: self.n].cpu().tolist()
            hi = max(ng)
            gen = eng.gen[: self.n, :hi].cpu() if hi else None
        new = []
        for i in range(self.n):
            new.append(gen[i, self.emitted[i]: ng[i]].tolist() if ng[i] > self.emitted[i] else [])
            self.emitted[i] = ng[i]
        return new, [bool(d) for d in done]

    def tokens(self, row: int) -> List[int]:
        ng = int(self.eng.rows["n_gen"][row])
        return self.eng.gen[row, :ng].cpu().tolist()

    def retire(self, rows: Sequence[int]) -> Dict[int, int]:
        """Drop ``rows``; returns {old row index: new row index} for the rows that moved into the holes."""
        eng = self.eng
        dead = sorted(set(int(x) for x in rows))
        if not dead:
            return {}
        keep = [i for i in range(self.n) if i not in set(dead)]
        n_new = len(keep)
        moves = {}
        holes = [h for h in dead if h < n_new]
        movers = [j for j in keep if j >= n_new]
        for h, j in zip(holes, movers):
            moves[j] = h
        for h in dead:
            self.free_slots.append(self.row_slot[h])
        if moves:
            r = eng.rows
            with torch.cuda.stream(eng.stream):
                # index tensors made on the engine's stream: the copies below run there, so the caching allocator
                # cannot hand these blocks out again before the gathers have read them
                src = torch.tensor(list(moves.keys()), device=eng.device, dtype=torch.long)
                dst = torch.tensor(list(moves.values()), device=eng.device, dtype=torch.long)
                for key in ("tok", "pos", "slot", "n_gen", "max_new", "done"):
                    r[key][dst] = r[key][src]
                h64 = r["hist"].view(-1, 64)
                h64[dst] = h64[src]
                eng.gen[dst] = eng.gen[src]
                from .. import ops

                sp = eng.sample_params.view(-1, ops.SAMPLE_BYTES)
                sp[dst] = sp[src]
            for j, h in moves.items():
                self.row_slot[h] = self.row_slot[j]
                self.emitted[h] = self.emitted[j]
                self.prompt_tokens[h] = self.prompt_tokens[j]
                self.options[h] = self.options[j]
        with torch.cuda.stream(eng.stream):
            eng.rows["slot"][n_new: self.n].fill_(-1)  # vacated rows: skipped by the sampler
        self.n = n_new
        del self.row_slot[n_new:], self.emitted[n_new:], self.prompt_tokens[n_new:], self.options[n_new:]
        return moves
