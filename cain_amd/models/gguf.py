"""GGUF model files (llama.cpp / Ollama's format) for the study families: reader, dequantisers, config and weight
mapping, tokenizer, and a small writer.

The reference gets its models from Ollama (``/root/reference/experiment/RunnerConfig.py:80``): GGUF blobs, mostly
4-bit K-quants.  ``load_gguf(path)`` turns such a file into this engine's ``ModelConfig`` + ``ModelWeights``
(+ tokenizer), so a user of the reference can point the engine at the same blobs (``CAIN_CHECKPOINTS`` accepts a
``.gguf`` path as well as a Hugging Face directory; ``DecodeEngine.from_pretrained`` too).  The weights are
dequantised to bf16 at load; the engine's ``weight_dtype="fp4"`` then re-quantises them to MXFP4, its own 4-bit
format (one e8m0 scale per 32 weights, where Q4_K has a 6-bit scale and min per 32 under fp16 super-scales).

* Container: GGUF v2 / v3, little-endian, every metadata value type, ``general.alignment``.  Tensors are read
  through ``numpy.memmap`` (nothing executes from the file).
* Tensor types: F32, F16, BF16, Q8_0, Q4_0, Q4_1, Q5_0, Q5_1, Q2_K, Q3_K, Q4_K, Q5_K, Q6_K (Ollama's q4_0 /
  q4_K_M defaults and its q2_K / q3_K_* / q5_* / q6_K / q8_0 tags).  Others (IQ*, Q8_K, ...) are refused.  Each
  decoder follows the ggml block layout in torch ops over all blocks of a tensor slice, on the load device: the
  quantised bytes go to the GPU and are decoded there.
* Architectures: ``llama`` (Llama 3.1 and Mistral: llama.cpp converts both as ``llama``, with q / k rows permuted
  to interleaved RoPE pairs, undone here -- the same inverse transformers applies, ``tests/test_gguf.py``),
  ``qwen2``, ``gemma`` (norm gains stored as 1 + w: w is restored) and ``phi3`` (fused ``attn_qkv``; ``ffn_up``
  holds gate then up).  Llama 3.1's RoPE scaling arrives as the ``rope_freqs`` tensor of per-frequency divisors
  (``ModelConfig.rope_freq_factors``).  Phi-3 long-rope factors are refused.
* Tokenizer: the ``tokenizer.ggml.*`` vocabulary through transformers' GGUF tokenizer converters
  (``transformers.integrations.ggml``), wrapped as ``HFTokenizer``.

Parity: no GGUF reader is importable here (the ``gguf`` package is absent, no network), so the block formats are
pinned by round trips through this module's own quantisers and by a per-element reference decoder in the tests --
"parity unpinned" against llama.cpp itself.  The tensor-name / permutation / gain conventions are pinned against
transformers' GGUF processors and, end to end, against transformers' model classes (tests/test_gguf.py).
"""
from __future__ import annotations

import json
import os
import re
import struct
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from .config import ModelConfig
from .weights import LayerWeights, ModelWeights

GGUF_MAGIC = b"GGUF"
SLICE_ELEMS = 1 << 24  # elements dequantised per slice of a tensor (GGUFFile.tensor)

# ggml tensor types: id -> (name, elements per block, bytes per block)
GGML_TYPES: Dict[int, Tuple[str, int, int]] = {
    0: ("F32", 1, 4), 1: ("F16", 1, 2), 2: ("Q4_0", 32, 18), 3: ("Q4_1", 32, 20), 6: ("Q5_0", 32, 22),
    7: ("Q5_1", 32, 24), 8: ("Q8_0", 32, 34), 10: ("Q2_K", 256, 84), 11: ("Q3_K", 256, 110), 12: ("Q4_K", 256, 144),
    13: ("Q5_K", 256, 176), 14: ("Q6_K", 256, 210), 30: ("BF16", 1, 2),
}
TYPE_ID = {v[0]: k for k, v in GGML_TYPES.items()}

# metadata value types
_SCALAR = {0: "<B", 1: "<b", 2: "<H", 3: "<h", 4: "<I", 5: "<i", 6: "<f", 7: "<?", 10: "<Q", 11: "<q", 12: "<d"}
_STRING, _ARRAY = 8, 9


@dataclass
class GGUFTensor:
    name: str
    shape: Tuple[int, ...]   # torch order (outermost first): ggml ne reversed
    type: int
    offset: int              # absolute file offset of the data
    nbytes: int

    @property
    def type_name(self) -> str:
        return GGML_TYPES.get(self.type, (f"type{self.type}",))[0]


class GGUFFile:
    """Metadata and tensor directory of a GGUF file; tensor data on demand (``numpy.memmap``)."""

    def __init__(self, path: Union[str, os.PathLike]):
        self.path = str(path)
        with open(self.path, "rb") as f:
            if f.read(4) != GGUF_MAGIC:
                raise ValueError(f"{path}: not a GGUF file")
            self.version, = struct.unpack("<I", f.read(4))
            if self.version not in (2, 3):
                raise ValueError(f"{path}: GGUF version {self.version} is not supported (2, 3 are)")
            n_tensors, n_kv = struct.unpack("<QQ", f.read(16))
            self.metadata: Dict[str, Any] = {}
            for _ in range(n_kv):
                key = self._str(f)
                self.metadata[key] = self._value(f, struct.unpack("<I", f.read(4))[0])
            infos = []
            for _ in range(n_tensors):
                name = self._str(f)
                nd, = struct.unpack("<I", f.read(4))
                ne = struct.unpack(f"<{nd}Q", f.read(8 * nd))
                ttype, off = struct.unpack("<IQ", f.read(12))
                infos.append((name, tuple(int(x) for x in ne), ttype, off))
            align = int(self.metadata.get("general.alignment", 32))
            base = (f.tell() + align - 1) // align * align
        self.tensors: Dict[str, GGUFTensor] = {}
        for name, ne, ttype, off in infos:
            n = int(np.prod(ne)) if ne else 1
            _, bs, bb = GGML_TYPES.get(ttype, ("?", 1, 0))
            self.tensors[name] = GGUFTensor(name, tuple(reversed(ne)), ttype, base + off, n // bs * bb)

    @staticmethod
    def _str(f) -> str:
        n, = struct.unpack("<Q", f.read(8))
        return f.read(n).decode("utf-8", errors="replace")

    def _value(self, f, vt: int):
        if vt in _SCALAR:
            fmt = _SCALAR[vt]
            return struct.unpack(fmt, f.read(struct.calcsize(fmt)))[0]
        if vt == _STRING:
            return self._str(f)
        if vt == _ARRAY:
            et, n = struct.unpack("<IQ", f.read(12))
            if et in _SCALAR and et != 7:
                dt = np.dtype(_SCALAR[et])
                return np.frombuffer(f.read(n * dt.itemsize), dtype=dt).tolist()
            return [self._value(f, et) for _ in range(n)]
        raise ValueError(f"unknown GGUF metadata type {vt}")

    def raw(self, name: str) -> np.ndarray:
        t = self.tensors[name]
        return np.memmap(self.path, dtype=np.uint8, mode="r", offset=t.offset, shape=(t.nbytes,))

    def tensor(self, name: str, device="cpu", dtype: torch.dtype = torch.float32) -> torch.Tensor:
        """``name`` dequantised (torch order) as ``dtype`` on ``device``: the quantised bytes travel, the blocks are
        decoded there."""
        t = self.tensors.get(name)
        if t is None:
            raise KeyError(f"GGUF file has no tensor {name!r}")
        n = int(np.prod(t.shape))
        _, bs, bb = GGML_TYPES.get(t.type, ("?", 1, 0))
        raw = self.raw(name)
        out = torch.empty(n, dtype=dtype, device=device)
        # in slices of whole blocks: a 128k x 4096 Q4_K embedding would otherwise hold ~4x its fp32 size in temporaries
        step = max(1, SLICE_ELEMS // bs) * bs
        for e0 in range(0, n, step):
            e1 = min(n, e0 + step)
            out[e0:e1] = dequantize(raw[e0 // bs * bb: e1 // bs * bb], t.type, e1 - e0, device=device)
        return out.reshape(t.shape)

    def has(self, name: str) -> bool:
        return name in self.tensors


# ---------------------------------------------------------------------------------------------------- dequantisers
# torch ops over all blocks of a slice, on the tensor's device: the GPU dequantises a 128k x 4096 Q4_K embedding in
# milliseconds, the CPU (multi-threaded) in about a second.  ``b`` is a uint8 [blocks, bytes per block] tensor.
def _f16(b: torch.Tensor) -> torch.Tensor:
    return b.contiguous().view(torch.float16).float()


def _nibbles(qs: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    return (qs & 0x0F).to(torch.int16), (qs >> 4).to(torch.int16)


def _k_scale_min(sc: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """The 8 six-bit (scale, min) pairs of a K-quant super-block's 12 packed bytes -> two [n, 8] tensors."""
    sc = sc.to(torch.int16)
    d = torch.cat([sc[:, 0:4] & 63, (sc[:, 8:12] & 0x0F) | ((sc[:, 0:4] >> 6) << 4)], 1)
    m = torch.cat([sc[:, 4:8] & 63, (sc[:, 8:12] >> 4) | ((sc[:, 4:8] >> 6) << 4)], 1)
    return d.float(), m.float()


def dequantize(raw, ttype: int, n: int, device=None) -> torch.Tensor:
    """fp32 values (a torch tensor on ``device``, default the bytes' device) of ``n`` elements stored as ggml type
    ``ttype`` in the bytes ``raw`` (numpy or torch uint8)."""
    name, bs, bb = GGML_TYPES.get(ttype, (f"type{ttype}", 0, 0))
    if isinstance(raw, np.ndarray):
        raw = torch.from_numpy(np.array(raw, dtype=np.uint8))  # a copy: file maps are read-only
    if device is not None:
        raw = raw.to(device)
    if name == "F32":
        return raw[: 4 * n].contiguous().view(torch.float32).clone()
    if name == "F16":
        return _f16(raw[: 2 * n])
    if name == "BF16":
        return raw[: 2 * n].contiguous().view(torch.bfloat16).float()
    if name not in _DEQUANT:
        raise NotImplementedError(f"GGUF tensor type {name} is not supported")
    if n % bs:
        raise ValueError(f"{name}: {n} elements is not a whole number of {bs}-element blocks")
    blocks = raw[: n // bs * bb].reshape(-1, bb)
    return _DEQUANT[name](blocks).reshape(-1)


def _q8_0(b):
    return _f16(b[:, :2]) * b[:, 2:].view(torch.int8).float()


def _q4_0(b):
    lo, hi = _nibbles(b[:, 2:])
    return _f16(b[:, :2]) * (torch.cat([lo, hi], 1) - 8).float()


def _q4_1(b):
    lo, hi = _nibbles(b[:, 4:])
    return _f16(b[:, :2]) * torch.cat([lo, hi], 1).float() + _f16(b[:, 2:4])


def _q5_hi(qh: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    bits = qh.contiguous().view(torch.int32).to(torch.int64)  # [n, 1]
    j = torch.arange(16, device=qh.device, dtype=torch.int64)
    return (((bits >> j) & 1) << 4).to(torch.int16), (((bits >> (j + 16)) & 1) << 4).to(torch.int16)


def _q5_0(b):
    h0, h1 = _q5_hi(b[:, 2:6])
    lo, hi = _nibbles(b[:, 6:])
    return _f16(b[:, :2]) * (torch.cat([lo | h0, hi | h1], 1) - 16).float()


def _q5_1(b):
    h0, h1 = _q5_hi(b[:, 4:8])
    lo, hi = _nibbles(b[:, 8:])
    return _f16(b[:, :2]) * torch.cat([lo | h0, hi | h1], 1).float() + _f16(b[:, 2:4])


def _q4_k(b):
    d, dmin = _f16(b[:, 0:2]), _f16(b[:, 2:4])
    sc, mn = _k_scale_min(b[:, 4:16])
    lo, hi = _nibbles(b[:, 16:144].reshape(-1, 4, 32))  # 4 groups of 64 values: sub-blocks 2g (low), 2g + 1 (high)
    q = torch.stack([lo, hi], 2).reshape(-1, 8, 32).float()
    return (d[:, :, None] * sc[:, :, None] * q - dmin[:, :, None] * mn[:, :, None]).reshape(-1, 256)


def _q5_k(b):
    d, dmin = _f16(b[:, 0:2]), _f16(b[:, 2:4])
    sc, mn = _k_scale_min(b[:, 4:16])
    qh = b[:, 16:48].to(torch.int16)[:, None, :]  # bit 2g / 2g + 1 of byte l: sub-block 2g / 2g + 1
    lo, hi = _nibbles(b[:, 48:176].reshape(-1, 4, 32))
    g = torch.arange(4, device=b.device, dtype=torch.int16)[None, :, None]
    q = torch.stack([lo + (((qh >> (2 * g)) & 1) << 4), hi + (((qh >> (2 * g + 1)) & 1) << 4)], 2)
    q = q.reshape(-1, 8, 32).float()
    return (d[:, :, None] * sc[:, :, None] * q - dmin[:, :, None] * mn[:, :, None]).reshape(-1, 256)


def _l16(device) -> torch.Tensor:
    return torch.arange(32, device=device) // 16  # lane l of a 32-value group -> its 16-value sub-block


def _q6_k(b):
    ql = b[:, 0:128].reshape(-1, 2, 64).to(torch.int16)  # two halves of 128 values
    qh = b[:, 128:192].reshape(-1, 2, 32).to(torch.int16)
    sc = b[:, 192:208].view(torch.int8).float().reshape(-1, 2, 4, 2)
    d = _f16(b[:, 208:210])
    q1 = (ql[:, :, :32] & 0xF) | ((qh & 3) << 4)
    q2 = (ql[:, :, 32:] & 0xF) | (((qh >> 2) & 3) << 4)
    q3 = (ql[:, :, :32] >> 4) | (((qh >> 4) & 3) << 4)
    q4 = (ql[:, :, 32:] >> 4) | (((qh >> 6) & 3) << 4)
    q = (torch.stack([q1, q2, q3, q4], 2) - 32).float()  # [n, half, quarter k, 32]: scale sc[half, 2k + l // 16]
    return (d[:, :, None, None] * sc[:, :, :, _l16(b.device)] * q).reshape(-1, 256)


def _q2_k(b):
    sc = b[:, 0:16].to(torch.int16).reshape(-1, 2, 4, 2)  # 16 sub-blocks of 16: low nibble scale, high nibble min
    qs = b[:, 16:80].reshape(-1, 2, 32).to(torch.int16)   # two halves of 128 values
    d, dmin = _f16(b[:, 80:82]), _f16(b[:, 82:84])
    shift = (2 * torch.arange(4, device=b.device, dtype=torch.int16))[None, None, :, None]
    q = ((qs[:, :, None, :] >> shift) & 3).float()       # [n, half, j, 32]: value 128 h + 32 j + l
    s = sc[:, :, :, _l16(b.device)]                       # scale index 8 h + 2 j + l // 16
    return (d[:, :, None, None] * (s & 0xF).float() * q - dmin[:, :, None, None] * (s >> 4).float()).reshape(-1, 256)


def _q3_k(b):
    hm = b[:, 0:32].to(torch.int16)                       # high bit of value (h, j, l): bit 4 h + j of byte l
    qs = b[:, 32:96].reshape(-1, 2, 32).to(torch.int16)
    raw = b[:, 96:108].contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF  # the packed 6-bit scales
    d = _f16(b[:, 108:110])
    k1, k2 = 0x03030303, 0x0F0F0F0F
    a0, a1, t = raw[:, 0], raw[:, 1], raw[:, 2]
    aux = torch.stack([(a0 & k2) | (((t >> 0) & k1) << 4), (a1 & k2) | (((t >> 2) & k1) << 4),
                       ((a0 >> 4) & k2) | (((t >> 4) & k1) << 4), ((a1 >> 4) & k2) | (((t >> 6) & k1) << 4)], 1)
    scales = aux.to(torch.int32).contiguous().view(torch.int8).float().reshape(-1, 2, 4, 2) - 32.0
    ar = torch.arange(4, device=b.device, dtype=torch.int16)
    lo = (qs[:, :, None, :] >> (2 * ar)[None, None, :, None]) & 3  # [n, half, j, 32]
    bit = (4 * torch.arange(2, device=b.device, dtype=torch.int16))[None, :, None, None] + ar[None, None, :, None]
    hi = (hm[:, None, None, :] >> bit) & 1
    q = (lo - torch.where(hi == 1, 0, 4)).float()
    return (d[:, :, None, None] * scales[:, :, :, _l16(b.device)] * q).reshape(-1, 256)


_DEQUANT = {"Q8_0": _q8_0, "Q4_0": _q4_0, "Q4_1": _q4_1, "Q5_0": _q5_0, "Q5_1": _q5_1, "Q2_K": _q2_k, "Q3_K": _q3_k,
            "Q4_K": _q4_k, "Q5_K": _q5_k, "Q6_K": _q6_k}


# ---------------------------------------------------------------------------------------------------- quantisers
def quantize_q8_0(x: np.ndarray) -> np.ndarray:
    """ggml Q8_0 blocks of ``x`` (fp32, length a multiple of 32): d = amax / 127, q = round(x / d)."""
    x = np.asarray(x, np.float32).reshape(-1, 32)
    amax = np.abs(x).max(1, keepdims=True)
    d = amax / 127.0
    inv = np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0)
    q = np.clip(np.round(x * inv), -127, 127).astype(np.int8)
    return np.concatenate([d.astype(np.float16).view(np.uint8), q.view(np.uint8)], 1).reshape(-1)


def quantize_q4_0(x: np.ndarray) -> np.ndarray:
    """ggml Q4_0 blocks: d = signed max / -8, q = clamp(round(x / d) + 8, 0, 15), low nibbles the first 16."""
    x = np.asarray(x, np.float32).reshape(-1, 32)
    idx = np.abs(x).argmax(1)
    mx = x[np.arange(len(x)), idx][:, None]
    d = mx / -8.0
    inv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0)
    q = np.clip(np.floor(x * inv + 8.5), 0, 15).astype(np.uint8)
    qs = q[:, :16] | (q[:, 16:] << 4)
    return np.concatenate([d.astype(np.float16).view(np.uint8), qs], 1).reshape(-1)


def quantize_q4_k(x: np.ndarray) -> np.ndarray:
    """Q4_K blocks (models/q4.py's min/max fit) of ``x`` (length a multiple of 256)."""
    from .q4 import quantize_q4_k as q4k

    return q4k(torch.from_numpy(np.asarray(x, np.float32).reshape(-1, 256))).numpy().reshape(-1)


_QUANT = {"Q8_0": quantize_q8_0, "Q4_0": quantize_q4_0, "Q4_K": quantize_q4_k}


# ---------------------------------------------------------------------------------------------------- writer
def write_gguf(path: Union[str, os.PathLike], metadata: Dict[str, Any], tensors: Dict[str, Tuple[np.ndarray, str]],
               alignment: int = 32) -> None:
    """A GGUF v3 file: ``metadata`` (str / int / float / bool / list values) and ``tensors`` name -> (array in torch
    order, type name among F32 / F16 / BF16 / Q8_0 / Q4_0).  Used by the tests and by ``export_gguf``."""
    def s(x: str) -> bytes:
        b = x.encode("utf-8")
        return struct.pack("<Q", len(b)) + b

    def val(v) -> bytes:
        if isinstance(v, bool):
            return struct.pack("<I?", 7, v)
        if isinstance(v, int):
            return struct.pack("<Iq", 11, v) if v < 0 else struct.pack("<IQ", 10, v) if v >= 2 ** 32 else \
                struct.pack("<II", 4, v)
        if isinstance(v, float):
            return struct.pack("<If", 6, v)
        if isinstance(v, str):
            return struct.pack("<I", _STRING) + s(v)
        if isinstance(v, (list, tuple)):
            if all(isinstance(e, str) for e in v):
                return struct.pack("<IIQ", _ARRAY, _STRING, len(v)) + b"".join(s(e) for e in v)
            if all(isinstance(e, int) and not isinstance(e, bool) for e in v):
                return struct.pack("<IIQ", _ARRAY, 5, len(v)) + np.asarray(v, "<i4").tobytes()
            return struct.pack("<IIQ", _ARRAY, 6, len(v)) + np.asarray(v, "<f4").tobytes()
        raise TypeError(f"metadata value {v!r}")

    meta = dict(metadata, **{"general.alignment": alignment})
    blobs, infos, off = [], [], 0
    for name, (arr, tname) in tensors.items():
        a = np.asarray(arr, np.float32)
        if tname == "F32":
            data = a.astype("<f4").tobytes()
        elif tname == "F16":
            data = a.astype("<f2").tobytes()
        elif tname == "BF16":  # round to nearest even, as torch does
            data = torch.from_numpy(a.reshape(-1).copy()).to(torch.bfloat16).view(torch.int16).numpy().tobytes()
        else:
            data = _QUANT[tname](a.reshape(-1)).tobytes()
        ne = tuple(reversed(a.shape))
        infos.append(s(name) + struct.pack("<I", len(ne)) + struct.pack(f"<{len(ne)}Q", *ne) +
                     struct.pack("<IQ", TYPE_ID[tname], off))
        blobs.append(data)
        off += (len(data) + alignment - 1) // alignment * alignment
    head = GGUF_MAGIC + struct.pack("<IQQ", 3, len(tensors), len(meta))
    head += b"".join(s(k) + val(v) for k, v in meta.items()) + b"".join(infos)
    with open(path, "wb") as f:
        f.write(head)
        f.write(b"\0" * ((-len(head)) % alignment))
        for data in blobs:
            f.write(data)
            f.write(b"\0" * ((-len(data)) % alignment))


# ---------------------------------------------------------------------------------------------------- model mapping
ARCHS = ("llama", "qwen2", "gemma", "phi3")


def permute_qk(w: torch.Tensor, n_head: int) -> torch.Tensor:
    """llama.cpp's q / k row order for arch ``llama`` (each head's rotate-half pairs interleaved): HF -> GGUF."""
    return w.reshape(n_head, 2, w.shape[0] // n_head // 2, *w.shape[1:]).transpose(1, 2).reshape(w.shape)


def unpermute_qk(w: torch.Tensor, n_head: int) -> torch.Tensor:
    """Inverse of ``permute_qk``: GGUF -> the rotate-half row order the engine and transformers use."""
    return w.reshape(n_head, w.shape[0] // n_head // 2, 2, *w.shape[1:]).transpose(1, 2).reshape(w.shape)


def config_from_gguf(g: GGUFFile, name: Optional[str] = None) -> ModelConfig:
    md = g.metadata
    arch = md.get("general.architecture")
    if arch not in ARCHS:
        raise ValueError(f"unsupported GGUF architecture {arch!r}; supported: {ARCHS}")

    def k(key, default=None):
        return md.get(f"{arch}.{key}", default)

    d = int(k("embedding_length"))
    n_heads = int(k("attention.head_count"))
    n_kv = int(k("attention.head_count_kv", n_heads))
    head_dim = int(k("attention.key_length") or k("rope.dimension_count") or d // n_heads)
    if int(k("rope.dimension_count", head_dim)) != head_dim:
        raise NotImplementedError("partial rotary embeddings are not supported")
    if g.has("rope_factors_long.weight") or g.has("rope_factors_short.weight"):
        raise NotImplementedError("long-rope (Phi-3 128k) RoPE factors are not supported")
    if k("rope.scaling.type") not in (None, "none"):
        raise NotImplementedError(f"RoPE scaling {k('rope.scaling.type')!r} is not supported")
    factors = tuple(float(x) for x in g.tensor("rope_freqs.weight").reshape(-1)) if g.has("rope_freqs.weight") \
        else None
    vocab = int(g.tensors["token_embd.weight"].shape[0])  # the embedding's rows (GGUF pads the vocabulary to them)
    ctx = int(k("context_length", 8192))
    window = k("attention.sliding_window")
    if window and int(window) < ctx:
        ctx = int(window)
    gemma = arch == "gemma"
    cfg = ModelConfig(
        name=name or md.get("general.name", arch), display_name=md.get("general.name", name or arch),
        n_layers=int(k("block_count")), d_model=d, n_heads=n_heads, n_kv_heads=n_kv, head_dim=head_dim,
        ffn=int(k("feed_forward_length")), vocab=vocab, act="gelu_tanh" if gemma else "silu",
        tie_embeddings=not g.has("output.weight"), qkv_bias=g.has("blk.0.attn_q.bias") or g.has("blk.0.attn_qkv.bias"),
        rope_theta=float(k("rope.freq_base", 10000.0)), norm_eps=float(k("attention.layer_norm_rms_epsilon", 1e-5)),
        norm_add_one=gemma, embed_scale=gemma, max_context=ctx,
        bos_id=int(md.get("tokenizer.ggml.bos_token_id", 1)), eos_id=int(md.get("tokenizer.ggml.eos_token_id", 2)),
        rope_freq_factors=factors, family=arch)
    from .hf import with_stop_ids

    return with_stop_ids(cfg, gguf_stop_ids(g))


def load_gguf_weights(g: GGUFFile, cfg: ModelConfig, device="cpu", dtype=torch.bfloat16) -> ModelWeights:
    arch = g.metadata["general.architecture"]

    def w(name: str) -> torch.Tensor:
        return g.tensor(name, device=device, dtype=dtype)

    def norm(name: str) -> torch.Tensor:
        t = g.tensor(name, device=device)
        return (t - 1.0 if arch == "gemma" else t).to(dtype)  # GGUF Gemma stores 1 + w

    f = cfg.ffn
    layers = []
    for i in range(cfg.n_layers):
        p = f"blk.{i}."
        if g.has(p + "attn_qkv.weight"):
            wqkv = w(p + "attn_qkv.weight")
            bqkv = w(p + "attn_qkv.bias") if g.has(p + "attn_qkv.bias") else None
        else:
            q, kk = w(p + "attn_q.weight"), w(p + "attn_k.weight")
            if arch == "llama":
                q, kk = unpermute_qk(q, cfg.n_heads), unpermute_qk(kk, cfg.n_kv_heads)
            wqkv = torch.cat([q, kk, w(p + "attn_v.weight")], 0)
            bqkv = (torch.cat([w(p + f"attn_{x}.bias") for x in "qkv"], 0) if g.has(p + "attn_q.bias") else None)
        if g.has(p + "ffn_gate.weight"):
            w_gate, w_up = w(p + "ffn_gate.weight"), w(p + "ffn_up.weight")
        else:  # phi3: ffn_up = [gate; up]
            gu = w(p + "ffn_up.weight")
            w_gate, w_up = gu[:f].contiguous(), gu[f:].contiguous()
        layers.append(LayerWeights(attn_norm=norm(p + "attn_norm.weight"), wqkv=wqkv, bqkv=bqkv,
                                   wo=w(p + "attn_output.weight"), mlp_norm=norm(p + "ffn_norm.weight"),
                                   w_gate=w_gate, w_up=w_up, w_down=w(p + "ffn_down.weight")))
        want = (cfg.qkv_dim, cfg.d_model)
        if tuple(wqkv.shape) != want or tuple(w_gate.shape) != (f, cfg.d_model):
            raise ValueError(f"layer {i}: qkv {tuple(wqkv.shape)} / gate {tuple(w_gate.shape)} do not match the "
                             f"metadata ({want}, {(f, cfg.d_model)})")
    embed = w("token_embd.weight")
    lm_head = w("output.weight") if g.has("output.weight") else embed
    return ModelWeights(cfg, embed, norm("output_norm.weight"), lm_head, layers)


def load_gguf_tokenizer(g: GGUFFile, cfg: Optional[ModelConfig] = None):
    """The file's vocabulary as a tokenizer (transformers' GGUF converters), or None without one."""
    md = g.metadata
    if "tokenizer.ggml.tokens" not in md:
        return None
    from transformers.integrations.ggml import GGUF_TO_FAST_CONVERTERS

    arch = md["general.architecture"]
    fields = {"tokenizer_type": md.get("tokenizer.ggml.model"), "tokens": md["tokenizer.ggml.tokens"]}
    for src, dst in (("scores", "scores"), ("token_type", "token_type"), ("merges", "merges"),
                     ("bos_token_id", "bos_token_id"), ("eos_token_id", "eos_token_id"),
                     ("unknown_token_id", "unk_token_id"), ("padding_token_id", "pad_token_id"),
                     ("add_space_prefix", "add_prefix_space")):
        if f"tokenizer.ggml.{src}" in md:
            fields[dst] = md[f"tokenizer.ggml.{src}"]
    for k in ("bos_token_id", "eos_token_id", "unk_token_id", "pad_token_id"):  # the converters read all four
        fields.setdefault(k, None)
    conv = GGUF_TO_FAST_CONVERTERS.get({"gemma": "gemma2"}.get(arch, arch))
    if conv is None:
        return None
    from .tokenizer import HFTokenizer

    bos = md.get("tokenizer.ggml.bos_token_id")
    tok = HFTokenizer.from_tokenizer(conv(fields).converted(), int(bos) if isinstance(bos, int) else
                                     (cfg.bos_id if cfg else None))
    # BOS as llama.cpp adds it: tokenizer.ggml.add_bos_token, else its per-vocabulary default (SentencePiece "llama"
    # vocabularies -- Llama 2, Mistral, Gemma, Phi-3 -- add one; byte-level BPE "gpt2" ones -- Qwen2 -- do not;
    # Llama-3 files carry the key set to true).  The converters attach no post-processor, so encode() prepends it.
    add_bos = md.get("tokenizer.ggml.add_bos_token")
    tok.add_bos_token = bool(add_bos) if add_bos is not None else md.get("tokenizer.ggml.model") == "llama"
    tok.chat_template = md.get("tokenizer.chat_template") or None
    toks = md["tokenizer.ggml.tokens"]
    for key, field in (("bos_token", "bos_token_id"), ("eos_token", "eos_token_id")):
        i = md.get(f"tokenizer.ggml.{field}")
        if isinstance(i, int) and 0 <= i < len(toks):
            tok.special_tokens[key] = toks[i]
    return tok


def load_gguf(path: Union[str, os.PathLike], name: Optional[str] = None, device="cpu", dtype=torch.bfloat16):
    """(config, weights, tokenizer or None) of a GGUF file."""
    g = GGUFFile(path)
    cfg = config_from_gguf(g, name=name or Path(path).stem)
    return cfg, load_gguf_weights(g, cfg, device=device, dtype=dtype), load_gguf_tokenizer(g, cfg)


def gguf_stop_ids(g: GGUFFile) -> List[int]:
    """End ids beside EOS: llama.cpp's ``tokenizer.ggml.eot_token_id`` / ``eom_token_id`` and the vocabulary's
    turn-end tokens (hf.TURN_END_TOKENS)."""
    from .hf import TURN_END_TOKENS

    md = g.metadata
    ids = [int(md[k]) for k in ("tokenizer.ggml.eot_token_id", "tokenizer.ggml.eom_token_id") if k in md]
    toks = md.get("tokenizer.ggml.tokens") or []
    index = {t: i for i, t in enumerate(toks) if t in TURN_END_TOKENS}
    return ids + [index[t] for t in TURN_END_TOKENS if t in index]


def gguf_tokenizer_fields(tokenizer_json: Dict[str, Any], bos_id: Optional[int] = None, eos_id: Optional[int] = None,
                          chat_template: Optional[str] = None) -> Optional[Dict[str, Any]]:
    """``tokenizer.ggml.*`` metadata for a Hugging Face ``tokenizer.json`` (the inverse of what load_gguf_tokenizer
    reads, in llama.cpp's layout), or None when the vocabulary has no GGUF form:

    * byte-level BPE (Llama 3, Qwen2): model "gpt2", tokens by id, merges, control types for added special tokens;
    * SentencePiece-style BPE with byte fallback (Llama 2, Mistral, Gemma, Phi-3): model "llama", tokens by id,
      scores = minus the rank of the merge producing the piece (0 for the base pieces; llama.cpp's SPM tokenizer
      merges by score), byte pieces typed 6 (byte), special tokens 3 (control).
    """
    model = tokenizer_json.get("model") or {}
    if model.get("type") != "BPE":
        return None
    vocab: Dict[str, int] = dict(model.get("vocab") or {})
    special = set()
    for t in tokenizer_json.get("added_tokens") or []:
        vocab[t["content"]] = int(t["id"])
        if t.get("special"):
            special.add(t["content"])
    n = max(vocab.values()) + 1 if vocab else 0
    tokens = [f"[PAD{i}]" for i in range(n)]
    for t, i in vocab.items():
        tokens[i] = t
    merges = [m if isinstance(m, str) else " ".join(m) for m in model.get("merges") or []]

    def has_byte_level(node) -> bool:
        if not isinstance(node, dict):
            return False
        if node.get("type") == "ByteLevel":
            return True
        return any(has_byte_level(x) for x in node.get("pretokenizers") or node.get("decoders") or [])

    types = [3 if t in special else 1 for t in tokens]
    out: Dict[str, Any] = {"tokenizer.ggml.tokens": tokens, "tokenizer.ggml.token_type": types}
    if has_byte_level(tokenizer_json.get("pre_tokenizer")):
        out.update({"tokenizer.ggml.model": "gpt2", "tokenizer.ggml.merges": merges})
    elif model.get("byte_fallback"):
        scores = [0.0] * n
        for rank, m in enumerate(merges):
            i = vocab.get(m.replace(" ", ""))
            if i is not None and scores[i] == 0.0:
                scores[i] = -float(rank + 1)
        for i, t in enumerate(tokens):
            if re.fullmatch(r"<0x[0-9A-F]{2}>", t):
                types[i] = 6
        out.update({"tokenizer.ggml.model": "llama", "tokenizer.ggml.scores": scores})
    else:
        return None
    if bos_id is not None:
        out["tokenizer.ggml.bos_token_id"] = int(bos_id)
        # the checkpoint's own BOS rule: its post-processor template names the BOS token
        out["tokenizer.ggml.add_bos_token"] = tokens[bos_id] in json.dumps(tokenizer_json.get("post_processor") or {})
    if eos_id is not None:
        out["tokenizer.ggml.eos_token_id"] = int(eos_id)
    if chat_template:
        out["tokenizer.chat_template"] = chat_template
    return out


def export_gguf(mw: ModelWeights, path: Union[str, os.PathLike], arch: str, tensor_type: str = "F16",
                tokenizer_fields: Optional[Dict[str, Any]] = None, context_length: Optional[int] = None) -> None:
    """Write ``mw`` as a GGUF file of ``arch`` with llama.cpp's conventions (the inverse of ``load_gguf``): q / k
    rows permuted for ``llama``, Gemma gains as 1 + w, Phi-3's fused qkv / gate-up, Llama-3 scaling as a
    ``rope_freqs`` tensor.  2-D weights in ``tensor_type`` (F32 / F16 / BF16 / Q8_0 / Q4_0), norms in F32."""
    from .config import rope_inv_freq

    cfg = mw.cfg
    if arch not in ARCHS:
        raise ValueError(f"arch must be one of {ARCHS}")
    md: Dict[str, Any] = {
        "general.architecture": arch, "general.name": cfg.name,
        f"{arch}.block_count": cfg.n_layers, f"{arch}.context_length": int(context_length or cfg.max_context),
        f"{arch}.embedding_length": cfg.d_model, f"{arch}.feed_forward_length": cfg.ffn,
        f"{arch}.attention.head_count": cfg.n_heads, f"{arch}.attention.head_count_kv": cfg.n_kv_heads,
        f"{arch}.attention.key_length": cfg.head_dim, f"{arch}.attention.value_length": cfg.head_dim,
        f"{arch}.rope.dimension_count": cfg.head_dim, f"{arch}.rope.freq_base": float(cfg.rope_theta),
        f"{arch}.attention.layer_norm_rms_epsilon": float(cfg.norm_eps),
        "tokenizer.ggml.bos_token_id": cfg.bos_id, "tokenizer.ggml.eos_token_id": cfg.eos_id,
    }
    md.update(tokenizer_fields or {})
    T: Dict[str, Tuple[np.ndarray, str]] = {}

    def put(name, t, typ=None):
        T[name] = (t.detach().float().cpu().numpy(), typ or (tensor_type if t.dim() == 2 else "F32"))

    def gain(t):
        return t.float() + 1.0 if arch == "gemma" else t

    if cfg.rope_scaling is not None or cfg.rope_freq_factors is not None:
        import dataclasses
        base = rope_inv_freq(dataclasses.replace(cfg, rope_scaling=None, rope_freq_factors=None))
        put("rope_freqs.weight", torch.tensor(base / rope_inv_freq(cfg), dtype=torch.float32), "F32")
    put("token_embd.weight", mw.embed)
    if not cfg.tie_embeddings:
        put("output.weight", mw.lm_head)
    put("output_norm.weight", gain(mw.final_norm))
    for i, lw in enumerate(mw.layers):
        p = f"blk.{i}."
        put(p + "attn_norm.weight", gain(lw.attn_norm))
        put(p + "ffn_norm.weight", gain(lw.mlp_norm))
        q, k, v = lw.wqkv.split([cfg.q_dim, cfg.kv_dim, cfg.kv_dim], 0)
        if arch == "phi3":
            put(p + "attn_qkv.weight", lw.wqkv)
            put(p + "ffn_up.weight", torch.cat([lw.w_gate, lw.w_up], 0))
        else:
            if arch == "llama":
                q, k = permute_qk(q, cfg.n_heads), permute_qk(k, cfg.n_kv_heads)
            put(p + "attn_q.weight", q)
            put(p + "attn_k.weight", k)
            put(p + "attn_v.weight", v)
            put(p + "ffn_gate.weight", lw.w_gate)
            put(p + "ffn_up.weight", lw.w_up)
        if lw.bqkv is not None:
            bq, bk, bv = lw.bqkv.split([cfg.q_dim, cfg.kv_dim, cfg.kv_dim], 0)
            put(p + "attn_q.bias", bq, "F32")
            put(p + "attn_k.bias", bk, "F32")
            put(p + "attn_v.bias", bv, "F32")
        put(p + "attn_output.weight", lw.wo)
        put(p + "ffn_down.weight", lw.w_down)
    write_gguf(path, md, T)


def is_gguf(path: Union[str, os.PathLike]) -> bool:
    p = Path(path)
    if not p.is_file():
        return False
    with open(p, "rb") as f:
        return f.read(4) == GGUF_MAGIC
