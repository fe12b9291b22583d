"""int8 key/value cache and its wire format.

The int8 forward of the reference already returns its quantised operands (attention_int8.py:259-262:
``q_i8, k_i8T, v_i8, sq, sk, sv, Bq, Bkv``).  For inference the key/value half of that tuple is the
natural cache: keys and values are quantised once, per 32-token block, and every later query block
attends to them without touching fp16 K/V again.  This module keeps that state in HBM
(:class:`QuantizedKV`), grows it in 32-token blocks, runs the HIP forward against it, and moves it in
one self-describing byte buffer.

Wire format (little-endian, version 1)::

    offset 0   8 B   magic  b"QATTNKV1"
    offset 8   4 B   header length H (uint32)
    offset 12  H B   UTF-8 JSON header: {"batch", "kv_heads", "tokens", "head_dim", "block": 32,
                     "smoothed": bool, "sections": {name: [offset, nbytes, dtype, shape]}}
    then the sections, each 256-byte aligned, offsets from the start of the buffer:
      k_i8    int8    [batch, kv_heads, tokens, head_dim]   row-major (the reference's k_i8T, untransposed)
      v_i8    int8    [batch, kv_heads, tokens, head_dim]
      sk, sv  float16 [batch * kv_heads * tokens / 32]      one scale per 32-token block,
                                                            index (b * kv_heads + h) * tokens / 32 + s / 32
      k_mean  float16 [batch, kv_heads, 1, head_dim]        only when "smoothed" (SageAttention k-smoothing)

The forward's P.V operand is not stored either: :meth:`QuantizedKV.vt` rebuilds the int8 V^T
operand image from v_i8 on the GPU (``qattn_int8_v_image``), bit-identically to the quantiser's own
output; :meth:`QuantizedKV.vdq` gives the dequantised values f16(v_i8 * sv) (``qattn_int8_dequant``).

Causal attention against a cache aligns the LAST query with the LAST key (query i of the Sq new
ones sits at position Sk - Sq + i and keeps the keys up to it: ``causal = 2`` of
qattn_int8_attn_fwd_ex), so a decode step sees the whole prefix.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib

MAGIC = b"QATTNKV1"
BLOCK = 32
_ALIGN = 256
_DTYPES = {"int8": torch.int8, "float16": torch.float16}

__all__ = ["QuantizedKV", "quantize_kv", "attention_int8_cached"]


@dataclass
class QuantizedKV:
    """Quantised keys/values of ``batch x kv_heads`` heads with ``tokens`` tokens each (device tensors).

    ``k_i8`` / ``v_i8``: int8 [B, Hkv, S, D]; ``sk`` / ``sv``: fp16 [B * Hkv * S / 32];
    ``k_mean``: fp16 [B, Hkv, 1, D] when the keys were smoothed before quantisation, else None.
    """

    k_i8: torch.Tensor
    v_i8: torch.Tensor
    sk: torch.Tensor
    sv: torch.Tensor
    k_mean: Optional[torch.Tensor] = None
    _vdq: Optional[torch.Tensor] = None
    _vt: Optional[torch.Tensor] = None

    @property
    def shape(self):
        return tuple(self.k_i8.shape)

    def vdq(self) -> torch.Tensor:
        """f16(v_i8 * sv) [B*Hkv*S, D], the dequantised values (rebuilt on demand, cached)."""
        if self._vdq is None:
            B, H, S, D = self.shape
            _lib.require_gpu(self.v_i8, self.sv)
            out = torch.empty((B * H * S, D), dtype=torch.float16, device=self.v_i8.device)
            _lib.call("qattn_int8_dequant", _lib.ptr(self.v_i8), _lib.ptr(self.sv), _lib.ptr(out),
                      B * H * S, D, _lib.stream_of(self.v_i8))
            self._vdq = out
        return self._vdq

    def vt(self) -> torch.Tensor:
        """The int8 V^T operand image of v_i8 [B*Hkv*S, D] bytes, the forward's P.V operand."""
        if self._vt is None:
            B, H, S, D = self.shape
            _lib.require_gpu(self.v_i8)
            out = torch.empty((B * H * S, D), dtype=torch.int8, device=self.v_i8.device)
            vi = self.v_i8.contiguous()   # (bound: it must outlive the launch)
            _lib.call("qattn_int8_v_image", _lib.ptr(vi), _lib.ptr(out), B * H * S, D,
                      _lib.stream_of(self.v_i8))
            self._vt = out
        return self._vt

    def drop_operands(self) -> None:
        """Free the cached P.V operand images (rebuilt on the next use); the cache proper is k_i8,
        v_i8, sk, sv (and k_mean)."""
        self._vdq = None
        self._vt = None

    # ------------------------------------------------------------------------------ growth
    def append(self, k: torch.Tensor, v: torch.Tensor) -> "QuantizedKV":
        """Quantise ``k, v`` [B, Hkv, n, D] (n % 32 == 0) and append them along the token axis.

        Quantisation is per 32-token block, so for an unsmoothed cache the result is bit-identical to
        quantising the concatenated sequence.  A smoothed cache subtracts its stored ``k_mean`` (the
        mean of the tokens it was created from) from the new keys; softmax is invariant to that
        shift, but the indices differ from smoothing with the mean of the longer sequence.
        """
        B, H, S, D = self.shape
        if k.shape[:2] != (B, H) or k.shape[3] != D or k.shape != v.shape or k.shape[2] % BLOCK:
            raise _lib.QAttnError("qattn kv cache: appended blocks must be [B, Hkv, 32*n, D]")
        new = quantize_kv(k, v, smooth=False, k_mean=self.k_mean)
        n = k.shape[2]
        cat = lambda a, b_: torch.cat([a, b_], dim=2)  # noqa: E731
        sk = torch.cat([self.sk.view(B, H, S // BLOCK), new.sk.view(B, H, n // BLOCK)], 2).reshape(-1)
        sv = torch.cat([self.sv.view(B, H, S // BLOCK), new.sv.view(B, H, n // BLOCK)], 2).reshape(-1)
        return QuantizedKV(cat(self.k_i8, new.k_i8), cat(self.v_i8, new.v_i8), sk, sv, self.k_mean)

    # ------------------------------------------------------------------------------ wire format
    def to_bytes(self) -> torch.Tensor:
        """Serialise into one uint8 tensor on the cache's device (see the module docstring)."""
        B, H, S, D = self.shape
        parts = [("k_i8", self.k_i8), ("v_i8", self.v_i8), ("sk", self.sk), ("sv", self.sv)]
        if self.k_mean is not None:
            parts.append(("k_mean", self.k_mean))
        sections, off = {}, 0
        for name, t in parts:
            nbytes = t.numel() * t.element_size()
            sections[name] = [off, nbytes, str(t.dtype).replace("torch.", ""), list(t.shape)]
            off += (nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
        header = {"batch": B, "kv_heads": H, "tokens": S, "head_dim": D, "block": BLOCK,
                  "smoothed": self.k_mean is not None, "sections": {}}
        # section offsets are absolute: header size first, then shift
        hdr = json.dumps(header).encode()
        base = 0
        for _ in range(3):   # the header length depends on the offsets it holds
            base = (12 + len(hdr) + _ALIGN - 1) // _ALIGN * _ALIGN
            header["sections"] = {k_: [o + base, n, dt, sh] for k_, (o, n, dt, sh) in sections.items()}
            hdr = json.dumps(header).encode()
        assert (12 + len(hdr) + _ALIGN - 1) // _ALIGN * _ALIGN == base
        buf = torch.zeros(base + off, dtype=torch.uint8, device=self.k_i8.device)
        prefix = MAGIC + len(hdr).to_bytes(4, "little") + hdr
        buf[:len(prefix)] = torch.frombuffer(bytearray(prefix), dtype=torch.uint8).to(buf.device)
        for name, t in parts:
            o, n = header["sections"][name][:2]
            buf[o:o + n] = t.contiguous().view(-1).view(torch.uint8)
        return buf

    @staticmethod
    def from_bytes(buf: torch.Tensor, device=None) -> "QuantizedKV":
        """Parse a buffer written by :meth:`to_bytes` (sections become views of ``buf``, moved to
        ``device`` if given)."""
        if device is not None:
            buf = buf.to(device)
        head = bytes(buf[:12].cpu().tolist())
        if head[:8] != MAGIC:
            raise _lib.QAttnError("qattn kv cache: bad magic (not a QATTNKV1 buffer)")
        hlen = int.from_bytes(head[8:12], "little")
        header = json.loads(bytes(buf[12:12 + hlen].cpu().tolist()).decode())
        if header.get("block") != BLOCK:
            raise _lib.QAttnError("qattn kv cache: unsupported block size")
        t = {}
        for name, (o, n, dt, sh) in header["sections"].items():
            t[name] = buf[o:o + n].view(_DTYPES[dt]).view(sh)
        return QuantizedKV(t["k_i8"], t["v_i8"], t["sk"], t["sv"], t.get("k_mean"))

    @staticmethod
    def from_forward_outputs(outputs, batch: int, kv_heads: int, k_mean=None) -> "QuantizedKV":
        """The cache held by the reference-shaped forward output
        ``(O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, Bq, Bkv)`` (attention_int8.py:259-262)."""
        _O, _lse, _qi, k_i8T, v_i8, _sq, sk, sv, _bq, bkv = outputs
        if bkv != BLOCK:
            raise _lib.QAttnError("qattn kv cache: Bkv must be 32")
        D = k_i8T.shape[0]
        S = k_i8T.shape[1] // (batch * kv_heads)
        k_i8 = k_i8T.t().contiguous().view(batch, kv_heads, S, D)
        return QuantizedKV(k_i8, v_i8.view(batch, kv_heads, S, D), sk, sv, k_mean)


def quantize_kv(k: torch.Tensor, v: torch.Tensor, smooth: bool = True,
                k_mean: Optional[torch.Tensor] = None) -> QuantizedKV:
    """Quantise fp16 ``k, v`` [B, Hkv, S, D] per 32-token block on the GPU (the forward's quantiser,
    attention_int8.py:188-195, 241-247).  ``smooth`` subtracts the per-head token mean from k first
    (SageAttention smoothing, as ``sage_attention_3_int8``); an explicit ``k_mean`` is used as given."""
    if k.shape != v.shape or k.dim() != 4:
        raise _lib.QAttnError("qattn kv cache: k and v must be [B, Hkv, S, D] of one shape")
    B, H, S, D = k.shape
    if S % BLOCK or D not in (64, 128):
        raise _lib.QAttnError("qattn kv cache: tokens must be a multiple of 32, head_dim 64 or 128")
    _lib.require_gpu(k, v)
    k = k.to(torch.float16).contiguous()
    v = v.to(torch.float16).contiguous()
    dev, st = k.device, _lib.stream_of(k)
    N = B * H * S
    if smooth and k_mean is None:
        k_mean = torch.empty((B, H, 1, D), dtype=torch.float16, device=dev)
        _lib.call("qattn_kmean", _lib.ptr(k), _lib.ptr(k_mean), B * H, S, D, st)
    k_i8 = torch.empty((B, H, S, D), dtype=torch.int8, device=dev)
    v_i8 = torch.empty((B, H, S, D), dtype=torch.int8, device=dev)
    sk = torch.empty((N // BLOCK,), dtype=torch.float16, device=dev)
    sv = torch.empty((N // BLOCK,), dtype=torch.float16, device=dev)
    km = None if k_mean is None else k_mean.to(torch.float16).contiguous()
    _lib.call("qattn_int8_quant", _lib.ptr(k), _lib.ptr(k_i8), _lib.ptr(sk), None, _lib.ptr(km), N, S, D,
              st)
    # v: indices, scales and the P.V operand image in one pass, 1 B per element
    vt = torch.empty((N, D), dtype=torch.int8, device=dev)
    _lib.call("qattn_int8_quant_vt", _lib.ptr(v), _lib.ptr(v_i8), _lib.ptr(sv), _lib.ptr(vt), N, D, st)
    return QuantizedKV(k_i8, v_i8, sk, sv, km, None, vt)


def attention_int8_cached(q: torch.Tensor, kv: QuantizedKV, causal: bool = False):
    """int8 attention of fp16 queries [B, Hq, Sq, D] against a quantised cache (inference; no autograd).

    Hq must be a multiple of the cache's heads (grouped-query attention).  ``causal``: the Sq queries
    are the LAST Sq positions (query i keeps keys <= Sk - Sq + i), Sq <= Sk.  Returns (O fp16
    [B, Hq, Sq, D], lse fp16 [B*Hq*Sq]); without ``causal`` identical to the forward on the un-cached
    tensors (bit-identical when one key split covers the cache).
    Non-causal at head_dim 128 runs in the decoding layout (_decode_split: the
    grouped query heads of a key/value head in one workgroup, long caches split over the keys and
    merged); the results equal the one-pass forward's up to the merge's rounding (<= 2e-3).
    """
    B, Hkv, Sk, D = kv.shape
    if q.dim() != 4 or q.shape[0] != B or q.shape[3] != D or q.shape[1] % Hkv or q.shape[2] % BLOCK:
        raise _lib.QAttnError("qattn kv cache: q must be [B, G*Hkv, 32*n, D] for the cache's B, Hkv, D")
    if causal and q.shape[2] > Sk:
        raise _lib.QAttnError("qattn kv cache: causal attention needs Sq <= the cached tokens")
    _lib.require_gpu(q, kv.k_i8)
    q = q.to(torch.float16).contiguous()
    Hq, Sq = q.shape[1], q.shape[2]
    N = B * Hq * Sq
    dev, st = q.device, _lib.stream_of(q)
    q_i8 = torch.empty((N, D), dtype=torch.int8, device=dev)
    sq = torch.empty((N // BLOCK,), dtype=torch.float16, device=dev)
    O = torch.empty((B, Hq, Sq, D), dtype=torch.float16, device=dev)
    lse = torch.empty((N,), dtype=torch.float16, device=dev)
    _lib.call("qattn_int8_quant", _lib.ptr(q), _lib.ptr(q_i8), _lib.ptr(sq), None, None, N, Sq, D, st)
    qks = float(torch.tensor(1.0 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
    mode = 2 if causal else 0          # bottom-right aligned causal mask
    if not causal and D == 128:
        _decode_split(q_i8, sq, kv, O, lse, B, Hq, Sq, qks, st)
        return O, lse
    _lib.call("qattn_int8_attn_fwd_ex", _lib.ptr(q_i8), _lib.ptr(sq), _lib.ptr(kv.k_i8),
              _lib.ptr(kv.sk), _lib.ptr(kv.vt()), _lib.ptr(kv.sv), _lib.ptr(O), _lib.ptr(lse),
              B * Hq, Sq, Sk, Hq // Hkv, mode, D, qks, st)
    return O, lse


def _split_plan(bhv: int, rows: int, sk: int) -> int:
    """Keys per split of the decoding forward: enough workgroups for two per CU (512), each split
    at least 32 key tiles (1024 keys: a workgroup's fixed prologue / epilogue cost is worth ~20
    tiles); sk (a multiple of 32) when one split suffices.  Measured on MI355X (tools/sweep_decode.py,
    D = 128): (B, Hq, Hkv, Sk) = (8, 32, 8, 8192) 1024 keys 56 us (512: 72, 2048: 60, one pass
    154); (8, 32, 32, 8192) 4096 keys 110 us (1024: 127, one pass 142); (1, 32, 8, 32768) 1024 keys
    49 us (512: 65, 2048: 56, one pass 578)."""
    wgs = bhv * -(-rows // 128)
    nsplit = max(1, min(sk // 1024, -(-512 // wgs)))
    return -(-(sk // 32) // nsplit) * 32


def _decode_split(q_i8, sq, kv, O, lse, B, Hq, Sq, qks, st):
    """Non-causal cached attention in the decoding layout.

    * Grouped query heads share one key/value head: the G = Hq / Hkv query heads of a key/value
      head are consecutive [Sq, D] blocks in memory, so they are run as ONE virtual head of G * Sq
      rows against that key/value head (group 1): the G heads' query blocks sit in one workgroup
      and read each key/value tile once (same rows, same scale blocks, same outputs).
    * Short query blocks against long caches are split over the keys (qattn_int8_attn_fwd_split)
      and merged (qattn_int8_split_combine), so that the grid fills the chip."""
    _, Hkv, Sk, D = kv.shape
    bhv, rows = B * Hkv, (Hq // Hkv) * Sq
    if bhv * rows == 0:
        return
    ks = _split_plan(bhv, rows, Sk)
    if ks >= Sk:
        _lib.call("qattn_int8_attn_fwd_ex", _lib.ptr(q_i8), _lib.ptr(sq), _lib.ptr(kv.k_i8),
                  _lib.ptr(kv.sk), _lib.ptr(kv.vt()), _lib.ptr(kv.sv), _lib.ptr(O), _lib.ptr(lse),
                  bhv, rows, Sk, 1, 0, D, qks, st)
        return
    nsplit = -(-Sk // ks)
    opart = torch.empty((nsplit, bhv * rows, D), dtype=torch.float16, device=O.device)
    ml = torch.empty((nsplit, bhv * rows, 2), dtype=torch.float32, device=O.device)
    _lib.call("qattn_int8_attn_fwd_split", _lib.ptr(q_i8), _lib.ptr(sq), _lib.ptr(kv.k_i8),
              _lib.ptr(kv.sk), _lib.ptr(kv.vt()), _lib.ptr(kv.sv), _lib.ptr(opart), _lib.ptr(ml),
              bhv, rows, Sk, 1, ks, D, qks, st)
    _lib.call("qattn_int8_split_combine", _lib.ptr(opart), _lib.ptr(ml), _lib.ptr(O), _lib.ptr(lse),
              bhv * rows, nsplit, D, st)
