"""MX-FP4 inference attention forward on gfx950 block-scaled MFMA.

The reference lists SageAttention3's FP4 attention (README.md:49-55) as its goal but ships only the
int8 variant; this module is the FP4 forward built on the CDNA4 ``v_mfma_scale_f32_32x32x64_f8f6f4``
instruction (4x the bf16 MFMA rate).  There is no reference interface to mirror, so the names
follow the int8 module: ``sage_attention_3_fp4(q, k, v)`` is the drop-in style entry, and
``mxfp4_attn_fwd`` exposes the quantised operands for tests and for KV reuse.

Numerics (csrc/mxfp4_attn.hip header): Q and K are MX-FP4 along head_dim (32-element blocks,
e8m0 scales); V along keys; P is re-quantised to MX-FP4 per query row and 32 keys inside the
kernel; the softmax state is fp32 and the row sum l adds the quantised P (on the matrix core).
The running max is kept as an integer raised lazily, so every rescale is a power of two and the
fp4 codes of P do not depend on the tile order of the max updates.  K is smoothed by its token mean first
(SageAttention), which leaves softmax unchanged and shrinks the K block ranges.  Forward only:
the outputs carry no autograd graph.
"""
from __future__ import annotations

import math

import torch

from . import _lib

__all__ = ["mxfp4_quantize_rows", "mxfp4_quantize_v", "mxfp4_attn_fwd", "sage_attention_3_fp4"]


def _qk_scale(head_dim: int) -> float:
    return float(torch.tensor(1.0 / math.sqrt(head_dim) * 1.44269504, dtype=torch.float32))


def mxfp4_quantize_rows(x: torch.Tensor, mean: torch.Tensor | None = None):
    """x [..., S, D] (fp16) -> (packed uint8 [rows, D/2], scales uint8 [rows, D/32]).

    ``mean`` [..., 1, D] (fp16, one row per leading index): quantise f16(x - mean) instead.
    """
    _lib.require_gpu(x)
    D = x.shape[-1]
    if D not in (64, 128):
        raise _lib.QAttnError("qattn mxfp4: head_dim must be 64 or 128")
    x = x.to(torch.float16).contiguous()
    rows = x.numel() // D
    seq = x.shape[-2] if x.dim() >= 2 else rows
    if mean is not None:
        mean = mean.to(torch.float16).contiguous()
        if mean.numel() * seq != x.numel():
            raise _lib.QAttnError("qattn mxfp4: mean must hold one row per sequence")
    q4 = torch.empty((rows, D // 2), dtype=torch.uint8, device=x.device)
    sc = torch.empty((rows, D // 32), dtype=torch.uint8, device=x.device)
    _lib.call("qattn_mxfp4_quant_rows", _lib.ptr(x), _lib.ptr(mean) if mean is not None else None,
              _lib.ptr(q4), _lib.ptr(sc), rows, seq, D, _lib.stream_of(x))
    return q4, sc


def mxfp4_quantize_v(v: torch.Tensor):
    """v [B, H, S, D] (fp16) -> (vt uint8 [B*H, S/64, D, 32], vs uint8 [B*H, S/64, D, 2])."""
    _lib.require_gpu(v)
    B, H, S, D = v.shape
    if S % 64:
        raise _lib.QAttnError("qattn mxfp4: key tokens must be a multiple of 64")
    if D not in (64, 128):
        raise _lib.QAttnError("qattn mxfp4: head_dim must be 64 or 128")
    v = v.to(torch.float16).contiguous()
    vt = torch.empty((B * H, S // 64, D, 32), dtype=torch.uint8, device=v.device)
    vs = torch.empty((B * H, S // 64, D, 2), dtype=torch.uint8, device=v.device)
    _lib.call("qattn_mxfp4_quant_vt", _lib.ptr(v), _lib.ptr(vt), _lib.ptr(vs), B * H, S, D,
              _lib.stream_of(v))
    return vt, vs


def _check(q, k, v):
    if q.dim() != 4 or k.shape != v.shape or q.shape[0] != k.shape[0] or q.shape[-1] != k.shape[-1]:
        raise _lib.QAttnError("qattn mxfp4: q [B,H,Sq,D], k = v [B,Hkv,Sk,D] expected")
    if q.shape[1] % k.shape[1]:
        raise _lib.QAttnError("qattn mxfp4: query heads must be a multiple of key/value heads")
    if q.shape[-1] != 128:
        raise _lib.QAttnError("qattn mxfp4: head_dim must be 128")
    if q.shape[2] % 32 or k.shape[2] % 64:
        raise _lib.QAttnError("qattn mxfp4: q tokens must be a multiple of 32, k tokens of 64")


@torch.no_grad()
def mxfp4_attn_fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, smooth_k: bool = True):
    """-> (O fp16 [B,H,Sq,D], lse fp32 [B*H, Sq] base 2, (q4, qs, k4, ks, vt, vs)).

    ``smooth_k`` quantises k - k_mean with k_mean the fp16 token mean per (batch, head)
    (qattn_kmean, as the int8 path); softmax is invariant to it.
    """
    _check(q, k, v)
    _lib.require_gpu(q, k, v)
    B, H, Sq, D = q.shape
    Hkv, Sk = k.shape[1], k.shape[2]
    k = k.to(torch.float16).contiguous()
    k_mean = None
    if smooth_k:   # f16 token mean per (batch, head), subtracted inside the quantiser
        k_mean = torch.empty((B, Hkv, 1, D), dtype=torch.float16, device=q.device)
        _lib.call("qattn_kmean", _lib.ptr(k), _lib.ptr(k_mean), B * Hkv, Sk, D, _lib.stream_of(k))
    q4, qs = mxfp4_quantize_rows(q)
    k4, ks = mxfp4_quantize_rows(k, k_mean)
    vt, vs = mxfp4_quantize_v(v)
    out = torch.empty((B, H, Sq, D), dtype=torch.float16, device=q.device)
    lse = torch.empty((B * H, Sq), dtype=torch.float32, device=q.device)
    _lib.call("qattn_mxfp4_attn_fwd", _lib.ptr(q4), _lib.ptr(qs), _lib.ptr(k4), _lib.ptr(ks),
              _lib.ptr(vt), _lib.ptr(vs), _lib.ptr(out), _lib.ptr(lse), B * H, Sq, Sk, H // Hkv, D,
              _qk_scale(D), _lib.stream_of(q))
    return out, lse, (q4, qs, k4, ks, vt, vs)


def sage_attention_3_fp4(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """softmax(q k^T / sqrt(D)) v with MX-FP4 operands (inference; fp16 output)."""
    return mxfp4_attn_fwd(q, k, v)[0]
