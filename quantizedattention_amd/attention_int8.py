"""Drop-in for ``attention_int8`` of selau642/QuantizedAttention, backed by gfx950 HIP kernels.

Public names (same signatures, argument meaning, outputs and assertion messages):
  SageAttention3_Int8_autograd_function   attention_int8.py:20-95
  helion_atten_int8_hl_dot_fwd            attention_int8.py:97-262
  helion_atten_int8_hl_dot_bwd            attention_int8.py:264-432
  sage_attention_3_int8                   attention_int8.py:434-451
  baseline_pytorch_attention              attention_int8.py:453-481

Semantics follow the build contract of SURVEY.md §8a (rows A4-A6): attention per (batch, head)
(F2), corrected backward (F4), SageAttention k-smoothing with the token mean (F1).  The
``helion_*`` names are kept for drop-in compatibility; no Helion/Triton is involved.

Generalised shapes (extensions the reference does not have): q [B, Hq, Sq, D] with
k, v [B, Hkv, Sk, D], Hq a multiple of Hkv (grouped-query attention: query head h reads key/value
head h // (Hq/Hkv)), Sq != Sk, and ``causal=True`` (keep key <= query, top-left aligned positions;
masked scores are excluded).  With Hq == Hkv, Sq == Sk and causal=False every function is exactly
the reference-shaped one.
"""
from __future__ import annotations

import math
import os
import weakref
from typing import Tuple

import torch
from torch.autograd import Function

from . import _lib
from ._baseline import baseline_pytorch_attention  # noqa: F401  (re-exported like the reference)

BQ = 32   # Bq  (register_tunable default, int8:155)
BKV = 32  # Bkv (int8:158)

__all__ = [
    "SageAttention3_Int8_autograd_function", "helion_atten_int8_hl_dot_fwd",
    "helion_atten_int8_hl_dot_bwd", "sage_attention_3_int8", "baseline_pytorch_attention",
]


def _qk_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim) * 1.44269504  # int8:151-153


def _check_shapes(q, k, v):
    batch, head, q_tokens, q_head_dim = q.shape
    _, _, k_tokens, k_head_dim = k.shape
    _, _, v_tokens, v_head_dim = v.shape
    assert k_tokens == v_tokens, "k and v tokens are different"
    assert k_head_dim == v_head_dim, "k head_dim and v head_dim are different"
    if q_head_dim != k_head_dim or q.shape[0] != k.shape[0] or k.shape[:2] != v.shape[:2]:
        raise _lib.QAttnError("qattn int8: q/k/v must share batch and head_dim, k/v their heads")
    if head % k.shape[1] != 0:
        raise _lib.QAttnError("qattn int8: query heads must be a multiple of key/value heads")
    if q_tokens % BQ != 0 or k_tokens % BKV != 0:
        raise _lib.QAttnError(f"qattn int8: token counts must each be a multiple of {BQ}")
    if q_head_dim not in (64, 128):
        raise _lib.QAttnError("qattn int8: head_dim must be 64 or 128")


# k-smoothing through qattn_int8_quant_k_smooth (one launch) instead of qattn_kmean +
# qattn_int8_quant_img (two): bit-identical (tests/test_gpu_int8.py), and no faster at config 3 (55
# against 54.5 us, 88 against ~83 us with the backward's image; HISTORY.md round 6), so off
FUSED_K_SMOOTH = False


def _int8_forward(q, k, v, smooth: bool, images: bool = False, causal: bool = False):
    """Quantise q, k, v and run the int8 attention forward (csrc/int8_attn_fwd.hip: both
    contractions on the int8 MFMA, P.V as the reference's hl.dot(P_int8, v_int8), int8:249).

    Returns (O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, k_mean, q_bf, k_bf); q_bf / k_bf are the exact
    bf16 images of q_i8 / k_i8 the backward reads (written by the same quantiser pass when
    ``images``, else None).
    """
    _check_shapes(q, k, v)
    _lib.require_gpu(q, k, v)
    q = q.to(torch.float16).contiguous()
    k = k.to(torch.float16).contiguous()
    v = v.to(torch.float16).contiguous()
    B, H, S, D = q.shape
    Hkv, Sk = k.shape[1], k.shape[2]
    N = B * H * S
    Nkv = B * Hkv * Sk
    dev = q.device
    st = _lib.stream_of(q)
    q_i8 = torch.empty((N, D), dtype=torch.int8, device=dev)
    k_i8 = torch.empty((Nkv, D), dtype=torch.int8, device=dev)
    v_i8 = torch.empty((Nkv, D), dtype=torch.int8, device=dev)
    sq = torch.empty((N // BQ,), dtype=torch.float16, device=dev)
    sk = torch.empty((Nkv // BKV,), dtype=torch.float16, device=dev)
    sv = torch.empty((Nkv // BKV,), dtype=torch.float16, device=dev)
    vt = torch.empty((Nkv, D), dtype=torch.int8, device=dev)   # the int8 V^T operand image of v
    O = torch.empty((B, H, S, D), dtype=torch.float16, device=dev)
    lse = torch.empty((N,), dtype=torch.float16, device=dev)
    q_bf = k_bf = None
    if images:
        q_bf = torch.empty((N, D), dtype=torch.bfloat16, device=dev)
        k_bf = torch.empty((Nkv, D), dtype=torch.bfloat16, device=dev)
    k_mean = None
    qks = float(torch.tensor(_qk_scale(D), dtype=torch.float32))
    # k (smoothed, with the backward's bf16 image when asked), then v with its P.V operand image
    # (two launches: one launch alternating k and v workgroups measured 105 against 31 + 45 us at
    # config 3, HISTORY.md round 5)
    if smooth:
        k_mean = torch.empty((B, Hkv, 1, D), dtype=torch.float16, device=dev)
        if FUSED_K_SMOOTH:   # k-mean and the smoothed quantiser in one launch (bit-identical)
            _lib.call("qattn_int8_quant_k_smooth", _lib.ptr(k), _lib.ptr(k_mean), _lib.ptr(k_i8),
                      _lib.ptr(sk), _lib.ptr(k_bf), B * Hkv, Sk, D, st)
        else:
            _lib.call("qattn_kmean", _lib.ptr(k), _lib.ptr(k_mean), B * Hkv, Sk, D, st)
            _lib.call("qattn_int8_quant_img", _lib.ptr(k), _lib.ptr(k_i8), _lib.ptr(sk), None,
                      _lib.ptr(k_bf), _lib.ptr(k_mean), Nkv, Sk, D, st)
    else:
        _lib.call("qattn_int8_quant_img", _lib.ptr(k), _lib.ptr(k_i8), _lib.ptr(sk), None, _lib.ptr(k_bf),
                  None, Nkv, Sk, D, st)
    _lib.call("qattn_int8_quant_vt", _lib.ptr(v), _lib.ptr(v_i8), _lib.ptr(sv), _lib.ptr(vt), Nkv, D, st)
    # q is quantised inside the attention kernel (q_i8, sq and the bf16 image written there)
    _lib.call("qattn_int8_attn_fwd_qf", _lib.ptr(q), _lib.ptr(q_i8), _lib.ptr(sq), _lib.ptr(q_bf),
              _lib.ptr(k_i8), _lib.ptr(sk), _lib.ptr(vt), _lib.ptr(sv), _lib.ptr(O), _lib.ptr(lse),
              B * H, S, Sk, H // Hkv, int(bool(causal)), D, qks, st)
    # k_i8T is returned as the [D, N] view of the row-major [N, D] tensor (same values/shape as
    # int8:165, zero-copy).
    return O, lse, q_i8, k_i8.t(), v_i8, sq, sk, sv, k_mean, q_bf, k_bf


# Largest dS workspace (bytes) the backward allocates to skip the dQ pass's recomputation of S,
# dP, P and dS (qattn_int8_attn_bwd_ws); larger problems recompute (qattn_int8_attn_bwd_ex).  The
# results are bit-identical either way.  1 B per score + 4 B per 32x32 tile: 2.2 GB at (4,32,4096).
# None: the library's shared cap (qattn_bwd_ws_cap: QATTN_BWD_WS_MAX, else 16 GiB; an allocation that
# fails falls back to recomputation), the same rule as the bf16 backward and the C++ operators.
WS_MAX_BYTES = None
# Key/value heads per chunk of the record backward (qattn_int8_attn_bwd_wsc): dK+dV then dQ per
# chunk, one chunk-sized workspace re-used by every chunk; 0: one pass over all heads; unset: auto
# (non-causal: chunks of >= 512 dK+dV workgroups, two per CU, measured 2-4 % faster than one pass
# at config 3 with a quarter of the workspace; causal: one pass, since a causal chunk's uneven
# workgroups leave a longer tail per launch, measured 10-170 % slower in chunks).
WS_CHUNK = os.environ.get("QATTN_BWD_WS_CHUNK")


def _ws_chunk(chunk, causal, bkv, sk):
    if chunk is None and WS_CHUNK is not None:
        chunk = int(WS_CHUNK)
    if chunk is None:
        chunk = 0 if causal else -(-512 // max(1, sk // 256))
    return bkv if chunk <= 0 else min(int(chunk), bkv)


def _int8_backward(dO, q_i8, sq, k_i8T, sk, v_i8, sv, O, lse, q_bf=None, k_bf=None, causal=False,
                   kv_heads=None, use_ws=None, ws_chunk=None, kv_len=None, ws_poison=None):
    """Corrected int8 backward; q_bf / k_bf: bf16 images from the forward (computed here if None).

    kv_heads: key/value heads (default: those of O); their token count follows from k_i8T.
    use_ws: dQ from the dS workspace (True), by recomputation (False), or by size (None).
    ws_chunk: key/value heads per workspace chunk (None: WS_CHUNK / auto; 0 = all heads at once).
    kv_len: key/value tokens, needed only to shape the (empty) gradients of an empty batch.
    ws_poison: a byte to fill the dS workspace with before the launch (protocol checks: every record
    the dQ pass reads must have been written by the dK+dV pass, so results cannot depend on it)."""
    O = O.to(torch.float16).contiguous()
    dO = dO.to(torch.float16).contiguous()
    _lib.require_gpu(dO, O, q_i8)
    B, H, S, D = O.shape
    Hkv = H if kv_heads is None else int(kv_heads)
    Nkv = k_i8T.shape[1]
    if B * H * S == 0 or Nkv == 0:
        # nothing attends: zero gradients (an empty batch gives empty ones)
        Sk = Nkv // (B * Hkv) if B * Hkv else int(kv_len if kv_len is not None else S)
        z = dict(dtype=torch.float16, device=O.device)
        return (torch.zeros((B, H, S, D), **z), torch.zeros((B, Hkv, Sk, D), **z),
                torch.zeros((B, Hkv, Sk, D), **z))
    if H % Hkv != 0 or Nkv % (B * Hkv) != 0:
        raise _lib.QAttnError("qattn int8 backward: inconsistent key/value heads")
    Sk = Nkv // (B * Hkv)
    N = B * H * S
    dev = O.device
    st = _lib.stream_of(O)
    k_i8 = k_i8T.t().contiguous()  # [N, D] (a no-op for the view our forward returns)
    q_i8 = q_i8.contiguous()
    v_i8 = v_i8.contiguous()
    dO_i8 = torch.empty((N, D), dtype=torch.int8, device=dev)
    sdO = torch.empty((N // BQ,), dtype=torch.float16, device=dev)
    LD = torch.empty((N, 2), dtype=torch.float32, device=dev)  # {lse, D} per row
    dO_bf = torch.empty((N, D), dtype=torch.bfloat16, device=dev)
    lse = lse.to(torch.float16).contiguous()
    _lib.call("qattn_int8_bwd_prep", _lib.ptr(dO), _lib.ptr(O), _lib.ptr(lse), _lib.ptr(dO_i8),
              _lib.ptr(sdO), _lib.ptr(LD), _lib.ptr(dO_bf), B * H, S, D, st)
    # exact bf16 images of the int8 operands read column-wise by the accumulating products
    if q_bf is None:
        q_bf = torch.empty((N, D), dtype=torch.bfloat16, device=dev)
        _lib.call("qattn_i8_to_bf16", _lib.ptr(q_i8), _lib.ptr(q_bf), N * D, st)
    if k_bf is None:
        k_bf = torch.empty((Nkv, D), dtype=torch.bfloat16, device=dev)
        _lib.call("qattn_i8_to_bf16", _lib.ptr(k_i8), _lib.ptr(k_bf), Nkv * D, st)
    dq = torch.empty((B, H, S, D), dtype=torch.float16, device=dev)
    dk = torch.empty((B, Hkv, Sk, D), dtype=torch.float16, device=dev)
    dv = torch.empty((B, Hkv, Sk, D), dtype=torch.float16, device=dev)
    qks = float(torch.tensor(_qk_scale(D), dtype=torch.float32))
    sms = float(torch.tensor(1.0 / math.sqrt(D), dtype=torch.float32))
    # (contiguous copies bound to names: they must outlive the launches that read them)
    sq, sk, sv = sq.contiguous(), sk.contiguous(), sv.contiguous()
    common = (_lib.ptr(dO_i8), _lib.ptr(sdO), _lib.ptr(q_i8), _lib.ptr(sq), _lib.ptr(k_i8),
              _lib.ptr(sk), _lib.ptr(v_i8), _lib.ptr(sv), _lib.ptr(LD),
              _lib.ptr(q_bf), _lib.ptr(k_bf), _lib.ptr(dO_bf), _lib.ptr(dq), _lib.ptr(dk), _lib.ptr(dv))
    shape = (B * H, S, Sk, H // Hkv, int(bool(causal)), D, qks, sms, st)
    chunk = _ws_chunk(ws_chunk, causal, B * Hkv, Sk)
    ws_bytes = _lib.load().qattn_int8_bwd_ws_bytes(chunk * (H // Hkv), S, Sk)
    # the records of one key/value head (its H / Hkv query heads) are addressed with 32-bit offsets
    region_ok = (H // Hkv) * (S // 32) * (Sk // 32) * 1024 < (1 << 31)
    if use_ws is None:
        cap = _lib.load().qattn_bwd_ws_cap() if WS_MAX_BYTES is None else WS_MAX_BYTES
        use_ws = 0 <= ws_bytes <= cap and region_ok
    elif use_ws and not (region_ok and ws_bytes >= 0):
        raise _lib.QAttnError("qattn int8 backward: dS workspace region exceeds 2 GiB per key/value "
                              "head; use the recomputing backward (use_ws=False)")
    ws = None
    if use_ws and ws_bytes > 0:
        # (None when there is no room: recompute dS in the dQ pass, same results)
        ws = _lib.try_workspace(ws_bytes, dev)
        if ws is not None and ws_poison is not None:
            ws.fill_(int(ws_poison) & 0xFF)
    if ws is not None and chunk < B * Hkv:
        _lib.call("qattn_int8_attn_bwd_wsc", *common, _lib.ptr(ws), chunk, *shape)
    elif ws is not None:
        _lib.call("qattn_int8_attn_bwd_ws", *common, _lib.ptr(ws), *shape)
    else:
        _lib.call("qattn_int8_attn_bwd_ex", *common, *shape)
    return dq, dk, dv


def helion_atten_int8_hl_dot_fwd(
    q_fp16_input: torch.Tensor,
    k_fp16_input: torch.Tensor,
    v_fp16_input: torch.Tensor,
    causal: bool = False,
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor,
           torch.Tensor, torch.Tensor, torch.Tensor, int, int]:
    """int8 forward (int8:101-262): returns (O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, Bq, Bkv).
    ``causal`` (and GQA / Sq != Sk shapes) are extensions, see the module docstring."""
    O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, _, _, _ = _int8_forward(
        q_fp16_input, k_fp16_input, v_fp16_input, smooth=False, causal=causal)
    return O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, BQ, BKV


def helion_atten_int8_hl_dot_bwd(
    dO_input_fp16: torch.Tensor,
    q_bh_int8: torch.Tensor,
    sq_bh_fp16: torch.Tensor,
    k_bh_int8_T: torch.Tensor,
    k_mean_bh_fp16: torch.Tensor,
    sk_bh_fp16: torch.Tensor,
    v_bh_int8: torch.Tensor,
    sv_bh_fp16: torch.Tensor,
    O_input_fp16: torch.Tensor,
    lse_input_fp16: torch.Tensor,
    Bq: int,
    Bkv: int,
    causal: bool = False,
    kv_heads: int | None = None,
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Corrected int8 backward (int8:268-432): returns fp16 (dq, dk, dv) [B,H,S,D].

    k_mean is accepted for signature compatibility; its term multiplies rowsum(dS) = 0 and is
    dropped (build contract).  Its head count (``[B, Hkv, 1, D]``) gives the key/value heads of a
    grouped-query call unless ``kv_heads`` is passed.
    """
    if Bq != BQ or Bkv != BKV:
        raise _lib.QAttnError("qattn int8 backward is built for Bq = Bkv = 32")
    if kv_heads is None and k_mean_bh_fp16 is not None and k_mean_bh_fp16.dim() == 4:
        kv_heads = k_mean_bh_fp16.shape[1]
    return _int8_backward(dO_input_fp16, q_bh_int8, sq_bh_fp16, k_bh_int8_T, sk_bh_fp16, v_bh_int8,
                          sv_bh_fp16, O_input_fp16, lse_input_fp16, causal=causal,
                          kv_heads=kv_heads)


# bf16 images of q_i8 / k_i8 written by the forward's quantiser pass, handed from forward() to
# setup_context() (a new-style forward has no ctx).  Keyed by id(q_i8); the entry is dropped with
# q_i8, so a forward whose setup_context never runs (a direct Function.forward call) leaks nothing.
_IMAGES: dict = {}


def _stash_images(q_i8, q_bf, k_bf):
    key = id(q_i8)
    _IMAGES[key] = (weakref.ref(q_i8), q_bf, k_bf)
    weakref.finalize(q_i8, _IMAGES.pop, key, None)


def _take_images(q_i8):
    e = _IMAGES.pop(id(q_i8), None)
    if e is None or e[0]() is not q_i8:
        return None, None
    return e[1], e[2]


class SageAttention3_Int8_autograd_function(Function):
    """int8:20-95, new-style like the reference: ``forward(q, k, v)`` (no ctx) + ``setup_context`` +
    ``backward``.  forward returns the 11-tuple (O, lse, k_mean, q_i8, k_i8T, v_i8, sq, sk, sv, Bq,
    Bkv); ``forward(q, k, v, causal)`` is an extension."""

    @staticmethod
    def forward(q_fp16, k_fp16, v_fp16, causal=False):
        # The bf16 images of q_i8 / k_i8 the backward reads come out of the same quantiser pass when
        # a gradient will be taken (handed to setup_context, not returned: the 11-tuple is the
        # reference's).
        images = any(t.requires_grad for t in (q_fp16, k_fp16, v_fp16))
        O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, k_mean, q_bf, k_bf = _int8_forward(
            q_fp16, k_fp16, v_fp16, smooth=True, images=images, causal=bool(causal))
        if images:
            _stash_images(q_i8, q_bf, k_bf)
        return O, lse, k_mean, q_i8, k_i8T, v_i8, sq, sk, sv, BQ, BKV

    @staticmethod
    def setup_context(ctx, inputs, output):
        k_fp16 = inputs[1]
        causal = bool(inputs[3]) if len(inputs) > 3 else False
        O, lse, k_mean, q_i8, k_i8T, v_i8, sq, sk, sv, Bq, Bkv = output
        ctx.mark_non_differentiable(lse, k_mean, sq, sk, sv)  # int8:52-56
        ctx.save_for_backward(O, lse, k_mean, q_i8, k_i8T, v_i8, sq, sk, sv)  # int8:58-64
        ctx.args = (Bq, Bkv)
        ctx.images = _take_images(q_i8)
        ctx.opts = (causal, k_fp16.shape[1], len(inputs) - 3, k_fp16.shape[2])

    @staticmethod
    def backward(ctx, dO_fp16, _lse, _k_mean, _q_i8, _k_i8T, _v_i8, _sq, _sk, _sv, _Bq, _Bkv):
        # plain tensors under torch.func transforms (_lib.plain); a no-op otherwise
        O, lse, k_mean, q_i8, k_i8T, v_i8, sq, sk, sv = (_lib.plain(t) for t in ctx.saved_tensors)
        Bq, Bkv = ctx.args
        if Bq != BQ or Bkv != BKV:
            raise _lib.QAttnError("qattn int8 backward is built for Bq = Bkv = 32")
        q_bf, k_bf = ctx.images   # (None, None): the backward rebuilds them from q_i8 / k_i8
        ctx.images = None
        causal, kv_heads, nopts, kv_len = ctx.opts
        with torch._C._DisableFuncTorch():
            dO_fp16 = torch.zeros_like(O) if dO_fp16 is None else _lib.plain(dO_fp16)
            dq, dk, dv = _int8_backward(dO_fp16, q_i8, sq, k_i8T, sk, v_i8, sv, O, lse, q_bf, k_bf,
                                        causal=causal, kv_heads=kv_heads, kv_len=kv_len)
        return (dq, dk, dv) + (None,) * nopts


def sage_attention_3_int8(q_fp16, k_fp16, v_fp16, causal: bool = False):
    """int8:434-451: SageAttention3 int8 attention with autograd; returns O fp16.
    ``causal`` (and GQA / Sq != Sk shapes) are extensions, see the module docstring."""
    if causal:
        return SageAttention3_Int8_autograd_function.apply(q_fp16, k_fp16, v_fp16, True)[0]
    return SageAttention3_Int8_autograd_function.apply(q_fp16, k_fp16, v_fp16)[0]
