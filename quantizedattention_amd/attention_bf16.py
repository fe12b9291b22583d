"""Drop-in for ``attention_bf16`` of selau642/QuantizedAttention, backed by gfx950 HIP kernels.

Public names (same signatures, outputs and assertion messages):
  FlashAttention_2_BF16_autograd_function   attention_bf16.py:16-85
  flash_atten_2_bf16                        attention_bf16.py:87-105
  helion_atten_bf16_fwd_training            attention_bf16.py:107-296
  helion_flash_atten_2_algo_4_bwd           attention_bf16.py:299-448
  baseline_pytorch_attention                attention_bf16.py:450-478

Forward: bf16 FlashAttention with the reference's "multiple-max" beta rule emulated at its pinned
k-tile of 16 (bf16:736).  Extension: k, v may have fewer heads than q (grouped-query
attention, query head h reads key/value head h // (Hq / Hkv)); dk, dv then sum over each group.  Backward: FA2 algorithm 4 with the build-contract fixes of SURVEY F3
(dS = P*(dP-D), sm_scale, deterministic dQ).
"""
from __future__ import annotations

import math
import os
from typing import Tuple

import torch
from torch.autograd import Function

from . import _lib
from ._baseline import baseline_pytorch_attention  # noqa: F401

__all__ = [
    "FlashAttention_2_BF16_autograd_function", "flash_atten_2_bf16",
    "helion_atten_bf16_fwd_training", "helion_flash_atten_2_algo_4_bwd",
    "baseline_pytorch_attention",
]

KT = 16  # k-tile of the beta rule (reference tuned config, bf16:736)


def _f32(x: float) -> float:
    return float(torch.tensor(x, dtype=torch.float32))


def _check(q, k, v):
    batch, head, q_tokens, q_head_dim = q.shape
    k_batch, k_head, k_tokens, k_head_dim = k.shape
    v_batch, v_head, v_tokens, v_head_dim = v.shape
    assert k_tokens == v_tokens, "input k_tokens must match v_tokens"  # bf16:154
    assert q_head_dim == k.size(-1) == v.size(-1), \
        "all head dimensions must match for q, k, v tensors"  # bf16:155
    if not (q.shape[0] == k.shape[0] and k.shape[:2] == v.shape[:2] and head % k.shape[1] == 0):
        raise _lib.QAttnError("qattn bf16: batch must match and q heads must be a multiple of k/v heads")
    if q_tokens % 32 or k_tokens % 32:
        raise _lib.QAttnError("qattn bf16: token counts must be multiples of 32")
    if q_head_dim not in (64, 128):
        raise _lib.QAttnError("qattn bf16: head_dim must be 64 or 128")


def helion_atten_bf16_fwd_training(
    q_fp16_input: torch.Tensor,
    k_fp16_input: torch.Tensor,
    v_bf16_input: torch.Tensor,
    causal: bool,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """bf16:111-296 -> (O fp32 [B,H,S,D], lse fp32 [B*H, S], base-2 units)."""
    _check(q_fp16_input, k_fp16_input, v_bf16_input)
    _lib.require_gpu(q_fp16_input, k_fp16_input, v_bf16_input)
    q = q_fp16_input.to(torch.float16).contiguous()
    k = k_fp16_input.to(torch.float16).contiguous()
    v = v_bf16_input.to(torch.bfloat16).contiguous()
    B, H, S, D = q.shape
    Sk = k.shape[2]
    O = torch.empty((B, H, S, D), dtype=torch.float32, device=q.device)
    lse = torch.empty((B * H, S), dtype=torch.float32, device=q.device)
    qks = _f32(1.0 / math.sqrt(D) * 1.44269504)
    # grouped-query attention (SURVEY §8f N2 extension): query head h reads k/v head h // (H / Hkv);
    # causal: the per-head V suffix sums stand in for the fully masked key tiles (include/qattn.h);
    # without room for them the kernel runs the whole masked tile loop (same results)
    ws = None
    if causal and Sk > 0:
        ws = _lib.try_workspace(_lib.load().qattn_bf16_fwd_ws_bytes(B * k.shape[1], Sk, D), q.device)
    _lib.call("qattn_bf16_fwd_ws_ex", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(O), _lib.ptr(lse),
              B * H, S, Sk, H // k.shape[1], int(bool(causal)), D, qks, _lib.ptr(ws), _lib.stream_of(q))
    return O, lse


def helion_flash_atten_2_algo_4_bwd(
    q_input: torch.Tensor,
    k_input: torch.Tensor,
    v_input: torch.Tensor,
    O_input: torch.Tensor,
    lse_input: torch.Tensor,
    causal: bool,
    dO_input: torch.Tensor,
):
    """bf16:309-448 (corrected) -> fp32 (dq, dk, dv)."""
    _check(q_input, k_input, v_input)
    _lib.require_gpu(q_input, k_input, v_input, O_input, lse_input, dO_input)
    q = q_input.to(torch.float16).contiguous()
    k = k_input.to(torch.float16).contiguous()
    v = v_input.to(torch.bfloat16).contiguous()
    O = O_input.to(torch.float32).contiguous()
    dO = dO_input.to(torch.float32).contiguous()
    lse = lse_input.to(torch.float32).contiguous()
    B, H, S, D = q.shape
    Sk = k.shape[2]
    dev = q.device
    st = _lib.stream_of(q)
    dO_bf = torch.empty((B, H, S, D), dtype=torch.bfloat16, device=dev)
    LD = torch.empty((B * H, S, 2), dtype=torch.float32, device=dev)
    _lib.call("qattn_bf16_bwd_prep", _lib.ptr(dO), _lib.ptr(O), _lib.ptr(lse), _lib.ptr(dO_bf),
              _lib.ptr(LD), B * H, S, D, st)
    q_bf = torch.empty(q.shape, dtype=torch.bfloat16, device=dev)
    k_bf = torch.empty(k.shape, dtype=torch.bfloat16, device=dev)
    _lib.call("qattn_f16_to_bf16", _lib.ptr(q), _lib.ptr(q_bf), q.numel(), st)
    _lib.call("qattn_f16_to_bf16", _lib.ptr(k), _lib.ptr(k_bf), k.numel(), st)
    dq = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    Hkv = k.shape[1]
    dk = torch.empty((B, Hkv, Sk, D), dtype=torch.float32, device=dev)
    dv = torch.empty((B, Hkv, Sk, D), dtype=torch.float32, device=dev)
    qks = _f32(1.0 / math.sqrt(D) * 1.44269504)
    sms = _f32(1.0 / math.sqrt(D))
    args = (_lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(dO_bf), _lib.ptr(LD), _lib.ptr(q_bf),
            _lib.ptr(k_bf), _lib.ptr(dq), _lib.ptr(dk), _lib.ptr(dv),
            B * H, S, Sk, H // Hkv, int(bool(causal)), D, qks, sms)
    entry = _BWD_ENTRY
    if entry == "auto":
        entry = "ws" if causal else "qattn_bf16_bwd_ex"
    ws = None
    if entry == "ws":
        ws_bytes = _lib.load().qattn_bf16_bwd_ws_bytes(B * H, S, Sk)
        cap = _lib.load().qattn_bwd_ws_cap() if WS_MAX_BYTES is None else WS_MAX_BYTES
        if 0 < ws_bytes <= cap:
            # (None when there is no room for the dS records: recompute dS in the dQ pass, same
            # results)
            ws = _lib.try_workspace(ws_bytes, dev)
    if ws is not None:
        _lib.call("qattn_bf16_bwd_ws_ex", *args, _lib.ptr(ws), st)
    else:
        _lib.call("qattn_bf16_bwd_ex" if entry == "ws" else entry, *args, st)
    return dq, dk, dv


# "auto" (default): causal -> "ws", else "qattn_bf16_bwd_ex".  "qattn_bf16_bwd_ex": fused dK+dV, dQ
# recomputing S and dP; "ws": the fused kernel also stores bf16 dS records (2 B per score, up to
# QATTN_BWD_WS_MAX bytes) and dQ reads them -- non-causal at config 3 the record traffic costs what
# the dQ pass saves, causal it is 7 % faster; "qattn_bf16_bwd_split_ex": separate dV
# and dK kernels.  All give bit-identical gradients.  QATTN_BF16_BWD_WS=1 / 0 forces ws on / off.
_BWD_ENTRY = {"1": "ws", "0": "qattn_bf16_bwd_ex"}.get(os.environ.get("QATTN_BF16_BWD_WS", ""), "auto")
# None: the library's shared cap (qattn_bwd_ws_cap), as the int8 backward and the C++ operators
WS_MAX_BYTES = None


class FlashAttention_2_BF16_autograd_function(Function):
    """bf16:16-85: forward in bf16 (returns O fp32, lse fp32), backward in fp32-accumulated MFMA."""

    @staticmethod
    def forward(q_fp16, k_fp16, v_bf16, causal):
        return helion_atten_bf16_fwd_training(q_fp16, k_fp16, v_bf16, causal)

    @staticmethod
    def setup_context(ctx, inputs, output):
        q_fp16, k_fp16, v_bf16, causal = inputs
        O_fp32, lse_fp32 = output
        ctx.mark_non_differentiable(lse_fp32)  # bf16:55
        ctx.save_for_backward(q_fp16, k_fp16, v_bf16, O_fp32, lse_fp32)  # bf16:56
        ctx.args = causal

    @staticmethod
    def backward(ctx, dO, _lse):
        # plain tensors under torch.func transforms (_lib.plain); a no-op otherwise
        q_fp16, k_fp16, v_bf16, O_fp32, lse_fp32 = (_lib.plain(t) for t in ctx.saved_tensors)
        causal = ctx.args
        with torch._C._DisableFuncTorch():
            dO = torch.zeros_like(O_fp32) if dO is None else _lib.plain(dO)
            dq, dk, dv = helion_flash_atten_2_algo_4_bwd(q_fp16, k_fp16, v_bf16, O_fp32, lse_fp32,
                                                         causal, dO)
        return dq, dk, dv, None  # bf16:85


def flash_atten_2_bf16(q_fp16, k_fp16, v_bf16, causal):
    """bf16:87-105: returns O fp32."""
    o_fp32, _lse_fp32 = FlashAttention_2_BF16_autograd_function.apply(q_fp16, k_fp16, v_bf16, causal)
    return o_fp32
