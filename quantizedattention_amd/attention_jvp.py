"""Drop-in for ``attention_jvp`` of selau642/QuantizedAttention, backed by a gfx950 HIP kernel.

Public names:
  helion_attention_jvp_forward_fp32   attention_jvp.py:24-195  (q,k,v,tq,tk,tv) -> (O, tO, lse)
  baseline_pytorch_attention          attention_jvp.py:197-215 (non-causal)

The kernel multiplies bf16 operands on MFMA with fp32 accumulation and fp32 softmax state
(BASELINE.json config 5: "attention_jvp fwd ... in bf16").  fp32 inputs are accepted and rounded to
bf16 on entry; outputs are fp32 as in the reference.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from ._baseline import baseline_pytorch_attention as _baseline

__all__ = ["helion_attention_jvp_forward_fp32", "baseline_pytorch_attention"]


def baseline_pytorch_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """jvp:197-215 (non-causal eager fp32 attention)."""
    return _baseline(q, k, v, q.shape[-1], False)


def helion_attention_jvp_forward_fp32(q_fp32_input, k_fp32_input, v_fp32_input,
                                      tan_q_fp32_input, tan_k_fp32_input, tan_v_fp32_input):
    """jvp:33-195 -> (O fp32 [B,H,S,D], tO fp32 [B,H,S,D], lse fp32 [B*H, S])."""
    batch, head, q_tokens, q_head_dim = q_fp32_input.shape
    k_batch, k_head, k_tokens, k_head_dim = k_fp32_input.shape
    v_batch, v_head, v_tokens, v_head_dim = v_fp32_input.shape
    assert k_tokens == v_tokens, "input k_tokens must match v_tokens"  # jvp:78
    assert q_head_dim == k_fp32_input.size(-1) == v_fp32_input.size(-1), \
        "all head dimensions must match for q, k, v tensors"  # jvp:79
    ins = (q_fp32_input, k_fp32_input, v_fp32_input, tan_q_fp32_input, tan_k_fp32_input,
           tan_v_fp32_input)
    _lib.require_gpu(*ins)
    if q_tokens % 32 or k_tokens % 64:
        raise _lib.QAttnError("qattn jvp: q tokens must be a multiple of 32, k tokens of 64")
    if q_head_dim not in (64, 128):
        raise _lib.QAttnError("qattn jvp: head_dim must be 64 or 128")
    for t, ref in zip(ins[3:], ins[:3]):
        if t.shape != ref.shape:
            raise _lib.QAttnError("qattn jvp: tangents must have the primals' shapes")
    q, k, v, tq, tk, tv = (t.to(torch.bfloat16).contiguous() for t in ins)
    B, H, S, D = q.shape
    O = torch.empty((B, H, S, D), dtype=torch.float32, device=q.device)
    tO = torch.empty_like(O)
    lse = torch.empty((B * H, S), dtype=torch.float32, device=q.device)
    qks = float(torch.tensor(1.0 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
    sm = float(torch.tensor(1.0 / math.sqrt(D), dtype=torch.float32))
    _lib.call("qattn_jvp_fwd", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(tq), _lib.ptr(tk),
              _lib.ptr(tv), _lib.ptr(O), _lib.ptr(tO), _lib.ptr(lse), B * H, S, k_tokens, D, 0, qks,
              sm, _lib.stream_of(q))
    return O, tO, lse
