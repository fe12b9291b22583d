"""The ``qattn::`` dispatcher operators ("C++ op layer").

The operators are defined and implemented in C++ (``csrc/torch/qattn_ops.cpp`` ->
``libqattn_torch.so``: ``TORCH_LIBRARY(qattn)`` schemas, CUDA-key kernels that allocate the outputs,
enter a HIP device guard and enqueue the C-ABI kernels of ``include/qattn.h`` on torch's current
stream).  This module loads that library and adds what belongs to the Python side of an operator:
its fake (meta) implementation, for graph capture (``torch.compile``, ``torch.export``, FX), and
the autograd rules of ``int8_fwd`` and ``bf16_fwd`` (their backward operators).

    torch.ops.qattn.int8_quant(x, block) -> (idx, scale)
    torch.ops.qattn.int8_fwd(q, k, v, smooth, causal) -> (O, lse, q_i8, k_i8, v_i8, sq, sk, sv)
    torch.ops.qattn.int8_bwd(dO, q_i8, sq, k_i8, sk, v_i8, sv, O, lse, causal, kv_heads)
        -> (dq, dk, dv)
    torch.ops.qattn.bf16_fwd(q, k, v, causal) -> (O, lse)
    torch.ops.qattn.bf16_bwd(q, k, v, O, lse, causal, dO) -> (dq, dk, dv)
    torch.ops.qattn.jvp_fwd(q, k, v, tq, tk, tv) -> (O, tO, lse)
    torch.ops.qattn.mxfp4_fwd(q, k, v) -> O

Shapes follow the drop-in functions (attention_int8.py:259-262 for the int8 outputs) except that
k_i8 is returned row-major [B*Hkv*Sk, D] (the drop-in's k_i8T is its transposed view: an operator
output may not be a view).  There is no CPU kernel, as for the drop-in functions: a CPU tensor
raises NotImplementedError from the dispatcher.  The Python wrappers below only forward to
``torch.ops.qattn`` (the names existing callers import).
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["int8_quant", "int8_fwd", "int8_bwd", "bf16_fwd", "bf16_bwd", "jvp_fwd", "mxfp4_fwd"]

_lib.load_ops()
_ops = torch.ops.qattn


# ---------------------------------------------------------------------------- fake kernels
@torch.library.register_fake("qattn::int8_quant")
def _(x, block):
    return (x.new_empty(x.shape, dtype=torch.int8),
            x.new_empty((*x.shape[:-2], x.shape[-2] // 32), dtype=torch.float16))


@torch.library.register_fake("qattn::int8_fwd")
def _(q, k, v, smooth, causal):
    B, H, S, D = q.shape
    Nq, Nkv = B * H * S, k.shape[0] * k.shape[1] * k.shape[2]
    e = lambda *s, dt: q.new_empty(s, dtype=dt)  # noqa: E731
    return (e(B, H, S, D, dt=torch.float16), e(Nq, dt=torch.float16), e(Nq, D, dt=torch.int8),
            e(Nkv, D, dt=torch.int8), e(Nkv, D, dt=torch.int8), e(Nq // 32, dt=torch.float16),
            e(Nkv // 32, dt=torch.float16), e(Nkv // 32, dt=torch.float16))


@torch.library.register_fake("qattn::int8_bwd")
def _(dO, q_i8, sq, k_i8, sk, v_i8, sv, O, lse, causal, kv_heads):
    B, H, S, D = O.shape
    Sk = k_i8.shape[0] // (B * kv_heads)
    return (O.new_empty((B, H, S, D), dtype=torch.float16),
            O.new_empty((B, kv_heads, Sk, D), dtype=torch.float16),
            O.new_empty((B, kv_heads, Sk, D), dtype=torch.float16))


@torch.library.register_fake("qattn::bf16_fwd")
def _(q, k, v, causal):
    B, H, S, D = q.shape
    return (q.new_empty((B, H, S, D), dtype=torch.float32),
            q.new_empty((B * H, S), dtype=torch.float32))


@torch.library.register_fake("qattn::bf16_bwd")
def _(q, k, v, O, lse, causal, dO):
    return (q.new_empty(q.shape, dtype=torch.float32), k.new_empty(k.shape, dtype=torch.float32),
            v.new_empty(v.shape, dtype=torch.float32))


@torch.library.register_fake("qattn::jvp_fwd")
def _(q, k, v, tq, tk, tv):
    B, H, S, D = q.shape
    return (q.new_empty((B, H, S, D), dtype=torch.float32),
            q.new_empty((B, H, S, D), dtype=torch.float32),
            q.new_empty((B * H, S), dtype=torch.float32))


@torch.library.register_fake("qattn::mxfp4_fwd")
def _(q, k, v):
    return q.new_empty(q.shape, dtype=torch.float16)


# ---------------------------------------------------------------------------- autograd rules
def _int8_setup(ctx, inputs, output):
    q, k, v, smooth, causal = inputs[:5]
    ctx.n_inputs = len(inputs)
    O, lse, q_i8, k_i8, v_i8, sq, sk, sv = output
    ctx.save_for_backward(O, lse, q_i8, k_i8, v_i8, sq, sk, sv)
    ctx.causal, ctx.kv_heads = causal, k.shape[1]
    ctx.dtypes = (q.dtype, k.dtype, v.dtype)
    ctx.kv_shape = k.shape


def _int8_backward_rule(ctx, dO, *_unused):
    # gradient of O only (the quantised outputs are not differentiable, int8:52-56); k smoothing
    # adds no gradient (softmax-invariant), so the same backward serves smooth and plain forwards
    O, lse, q_i8, k_i8, v_i8, sq, sk, sv = ctx.saved_tensors
    rest = (None,) * (ctx.n_inputs - 3)   # smooth, causal
    if dO is None:
        return (None, None, None) + rest
    qd, kd, vd = ctx.dtypes
    if O.numel() == 0 or k_i8.numel() == 0:   # nothing attends (an empty batch): zero gradients
        z = dict(device=O.device)
        return (torch.zeros(O.shape, dtype=qd, **z), torch.zeros(ctx.kv_shape, dtype=kd, **z),
                torch.zeros(ctx.kv_shape, dtype=vd, **z)) + rest
    dq, dk, dv = _ops.int8_bwd(dO.to(torch.float16), q_i8, sq, k_i8, sk, v_i8, sv, O, lse, ctx.causal,
                               ctx.kv_heads)
    return (dq.to(qd), dk.to(kd), dv.to(vd)) + rest


torch.library.register_autograd("qattn::int8_fwd", _int8_backward_rule, setup_context=_int8_setup)


def _bf16_setup(ctx, inputs, output):
    q, k, v, causal = inputs
    O, lse = output
    ctx.save_for_backward(q, k, v, O, lse)
    ctx.causal = causal


def _bf16_backward_rule(ctx, dO, _dlse):
    q, k, v, O, lse = ctx.saved_tensors
    if dO is None:
        return None, None, None, None
    dq, dk, dv = _ops.bf16_bwd(q, k, v, O, lse, ctx.causal, dO)
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), None


torch.library.register_autograd("qattn::bf16_fwd", _bf16_backward_rule, setup_context=_bf16_setup)


# ---------------------------------------------------------------------------- Python names
def int8_quant(x, block):
    """Per-32-token block quantiser (attention_int8.py:178-186): x fp16 [..., S, D] ->
    (idx int8 [..., S, D], scale fp16 [..., S/32]); s = f16(amax/127), idx = trunc(f16(x/s))."""
    return _ops.int8_quant(x, block)


def int8_fwd(q, k, v, smooth, causal):
    """SageAttention-3 int8 forward (attention_int8.py:97-262, per (batch, head)); the same kernels
    as ``sage_attention_3_int8``."""
    return _ops.int8_fwd(q, k, v, smooth, causal)


def int8_bwd(dO, q_i8, sq, k_i8, sk, v_i8, sv, O, lse, causal, kv_heads):
    """Corrected int8 backward (attention_int8.py:264-432); k_i8 row-major."""
    return _ops.int8_bwd(dO, q_i8, sq, k_i8, sk, v_i8, sv, O, lse, causal, kv_heads)


def bf16_fwd(q, k, v, causal):
    """FA2 forward with the corrected beta rule (attention_bf16.py:107-296): (O fp32, lse fp32)."""
    return _ops.bf16_fwd(q, k, v, causal)


def bf16_bwd(q, k, v, O, lse, causal, dO):
    """FA2 algorithm-4 backward, corrected (attention_bf16.py:299-448): fp32 grads."""
    return _ops.bf16_bwd(q, k, v, O, lse, causal, dO)


def jvp_fwd(q, k, v, tq, tk, tv):
    """Attention with its forward-mode tangent (attention_jvp.py:24-195): (O, tO, lse) fp32."""
    return _ops.jvp_fwd(q, k, v, tq, tk, tv)


def mxfp4_fwd(q, k, v):
    """MX-FP4 inference forward, k smoothed: O fp16."""
    return _ops.mxfp4_fwd(q, k, v)
