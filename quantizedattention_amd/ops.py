"""torch.library operators over the HIP kernels ("C++ op layer": the ``qattn::`` schemas).

The drop-in modules (attention_int8 / attention_bf16 / attention_jvp / attention_mxfp4) call the
C-ABI library directly.  This module registers the same computations as dispatcher operators, so
that graph capture (``torch.compile``, ``torch.export``, FX tracing) sees one opaque node per
kernel sequence instead of breaking the graph at a ctypes call.  Each operator has a fake (meta)
implementation giving output shapes and dtypes without running anything; ``int8_fwd`` and
``bf16_fwd`` carry autograd rules (their backward operators), so compiled training steps
differentiate through them.

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
output may not be a view).  The implementations are CUDA-only: there is no CPU kernel, as for
the drop-in functions.
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from . import attention_bf16 as _bf16
from . import attention_int8 as _i8
from . import attention_jvp as _jvp
from . import attention_mxfp4 as _fp4

__all__ = ["int8_quant", "int8_fwd", "int8_bwd", "bf16_fwd", "bf16_bwd", "jvp_fwd", "mxfp4_fwd"]

_LIB = "qattn"


# ------------------------------------------------------------------------------------ int8
@torch.library.custom_op(f"{_LIB}::int8_quant", mutates_args=(), device_types="cuda")
def int8_quant(x: Tensor, block: int) -> Tuple[Tensor, Tensor]:
    """Per-32-token block quantiser (attention_int8.py:178-186): x fp16 [..., S, D] ->
    (idx int8 [..., S, D], scale fp16 [..., S/32]); s = f16(amax/127), idx = trunc(f16(x/s))."""
    if block != 32:
        raise ValueError("qattn::int8_quant supports block = 32 (the reference's Bq = Bkv)")
    if x.dim() < 2 or x.shape[-2] % 32 != 0 or x.shape[-1] not in (64, 128):
        raise ValueError("qattn::int8_quant needs x [..., S, D] with S % 32 == 0 and D in (64, 128)")
    from . import _lib
    _lib.require_gpu(x)
    xh = x.to(torch.float16).contiguous()
    rows, D = xh.numel() // x.shape[-1], x.shape[-1]
    idx = torch.empty(xh.shape, dtype=torch.int8, device=x.device)
    scale = torch.empty((*xh.shape[:-2], xh.shape[-2] // 32), dtype=torch.float16, device=x.device)
    _lib.call("qattn_int8_quant", _lib.ptr(xh), _lib.ptr(idx), _lib.ptr(scale), None, None, rows,
              xh.shape[-2], D, _lib.stream_of(xh))
    return idx, scale


@int8_quant.register_fake
def _(x, block):
    return (x.new_empty(x.shape, dtype=torch.int8),
            x.new_empty((*x.shape[:-2], x.shape[-2] // 32), dtype=torch.float16))


@torch.library.custom_op(f"{_LIB}::int8_fwd", mutates_args=(), device_types="cuda")
def int8_fwd(q: Tensor, k: Tensor, v: Tensor, smooth: bool, causal: bool
             ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """SageAttention-3 int8 forward (attention_int8.py:97-262, per (batch, head))."""
    O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, _, _, _ = _i8._int8_forward(q, k, v, smooth=smooth,
                                                                      causal=causal)
    return O, lse, q_i8, k_i8T.t().contiguous(), v_i8, sq, sk, sv


@int8_fwd.register_fake
def _(q, k, v, smooth, causal):
    B, H, S, D = q.shape
    Nq, Nkv = B * H * S, k.shape[0] * k.shape[1] * k.shape[2]
    e = lambda *s, dt: q.new_empty(s, dtype=dt)  # noqa: E731
    return (e(B, H, S, D, dt=torch.float16), e(Nq, dt=torch.float16), e(Nq, D, dt=torch.int8),
            e(Nkv, D, dt=torch.int8), e(Nkv, D, dt=torch.int8), e(Nq // 32, dt=torch.float16),
            e(Nkv // 32, dt=torch.float16), e(Nkv // 32, dt=torch.float16))


@torch.library.custom_op(f"{_LIB}::int8_bwd", mutates_args=(), device_types="cuda")
def int8_bwd(dO: Tensor, q_i8: Tensor, sq: Tensor, k_i8: Tensor, sk: Tensor, v_i8: Tensor,
             sv: Tensor, O: Tensor, lse: Tensor, causal: bool, kv_heads: int
             ) -> Tuple[Tensor, Tensor, Tensor]:
    """Corrected int8 backward (attention_int8.py:264-432); k_i8 row-major."""
    return _i8._int8_backward(dO, q_i8, sq, k_i8.t(), sk, v_i8, sv, O, lse, causal=causal,
                              kv_heads=kv_heads)


@int8_bwd.register_fake
def _(dO, q_i8, sq, k_i8, sk, v_i8, sv, O, lse, causal, kv_heads):
    B, H, S, D = O.shape
    Sk = k_i8.shape[0] // (B * kv_heads)
    return (O.new_empty((B, H, S, D), dtype=torch.float16),
            O.new_empty((B, kv_heads, Sk, D), dtype=torch.float16),
            O.new_empty((B, kv_heads, Sk, D), dtype=torch.float16))


def _int8_setup(ctx, inputs, output):
    q, k, v, smooth, causal = inputs
    O, lse, q_i8, k_i8, v_i8, sq, sk, sv = output
    ctx.save_for_backward(O, lse, q_i8, k_i8, v_i8, sq, sk, sv)
    ctx.causal, ctx.kv_heads = causal, k.shape[1]
    ctx.dtypes = (q.dtype, k.dtype, v.dtype)


def _int8_backward_rule(ctx, dO, *_unused):
    # gradient of O only (the quantised outputs are not differentiable, int8:52-56); k smoothing
    # adds no gradient (softmax-invariant), so the same backward serves smooth and plain forwards
    O, lse, q_i8, k_i8, v_i8, sq, sk, sv = ctx.saved_tensors
    if dO is None:
        return None, None, None, None, None
    dq, dk, dv = int8_bwd(dO.to(torch.float16), q_i8, sq, k_i8, sk, v_i8, sv, O, lse, ctx.causal,
                          ctx.kv_heads)
    qd, kd, vd = ctx.dtypes
    return dq.to(qd), dk.to(kd), dv.to(vd), None, None


int8_fwd.register_autograd(_int8_backward_rule, setup_context=_int8_setup)


# ------------------------------------------------------------------------------------ bf16
@torch.library.custom_op(f"{_LIB}::bf16_fwd", mutates_args=(), device_types="cuda")
def bf16_fwd(q: Tensor, k: Tensor, v: Tensor, causal: bool) -> Tuple[Tensor, Tensor]:
    """FA2 forward with the corrected beta rule (attention_bf16.py:107-296): (O fp32, lse fp32)."""
    return _bf16.helion_atten_bf16_fwd_training(q, k, v, causal)


@bf16_fwd.register_fake
def _(q, k, v, causal):
    B, H, S, D = q.shape
    return (q.new_empty((B, H, S, D), dtype=torch.float32),
            q.new_empty((B * H, S), dtype=torch.float32))


@torch.library.custom_op(f"{_LIB}::bf16_bwd", mutates_args=(), device_types="cuda")
def bf16_bwd(q: Tensor, k: Tensor, v: Tensor, O: Tensor, lse: Tensor, causal: bool, dO: Tensor
             ) -> Tuple[Tensor, Tensor, Tensor]:
    """FA2 algorithm-4 backward, corrected (attention_bf16.py:299-448): fp32 grads."""
    return _bf16.helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, causal, dO)


@bf16_bwd.register_fake
def _(q, k, v, O, lse, causal, dO):
    return (q.new_empty(q.shape, dtype=torch.float32), k.new_empty(k.shape, dtype=torch.float32),
            v.new_empty(v.shape, dtype=torch.float32))


def _bf16_setup(ctx, inputs, output):
    q, k, v, causal = inputs
    O, lse = output
    ctx.save_for_backward(q, k, v, O, lse)
    ctx.causal = causal


def _bf16_backward_rule(ctx, dO, _dlse):
    q, k, v, O, lse = ctx.saved_tensors
    if dO is None:
        return None, None, None, None
    dq, dk, dv = bf16_bwd(q, k, v, O, lse, ctx.causal, dO)
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), None


bf16_fwd.register_autograd(_bf16_backward_rule, setup_context=_bf16_setup)


# ------------------------------------------------------------------------------------- jvp
@torch.library.custom_op(f"{_LIB}::jvp_fwd", mutates_args=(), device_types="cuda")
def jvp_fwd(q: Tensor, k: Tensor, v: Tensor, tq: Tensor, tk: Tensor, tv: Tensor
            ) -> Tuple[Tensor, Tensor, Tensor]:
    """Attention with its forward-mode tangent (attention_jvp.py:24-195): (O, tO, lse) fp32."""
    return _jvp.helion_attention_jvp_forward_fp32(q, k, v, tq, tk, tv)


@jvp_fwd.register_fake
def _(q, k, v, tq, tk, tv):
    B, H, S, D = q.shape
    return (q.new_empty((B, H, S, D), dtype=torch.float32),
            q.new_empty((B, H, S, D), dtype=torch.float32),
            q.new_empty((B * H, S), dtype=torch.float32))


# ----------------------------------------------------------------------------------- mxfp4
@torch.library.custom_op(f"{_LIB}::mxfp4_fwd", mutates_args=(), device_types="cuda")
def mxfp4_fwd(q: Tensor, k: Tensor, v: Tensor) -> Tensor:
    """MX-FP4 inference forward, k smoothed: O fp16."""
    return _fp4.sage_attention_3_fp4(q, k, v)


@mxfp4_fwd.register_fake
def _(q, k, v):
    return q.new_empty(q.shape, dtype=torch.float16)
