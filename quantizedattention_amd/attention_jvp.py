"""Drop-in for ``attention_jvp`` of selau642/QuantizedAttention, backed by a gfx950 HIP kernel.

Public names:
  helion_attention_jvp_forward_fp32   attention_jvp.py:24-195  (q,k,v,tq,tk,tv) -> (O, tO, lse)
  baseline_pytorch_attention          attention_jvp.py:197-215 (non-causal)
  AttentionJVP_autograd_function      SURVEY §8f N1: torch.autograd.Function whose ``jvp`` staticmethod
  attention_jvp                       routes forward-mode AD (torch.func.jvp, torch.autograd.forward_ad)
                                      to the kernel (README.md:19-22 of the reference promises this use)

Two numeric modes, chosen by the input dtype (outputs are fp32 in both, as in the reference):
  * bf16 inputs (BASELINE.json config 5): bf16 MFMA operands, fp32 accumulation and softmax state.
  * fp32 inputs: the fp32-accurate mode.  Every operand is split into two bf16 images (hi + lo,
    qattn_split_bf16) and each product runs as hi*hi + hi*lo + lo*hi on the MFMA (qattn_jvp_fwd_x3),
    which keeps ~16 significand bits per product (fp32 mode <= 1e-5 vs torch.func.jvp).
Other dtypes are cast to fp32 first.
"""
from __future__ import annotations

import math
import threading

import torch

from . import _lib
from ._baseline import baseline_pytorch_attention as _baseline

__all__ = ["helion_attention_jvp_forward_fp32", "baseline_pytorch_attention",
           "AttentionJVP_autograd_function", "attention_jvp"]


def baseline_pytorch_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """jvp:197-215 (non-causal eager fp32 attention)."""
    return _baseline(q, k, v, q.shape[-1], False)


def helion_attention_jvp_forward_fp32(q_fp32_input, k_fp32_input, v_fp32_input,
                                      tan_q_fp32_input, tan_k_fp32_input, tan_v_fp32_input):
    """jvp:33-195 -> (O fp32 [B,H,S,D], tO fp32 [B,H,S,D], lse fp32 [B*H, S])."""
    return _jvp(q_fp32_input, k_fp32_input, v_fp32_input,
                (tan_q_fp32_input, tan_k_fp32_input, tan_v_fp32_input))


# kernel launches by kind (tests count them: torch.func.jvp(attention_jvp, ...) is one launch)
LAUNCHES = {"primal": 0, "tangent": 0}


def _jvp(q_fp32_input, k_fp32_input, v_fp32_input, tangents, out_O=None):
    """The kernel call.  ``tangents`` None runs the primal-only kernel (qattn_jvp_primal_ex: O and
    lse, bit-identical to the tangent kernel's) and returns (O, None, lse).  ``out_O``: write O into
    this fp32 [B,H,S,D] contiguous tensor instead of a new one."""
    batch, head, q_tokens, q_head_dim = q_fp32_input.shape
    k_batch, k_head, k_tokens, k_head_dim = k_fp32_input.shape
    v_batch, v_head, v_tokens, v_head_dim = v_fp32_input.shape
    assert k_tokens == v_tokens, "input k_tokens must match v_tokens"  # jvp:78
    assert q_head_dim == k_fp32_input.size(-1) == v_fp32_input.size(-1), \
        "all head dimensions must match for q, k, v tensors"  # jvp:79
    prim = (q_fp32_input, k_fp32_input, v_fp32_input)
    ins = prim + (tuple(tangents) if tangents is not None else ())
    _lib.require_gpu(*ins)
    if q_tokens % 32 or k_tokens % 32:
        raise _lib.QAttnError("qattn jvp: q and k tokens must be multiples of 32")
    if q_head_dim not in (64, 128):
        raise _lib.QAttnError("qattn jvp: head_dim must be 64 or 128")
    for t, ref in zip(ins[3:], prim):
        if t.shape != ref.shape:
            raise _lib.QAttnError("qattn jvp: tangents must have the primals' shapes")
    B, H, S, D = q_fp32_input.shape
    # grouped-query attention (SURVEY §8f N2 extension): k, v may have fewer heads than q
    Hkv = k_head
    if k_batch != batch or v_batch != batch or v_head != Hkv or H % Hkv != 0:
        raise _lib.QAttnError("qattn jvp: k and v need q's batch and a head count dividing q's")
    group = H // Hkv
    dev = q_fp32_input.device
    if out_O is not None and (out_O.shape != (B, H, S, D) or out_O.dtype != torch.float32 or
                              not out_O.is_contiguous() or out_O.device != dev):
        raise _lib.QAttnError("qattn jvp: out_O must be a contiguous fp32 [B,H,S,D] tensor on q's device")
    O = out_O if out_O is not None else torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    LAUNCHES["primal" if tangents is None else "tangent"] += 1
    tO = torch.empty_like(O) if tangents is not None else None
    lse = torch.empty((B * H, S), dtype=torch.float32, device=dev)
    qks = float(torch.tensor(1.0 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
    sm = float(torch.tensor(1.0 / math.sqrt(D), dtype=torch.float32))
    st = _lib.stream_of(q_fp32_input)
    shape = (B * H, S, k_tokens, group, D, qks, sm, st)
    if all(t.dtype == torch.bfloat16 for t in ins):
        if k_tokens % 64:
            raise _lib.QAttnError("qattn jvp: k tokens must be a multiple of 64 for bf16 inputs")
        # keep the contiguous copies alive through the launch: a copy freed as soon as its address
        # is taken hands its block to the next input's copy (the caching allocator), and the
        # kernel would read the wrong tensor
        xs = [t.contiguous() for t in ins]
        ptrs = [_lib.ptr(t) for t in xs]
        if tangents is None:
            _lib.call("qattn_jvp_primal_ex", *ptrs, _lib.ptr(O), _lib.ptr(lse), *shape)
        else:
            _lib.call("qattn_jvp_fwd_ex", *ptrs, _lib.ptr(O), _lib.ptr(tO), _lib.ptr(lse), *shape)
        return O, tO, lse
    imgs = []
    for t in ins:
        x = t.to(torch.float32).contiguous()
        hi = torch.empty(x.shape, dtype=torch.bfloat16, device=dev)
        lo = torch.empty_like(hi)
        _lib.call("qattn_split_bf16", _lib.ptr(x), _lib.ptr(hi), _lib.ptr(lo), x.numel(), st)
        imgs += [hi, lo]
    if tangents is None:
        _lib.call("qattn_jvp_primal_x3_ex", *(_lib.ptr(t) for t in imgs), _lib.ptr(O), _lib.ptr(lse),
                  *shape)
    else:
        _lib.call("qattn_jvp_fwd_x3_ex", *(_lib.ptr(t) for t in imgs), _lib.ptr(O), _lib.ptr(tO),
                  _lib.ptr(lse), *shape)
    return O, tO, lse


_plain = _lib.plain

# Deferred forwards: when attention_jvp knows that the jvp rule will follow (a torch.func.jvp
# transform, or forward-mode dual inputs), the Function's forward returns an EMPTY O and the jvp rule
# fills it with the tangent kernel, which computes O and tO together: one launch per call.
_DEFER = threading.local()


def _key(q, k, v):
    return (q.data_ptr(), k.data_ptr(), v.data_ptr(), tuple(q.shape), tuple(k.shape))


def _jvp_follows(tensors) -> bool:
    """True when the Function's jvp rule will run right after its forward: the innermost functorch
    transform is torch.func.jvp AND an input is wrapped at that transform's level (so it carries a
    tangent there), or (no functorch transform) an input is a forward-AD dual tensor."""
    if torch._C._functorch.peek_interpreter_stack() is not None:
        from torch._functorch.pyfunctorch import retrieve_current_functorch_interpreter
        interp = retrieve_current_functorch_interpreter()
        if interp.key() != torch._C._functorch.TransformType.Jvp:
            return False
        level = interp.level()
        return any(torch._C._functorch.maybe_get_level(t) == level for t in tensors)
    import torch.autograd.forward_ad as fwAD
    return any(fwAD.unpack_dual(t).tangent is not None for t in tensors)


class AttentionJVP_autograd_function(torch.autograd.Function):
    """Attention O = softmax(q k^T / sqrt(D)) v whose forward-mode derivative is the kernel's tO.

    ``torch.func.jvp(attention_jvp, (q, k, v), (tq, tk, tv))`` and ``torch.autograd.forward_ad``
    dual tensors both dispatch to :meth:`jvp`.  Called through :func:`attention_jvp` under either,
    the forward defers O to the jvp rule's tangent kernel (one launch: O, tO and lse together);
    called plainly it runs the primal-only kernel (qattn_jvp_primal_ex: no tangent chains, O
    bit-identical to the tangent kernel's).  Reverse mode is not provided, as in the reference,
    which has no backward for this path.
    """

    @staticmethod
    def forward(q, k, v):
        q, k, v = _plain(q), _plain(k), _plain(v)
        if getattr(_DEFER, "on", False):
            with torch._C._DisableFuncTorch():
                B, H, S, D = q.shape
                O = torch.empty((B, H, S, D), dtype=torch.float32, device=q.device)
            _DEFER.pending = getattr(_DEFER, "pending", []) + [(_key(q, k, v), O, (q, k, v))]
            return O
        with torch._C._DisableFuncTorch():
            O, _tO, _lse = _jvp(q, k, v, None)
        return O

    @staticmethod
    def setup_context(ctx, inputs, output):
        q, k, v = inputs
        ctx.save_for_forward(q, k, v)

    @staticmethod
    def jvp(ctx, tq, tk, tv):
        # under torch.func.jvp the saved primals and the tangents arrive as functorch wrappers
        # (no storage) and new tensors would be wrapped too: the kernel runs on the plain tensors
        # with functorch disabled, and torch re-wraps the plain tO
        q, k, v = (_plain(t) for t in ctx.saved_tensors)
        tq, tk, tv = (None if t is None else _plain(t) for t in (tq, tk, tv))
        with torch._C._DisableFuncTorch():
            tq = torch.zeros_like(q) if tq is None else tq.to(q.dtype)
            tk = torch.zeros_like(k) if tk is None else tk.to(k.dtype)
            tv = torch.zeros_like(v) if tv is None else tv.to(v.dtype)
        # a deferred forward's O (see forward): filled here by the same launch as tO
        out_O = None
        pending = getattr(_DEFER, "pending", [])
        for i, (key, O, _) in enumerate(pending):
            if key == _key(q, k, v):
                out_O = O
                _DEFER.pending = pending[:i] + pending[i + 1:]
                break
        with torch._C._DisableFuncTorch():   # plain allocations for the kernel's buffers
            _O, tO, _lse = _jvp(q, k, v, (tq, tk, tv), out_O=out_O)
        return tO

    @staticmethod
    def backward(ctx, grad_O):
        raise RuntimeError("qattn jvp: reverse mode is not provided (forward-mode AD only)")


def attention_jvp(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """O fp32 [B,H,S,D]; differentiable in forward mode through the HIP tangent kernel (one launch
    per torch.func.jvp / forward-AD call)."""
    prev = getattr(_DEFER, "on", False)
    defer = _jvp_follows((q, k, v))
    _DEFER.on = defer
    n0 = len(getattr(_DEFER, "pending", []))
    try:
        out = AttentionJVP_autograd_function.apply(q, k, v)
    finally:
        _DEFER.on = prev
        # no deferred entry outlives the call that made it
        pending = getattr(_DEFER, "pending", [])
        left, _DEFER.pending = pending[n0:], pending[:n0]
    # a deferred O whose jvp rule did not run (no tangent reached this call after all) is filled by
    # the primal kernel
    for _k, O, (pq, pk, pv) in left:
        with torch._C._DisableFuncTorch():
            _jvp(pq, pk, pv, None, out_O=O)
    return out
