"""ctypes binding of libqattn.so — the C-ABI boundary declared in include/qattn.h.

The library is loaded after ``torch`` so that its ``libamdhip64.so.7`` dependency resolves to the
HIP runtime torch already mapped (one runtime per process; torch streams are valid handles).
There is no fallback: if the library is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "libqattn.so"

_c_long = ctypes.c_long
_c_int = ctypes.c_int
_c_float = ctypes.c_float
_vp = ctypes.c_void_p

# name -> argtypes (restype is always int status: 0 ok, 1 invalid argument, 2 launch failure)
SIGNATURES = {
    "qattn_abi_version": [],
    "qattn_source_hash": [],
    "qattn_int8_quant": [_vp, _vp, _vp, _vp, _vp, _c_long, _c_int, _c_int, _vp],
    "qattn_int8_quant_img": [_vp] * 6 + [_c_long, _c_int, _c_int, _vp],
    "qattn_int8_dequant": [_vp, _vp, _vp, _c_long, _c_int, _vp],
    "qattn_int8_quant_vt": [_vp, _vp, _vp, _vp, _c_long, _c_int, _vp],
    "qattn_int8_v_image": [_vp, _vp, _c_long, _c_int, _vp],
    "qattn_kmean": [_vp, _vp, _c_long, _c_long, _c_int, _vp],
    "qattn_int8_quant_k_smooth": [_vp] * 5 + [_c_long, _c_long, _c_int, _vp],
    "qattn_int8_attn_fwd": [_vp] * 8 + [_c_long, _c_long, _c_int, _c_float, _vp],
    "qattn_int8_attn_fwd_ex": [_vp] * 8 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int, _c_float,
                                                 _vp],
    "qattn_int8_attn_fwd_qf": [_vp] * 10 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int, _c_float, _vp],
    "qattn_int8_attn_fwd_split": [_vp] * 8 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int, _c_float,
                                               _vp],
    "qattn_int8_split_combine": [_vp] * 4 + [_c_long, _c_int, _c_int, _vp],
    "qattn_int8_attn_bwd_ex": [_vp] * 15 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int, _c_float,
                                             _c_float, _vp],
    "qattn_int8_attn_bwd_ws": [_vp] * 16 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int, _c_float,
                                             _c_float, _vp],
    "qattn_int8_bwd_ws_bytes": [_c_long, _c_long, _c_long],
    "qattn_bwd_ws_cap": [],
    "qattn_int8_attn_bwd_wsc": [_vp] * 16 + [_c_long, _c_long, _c_long, _c_long, _c_int, _c_int, _c_int,
                                              _c_float, _c_float, _vp],
    "qattn_int8_bwd_dkdv_ws": [_vp] * 14 + [_c_long, _c_long, _c_int, _c_float, _c_float, _vp],
    "qattn_int8_bwd_dq_ws": [_vp] * 4 + [_c_long, _c_long, _c_int, _c_float, _vp],
    "qattn_int8_bwd_prep": [_vp] * 7 + [_c_long, _c_long, _c_int, _vp],
    "qattn_i8_to_bf16": [_vp, _vp, _c_long, _vp],
    "qattn_int8_attn_bwd": [_vp] * 15 + [_c_long, _c_long, _c_int, _c_float, _c_float, _vp],
    "qattn_int8_bwd_dkdv": [_vp] * 13 + [_c_long, _c_long, _c_int, _c_float, _c_float, _vp],
    "qattn_int8_bwd_dv": [_vp] * 13 + [_c_long, _c_long, _c_int, _c_float, _c_float, _vp],
    "qattn_int8_bwd_dk": [_vp] * 13 + [_c_long, _c_long, _c_int, _c_float, _c_float, _vp],
    "qattn_int8_bwd_dq": [_vp] * 11 + [_c_long, _c_long, _c_int, _c_float, _c_float, _vp],
    "qattn_bf16_fwd": [_vp, _vp, _vp, _vp, _vp, _c_long, _c_long, _c_long, _c_int, _c_int, _c_float, _vp],
    "qattn_bf16_fwd_ex": [_vp] * 5 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int, _c_float, _vp],
    "qattn_bf16_fwd_ws_bytes": [_c_long, _c_long, _c_int],
    "qattn_bf16_fwd_ws_ex": [_vp] * 5 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int, _c_float,
                                          _vp, _vp],
    "qattn_bf16_bwd_ex": [_vp] * 10 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int, _c_float,
                                        _c_float, _vp],
    "qattn_bf16_bwd_ws_bytes": [_c_long, _c_long, _c_long],
    "qattn_bf16_bwd_ws_ex": [_vp] * 10 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int, _c_float,
                                           _c_float, _vp, _vp],
    "qattn_bf16_bwd_split_ex": [_vp] * 10 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_int,
                                              _c_float, _c_float, _vp],
    "qattn_bf16_bwd_prep": [_vp] * 5 + [_c_long, _c_long, _c_int, _vp],
    "qattn_f16_to_bf16": [_vp, _vp, _c_long, _vp],
    "qattn_bf16_bwd": [_vp] * 10 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_float, _c_float, _vp],
    "qattn_jvp_fwd": [_vp] * 9 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_float, _c_float, _vp],
    "qattn_jvp_fwd_x3": [_vp] * 15 + [_c_long, _c_long, _c_long, _c_int, _c_float, _c_float, _vp],
    "qattn_jvp_fwd_ex": [_vp] * 9 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_float, _c_float, _vp],
    "qattn_jvp_primal_ex": [_vp] * 5 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_float, _c_float, _vp],
    "qattn_jvp_primal_x3_ex": [_vp] * 8 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_float, _c_float,
                               _vp],
    "qattn_jvp_fwd_x3_ex": [_vp] * 15 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_float, _c_float,
                                         _vp],
    "qattn_split_bf16": [_vp, _vp, _vp, _c_long, _vp],
    "qattn_mxfp4_quant_rows": [_vp, _vp, _vp, _vp, _c_long, _c_long, _c_int, _vp],
    "qattn_mxfp4_quant_vt": [_vp, _vp, _vp, _c_long, _c_long, _c_int, _vp],
    "qattn_mxfp4_attn_fwd": [_vp] * 8 + [_c_long, _c_long, _c_long, _c_int, _c_int, _c_float, _vp],
}

# libqattn_dev.so (include/qattn_dev.h): fragment-layout probes for tests/test_gpu_layout.py
DEV_SIGNATURES = {
    "qattn_probe_mfma_i8": [_vp, _vp, _vp, _vp],
    "qattn_probe_mfma_f16": [_vp, _vp, _vp, _vp],
    "qattn_probe_tr16": [_vp, _vp, _vp],
    "qattn_probe_pk": [_vp, _vp, _vp, _vp],
    "qattn_probe_mfma_fp4": [_vp] * 6,
    "qattn_probe_fp4_cvt": [_vp] * 5,
    "qattn_probe_fwd_helpers": [_vp] * 7,
    "qattn_probe_quant_div": [_c_int, _c_int, _vp, _vp],
    "qattn_probe_few_wg_copy": [_vp, _vp, _c_long, _c_int, _vp],
    "qattn_probe_exp2_dom": [_vp, _vp, _vp],
}

# return types other than the int status code
RESTYPES = {"qattn_abi_version": ctypes.c_int, "qattn_source_hash": ctypes.c_char_p,
            "qattn_int8_bwd_ws_bytes": ctypes.c_long, "qattn_bf16_bwd_ws_bytes": ctypes.c_long,
            "qattn_bf16_fwd_ws_bytes": ctypes.c_long,
            "qattn_bwd_ws_cap": ctypes.c_long}

# include/qattn.h QATTN_ABI_VERSION: the argument lists SIGNATURES describes
ABI_VERSION = 6

_lib = None
_dev = None


class QAttnError(RuntimeError):
    pass


def load(path: os.PathLike | None = None) -> ctypes.CDLL:
    """Load (once) and type the library; raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("QATTN_LIB", LIB_PATH))
    if not p.exists():
        raise QAttnError(
            f"{p} not found: build it with `python -m quantizedattention_amd.build` "
            "(there is no CPU fallback)")
    lib = ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            raise QAttnError(f"{p} does not export {name} (stale build? rebuild it)")
        fn.argtypes = argtypes
        fn.restype = RESTYPES.get(name, ctypes.c_int)
    if lib.qattn_abi_version() != ABI_VERSION:
        raise QAttnError(f"{p}: C ABI version {lib.qattn_abi_version()}, this binding speaks "
                         f"{ABI_VERSION} (include/qattn.h QATTN_ABI_VERSION); rebuild the library")
    from . import _srchash
    if _srchash.available() and os.environ.get("QATTN_LIB") is None:
        built = lib.qattn_source_hash().decode()
        want = _srchash.library_hash()
        if built != want:
            raise QAttnError(
                f"{p} is stale: built from sources/flags {built[:12]}, the tree holds {want[:12]} "
                "(rebuild it with `python -m quantizedattention_amd.build`)")
    _lib = lib
    return lib


_ops_loaded = False


def load_ops() -> None:
    """Load (once) libqattn_torch.so, the TORCH_LIBRARY(qattn) operators (csrc/torch/qattn_ops.cpp),
    after libqattn.so whose C-ABI it calls; raises if it is absent or stale."""
    global _ops_loaded
    if _ops_loaded:
        return
    load()
    p = _PKG / "libqattn_torch.so"
    if not p.exists():
        raise QAttnError(f"{p} not found: build it with `python -m quantizedattention_amd.build` "
                         "(the qattn:: operators have no Python fallback)")
    import torch
    torch.ops.load_library(str(p))
    _ops_loaded = True


def load_dev() -> ctypes.CDLL:
    """The development library of layout probes (built beside libqattn.so); tests only."""
    global _dev
    if _dev is None:
        load()
        p = _PKG / "libqattn_dev.so"
        if not p.exists():
            raise QAttnError(f"{p} not found: build it with `python -m quantizedattention_amd.build`")
        lib = ctypes.CDLL(str(p))
        for name, argtypes in DEV_SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        _dev = lib
    return _dev


def exported_symbols() -> list[str]:
    lib = load()
    return [n for n in SIGNATURES if hasattr(lib, n)]


def ptr(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class _Stream(ctypes.c_void_p):
    """A hipStream_t argument that remembers its device (the device guard of ``call``)."""
    device_index = None


def stream_of(t: torch.Tensor):
    st = _Stream(torch.cuda.current_stream(t.device).cuda_stream)
    st.device_index = t.device.index
    return st


def call(name: str, *args) -> None:
    """Call a C-ABI entry; launches go to the device of its stream argument (the HIPGuard of SURVEY
    §8b: ``hipFuncSetAttribute`` and the launch act on the current device)."""
    fn = getattr(load_dev() if name in DEV_SIGNATURES else load(), name)
    dev = next((a.device_index for a in args if isinstance(a, _Stream)), None)
    if dev is not None and dev != torch.cuda.current_device():
        with torch.cuda.device(dev):
            rc = fn(*args)
    else:
        rc = fn(*args)
    if rc == 1:
        raise QAttnError(f"{name}: unsupported shape/argument (status 1)")
    if rc != 0:
        raise QAttnError(f"{name}: kernel launch failed (status {rc})")


def plain(t):
    """The tensor under any functorch wrappers (torch.func.grad / vjp / jvp hand custom Functions'
    backward and jvp rules GradTrackingTensors, which have no storage).  Kernel launches run on the
    plain tensors inside ``torch._C._DisableFuncTorch()``; torch wraps the plain results again."""
    if not isinstance(t, torch.Tensor):
        return t
    from torch._C._functorch import get_unwrapped, is_functorch_wrapped_tensor
    while is_functorch_wrapped_tensor(t):
        t = get_unwrapped(t)
    return t


def require_gpu(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if not t.is_cuda:
            raise QAttnError("qattn kernels run on the GPU only; got a tensor on "
                             f"{t.device} (no CPU fallback by design)")


# Backward workspaces (the dS records) refused by the allocator, per device: {device: smallest refused
# size}.  torch's caching allocator answers an allocation it cannot serve by freeing every cached
# block and retrying before it raises, so a training loop whose workspace never fits would flush the
# cache and stall on hipFree in every backward.  After one refusal, a workspace that large is only
# tried again when the device has room for it (free plus reserved-but-unused bytes).
_WS_REFUSED: dict = {}


def try_workspace(nbytes: int, device) -> torch.Tensor | None:
    """A uint8 workspace of ``nbytes`` on ``device``, or None when it does not fit (the caller then
    takes the recomputing path, with the same results)."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    refused = _WS_REFUSED.get(idx)
    if refused is not None and nbytes >= refused:
        free, _total = torch.cuda.mem_get_info(idx)
        spare = torch.cuda.memory_reserved(idx) - torch.cuda.memory_allocated(idx)
        if free + spare < nbytes:
            return None
    try:
        ws = torch.empty((nbytes,), dtype=torch.uint8, device=dev)
    except torch.cuda.OutOfMemoryError:
        _WS_REFUSED[idx] = nbytes if refused is None else min(refused, nbytes)
        return None
    if refused is not None and nbytes >= refused:
        _WS_REFUSED.pop(idx, None)
    return ws
