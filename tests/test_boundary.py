"""CPU tests of the C-ABI boundary and the Python mirror's host logic (no kernel launches).

* include/qattn.h declares exactly the symbols libqattn.so exports and _lib.SIGNATURES types,
  with matching parameter counts.
* The reference's error behaviour: same exception type and message for mismatched shapes
  (attention_int8.py:126-127, attention_bf16.py:154-155, attention_jvp.py:78-79).
* The product path refuses CPU tensors loudly (no CPU fallback).
"""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "qattn.h"
LIB = ROOT / "quantizedattention_amd" / "libqattn.so"


def header_decls():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(int|long|const char\s*\*)\s*(qattn_\w+)\s*\(([^)]*)\)\s*;", text):
        params = [p.strip() for p in m.group(3).split(",") if p.strip() and p.strip() != "void"]
        decls[m.group(2)] = params
    return decls


def header_returns():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return {m.group(2): re.sub(r"\s+", "", m.group(1))
            for m in re.finditer(r"\b(int|long|const char\s*\*)\s*(qattn_\w+)\s*\(([^)]*)\)\s*;", text)}


def test_header_parses():
    d = header_decls()
    assert "qattn_int8_attn_fwd" in d and "qattn_bf16_bwd" in d and "qattn_jvp_fwd" in d
    assert len(d) >= 15


def test_signatures_match_header():
    from quantizedattention_amd import _lib
    d = header_decls()
    assert set(d) == set(_lib.SIGNATURES), set(d) ^ set(_lib.SIGNATURES)
    for name, params in d.items():
        assert len(params) == len(_lib.SIGNATURES[name]), name
        for p, ct in zip(params, _lib.SIGNATURES[name]):
            if "*" in p:
                assert ct is ctypes.c_void_p, (name, p)
            elif p.startswith("long"):
                assert ct is ctypes.c_long, (name, p)
            elif p.startswith("int"):
                assert ct is ctypes.c_int, (name, p)
            elif p.startswith("float"):
                assert ct is ctypes.c_float, (name, p)
            else:
                raise AssertionError((name, p))


@pytest.mark.skipif(not LIB.exists(), reason="libqattn.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT\s+(qattn_\w+)", out))
    declared = set(header_decls())
    assert declared <= exported, declared - exported
    assert exported <= declared, f"undeclared exports: {exported - declared}"


@pytest.mark.skipif(not LIB.exists(), reason="libqattn.so not built")
def test_library_loads_and_types():
    from quantizedattention_amd import _lib
    lib = _lib.load()
    for name, ret in header_returns().items():
        want = {"long": ctypes.c_long, "int": ctypes.c_int, "constchar*": ctypes.c_char_p}[ret]
        assert getattr(lib, name).restype is want, name


@pytest.mark.skipif(not LIB.exists(), reason="libqattn.so not built (run __graft_entry__.build())")
def test_abi_version_and_source_hash():
    """The library speaks the header's ABI version and was built from the sources in the tree
    (_lib.load refuses it otherwise: a stale prebuilt library must not run)."""
    from quantizedattention_amd import _lib, _srchash
    lib = _lib.load()
    m = re.search(r"#define\s+QATTN_ABI_VERSION\s+(\d+)", HEADER.read_text())
    assert m and int(m.group(1)) == _lib.ABI_VERSION == lib.qattn_abi_version()
    assert lib.qattn_source_hash().decode() == _srchash.library_hash()


def test_int8_error_messages():
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    q = torch.zeros(1, 1, 64, 64, dtype=torch.float16)
    with pytest.raises(AssertionError, match="k and v tokens are different"):
        helion_atten_int8_hl_dot_fwd(q, q, torch.zeros(1, 1, 32, 64, dtype=torch.float16))
    with pytest.raises(AssertionError, match="k head_dim and v head_dim are different"):
        helion_atten_int8_hl_dot_fwd(q, q, torch.zeros(1, 1, 64, 128, dtype=torch.float16))


def test_bf16_error_messages():
    from quantizedattention_amd.attention_bf16 import helion_atten_bf16_fwd_training
    q = torch.zeros(1, 1, 64, 64, dtype=torch.float16)
    with pytest.raises(AssertionError, match="input k_tokens must match v_tokens"):
        helion_atten_bf16_fwd_training(q, q, torch.zeros(1, 1, 32, 64, dtype=torch.bfloat16), False)
    with pytest.raises(AssertionError, match="all head dimensions must match"):
        helion_atten_bf16_fwd_training(q, q, torch.zeros(1, 1, 64, 128, dtype=torch.bfloat16), False)


def test_jvp_error_messages():
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    q = torch.zeros(1, 1, 64, 64)
    with pytest.raises(AssertionError, match="input k_tokens must match v_tokens"):
        helion_attention_jvp_forward_fp32(q, q, torch.zeros(1, 1, 32, 64), q, q, q)


def test_no_cpu_fallback():
    from quantizedattention_amd import _lib
    from quantizedattention_amd.attention_bf16 import helion_atten_bf16_fwd_training
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    q = torch.zeros(1, 1, 64, 64, dtype=torch.float16)
    with pytest.raises(_lib.QAttnError, match="no CPU fallback"):
        helion_atten_int8_hl_dot_fwd(q, q, q)
    with pytest.raises(_lib.QAttnError, match="no CPU fallback"):
        helion_atten_bf16_fwd_training(q, q, q.bfloat16(), False)
    x = torch.zeros(1, 1, 64, 64)
    with pytest.raises(_lib.QAttnError, match="no CPU fallback"):
        helion_attention_jvp_forward_fp32(x, x, x, x, x, x)


def test_unsupported_shapes_rejected_before_launch():
    from quantizedattention_amd import _lib
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    with pytest.raises(_lib.QAttnError, match="multiple of 32"):
        q = torch.zeros(1, 1, 48, 64, dtype=torch.float16)
        helion_atten_int8_hl_dot_fwd(q, q, q)
    with pytest.raises(_lib.QAttnError, match="head_dim"):
        q = torch.zeros(1, 1, 64, 96, dtype=torch.float16)
        helion_atten_int8_hl_dot_fwd(q, q, q)


def test_oracle_not_imported_by_product():
    """The product package never imports the oracle (test infrastructure only)."""
    for p in (ROOT / "quantizedattention_amd").rglob("*.py"):
        src = p.read_text()
        assert not re.search(r"^\s*(from|import)\s+oracle\b", src, flags=re.M), p


@pytest.mark.skipif(not LIB.exists(), reason="libqattn.so not built")
def test_bwd_workspace_size():
    """qattn_int8_bwd_ws_bytes (host-only): 1 KiB record + 4 B scale per (head, q-tile, k-tile)."""
    from quantizedattention_amd import _lib
    lib = _lib.load()
    assert lib.qattn_int8_bwd_ws_bytes(4 * 32, 4096, 4096) == 128 * 128 * 128 * 1028
    assert lib.qattn_int8_bwd_ws_bytes(6, 96, 160) == 6 * 3 * 5 * 1028
    assert lib.qattn_int8_bwd_ws_bytes(2, 100, 64) == -1          # tokens not a multiple of 32
    assert lib.qattn_int8_bwd_ws_bytes(0, 64, 64) == 0
    # one key/value head's records are addressed with 32-bit offsets: (S/32)^2 KiB < 2 GiB
    assert lib.qattn_int8_bwd_ws_bytes(1, 46336, 46336) > 0          # 1448^2 KiB < 2 GiB
    assert lib.qattn_int8_bwd_ws_bytes(1, 65536, 65536) == -1         # 4 GiB region: recompute
    assert lib.qattn_int8_bwd_ws_bytes(8, 32768, 65536) == -1         # 2 GiB region
    # the grouped check is in the launcher: G = 8 query heads at S = 32768 is 8 GiB per kv head
    # (a non-null workspace pointer: the guard answers before anything touches memory or a device)
    assert lib.qattn_int8_attn_bwd_ws(*([None] * 15), ctypes.c_void_p(16), 8, 32768, 32768, 8, 0, 128,
                                      0.0, 0.0, None) == 1
    assert lib.qattn_bf16_bwd_ws_bytes(4 * 32, 4096, 4096) == 128 * 128 * 128 * 2048
    assert lib.qattn_bf16_bwd_ws_bytes(6, 96, 160) == 6 * 3 * 5 * 2048
    assert lib.qattn_bf16_bwd_ws_bytes(2, 100, 64) == -1


def test_call_guards_the_stream_device(monkeypatch):
    """_lib.call switches to the device of its stream argument for the launch (host-only check with
    a stand-in entry point and device hooks)."""
    import contextlib

    import torch

    from quantizedattention_amd import _lib
    seen = []

    class FakeLib:
        @staticmethod
        def qattn_probe(*args):
            seen.append(("launch", cur[0]))
            return 0
    cur = [0]

    @contextlib.contextmanager
    def fake_device(i):
        old, cur[0] = cur[0], i
        seen.append(("enter", i))
        yield
        cur[0] = old
    monkeypatch.setattr(_lib, "load", lambda: FakeLib)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: cur[0])
    monkeypatch.setattr(torch.cuda, "device", fake_device)
    st = _lib._Stream(0)
    st.device_index = 1
    _lib.call("qattn_probe", st)
    assert seen == [("enter", 1), ("launch", 1)]
    seen.clear()
    st.device_index = 0
    _lib.call("qattn_probe", st)
    assert seen == [("launch", 0)]
