"""MFMA / ds_read_tr16 fragment-map probes (the lane maps common.h assumes), asymmetric integer data."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_mfma_i8_layout(lib):
    from quantizedattention_amd import _lib
    g = torch.Generator().manual_seed(1)
    A = torch.randint(-100, 100, (32, 32), generator=g, dtype=torch.int8)
    B = torch.randint(-100, 100, (32, 32), generator=g, dtype=torch.int8)
    Ad, Bd = A.cuda(), B.cuda()
    C = torch.empty((32, 32), dtype=torch.int32, device="cuda")
    _lib.call("qattn_probe_mfma_i8", _lib.ptr(Ad), _lib.ptr(Bd), _lib.ptr(C), _lib.stream_of(C))
    ref = (A.long() @ B.long()).int()
    assert torch.equal(C.cpu(), ref)


def test_mfma_f16_layout(lib):
    from quantizedattention_amd import _lib
    g = torch.Generator().manual_seed(2)
    A = torch.randint(-8, 8, (32, 16), generator=g).half()
    B = torch.randint(-8, 8, (16, 32), generator=g).half()
    Ad, Bd = A.cuda(), B.cuda()  # keep the device copies alive until the kernel has run
    C = torch.empty((32, 32), dtype=torch.float32, device="cuda")
    _lib.call("qattn_probe_mfma_f16", _lib.ptr(Ad), _lib.ptr(Bd), _lib.ptr(C), _lib.stream_of(C))
    torch.cuda.synchronize()
    assert torch.equal(C.cpu(), A.float() @ B.float())


def test_ds_read_tr16(lib):
    from quantizedattention_amd import _lib
    M = torch.arange(16 * 64, dtype=torch.int32).to(torch.int16).reshape(16, 64)
    out = torch.empty((64, 4), dtype=torch.int16, device="cuda")
    Md = M.cuda()
    _lib.call("qattn_probe_tr16", _lib.ptr(Md), _lib.ptr(out), _lib.stream_of(out))
    torch.cuda.synchronize()
    exp = torch.empty((64, 4), dtype=torch.int16)
    for l in range(64):
        g, i = l >> 4, l & 15
        for q in range(4):
            exp[l, q] = M[4 * g + q, 16 * g + i]
    assert torch.equal(out.cpu(), exp)


def test_packed_half_helpers(lib):
    """exp2_pk / trunc_pk (e32 + SDWA WORD_1 pairs) equal per-element exp2 / trunc."""
    from quantizedattention_amd import _lib
    x = -torch.rand(128, generator=torch.Generator().manual_seed(3)).half() * 8
    xd = x.cuda()
    e = torch.empty_like(xd)
    t = torch.empty_like(xd)
    _lib.call("qattn_probe_pk", _lib.ptr(xd), _lib.ptr(e), _lib.ptr(t), _lib.stream_of(xd))
    torch.cuda.synchronize()
    assert torch.allclose(e.cpu().float(), torch.exp2(x.float()), rtol=2e-3, atol=0)
    assert torch.equal(t.cpu().float(), torch.trunc((x * 127).float()))


def test_int8_fwd_softmax_helpers(lib):
    """p_operand8: f16(trunc(127 e) * sp) via the round-toward-zero packed fma (bit-exact);
    fma_mix8: f16(a*c + n) with one rounding (bit-exact vs an fp64 reference rounded to f16)."""
    from quantizedattention_amd import _lib
    g = torch.Generator().manual_seed(5)
    e = torch.rand(256, generator=g).half()
    e[::17] = 1.0          # the row maximum: 127 exactly
    e[5] = 0.0
    sp = (torch.rand(16, generator=g) * 2 + 1e-3).half()
    a = (torch.randn(256, generator=g) * 3e5).round()
    cn = torch.stack([torch.rand(16, generator=g) * 1e-4, -torch.rand(16, generator=g) * 8], 1).float()
    ed, spd, ad, cnd = e.cuda(), sp.cuda(), a.cuda(), cn.reshape(-1).cuda()
    w = torch.empty(256, dtype=torch.float16, device="cuda")
    d = torch.empty(256, dtype=torch.float16, device="cuda")
    _lib.call("qattn_probe_fwd_helpers", _lib.ptr(ed), _lib.ptr(spd), _lib.ptr(w), _lib.ptr(ad),
              _lib.ptr(cnd), _lib.ptr(d), _lib.stream_of(ed))
    torch.cuda.synchronize()
    lane = torch.arange(256) // 16
    exp_w = (torch.trunc(e.double() * 127) * sp[lane].double()).half()
    assert torch.equal(w.cpu().view(torch.int16), exp_w.view(torch.int16))
    exp_d = (a.double() * cn[lane, 0].double() + cn[lane, 1].double()).half()
    assert torch.equal(d.cpu().view(torch.int16), exp_d.view(torch.int16))


def test_quant_div_exhaustive(lib):
    """The quantisers' division-free index (common.h quant8: reciprocal + one Newton step) equals
    trunc(f16(fp32(x) / s)) with the IEEE fp32 division for every finite fp16 x with |x| < 127.5 s
    (a block holds |x / s| <= 127.07) and
    every fp16 scale s >= 0 (bit patterns 0 .. 0x7BFF; s = 0 gives idx 0)."""
    from quantizedattention_amd import _lib
    bad = torch.zeros((8,), dtype=torch.int32, device="cuda")
    st = _lib.stream_of(bad)
    for lo in range(0, 0x7C00, 0x2000):
        _lib.call("qattn_probe_quant_div", lo, min(lo + 0x2000, 0x7C00), _lib.ptr(bad), st)
    torch.cuda.synchronize()
    b = bad.cpu().tolist()
    assert b[0] == 0, (f"{b[0]} mismatches; first: s=0x{b[1]:04x} x=0x{b[2]:04x} ref={b[3]} "
                       f"byte={b[4]} image=0x{b[5] & 0xffffffff:08x}")


def test_exp2_cr_on_f16_domain(lib):
    """v_exp_f32 plus the correction table csrc/exp2_corr.h (the literal P chain's exp2_cr) is the
    correctly rounded exp2 on every fp16 argument in [-32, 0]; v_exp_f16 is correctly rounded on every
    finite fp16 argument.  (The oracle's exp2 is the correctly rounded one, oracle/restate.py _exp2.)"""
    import re
    from pathlib import Path
    import numpy as np
    from quantizedattention_amd import _lib
    e32 = torch.empty(65536, dtype=torch.int32, device="cuda")
    e16 = torch.empty(65536, dtype=torch.int16, device="cuda")
    _lib.call("qattn_probe_exp2_dom", _lib.ptr(e32), _lib.ptr(e16), _lib.stream_of(e32))
    torch.cuda.synchronize()
    g32 = e32.cpu().numpy().view(np.uint32).astype(np.int64)
    g16 = e16.cpu().numpy().view(np.float16)
    hdr = (Path(__file__).resolve().parents[1] / "quantizedattention_amd" / "csrc" / "exp2_corr.h").read_text()
    body = hdr[hdr.index("g_exp2_corr[EXP2_CORR_WORDS] = {"):]
    words = np.array([int(w, 16) for w in re.findall(r"0x([0-9a-f]{8})u", body)], dtype=np.uint64)
    n = 0x5001
    i = np.arange(n)
    corr = ((words[i // 4] >> (8 * (i % 4)).astype(np.uint64)) & 0xff).astype(np.uint8).view(np.int8)
    hb = (0x8000 | i).astype(np.uint16)
    x = hb.view(np.float16).astype(np.float64)
    cr = np.exp2(x).astype(np.float32).view(np.uint32).astype(np.int64)
    fixed = g32[hb.astype(np.int64)] + corr.astype(np.int64)
    assert np.array_equal(fixed, cr), int((fixed != cr).sum())
    h = np.arange(65536, dtype=np.uint32).astype(np.uint16).view(np.float16)
    fin = np.isfinite(h)
    with np.errstate(over="ignore"):
        cr16 = np.exp2(h.astype(np.float64)).astype(np.float16)
    assert np.array_equal(g16[fin].view(np.uint16), cr16[fin].view(np.uint16))
