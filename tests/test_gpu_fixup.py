"""The int8 forward's deferred-vote fixup paths, on inputs that make the votes hold.

The fast pass takes the fast P_i8 chain on every tile and writes each tile's vote down; the epilogue
takes the votes again against the final row sums and marks a wave for which one still holds
(csrc/int8_attn_fwd.hip, DESIGN.md §3 "the reference's chain where it matters").  The marked waves
are recomputed with the reference's literal P chain (attention_int8.py:197-237):
  * by a second launch on the pre-quantised entry (qattn_int8_attn_fwd_ex; marks in lse as the fp16
    NaN pattern FIX_LSE16 = 0x7e5a),
  * inline, in the same workgroup, on the q-fused entry (qattn_int8_attn_fwd_qf, the drop-ins' path),
  * by a second launch of the key-split decoding entry (qattn_int8_attn_fwd_split; marks in the
    split state's m as the fp32 NaN pattern FIX_M32 = 0x7fc0e5a5).
QATTN_FWD_SKIP_FIXUP=1 (a diagnostic switch of the library) leaves the second launches out, so the
marks can be counted.  On random config-3 inputs no wave is marked; here, with q = k and keys scaled
by a ramp (peaked rows whose own key carries most of the row), waves are.
"""
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

FIX_LSE16 = 0x7e5a
FIX_M32 = 0x7fc0e5a5


def _peaked(B, H, S, D, seed, scale=24.0):
    """Even heads peaked (q = k, keys scaled by a ramp: every wave is marked), odd heads plain random
    (no wave is marked, as at config 3), so both kinds of rows are checked."""
    g = torch.Generator().manual_seed(seed)
    ramp = (1.0 + torch.arange(S, dtype=torch.float32) / scale).view(1, 1, S, 1)
    k = torch.randn((B, H, S, D), generator=g) * ramp
    q = k.clone()
    plain = torch.arange(H) % 2 == 1
    q[:, plain] = torch.randn((B, int(plain.sum()), S, D), generator=g)
    k[:, plain] = torch.randn((B, int(plain.sum()), S, D), generator=g)
    v = torch.randn((B, H, S, D), generator=g).half()
    return q.half(), k.half(), v


def _quantise(q, k, v):
    from quantizedattention_amd import _lib
    B, H, S, D = q.shape
    N = B * H * S
    dev = q.device
    st = _lib.stream_of(q)
    out = {n: torch.empty((N, D), dtype=torch.int8, device=dev) for n in ("qi", "ki", "vi", "vt")}
    for n in ("sq", "sk", "sv"):
        out[n] = torch.empty((N // 32,), dtype=torch.float16, device=dev)
    _lib.call("qattn_int8_quant", _lib.ptr(q), _lib.ptr(out["qi"]), _lib.ptr(out["sq"]), None, None, N, S, D, st)
    _lib.call("qattn_int8_quant", _lib.ptr(k), _lib.ptr(out["ki"]), _lib.ptr(out["sk"]), None, None, N, S, D, st)
    _lib.call("qattn_int8_quant_vt", _lib.ptr(v), _lib.ptr(out["vi"]), _lib.ptr(out["sv"]), _lib.ptr(out["vt"]),
              N, D, st)
    return out


def _qks(D):
    return float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))


def _fwd_ex(t, q, causal, skip):
    from quantizedattention_amd import _lib
    B, H, S, D = q.shape
    O = torch.full((B, H, S, D), float("nan"), dtype=torch.float16, device=q.device)
    lse = torch.full((B * H * S,), float("nan"), dtype=torch.float16, device=q.device)
    os.environ["QATTN_FWD_SKIP_FIXUP"] = "1" if skip else "0"
    try:
        _lib.call("qattn_int8_attn_fwd_ex", _lib.ptr(t["qi"]), _lib.ptr(t["sq"]), _lib.ptr(t["ki"]),
                  _lib.ptr(t["sk"]), _lib.ptr(t["vt"]), _lib.ptr(t["sv"]), _lib.ptr(O), _lib.ptr(lse),
                  B * H, S, S, 1, int(causal), D, _qks(D), _lib.stream_of(q))
        torch.cuda.synchronize()
    finally:
        os.environ.pop("QATTN_FWD_SKIP_FIXUP", None)
    return O, lse


@pytest.mark.parametrize("D,causal", [(128, False), (128, True), (64, False), (64, True)])
def test_fixup_runs_and_matches_inline(lib, D, causal):
    from oracle import restate as R
    from quantizedattention_amd import _lib
    B, H, S = 1, 4, 512
    q, k, v = _peaked(B, H, S, D, seed=61 + D)
    qc, kc, vc = q.cuda(), k.cuda(), v.cuda()
    t = _quantise(qc, kc, vc)
    O0, l0 = _fwd_ex(t, qc, causal, skip=True)
    marked = l0.view(torch.int16).to(torch.int32).bitwise_and(0xffff) == FIX_LSE16
    n_rows = int(marked.sum())
    print(f"D={D} causal={causal}: {n_rows // 32} of {B * H * S // 32} waves marked")
    assert n_rows > 0 and n_rows % 32 == 0, "the peaked input must mark waves (else nothing is tested)"
    assert n_rows < B * H * S, "the plain heads must keep unmarked waves"
    O1, l1 = _fwd_ex(t, qc, causal, skip=False)
    # the fixup leaves no mark, and touches exactly the marked waves' rows
    assert not (l1.view(torch.int16).to(torch.int32).bitwise_and(0xffff) == FIX_LSE16).any()
    assert torch.isfinite(O1).all() and torch.isfinite(l1).all()
    rows = marked.view(B, H, S)
    assert torch.equal(O0[~rows], O1[~rows]) and torch.equal(l0[~marked], l1[~marked])
    assert not torch.equal(O0[rows], O1[rows]), "the fixup pass changed nothing on the marked rows"
    # the inline fixup of the q-fused entry (the drop-ins' path) gives the same bits
    Oq = torch.empty_like(O1)
    lq = torch.empty_like(l1)
    qi2, sq2 = torch.empty_like(t["qi"]), torch.empty_like(t["sq"])
    _lib.call("qattn_int8_attn_fwd_qf", _lib.ptr(qc), _lib.ptr(qi2), _lib.ptr(sq2), None, _lib.ptr(t["ki"]),
              _lib.ptr(t["sk"]), _lib.ptr(t["vt"]), _lib.ptr(t["sv"]), _lib.ptr(Oq), _lib.ptr(lq),
              B * H, S, S, 1, int(causal), D, _qks(D), _lib.stream_of(qc))
    torch.cuda.synchronize()
    assert torch.equal(qi2, t["qi"]) and torch.equal(sq2, t["sq"])
    assert torch.equal(Oq, O1) and torch.equal(lq, l1)
    # the redone rows follow the reference's literal chain: closer to the oracle than the fast pass
    ref = R.int8_fwd(q, k, v, causal=causal)
    Or = ref[0].float().cuda()
    e_fast = (O0.float() - Or).abs()[rows].max().item()
    e_fix = (O1.float() - Or).abs()[rows].max().item()
    vmax = v.float().abs().max().item()
    print(f"   marked rows: |O_fast - O_ref| {e_fast:.2e}, |O_fixed - O_ref| {e_fix:.2e} (max|v| {vmax:.2f})")
    assert e_fix <= 1e-2 * vmax
    assert e_fix <= e_fast


def test_split_fixup_marks_and_merge(lib):
    """Key-split decoding: marks in the split state's m (FIX_M32), redone by the second launch; the
    merged output stays within the merge's rounding of the one-pass forward."""
    from quantizedattention_amd import _lib
    B, H, S, D = 1, 2, 1024, 128
    q, k, v = _peaked(B, H, S, D, seed=67)
    qc, kc, vc = q.cuda(), k.cuda(), v.cuda()
    t = _quantise(qc, kc, vc)
    ks = 256
    nsplit = S // ks
    rows = B * H * S
    O_one, l_one = _fwd_ex(t, qc, False, skip=False)

    def split(skip):
        opart = torch.empty((nsplit, rows, D), dtype=torch.float16, device="cuda")
        ml = torch.empty((nsplit, rows, 2), dtype=torch.float32, device="cuda")
        os.environ["QATTN_FWD_SKIP_FIXUP"] = "1" if skip else "0"
        try:
            _lib.call("qattn_int8_attn_fwd_split", _lib.ptr(t["qi"]), _lib.ptr(t["sq"]), _lib.ptr(t["ki"]),
                      _lib.ptr(t["sk"]), _lib.ptr(t["vt"]), _lib.ptr(t["sv"]), _lib.ptr(opart), _lib.ptr(ml),
                      B * H, S, S, 1, ks, D, _qks(D), _lib.stream_of(qc))
            torch.cuda.synchronize()
        finally:
            os.environ.pop("QATTN_FWD_SKIP_FIXUP", None)
        return opart, ml

    _, ml0 = split(True)
    m_bits = ml0[..., 0].contiguous().view(torch.int32)
    n_marked = int((m_bits == FIX_M32).sum())
    print(f"split: {n_marked // 32} of {nsplit * rows // 32} split waves marked")
    assert 0 < n_marked < nsplit * rows
    opart, ml = split(False)
    m_bits = ml[..., 0].contiguous().view(torch.int32)
    assert not (m_bits == FIX_M32).any()
    O = torch.empty((rows, D), dtype=torch.float16, device="cuda")
    lse = torch.empty((rows,), dtype=torch.float16, device="cuda")
    _lib.call("qattn_int8_split_combine", _lib.ptr(opart), _lib.ptr(ml), _lib.ptr(O), _lib.ptr(lse), rows,
              nsplit, D, _lib.stream_of(qc))
    torch.cuda.synchronize()
    assert torch.isfinite(O).all() and torch.isfinite(lse).all()
    d = (O.float() - O_one.view(rows, D).float()).abs().max().item()
    print(f"   |O_split - O_one| {d:.2e}")
    assert d <= 2e-3 * max(1.0, v.float().abs().max().item())
