"""Numerical emulation of the int8 forward kernel (int8_attn_fwd.hip, PV_I8, non-causal) on the CPU.

A study tool, not a test: it reproduces the kernel's rounding points (the fast P chain on the f16
exponential, the deferred running max, the per-tile dequantisation) and a candidate "literal" chain
(the reference's P_i8 = trunc(exp2(f16(S - m)) / sp), int8:197-237, with correctly rounded exp2) on
tiles chosen by a wave-uniform vote, and compares O / lse with oracle.restate.int8_fwd.  v_exp_f16 is
correctly rounded on every fp16 argument (tools/exp2_probe.py), so the fast chain is emulated exactly
up to fp32 summation order.

  python tools/fwd_emul.py            # the peaked / fuzz / config-3 studies, for several vote bars K
"""
from __future__ import annotations

import math
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import restate as R  # noqa: E402

KMAG = 12582912.0
F16, F32 = np.float16, np.float32


def h(x):      # round to f16 (numpy: one rounding from float64)
    return np.asarray(x, dtype=np.float64).astype(F16).astype(np.float64)


def f(x):      # round to f32
    return np.asarray(x, dtype=np.float64).astype(F32).astype(np.float64)


def exp2_cr32(x):
    with np.errstate(under="ignore", over="ignore"):
        return f(np.exp2(x))


def exp2_cr16(x):
    with np.errstate(under="ignore", over="ignore"):
        return h(np.exp2(x))


def kmag_scale(c):
    b = np.asarray(c, dtype=F32).view(np.uint32) & np.uint32(0xFFFFFFFE)
    return b.view(F32).astype(np.float64)


def emulate(qi, sq, ki, sk, vi, sv, qks, K=None, thr=8.0, lse_from_mt=False, wave=32, NC=0):
    """One head: qi [S,D], ki/vi [Sk,D] int8 (as int64 arrays), sq/sk/sv f16 per 32-row block.
    K: the vote bar (a tile takes the literal chain when some row of its wave has er*K > l);
    None = never (the current kernel), 0 = always.  Returns O (f16 as f64), lse, literal fraction."""
    S, D = qi.shape
    Sk = ki.shape[0]
    nt = Sk // 32
    rows = np.arange(S)
    sqr = sq.astype(np.float64)[rows // 32]                     # per-row q scale
    m = np.full(S, -np.inf)
    m_thr = np.full(S, -np.inf)
    mt = np.full(S, -np.inf)
    lrow = np.zeros(S)
    O = np.zeros((S, D))
    nlit = 0
    nredo = 0
    qks32 = float(np.float32(qks))
    nw = S // wave
    cands = [[] for _ in range(nw)]   # per wave: deferred candidates (tile, fast and literal parts)
    for t in range(nt):
        ks = slice(32 * t, 32 * t + 32)
        X = (qi @ ki[ks].T).astype(np.float64)                   # exact integer dot
        skt = float(sk[t])
        ckt = f(skt * qks32)
        c = kmag_scale(f(sqr * ckt))
        S16 = h(f(X * c[:, None]))
        rm = S16.max(1)
        # deferred running max (per wave: every row of the wave moves when one row passes m_thr)
        mv = (rm > m_thr).reshape(-1, wave).any(1).repeat(wave)
        nm = np.where(mv, np.maximum(m, rm), m)
        r = np.where(mv, exp2_cr32(h(m - nm)), 1.0)
        r = np.where(np.isneginf(m) & mv, 0.0, r)
        m = nm
        m_thr = np.where(mv, h(m + thr), m_thr)
        lrow *= r
        O *= r[:, None]
        for w_ in range(nw):   # deferred candidates rescale with O
            rs = slice(w_ * wave, (w_ + 1) * wave)
            for cd in cands[w_]:
                cd["scale"] *= r[rs]
        er = exp2_cr32(h(rm - m))
        if K is None:
            lit = np.zeros(S, bool)
        elif K == 0:
            lit = np.ones(S, bool)
        else:
            lit = (er * K > lrow).reshape(-1, wave).any(1).repeat(wave)
        # NC > 0: the first NC voting tiles of a wave go fast now and are redone at the end if the
        # final row sum still says so (deferred vote); later ones go literal now
        defer = np.zeros(S, bool)
        if NC > 0 and K not in (None, 0):
            for w_ in range(nw):
                rs = slice(w_ * wave, (w_ + 1) * wave)
                if lit[rs][0] and len(cands[w_]) < NC:
                    defer[rs] = True
            lit = lit & ~defer
        nlit += lit.reshape(-1, wave)[:, 0].sum()
        # fast chain
        d = h(S16 - rm[:, None])
        e = exp2_cr16(d)
        Pi = np.floor(127.0 * e)
        cpv = er * f(float(sv[t]) * f(1.0 / 127.0))
        lt = er * e.sum(1)
        # literal chain (the reference's, int8:197-237, exp2 correctly rounded)
        if defer.any():
            Sr = h(f(f(f(X * sqr[:, None]) * skt) * qks32))
            rmr = Sr.max(1)
            nmr = np.maximum(mt, rmr)
            P = exp2_cr32(h(Sr - nmr[:, None]))
            sp = f(exp2_cr32(h(rmr - nmr)) / 127.0)
            with np.errstate(divide="ignore", invalid="ignore"):
                Pir = np.where(sp[:, None] > 0, np.trunc(f(P / np.where(sp > 0, sp, 1.0)[:, None])), 0.0)
            wv = exp2_cr32(nmr - m)
            Vt = vi[ks].astype(np.float64)
            for w_ in range(nw):
                rs = slice(w_ * wave, (w_ + 1) * wave)
                if defer[rs][0]:
                    cands[w_].append(dict(
                        fastO=(Pi[rs] @ Vt) * cpv[rs, None], fastl=lt[rs], er=er[rs],
                        litO=(Pir[rs] @ Vt) * (f(sp[rs] * float(sv[t])) * wv[rs])[:, None],
                        litl=f(P[rs].sum(1)) * wv[rs], scale=np.ones(wave)))
            mt = np.where(defer, nmr, mt)
        if lit.any():
            Sr = h(f(f(f(X * sqr[:, None]) * skt) * qks32))
            rmr = Sr.max(1)
            nmr = np.maximum(mt, rmr)
            P = exp2_cr32(h(Sr - nmr[:, None]))
            sp = f(exp2_cr32(h(rmr - nmr)) / 127.0)
            with np.errstate(divide="ignore", invalid="ignore"):
                Pir = np.where(sp[:, None] > 0, np.trunc(f(P / np.where(sp > 0, sp, 1.0)[:, None])), 0.0)
            w = exp2_cr32(nmr - m)          # reference units (nmr) -> ours (m)
            ltr = f(P.sum(1)) * w
            cpvr = f(sp * float(sv[t])) * w
            Pi = np.where(lit[:, None], Pir, Pi)
            lt = np.where(lit, ltr, lt)
            cpv = np.where(lit, cpvr, cpv)
            mt = np.where(lit, nmr, np.maximum(mt, rm))
        else:
            mt = np.maximum(mt, rm)
        lrow += lt
        O += (Pi @ vi[ks].astype(np.float64)) * cpv[:, None]
    for w_ in range(nw):   # the deferred vote on the final row sums
        rs = slice(w_ * wave, (w_ + 1) * wave)
        for cd in cands[w_]:
            if np.any(cd["er"] * cd["scale"] * K > lrow[rs]):
                nredo += 1
                O[rs] += (cd["litO"] - cd["fastO"]) * cd["scale"][:, None]
                lrow[rs] += (cd["litl"] - cd["fastl"]) * cd["scale"]
    if lse_from_mt:
        lref = f(lrow * exp2_cr32(m - mt))
        lse = h(mt + h(np.log2(lref)))
    else:
        lse = h(m + h(np.log2(lrow)))
    return h(O / lrow[:, None]), lse, nlit / (S // wave * nt)


def emulate_fwd(q, k, v, **kw):
    """Like R.int8_fwd (non-causal): returns (O [B,H,S,D] f64, lse [N], literal fraction)."""
    B, H, S, D = q.shape
    Hkv, Sk = k.shape[1], k.shape[2]
    G = H // Hkv
    qi, sq = R.quant_blocks(q.reshape(B * H, S, D))
    ki, sk = R.quant_blocks(k.reshape(B * Hkv, Sk, D))
    vi, sv = R.quant_blocks(v.reshape(B * Hkv, Sk, D))
    qks = R.qk_scale(D)
    Os, ls, fr = [], [], []
    for bh in range(B * H):
        kv = bh // G
        o, l, fl = emulate(qi[bh].numpy().astype(np.int64), sq[bh].numpy(), ki[kv].numpy().astype(np.int64),
                           sk[kv].numpy(), vi[kv].numpy().astype(np.int64), sv[kv].numpy(), qks, **kw)
        Os.append(o)
        ls.append(l)
        fr.append(fl)
    return np.stack(Os).reshape(B, H, S, D), np.concatenate(ls), float(np.mean(fr))


def _ulp16(x):
    return 2.0 ** (math.floor(math.log2(max(1.0, x))) - 10)


def study(name, q, k, v, Ks, vs=1.0):
    ref = R.int8_fwd(q, k, v)
    Or, lr = ref[0].double().numpy(), ref[1].double().numpy()
    ulp = _ulp16(np.abs(lr).max())
    for K in Ks:
        for lm in (False, True):
            O, l, fr = emulate_fwd(q, k, v, K=K, lse_from_mt=lm)
            dO = np.abs(O - Or).max() / vs
            dl = np.abs(l - lr).max() / ulp
            print(f"{name:34s} K={str(K):5s} lse_mt={int(lm)}  |dO|/vs {dO:.2e}  |dlse| {dl:.1f} ulp  "
                  f"literal tiles {100 * fr:.1f} %")


def main():
    Ks = [None, 0, 2, 4, 8, 16]
    g = torch.Generator().manual_seed(44)
    S = 256
    for D in (128, 64):
        g = torch.Generator().manual_seed(44)
        ramp = (1.0 + torch.arange(S, dtype=torch.float32) / 24.0).view(1, 1, S, 1)
        k = (torch.randn((1, 2, S, D), generator=g) * ramp).half()
        for qn, q in (("q=k", k.clone()), ("q rand*2", (torch.randn((1, 2, S, D), generator=g) * 2.0).half())):
            v = torch.randn((1, 2, S, D), generator=g).half()
            study(f"peaked D={D} {qn}", q, k, v, Ks)
    # test_zero_and_constant_inputs: q = k random, v constant
    g = torch.Generator(device="cpu").manual_seed(41)
    k = torch.randn((1, 2, 256, 128), generator=g).half()
    study("q=k, v=0.75", k, k, torch.full_like(k, 0.75), Ks)
    # the non-causal fuzz cases of tests/test_gpu_fuzz.py
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
    from test_gpu_fuzz import _case
    for i in range(24):
        q, k, v, causal = _case(i)
        if causal:
            continue
        vs = max(1.0, v.float().abs().max().item() / 4)
        study(f"fuzz {i} {tuple(q.shape)} Sk={k.shape[2]}", q, k, v, [None, 4, 8, 16], vs)
    # config-3 statistics: random heads at full length (literal fraction and error)
    g = torch.Generator().manual_seed(7)
    q, k, v = (torch.randn((1, 1, 4096, 128), generator=g).half() for _ in range(3))
    k = (k.float() - k.float().mean(2, keepdim=True)).half()
    study("cfg3 head (smoothed k)", q, k, v, [None, 4, 8, 16])


if __name__ == "__main__":
    main()
