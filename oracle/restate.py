"""CPU restatement of selau642/QuantizedAttention's attention kernels.

TEST INFRASTRUCTURE ONLY.  Nothing in ``quantizedattention_amd`` may import this module: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and only as
the checker / reported CPU baseline, never as a product path.

Every function restates one reference kernel with eager-torch rounding points made explicit
(SURVEY.md Appendix A).  Citations are ``file:line`` in the reference tree
(selau642/QuantizedAttention @ 2026-01-30).

Parity status
-------------
The reference kernels cannot run here: every module imports ``helion`` (not installed, not
installable offline), and stand-ins for absent libraries are not used.  This restatement is
therefore pinned only by (a) the reference's own published test statistics (attention_jvp.py:
305-317, attention_bf16.py:563), checked in ``tests/test_oracle.py``, and (b) the reference's
own fp32 oracle ``baseline_pytorch_attention`` (restated below).  Bit-level parity with the
reference's kernels is **unpinned** (DESIGN.md §3).  The survey probe found
this rounding contract bit-identical to the reference run eagerly; that probe is not re-run here.

Deliberate deviations from the literal reference (the build contract):
* int8 forward attends per (batch, head) (reference flattens B·H·S, finding F2).
* backward kernels use dS = P∘(dP−D) and sm_scale, accumulate deterministically (F3/F4).
* sage_attention_3_int8 smoothing uses mean over tokens (reference crashes, F1).
"""
from __future__ import annotations

import math

import torch

LOG2E_LITERAL = 1.44269504  # bf16:190, int8:153, jvp:125
BF16_1EM3 = float(torch.tensor(1e-3).bfloat16())  # eager `bf16 - 1e-3` rounds the scalar to bf16 first


def qk_scale(head_dim: int) -> float:
    """fp32 value of ``sm_scale * 1.44269504`` as multiplied into fp32/bf16 tensors (bf16:188-190)."""
    return float(torch.tensor(1.0 / math.sqrt(head_dim) * LOG2E_LITERAL, dtype=torch.float32))


def sm_scale(head_dim: int) -> float:
    return float(torch.tensor(1.0 / math.sqrt(head_dim), dtype=torch.float32))


def _bf(x):
    return x.to(torch.bfloat16)


def _h(x):
    return x.to(torch.float16)


def _f(x):
    return x.to(torch.float32)


def _exp2(x):
    """fp32 exp2 correctly rounded: float64 exp2 rounded once to fp32.

    The int8 chains evaluate exp2 only at fp16 arguments (f16 differences, int8:211-237, 360), and on
    every fp16 argument the float64 value lies at least 2^-39 (relative) from an fp32 rounding
    midpoint (tools/exp2_probe.py), far beyond float64 exp2's error: the rounding is exact.  The
    reference's torch.exp2 is whatever its platform computes (within an ulp); that last ulp decides
    trunc(P / sp) between 126 and 127 for a tile's maximum key (tests/test_oracle_sensitivity.py), so
    the restatement pins the exact value, and the HIP kernels compute the same one."""
    return torch.exp2(_f(x).double()).float()


# --------------------------------------------------------------------------------------------
# A8: the reference's own fp32 oracle (bf16:450-478 == int8:453-481; jvp:197-215 is causal=False)
# --------------------------------------------------------------------------------------------
def baseline_pytorch_attention(q, k, v, head_dim=None, causal=False):
    """fp32 matmul/sqrt(D) -> strict-lower causal fill -128*ln2 -> softmax -> matmul (bf16:450-478)."""
    if head_dim is None:
        head_dim = q.shape[-1]
    p = torch.matmul(q, k.transpose(2, 3)) / math.sqrt(head_dim)
    if causal:
        qn, kn = p.shape[-2], p.shape[-1]
        mask = torch.arange(qn, device=q.device)[:, None] - torch.arange(kn, device=q.device)[None, :]
        p = torch.where(mask[None, None] > 0, p, -128 * torch.log(torch.tensor([2.0], device=q.device)))
    p = torch.softmax(p.to(torch.float32), dim=-1).to(torch.float32)
    return torch.matmul(p, v)


# --------------------------------------------------------------------------------------------
# A1: bf16 forward with the "multiple-max" beta rule (bf16:107-296), Appendix A.1
# --------------------------------------------------------------------------------------------
def bf16_fwd(q, k, v, causal=False, kt=16):
    """Restates helion_atten_bf16_fwd_training (bf16:111-296).

    q, k fp16 [B,H,S,D]; v bf16 [B,H,Sk,D].  Returns (O fp32 [B,H,S,D], lse fp32 [B*H,S]).
    ``kt`` is the k-tile width the beta rule is applied at (reference default unpinned, F8; the
    only pinned config, bf16:736, uses 16).
    """
    if k.shape[1] != q.shape[1]:   # grouped-query attention (N2 extension): expand k/v heads
        G = q.shape[1] // k.shape[1]
        k, v = k.repeat_interleave(G, dim=1), v.repeat_interleave(G, dim=1)
    B, H, S, D = q.shape
    Sk = k.shape[2]
    BH = B * H
    qks = qk_scale(D)
    qf = _f(q.reshape(BH, S, D))
    kf = _f(k.reshape(BH, Sk, D))
    vf = _f(v.reshape(BH, Sk, D))
    m = torch.full((BH, S, 1), float("-inf"), dtype=torch.bfloat16)  # bf16:197
    l = torch.ones((BH, S, 1), dtype=torch.float32)  # bf16:198
    O = torch.zeros((BH, S, D), dtype=torch.float32)  # bf16:199
    qidx = torch.arange(S)
    neg126 = torch.tensor(-126.0, dtype=torch.bfloat16)
    zero = torch.tensor(0.0, dtype=torch.bfloat16)
    for k0 in range(0, Sk, kt):
        k1 = min(k0 + kt, Sk)
        Sb = _bf(_h(qf @ kf[:, k0:k1].transpose(1, 2)))  # bf16:215-216
        if causal:  # bf16:222-233 (tile guard begin_q<end_k is a no-op on unmasked tiles)
            mask = (qidx[:, None] - torch.arange(k0, k1)[None, :]) > 0
            Sb = torch.where(mask[None], Sb, neg126)
        nm = torch.maximum(m, _bf(_f(Sb.amax(-1, keepdim=True)) * qks))  # bf16:236-239
        thr = _bf(_f(nm) - BF16_1EM3)  # bf16:248 (scalar rounded to bf16 by eager sub)
        multi = (Sb >= thr).sum(-1, keepdim=True) > 1  # bf16:248-250
        nm = torch.where(multi & (nm > 0), _bf(2.0 * _f(nm)), nm)  # bf16:252-256
        nm = torch.where(multi & (nm < 0), zero, nm)  # bf16:258-264
        Sp = _bf(_f(_bf(_f(Sb) * qks)) - _f(nm))  # bf16:267
        P = _bf(torch.exp2(_f(Sp)))  # bf16:269
        lt = _f(P).sum(-1, keepdim=True)  # bf16:274
        r = _bf(torch.exp2(_f(_bf(_f(m) - _f(nm)))))  # bf16:276
        m = nm
        l = l * _f(r) + lt  # bf16:279
        O = O * _f(r)  # bf16:280
        O = O + _f(P) @ vf[:, k0:k1]  # bf16:285
    lse = _f(m).squeeze(-1) + torch.log2(l).squeeze(-1)  # bf16:288
    O = O / l  # bf16:293
    return O.view(B, H, S, D), lse


# --------------------------------------------------------------------------------------------
# A3 (build contract): corrected FA2 backward in fp32 (bf16:299-448 with F3 fixed)
# --------------------------------------------------------------------------------------------
def bf16_bwd(q, k, v, O, lse, causal, dO):
    """Grouped-query wrapper (N2 extension): expand k/v to the query heads, sum dk/dv per group."""
    Hq, Hkv = q.shape[1], k.shape[1]
    if Hkv == Hq:
        return _bf16_bwd_heads(q, k, v, O, lse, causal, dO)
    G = Hq // Hkv
    dq, dk, dv = _bf16_bwd_heads(q, k.repeat_interleave(G, dim=1), v.repeat_interleave(G, dim=1), O, lse,
                                 causal, dO)
    B, _, Sk, D = dk.shape
    return dq, dk.view(B, Hkv, G, Sk, D).sum(2), dv.view(B, Hkv, G, Sk, D).sum(2)


def _bf16_bwd_heads(q, k, v, O, lse, causal, dO):
    """Corrected restatement of helion_flash_atten_2_algo_4_bwd (bf16:309-448).

    Same inputs/outputs as the reference (fp32 grads).  Fixes: dS = P*(dP-D) instead of
    S*(dP-D) (bf16:421); scale sm_scale instead of qk_scale (bf16:428-441).  The causal fill stays
    the reference's -128 in scaled units (bf16:379-389).
    """
    B, H, S, D = q.shape
    Sk = k.shape[2]
    BH = B * H
    qks = qk_scale(D)
    sms = sm_scale(D)
    qf = _f(q).reshape(BH, S, D)  # bf16:342-344
    kf = _f(k).reshape(BH, Sk, D)
    vf = _f(v).reshape(BH, Sk, D)
    Of = _f(O).reshape(BH, S, D)
    dOf = _f(dO).reshape(BH, S, D)
    St = qks * (qf @ kf.transpose(1, 2))  # bf16:376-377
    if causal:
        mask = (torch.arange(S)[:, None] - torch.arange(Sk)[None, :]) > 0
        St = torch.where(mask[None], St, torch.tensor(-128.0))
    P = torch.exp2(St - lse.reshape(BH, S, 1))  # bf16:392
    dv = P.transpose(1, 2) @ dOf  # bf16:399
    dP = dOf @ vf.transpose(1, 2)  # bf16:405
    Dr = (dOf * Of).sum(-1, keepdim=True)  # bf16:416
    dS = P * (dP - Dr)  # corrected bf16:421
    dq = sms * (dS @ kf)  # corrected bf16:427-432
    dk = sms * (dS.transpose(1, 2) @ qf)  # corrected bf16:436-441
    return dq.view(B, H, S, D), dk.view(B, H, Sk, D), dv.view(B, H, Sk, D)


# --------------------------------------------------------------------------------------------
# A4: int8 per-block quantiser + SageAttention3-style forward (int8:97-262), Appendix A.2
# --------------------------------------------------------------------------------------------
def quant_blocks(x, block=32):
    """Per-block int8 quantisation exactly as int8:180-183 / 190-194 / 242-246 in eager torch.

    x: fp16 [..., N, D] with N % block == 0.  Returns (idx int8 [..., N, D], scale fp16 [..., N/block]).
    s = RNE_fp16(fp32(amax|X|) / 127); idx = trunc(RNE_fp16(fp32(x) / fp32(s))).  An all-zero block
    (s == 0, where the reference divides 0/0) quantises to idx 0 (build-defined edge case).
    """
    *lead, N, D = x.shape
    assert N % block == 0
    xb = x.reshape(*lead, N // block, block * D)
    amax = xb.abs().amax(-1)  # exact in fp16
    s = _h(_f(amax) / 127.0)
    q = _f(_h(_f(xb) / _f(s)[..., None]))
    q = torch.where(s[..., None] == 0, torch.zeros_like(q), q)
    idx = torch.trunc(q).to(torch.int8)
    return idx.reshape(*lead, N, D), s


def int8_fwd(q, k, v, block=32, causal=False, causal_offset=0):
    """Per-(batch, head) restatement of helion_atten_int8_hl_dot_fwd (int8:101-262).

    q, k, v fp16 [B,H,S,D], S % 32 == 0.  Returns the reference's 10-tuple
    (O fp16 [B,H,S,D], lse fp16 [N], q_i8 [N,D], k_i8T [D,N], v_i8 [N,D], sq, sk, sv fp16 [N/32],
    Bq, Bkv) with N = B*H*S and block index (b*H+h)*S/32 + s/32 (int8:161-168).  Attention is per
    (b, h) (build contract); quantisation is identical to the flattened reference
    whenever S % 32 == 0.

    Extensions (no reference counterpart): k, v may have Hkv = H / G heads (query
    head h reads key/value head h // G) and Sk != S tokens; ``causal`` drops key > query (top-left
    aligned) by excluding those scores (P = 0; a tile with no kept key has sp = 0);
    ``causal_offset`` shifts the diagonal (query i keeps keys <= i + causal_offset: Sk - Sq aligns the
    last query with the last key, the key/value-cache decode of SURVEY §8f N3).
    """
    B, H, S, D = q.shape
    Hkv, Sk = k.shape[1], k.shape[2]
    G = H // Hkv
    BH = B * H
    qks = qk_scale(D)
    qi, sq = quant_blocks(q.reshape(BH, S, D), block)  # int8:178-186
    ki_kv, sk_kv = quant_blocks(k.reshape(B * Hkv, Sk, D), block)  # int8:188-195
    vi_kv, sv_kv = quant_blocks(v.reshape(B * Hkv, Sk, D), block)  # int8:241-247
    kvh = torch.arange(BH) // G  # key/value head of each query head
    ki, sk, vi, sv = ki_kv[kvh], sk_kv[kvh], vi_kv[kvh], sv_kv[kvh]
    nq = S // block
    O = torch.zeros((BH, S, D), dtype=torch.float32)  # int8:172
    l = torch.ones((BH, S, 1), dtype=torch.float32)  # int8:173
    m = torch.full((BH, S, 1), float("-inf"), dtype=torch.float16)  # int8:174
    qd = qi.double()
    sqf = _f(sq).repeat_interleave(block, dim=1)[..., None]  # per-row view of the q block scale
    for t in range(Sk // block):
        k0, k1 = t * block, (t + 1) * block
        acc = _f(qd @ ki[:, k0:k1].double().transpose(1, 2))  # int8:197 (exact integer dot)
        Sf = ((acc * sqf) * _f(sk[:, t])[:, None, None]) * qks  # int8:200
        S16 = _h(Sf)  # int8:203
        if causal:
            keep = torch.arange(k0, k1)[None, :] <= torch.arange(S)[:, None] + causal_offset
            S16 = torch.where(keep[None], S16, torch.full_like(S16, float("-inf")))
        rm = S16.amax(-1, keepdim=True)  # int8:205
        nm = torch.maximum(m, rm)  # int8:206-209
        P = _exp2(_h(_f(S16) - _f(nm)))  # int8:211-213
        lt = P.sum(-1, keepdim=True)  # int8:215
        r = _exp2(_h(_f(m) - _f(nm)))  # int8:217-219
        m = nm  # int8:221
        l = l * r + lt  # int8:223
        O = O * r  # int8:225
        sp = _exp2(_h(_f(rm) - _f(m))) / 127  # int8:232-234
        Pi = torch.where(sp > 0, torch.trunc(P / torch.where(sp > 0, sp, 1.0)), 0.0)  # int8:236-237
        pv = _f(Pi.double() @ vi[:, k0:k1].double())  # int8:249
        O = O + (pv * sp) * _f(sv[:, t])[:, None, None]  # int8:249-250
    lse = _h(_f(m.squeeze(-1)) + _f(_h(torch.log2(l).squeeze(-1))))  # int8:252
    Oh = _h(O / l)  # int8:256-257
    N = BH * S
    Nkv = B * Hkv * Sk
    return (Oh.view(B, H, S, D), lse.reshape(N), qi.reshape(N, D), ki_kv.reshape(Nkv, D).t(),
            vi_kv.reshape(Nkv, D), sq.reshape(-1), sk_kv.reshape(-1), sv_kv.reshape(-1), block, block)


def k_smooth(k):
    """SageAttention k-smoothing (build contract for int8:24-25, which crashes, F1).

    k_mean = fp16(mean over tokens) [B,H,1,D]; k_s = fp16(k - k_mean).
    """
    km = _h(_f(k).mean(dim=-2, keepdim=True))
    return _h(_f(k) - _f(km)), km


def int8_bwd(dO, q_i8, sq, k_i8T, k_mean, sk, v_i8, sv, O, lse, Bq=32, Bkv=32, causal=False,
             kv_heads=None):
    """Corrected per-(b,h) restatement of helion_atten_int8_hl_dot_bwd (int8:268-432).

    Follows the reference's quantisation recipe (P and dS per Bq x Bkv tile, dO per Bq-row block,
    q/k/v int8 from the forward) with the build-contract fixes: dS = P*(dP-D)
    (int8:399), sm_scale (int8:417,424), per-(b,h) accumulation of dq/dk/dv in fp32 over all tiles
    (int8:420,427,428 overwrite / race), no k_mean term (int8:408-410; it multiplies rowsum(dS)=0).
    Returns fp16 dq, dk, dv [B,H,S,D].  Extensions as int8_fwd: key/value heads ``kv_heads`` (default
    k_mean's, else H; dk, dv of a key/value head sum over its query heads in fp32), Sk != S from
    k_i8T, ``causal`` (masked P = 0 before the tile quantisation).
    """
    B, H, S, D = O.shape
    BH = B * H
    N = BH * S
    if kv_heads is None:
        kv_heads = k_mean.shape[1] if k_mean is not None and k_mean.dim() == 4 else H
    Hkv = kv_heads
    G = H // Hkv
    Sk = k_i8T.shape[1] // (B * Hkv)
    kvh = torch.arange(BH) // G
    sms = sm_scale(D)
    qks = qk_scale(D)
    qi = q_i8.reshape(BH, S, D).double()
    ki = k_i8T.t().reshape(B * Hkv, Sk, D).double()[kvh]
    vi = v_i8.reshape(B * Hkv, Sk, D).double()[kvh]
    sq = _f(sq.reshape(BH, S // Bq))
    sk = _f(sk.reshape(B * Hkv, Sk // Bkv))[kvh]
    sv = _f(sv.reshape(B * Hkv, Sk // Bkv))[kvh]
    dOh = dO.reshape(BH, S, D)
    Oh = O.reshape(BH, S, D)
    lse = lse.reshape(BH, S)
    dq = torch.zeros((BH, S, D))
    dk = torch.zeros((BH, Sk, D))
    dv = torch.zeros((BH, Sk, D))
    dOi, sdO = quant_blocks(dOh, Bq)  # int8:372-374
    dOi = dOi.double()
    sdO = _f(sdO)
    # D = rowsum(dO*O) in fp16 (int8:398): elementwise fp16 product, fp32-accumulated sum -> fp16
    Dr = _f(_h(_f(_h(_f(dOh) * _f(Oh))).sum(-1)))
    for kt in range(Sk // Bkv):
        ks = slice(kt * Bkv, (kt + 1) * Bkv)
        for qt in range(S // Bq):
            qs = slice(qt * Bq, (qt + 1) * Bq)
            acc = _f(qi[:, qs] @ ki[:, ks].transpose(1, 2))  # int8:352
            S16 = _h(((acc * sq[:, qt, None, None]) * sk[:, kt, None, None]) * qks)  # int8:353-355
            P = _exp2(_h(_f(S16) - _f(lse[:, qs])[..., None]))  # int8:360
            if causal:
                keep = torch.arange(ks.start, ks.stop)[None, :] <= torch.arange(qs.start, qs.stop)[:, None]
                P = torch.where(keep[None], P, torch.zeros_like(P))
            sP = P.abs().flatten(1).amax(-1) / 127  # int8:363
            sP_safe = torch.where(sP == 0, torch.ones_like(sP), sP)
            Pi = torch.trunc(P / sP_safe[:, None, None]).double()  # int8:364-365
            dvt = ((_f(Pi.transpose(1, 2) @ dOi[:, qs]) * sdO[:, qt, None, None])
                   * sP[:, None, None])  # int8:375-377
            dv[:, ks] += dvt
            dP = (_f(dOi[:, qs] @ vi[:, ks].transpose(1, 2)) * sdO[:, qt, None, None]) \
                * sv[:, kt, None, None]  # int8:382-384
            dS = P * (dP - Dr[:, qs, None])  # corrected int8:399
            sdS = dS.abs().flatten(1).amax(-1) / 127  # int8:403
            sdS_safe = torch.where(sdS == 0, torch.ones_like(sdS), sdS)
            dSi = torch.trunc(dS / sdS_safe[:, None, None]).double()  # int8:404-405
            dqt = ((_f(dSi @ ki[:, ks]) * sdS[:, None, None]) * sk[:, kt, None, None]) * sms
            dq[:, qs] += dqt  # int8:416-420 (sm_scale, fp32 accumulation, no k_mean term)
            dkt = ((_f(dSi.transpose(1, 2) @ qi[:, qs]) * sdS[:, None, None])
                   * sq[:, qt, None, None]) * sms
            dk[:, ks] += dkt  # int8:423-427
    dk = dk.view(B * Hkv, G, Sk, D).sum(1)
    dv = dv.view(B * Hkv, G, Sk, D).sum(1)
    return _h(dq).view(B, H, S, D), _h(dk).view(B, Hkv, Sk, D), _h(dv).view(B, Hkv, Sk, D)


# --------------------------------------------------------------------------------------------
# A7: forward-mode tangent attention (jvp:24-195), Appendix A.3
# --------------------------------------------------------------------------------------------
def jvp_fwd(q, k, v, tq, tk, tv, kt=16):
    """Restates helion_attention_jvp_forward_fp32 (jvp:33-195) in fp32 (non-causal)."""
    B, H, S, D = q.shape
    Sk = k.shape[2]
    BH = B * H
    qks = qk_scale(D)
    sms = 1.0 / math.sqrt(D)  # jvp:123 (python double, rounded where multiplied into fp32)
    qf, tqf = _f(q).reshape(BH, S, D), _f(tq).reshape(BH, S, D)
    kf, tkf = _f(k).reshape(BH, Sk, D), _f(tk).reshape(BH, Sk, D)
    vf, tvf = _f(v).reshape(BH, Sk, D), _f(tv).reshape(BH, Sk, D)
    m = torch.full((BH, S, 1), float("-inf"))  # jvp:130
    l = torch.zeros((BH, S, 1))  # jvp:131
    O = torch.zeros((BH, S, D))
    r = torch.zeros((BH, S, 1))
    A = torch.zeros((BH, S, D))
    Bacc = torch.zeros((BH, S, D))
    for k0 in range(0, Sk, kt):
        ks = slice(k0, min(k0 + kt, Sk))
        kT, tkT = kf[:, ks].transpose(1, 2), tkf[:, ks].transpose(1, 2)
        St = qf @ kT  # jvp:148
        tS = ((tqf @ kT) + (qf @ tkT)) * sms  # jvp:149-153
        nm = torch.maximum(m, St.amax(-1, keepdim=True) * qks)  # jvp:155-158
        P = torch.exp2(St * qks - nm)  # jvp:160-161
        lt = P.sum(-1, keepdim=True)  # jvp:162
        rs = torch.exp2(m - nm)  # jvp:164
        l = l * rs + lt  # jvp:165
        m = nm
        O = O * rs + P @ vf[:, ks]  # jvp:167-171
        A = A * rs + P @ tvf[:, ks]  # jvp:173-174
        Hm = P * tS  # jvp:176
        r = r * rs + Hm.sum(-1, keepdim=True)  # jvp:178
        Bacc = Bacc * rs + Hm @ vf[:, ks]  # jvp:180-181
    lse = m.squeeze(-1) + torch.log2(l).squeeze(-1)  # jvp:183
    Of = O / l  # jvp:188
    tO = (A + Bacc - r * Of) / l  # jvp:190
    return Of.view(B, H, S, D), tO.view(B, H, S, D), lse


# --------------------------------------------------------------------------------------------
# Truth references used for gradient / tangent parity (fp32 autograd of A8)
# --------------------------------------------------------------------------------------------
def attention_grads_truth(q, k, v, dO, causal=False):
    """fp32 autograd gradients of baseline_pytorch_attention (the reference tests' truth)."""
    qf, kf, vf = (_f(t).detach().clone().requires_grad_(True) for t in (q, k, v))
    out = baseline_pytorch_attention(qf, kf, vf, q.shape[-1], causal)
    out.backward(_f(dO))
    return qf.grad, kf.grad, vf.grad


def jvp_truth(q, k, v, tq, tk, tv):
    """torch.func.jvp of the non-causal baseline (jvp:254-258)."""
    f = lambda a, b, c: baseline_pytorch_attention(a, b, c, None, False)
    return torch.func.jvp(f, (_f(q), _f(k), _f(v)), (_f(tq), _f(tk), _f(tv)))
