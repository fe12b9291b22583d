"""CPU restatement of the MX-FP4 attention forward.

TEST INFRASTRUCTURE ONLY -- imported by ``tests/`` alone, as the checker.

The reference names SageAttention3's FP4 path (README.md:49-55) but contains no FP4 kernel, so
there is nothing in it to restate: this module restates the definition the HIP kernels implement
(the quantisation contract in quantizedattention_amd/csrc/mxfp4_attn.hip).  Parity
with the reference is **unpinned** (no reference FP4 outputs exist); the tests pin the kernels to
this definition (quantisers bit-exact, attention within a stated tolerance) and the definition to
exact fp32 attention (accuracy bound).

Format: OCP MX v1.0 e2m1 elements with one e8m0 power-of-two scale per block of 32:
    e = floor(log2 amax) - 2   (amax == 0: e = -127),   code = RNE(saturate(x / 2^e)) on the grid
    {0, 0.5, 1, 1.5, 2, 3, 4, 6}, ties to the even code.
"""
from __future__ import annotations

import math

import torch

E2M1 = torch.tensor([0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0], dtype=torch.float64)
LOG2E_LITERAL = 1.44269504


def qk_scale(head_dim: int) -> float:
    return float(torch.tensor(1.0 / math.sqrt(head_dim) * LOG2E_LITERAL, dtype=torch.float32))


def e8m0(amax: torch.Tensor) -> torch.Tensor:
    """Biased e8m0 byte (int64) of floor(log2 amax) - 2, clamped to [0, 254]; amax == 0 -> 0."""
    a = amax.to(torch.float32)
    _, ex = torch.frexp(a)                 # a = m * 2^ex with m in [0.5, 1): floor(log2 a) = ex - 1
    e = ex.to(torch.int64) - 1 - 2 + 127
    return torch.where(a > 0, e.clamp(0, 254), torch.zeros_like(e))


def scale_value(b: torch.Tensor) -> torch.Tensor:
    return torch.pow(2.0, b.to(torch.float64) - 127)


def rne_e2m1(y: torch.Tensor) -> torch.Tensor:
    """Nibble code (int64, sign in bit 3) of RNE(saturate(y)) on the e2m1 grid."""
    a = y.abs().to(torch.float64).clamp(max=6.0)
    d = (a[..., None] - E2M1).abs()
    best = d.min(-1, keepdim=True).values
    tie = (d == best)
    # among the tied grid points prefer the even code (mantissa bit 0): indices 0, 2, 4, 6
    even = torch.tensor([1, 0, 1, 0, 1, 0, 1, 0], dtype=torch.bool)
    pick = torch.where(tie.sum(-1, keepdim=True) > 1, tie & even, tie)
    code = pick.to(torch.int64).argmax(-1)
    return code + 8 * torch.signbit(y).to(torch.int64)   # the sign survives a zero result (-0 = 8)


def decode(code: torch.Tensor) -> torch.Tensor:
    v = E2M1[code & 7]   # code 8 (-0) decodes to 0
    return torch.where(code >= 8, -v, v)


def quant_block32(x: torch.Tensor):
    """x [..., 32] -> (codes int64 [..., 32], scale byte int64 [...])."""
    b = e8m0(x.to(torch.float32).abs().amax(-1))
    codes = rne_e2m1(x.to(torch.float64) / scale_value(b)[..., None])
    return codes, b


def pack_nibbles(codes: torch.Tensor) -> torch.Tensor:
    """[..., 2n] codes -> [..., n] uint8, element 2i in the low nibble."""
    return (codes[..., 0::2] | (codes[..., 1::2] << 4)).to(torch.uint8)


def quant_rows(x: torch.Tensor):
    """Q / K quantiser: x fp16 [rows, D] -> (packed uint8 [rows, D/2], scales uint8 [rows, D/32])."""
    rows, D = x.shape
    codes, b = quant_block32(x.reshape(rows, D // 32, 32))
    return pack_nibbles(codes.reshape(rows, D)), b.to(torch.uint8)


def vt_key_order() -> torch.Tensor:
    """[2, 32]: key (within a 64-key tile) of nibble j of half h (the S^T accumulator order)."""
    j = torch.arange(32)
    return torch.stack([32 * (j >> 4) + 8 * ((j >> 2) & 3) + 4 * h + (j & 3) for h in (0, 1)])


def quant_vt(v: torch.Tensor):
    """V quantiser: v fp16 [BH, Sk, D] -> (vt uint8 [BH, Sk/64, D, 32], vs uint8 [BH, Sk/64, D, 2])."""
    BH, Sk, D = v.shape
    ng = Sk // 64
    vg = v.reshape(BH, ng, 64, D).permute(0, 1, 3, 2)            # [BH, ng, D, 64 keys]
    blocks = vg[..., vt_key_order()]                              # [BH, ng, D, 2, 32]
    codes, b = quant_block32(blocks)
    return pack_nibbles(codes).reshape(BH, ng, D, 32), b.to(torch.uint8)


def _unpack(p: torch.Tensor) -> torch.Tensor:
    p = p.to(torch.int64)
    return torch.stack([p & 15, p >> 4], -1).reshape(*p.shape[:-1], -1)


def deq_rows(packed, scales):
    rows = packed.shape[0]
    c = decode(_unpack(packed)).reshape(rows, -1, 32)
    return (c * scale_value(scales.to(torch.int64))[..., None]).reshape(rows, -1)


def deq_vt(vt, vs):
    """-> dequantised V [BH, Sk, D] (float64)."""
    BH, ng, D, _ = vt.shape
    c = decode(_unpack(vt)).reshape(BH, ng, D, 2, 32) * scale_value(vs.to(torch.int64))[..., None]
    out = torch.zeros((BH, ng, D, 64), dtype=torch.float64)
    out[..., vt_key_order()] = c
    return out.permute(0, 1, 3, 2).reshape(BH, ng * 64, D)


def mxfp4_fwd(q, k, v, mslack=8.0):
    """q fp16 [B,H,Sq,D], k/v fp16 [B,Hkv,Sk,D] (H % Hkv == 0, Sk % 64 == 0) ->
    (O fp16 [B,H,Sq,D], lse fp32 [B*H, Sq] base 2, (q4, qs, k4, ks, vt, vs)).

    Per 64-key tile t (the kernel's order, csrc/mxfp4_attn.hip header): S = deq(Q) deq(K)^T in
    fp32; if rowmax(fp32(S * qks)) > m + mslack: m' = ceil(that max), O and l scaled by
    2^(m - m'); P = exp2(fp32(S * qks - m)) (one rounding, the kernel's fma); P is MX-quantised per
    query row in two blocks of 32 (the keys whose bit 2 is 0 / 1); l += sum(deq P);
    O += deq(P) deq(V).
    """
    B, H, Sq, D = q.shape
    Hkv, Sk = k.shape[1], k.shape[2]
    G = H // Hkv
    BH = B * H
    qks = qk_scale(D)
    q4, qs = quant_rows(q.reshape(BH * Sq, D))
    k4, ks = quant_rows(k.reshape(B * Hkv * Sk, D))
    vt, vs = quant_vt(v.reshape(B * Hkv, Sk, D))
    kvh = torch.arange(BH) // G
    dq = deq_rows(q4, qs).reshape(BH, Sq, D)
    dk = deq_rows(k4, ks).reshape(B * Hkv, Sk, D)[kvh]
    dv = deq_vt(vt, vs)[kvh]
    m = torch.full((BH, Sq, 1), float("-inf"), dtype=torch.float64)
    l = torch.zeros((BH, Sq, 1), dtype=torch.float64)
    O = torch.zeros((BH, Sq, D), dtype=torch.float64)
    order = vt_key_order()
    for t in range(Sk // 64):
        k0 = 64 * t
        acc = (dq @ dk[:, k0:k0 + 64].transpose(1, 2)).to(torch.float32)    # MFMA fp32 result
        mx = (acc * qks).amax(-1, keepdim=True).double()                   # fp32 products
        raise_ = mx > m + mslack
        nm = torch.where(raise_, torch.ceil(mx), m)
        r = torch.where(torch.isinf(m), torch.zeros_like(m), torch.pow(2.0, m - nm))
        O, l, m = O * r, l * r, nm
        # fma(acc, qks, -m): the exact value rounded once to fp32
        P = torch.exp2((acc.double() * qks - m).to(torch.float32))       # fp32 [BH, Sq, 64]
        codes, b = quant_block32(P[..., order])
        Pd = torch.zeros((BH, Sq, 64), dtype=torch.float64)
        Pd[..., order] = decode(codes) * scale_value(b)[..., None]
        l = l + Pd.sum(-1, keepdim=True)
        O = O + Pd @ dv[:, k0:k0 + 64]
    lse = (m + torch.log2(l)).squeeze(-1).to(torch.float32)
    Oh = (O / l).to(torch.float16)
    return Oh.view(B, H, Sq, D), lse, (q4, qs, k4, ks, vt, vs)
