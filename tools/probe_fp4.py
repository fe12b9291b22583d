"""Probe the gfx950 MX-FP4 MFMA operand layout and the scaled fp4 converts (dev tool)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd import _lib  # noqa: E402

FP4 = np.array([0, 0.5, 1, 1.5, 2, 3, 4, 6, -0.0, -0.5, -1, -1.5, -2, -3, -4, -6], dtype=np.float64)
P = _lib.ptr
st = _lib.stream_of(torch.zeros(1, device="cuda"))
rng = np.random.default_rng(0)

# ---- converts: which way does the scale act?
x = rng.uniform(-8, 8, 512).astype(np.float32)
s = np.array([2.0 ** rng.integers(-2, 3) for _ in range(64)], dtype=np.float32)
xt, sct = torch.tensor(x, device="cuda"), torch.tensor(s, device="cuda")
packed = torch.zeros(64, dtype=torch.int32, device="cuda")
back = torch.zeros(512, dtype=torch.float32, device="cuda")
_lib.call("qattn_probe_fp4_cvt", P(xt), P(sct), P(packed), P(back), st)
torch.cuda.synchronize()
pk = packed.cpu().numpy().view(np.uint32)
nib = np.array([(pk[i] >> (4 * j)) & 15 for i in range(64) for j in range(8)])
vals = FP4[nib]
sc = np.repeat(s, 8)


def rne_fp4(v):
    mags = np.array([0, 0.5, 1, 1.5, 2, 3, 4, 6])
    out = []
    for t in v:
        a = min(abs(t), 6.0)
        d = np.abs(mags - a)
        best = np.flatnonzero(d == d.min())
        if len(best) > 1:   # tie: even mantissa (indices 0, 2, 4, 6 have mantissa bit 0)
            best = [b for b in best if b % 2 == 0]
        out.append(np.copysign(mags[best[0]], t))
    return np.array(out)


for name, scaled in (("x / s", x / sc), ("x * s", x * sc)):
    print(f"cvt hypothesis code = rne(sat({name})): matches {np.mean(rne_fp4(scaled) == np.abs(vals) * np.sign(vals) + 0 * vals):.4f}"
          f"  (nibble value == rne: {np.mean(np.isclose(rne_fp4(scaled), vals)):.4f})")
bk = back.cpu().numpy()
print("decode: back == code * s:", np.allclose(bk, vals * sc), " back == code / s:", np.allclose(bk, vals / sc))

# ---- block-scaled MFMA: A 32x64, B 64x32 in fp4 with one scale per (row, 32-k block)
A = rng.integers(0, 16, (32, 64))
B = rng.integers(0, 16, (64, 32))
ea = rng.integers(124, 131, (32, 2))     # e8m0 exponents
eb = rng.integers(124, 131, (2, 32))
Af = FP4[A] * 2.0 ** (np.repeat(ea, 32, axis=1) - 127)
Bf = FP4[B] * 2.0 ** (np.repeat(eb, 32, axis=0) - 127)
ref = Af @ Bf


def pack_rows(M):  # 32 nibbles -> 16 bytes, low nibble first
    b = M[:, 0::2] | (M[:, 1::2] << 4)
    return b.astype(np.uint8)


lanesA = np.zeros((64, 16), np.uint8)
lanesB = np.zeros((64, 16), np.uint8)
sa = np.zeros(64, np.uint32)
sb = np.zeros(64, np.uint32)
for l in range(64):
    r, h = l & 31, l >> 5
    lanesA[l] = pack_rows(A[r:r + 1, 32 * h:32 * h + 32])[0]
    lanesB[l] = pack_rows(B[32 * h:32 * h + 32, r][None, :])[0]
    sa[l] = ea[r, h]
    sb[l] = eb[h, r]
At = torch.tensor(lanesA.view(np.int32), device="cuda")
Bt = torch.tensor(lanesB.view(np.int32), device="cuda")
C = torch.zeros((64, 16), dtype=torch.float32, device="cuda")
_lib.call("qattn_probe_mfma_fp4", P(At), P(Bt), P(torch.tensor(sa.view(np.int32), device="cuda")),
          P(torch.tensor(sb.view(np.int32), device="cuda")), P(C), st)
torch.cuda.synchronize()
Cn = C.cpu().numpy()
got = np.zeros((32, 32))
for l in range(64):
    for rg in range(16):
        got[(rg & 3) + 8 * (rg >> 2) + 4 * (l >> 5), l & 31] = Cn[l, rg]
print("MFMA layout hypothesis (A[l&31][32(l>>5)+j], B[32(l>>5)+j][l&31], nibble j low-first, "
      "scale byte 0 = e8m0 of the lane's block):", np.allclose(got, ref), "max err", np.abs(got - ref).max())

# ---- hypothesis search with random e8m0 scales: data map (lane half h, nibble j -> k) x scale
# provider (the scale of row/col r, 32-k block b is byte 0 of lane r + 32*b)
maps = {
    "32h+j": lambda h, j: 32 * h + j,
    "2j+h": lambda h, j: 2 * j + h,
    "16(j>>3)+8h+(j&7)": lambda h, j: 16 * (j >> 3) + 8 * h + (j & 7),
    "32(j>>4)+16h+(j&15)": lambda h, j: 32 * (j >> 4) + 16 * h + (j & 15),
    "8(j>>2)+4h+(j&3)": lambda h, j: 8 * (j >> 2) + 4 * h + (j & 3),
    "4(j>>1)+2h+(j&1)": lambda h, j: 4 * (j >> 1) + 2 * h + (j & 1),
}
A = rng.integers(0, 16, (32, 64))
B = rng.integers(0, 16, (64, 32))
ea = rng.integers(124, 131, (32, 2))
eb = rng.integers(124, 131, (2, 32))
sa = np.zeros(64, np.uint32)
sb = np.zeros(64, np.uint32)
for l in range(64):
    sa[l] = ea[l & 31, l >> 5]
    sb[l] = eb[l >> 5, l & 31]
sat = torch.tensor(sa.view(np.int32), device="cuda")
sbt = torch.tensor(sb.view(np.int32), device="cuda")
ref = (FP4[A] * 2.0 ** (np.repeat(ea, 32, axis=1) - 127)) @ (FP4[B] * 2.0 ** (np.repeat(eb, 32, axis=0) - 127))
for mname, m in maps.items():
    lanesA = np.zeros((64, 32), np.int64)
    lanesB = np.zeros((64, 32), np.int64)
    for l in range(64):
        r, h = l & 31, l >> 5
        for j in range(32):
            lanesA[l, j] = A[r, m(h, j)]
            lanesB[l, j] = B[m(h, j), r]
    pack = lambda L: (L[:, 0::2] | (L[:, 1::2] << 4)).astype(np.uint8)  # noqa: E731
    At = torch.tensor(np.ascontiguousarray(pack(lanesA)).view(np.int32), device="cuda")
    Bt = torch.tensor(np.ascontiguousarray(pack(lanesB)).view(np.int32), device="cuda")
    C = torch.zeros((64, 16), dtype=torch.float32, device="cuda")
    _lib.call("qattn_probe_mfma_fp4", P(At), P(Bt), P(sat), P(sbt), P(C), st)
    torch.cuda.synchronize()
    Cn = C.cpu().numpy()
    got = np.zeros((32, 32))
    for l in range(64):
        for rg in range(16):
            got[(rg & 3) + 8 * (rg >> 2) + 4 * (l >> 5), l & 31] = Cn[l, rg]
    print(f"scaled map {mname:24s}: match {np.allclose(got, ref)}  max err {np.abs(got - ref).max():.3g}")
