"""Generate the committed golden fixtures under tests/golden/ (run from the repo root):

    python tests/golden/gen_golden.py

Fixtures are DATA (seeded inputs and expected outputs), produced by:
  * ``quant_kat.json`` — known-answer vectors for the int8 block quantiser (attention_int8.py:180-183,
    190-194, 242-246) computed by an independent numpy implementation below (explicit float32 divide,
    round-to-nearest-even to float16, truncate toward zero).  It shares no code with oracle/restate.py,
    so the test that compares the two pins the oracle's quantiser.
  * ``oracle_small.pt`` — seeded small-shape inputs with the outputs of oracle/restate.py (the CPU
    restatement) for every hot-path function: a regression anchor for the oracle and the fixed
    vectors the GPU parity tests check the HIP kernels against.

The reference kernels themselves cannot run here (they import ``helion``, which is absent), so no
fixture holds reference-kernel output; see DESIGN.md §3 ("parity pinning").
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import restate as R  # noqa: E402


def np_quant(x16: np.ndarray, block: int = 32):
    """Independent numpy quantiser: x16 float16 [N, D] -> (idx int8 [N, D], scale float16 [N/block])."""
    n, d = x16.shape
    idx = np.zeros((n, d), dtype=np.int8)
    sc = np.zeros(n // block, dtype=np.float16)
    for b in range(n // block):
        blk = x16[b * block:(b + 1) * block]
        amax = np.float32(np.abs(blk).max())
        s = np.float16(amax / np.float32(127.0))
        sc[b] = s
        if s == 0:
            continue
        q = (blk.astype(np.float32) / np.float32(s)).astype(np.float16).astype(np.float32)
        idx[b * block:(b + 1) * block] = np.trunc(q).astype(np.int8)
    return idx, sc


def quant_kats():
    rng = np.random.default_rng(7)
    cases = []
    # 1: plain gaussian block
    cases.append(("gaussian", rng.standard_normal((32, 64)).astype(np.float16)))
    # 2: values exactly at multiples of the scale and half-way points (truncation vs rounding)
    s = np.float16(1.0 / 127.0)
    base = np.arange(-63, 65, dtype=np.float32)[None, :].repeat(32, 0)[:, :64]
    x = (base * np.float32(s) + np.float32(s) * np.float32(0.5)).astype(np.float16)
    x[0, 0] = np.float16(1.0)
    cases.append(("halfway", x))
    # 3: all-zero block (reference divides 0/0; build-defined idx 0, scale 0)
    cases.append(("zeros", np.zeros((32, 64), dtype=np.float16)))
    # 4: one large outlier, rest tiny (scale dominated by the outlier; most idx 0)
    x = (rng.standard_normal((32, 64)) * 1e-3).astype(np.float16)
    x[5, 17] = np.float16(-300.0)
    cases.append(("outlier", x))
    # 5: fp16 extremes and subnormals
    x = np.zeros((32, 64), dtype=np.float16)
    x[0, :8] = np.array([65504, -65504, 6e-8, -6e-8, 1e-4, -1e-4, 3.14, -2.71], dtype=np.float16)
    cases.append(("extremes", x))
    # 6: two blocks, D=128
    cases.append(("two_blocks_d128", rng.standard_normal((64, 128)).astype(np.float16) * np.float16(4)))
    out = []
    for name, x in cases:
        idx, sc = np_quant(x)
        out.append({"name": name, "shape": list(x.shape),
                    "x_f16_bits": x.view(np.uint16).ravel().tolist(),
                    "idx": idx.ravel().tolist(), "scale_f16_bits": sc.view(np.uint16).tolist()})
    return out


def oracle_small():
    g = torch.Generator().manual_seed(2024)
    rnd = lambda *s: torch.randn(s, generator=g)  # noqa: E731
    fx = {}
    # int8 forward, (1,2,128,64) and (1,2,64,128), plain and k-smoothed
    for tag, shape in (("i8a", (1, 2, 128, 64)), ("i8b", (1, 2, 64, 128))):
        q, k, v = (rnd(*shape).half() for _ in range(3))
        fx[f"{tag}.q"], fx[f"{tag}.k"], fx[f"{tag}.v"] = q, k, v
        out = R.int8_fwd(q, k, v)
        for n, t in zip(("O", "lse", "q_i8", "k_i8T", "v_i8", "sq", "sk", "sv"), out[:8]):
            fx[f"{tag}.{n}"] = t.contiguous()
        ks, km = R.k_smooth(k)
        outs = R.int8_fwd(q, ks, v)
        fx[f"{tag}.smooth.O"] = outs[0].contiguous()
        fx[f"{tag}.smooth.k_mean"] = km.contiguous()
        dO = (rnd(*shape) * 0.1).half()
        fx[f"{tag}.dO"] = dO
        dq, dk, dv = R.int8_bwd(dO, outs[2], outs[5], outs[3], km, outs[6], outs[4], outs[7],
                                outs[0], outs[1])
        fx[f"{tag}.smooth.dq"], fx[f"{tag}.smooth.dk"], fx[f"{tag}.smooth.dv"] = dq, dk, dv
    # bf16 forward (beta rule at KT=16) + corrected backward, (1,2,128,64), causal and not
    q, k, v = (rnd(1, 2, 128, 64) for _ in range(3))
    fx["bf.q"], fx["bf.k"], fx["bf.v"] = q.half(), k.half(), v.bfloat16()
    dO = rnd(1, 2, 128, 64)
    fx["bf.dO"] = dO
    for c in (0, 1):
        O, lse = R.bf16_fwd(q.half(), k.half(), v.bfloat16(), bool(c), kt=16)
        fx[f"bf.c{c}.O"], fx[f"bf.c{c}.lse"] = O.contiguous(), lse.contiguous()
        dq, dk, dv = R.bf16_bwd(q.half(), k.half(), v.bfloat16(), O, lse, bool(c), dO)
        fx[f"bf.c{c}.dq"], fx[f"bf.c{c}.dk"], fx[f"bf.c{c}.dv"] = dq, dk, dv
    # jvp (1,2,64,64), randn tangents
    ts = [rnd(1, 2, 64, 64) for _ in range(6)]
    for n, t in zip(("q", "k", "v", "tq", "tk", "tv"), ts):
        fx[f"jvp.{n}"] = t
    O, tO, lse = R.jvp_fwd(*ts)
    fx["jvp.O"], fx["jvp.tO"], fx["jvp.lse"] = O, tO, lse
    return fx


def main():
    with open(os.path.join(HERE, "quant_kat.json"), "w") as f:
        json.dump(quant_kats(), f, separators=(",", ":"))
    torch.save(oracle_small(), os.path.join(HERE, "oracle_small.pt"))
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
