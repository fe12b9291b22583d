"""Drive tools/ubench/mix.hip (dev tool): every wave mixes 8 MFMAs of one shape with P vector
instructions of one type after each MFMA; prints cycles per SIMD per wave-iteration at 1..4 waves
per SIMD.  Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o libmix.so mix.hip

    python tools/ubench/mix.py [ops] [shapes]     (comma lists of indices)"""
import ctypes
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libmix.so"))
lib.mix.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_int]
ops = ["v_fma_f32", "v_pk_fma_f32", "v_pk_fma_f16", "v_exp_f16", "v_pk_add_f16", "v_cvt_pk_f16_f32",
       "v_max3_i32", "v_perm_b32", "v_exp_f32", "v_pk_mul_f32", "v_fma_mix_f32", "v_mov_b32", "v_fma_mixlo_f16", "v_exp_f16_sdwa", "ds_read_b64",
       "v_add_u32", "s_nop0"]
shapes = ["i8_32x32x32", "i8_16x16x64", "f16_32x32x16", "f16_16x16x32"]
pvals = [0, 4, 8, 12, 16, 24]
sel_ops = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else range(len(ops))
sel_sh = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else range(len(shapes))
iters, nb = 200, 256
for s in sel_sh:
    for o in sel_ops:
        for pi, p in enumerate(pvals):
            if p == 0 and o != sel_ops[0]:
                continue
            row = []
            for w in (1, 2, 3, 4):
                out = torch.zeros(nb * 4 * w * 2, dtype=torch.int64, device="cuda")
                assert lib.mix(o, s, pi, w, iters, ctypes.c_void_p(out.data_ptr()), nb) == 0
                cyc = out.view(nb, 4 * w, 2)[..., 0].float() / iters
                # the CU's span (its slowest wave) per wave-iteration of one SIMD
                row.append(float(cyc.max(dim=1).values.mean()) / w)
            name = ops[o] if p else "-"
            print(f"{shapes[s]:13s} 8 MFMA + {8 * p:3d} {name:16s} per SIMD per wave-iter: "
                  + "  ".join(f"W{w}={c:7.1f}" for w, c in zip((1, 2, 3, 4), row)), flush=True)
