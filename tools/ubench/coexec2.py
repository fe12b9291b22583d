"""Drive tools/ubench/coexec2.hip (dev tool): MFMA-only waves beside vector waves of one instruction
type; prints cycles per iteration (12 MFMAs / 144 vector instructions) of each wave group."""
import ctypes
import os

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libcoexec2.so"))
lib.coexec2.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int]
ops = ["v_fma_f32", "v_pk_fma_f16", "v_pk_add_f16", "v_pk_max_f16", "v_exp_f16", "v_exp_f32",
       "v_fma_mixlo_f16", "v_add_f16", "v_max_i32", "v_cvt_f32_f16", "v_perm_b32", "v_pk_fma_f32",
       "v_pk_mul_f32", "v_cvt_pk_f16_f32", "v_fma_mix_f32", "v_cvt_f16_f32", "v_pk_mul_f16", "v_max3_i32",
       "v_fmac_f32", "v_mul_f32"]
import sys
sel = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else range(len(ops))
iters, nb = 300, 256
for k in sel:
    name = ops[k]
    for w, mi in ((2, iters), (2, 0), (1, -1)):
        if True:
            out = torch.zeros(nb * 4 * w * 2, dtype=torch.int64, device="cuda")
            assert lib.coexec2(k, w, iters, mi, ctypes.c_void_p(out.data_ptr()), nb) == 0
            cyc = out.view(nb, w, 4, 2)[..., 0].float() / iters
            g = cyc.mean(dim=(0, 2)).tolist()
            tag = "with MFMA wave" if mi > 0 else ("MFMA wave idle" if mi == 0 else "MIXED (1 wave)")
            if mi < 0:
                print(f"{name:16s} {tag:15s}: 12 MFMA + 144 vector per iteration {g[0]:7.1f} "
                      f"(({g[0]:.0f} - 384) / 144 = {(g[0] - 384) / 144:.2f} cyc/instr beyond the MFMAs)", flush=True)
            else:
                print(f"{name:16s} W={w} {tag:15s}: MFMA wave {g[0]:7.1f}  vector waves " +
                      " ".join(f"{x:7.1f}" for x in g[1:]) + f"  ({sum(g[1:]) and g[1] / 144:.2f} cyc/instr)",
                      flush=True)
