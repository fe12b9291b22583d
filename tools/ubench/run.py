"""Drive tools/ubench: cycles per instruction per wave with 1 or 2 waves per SIMD, alone and beside
an MFMA-only wave on the same SIMD.  Build first: tools/ubench/build.sh"""
import ctypes
import os

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libubench.so"))
lib.ubench.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int]
names = ["v_mul_f32", "v_fma_f32", "v_cvt_f32_i32", "v_trunc_f32", "v_exp_f32", "v_cvt_pk_bf16_f32",
         "v_max3_f32", "v_exp_f16", "v_pk_fma_f16", "v_pk_add_f16", "v_dot2c_f32_f16",
         "v_fma_mixlo_f16", "v_max_f32", "v_mov_b32", "v_add_u32", "v_cvt_f32_f16", "v_pk_mul_f32", "v_pk_add_f32", "v_pk_fma_f32",
         "v_cvt_f32_bf16", "v_med3_f32", "v_dot2_f32_bf16"]
iters = 2000
nb = 256
for k, name in enumerate(names):
    res = []
    for wps, mw in ((1, 0), (2, 0), (2, 1)):
        out = torch.zeros(nb * 4 * wps * 2, dtype=torch.int64, device="cuda")
        assert lib.ubench(k, wps, mw, iters, ctypes.c_void_p(out.data_ptr()), nb) == 0
        cyc = out.view(-1, 2)[:, 0].float().cpu()
        nw = 4 * wps
        per_wave = cyc.view(nb, nw)
        valu = per_wave[:, 4 * mw:] if mw else per_wave
        res.append(float(valu.mean()) / (iters * 16))
        if mw:
            mf = per_wave[:, :4 * mw]
            res.append(float(mf.mean()) / (iters * 16))
    print(f"{name:20s} 1w/SIMD {res[0]:5.2f}  2w/SIMD {res[1]:5.2f}  beside-MFMA-wave {res[2]:5.2f} "
          f"(mfma wave {res[3]:5.1f} cyc/mfma)", flush=True)
