"""Calibrate s_memtime ticks against wall time with an MFMA-only ubench launch (dev tool)."""
import ctypes
import os

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libubench.so"))
lib.ubench.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int]
nb = 256
for iters in (20000, 40000):
    out = torch.zeros(nb * 4 * 2, dtype=torch.int64, device="cuda")
    lib.ubench(0, 1, 1, iters, ctypes.c_void_p(out.data_ptr()), nb)   # warm
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    lib.ubench(0, 1, 1, iters, ctypes.c_void_p(out.data_ptr()), nb)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b)
    ticks = out.view(-1, 2)[:, 0].float().cpu().view(nb, 4)
    n_mfma = iters * 16
    print(f"iters {iters}: wall {ms:.3f} ms, ticks/wave {ticks.mean():.0f} -> tick rate "
          f"{ticks.mean() / (ms * 1e-3) / 1e9:.3f} GHz; ticks/MFMA {ticks.mean() / n_mfma:.2f}; "
          f"if 32 shader cycles per i8 32x32x32 MFMA the clock is "
          f"{n_mfma * 32 / (ms * 1e-3) / 1e9:.3f} GHz", flush=True)
