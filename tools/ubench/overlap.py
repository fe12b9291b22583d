"""Drive tools/ubench/overlap.hip: cycles per loop iteration per wave, 1..3 waves per SIMD."""
import ctypes
import os

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "liboverlap.so"))
lib.overlap.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int]
names = ["12 MFMA (4 chains)", "128 VALU", "12 MFMA + 128 VALU (blocked)", "12 MFMA + 128 VALU (interleaved)",
         "12 MFMA (1 chain)", "12 MFMA 1 chain + 128 VALU interleaved", "12 MFMA + 64 VALU interleaved",
         "64 VALU"]
iters, nb = 500, 256
for k, name in enumerate(names):
    res = []
    for w in (1, 2, 3, 4):
        out = torch.zeros(nb * 4 * w * 2, dtype=torch.int64, device="cuda")
        assert lib.overlap(k, w, iters, ctypes.c_void_p(out.data_ptr()), nb) == 0
        res.append(float(out.view(-1, 2)[:, 0].float().mean()) / iters)
    print(f"{name:42s} cycles/iter/wave @1,2,3,4 waves/SIMD: " + "  ".join(f"{x:7.1f}" for x in res)
          + "   per-SIMD: " + "  ".join(f"{x / w:7.1f}" for x, w in zip(res, (1, 2, 3, 4))), flush=True)
