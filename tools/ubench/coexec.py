"""Drive tools/ubench/coexec.hip: per-wave cycles per iteration, role split vs mixed (dev tool)."""
import ctypes
import os

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libcoexec.so"))
lib.coexec.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int]
names = ["MFMA only on waves 0-3 (VALU waves idle)", "mixed: 12 MFMA + 144 VALU per wave",
         "split: 0-3 MFMA, rest 144 VALU", "every wave 12 MFMA", "every wave 4 MFMA + 144 VALU"]
iters, nb = 400, 256
for k, name in enumerate(names):
    for w in (1, 2, 3):
        out = torch.zeros(nb * 4 * w * 2, dtype=torch.int64, device="cuda")
        assert lib.coexec(k, w, iters, ctypes.c_void_p(out.data_ptr()), nb) == 0
        cyc = out.view(nb, w, 4, 2)[..., 0].float() / iters   # [block, wave-group, simd]
        per_group = cyc.mean(dim=(0, 2)).tolist()
        print(f"{name:42s} W={w}: cycles/iter by wave group " + " ".join(f"{x:7.1f}" for x in per_group),
              flush=True)
