"""Per-kernel HIP-event times of the int8 path at config 3 (bench.int8_kernel_times), dev tool.

    python tools/time_int8_kernels.py [name-substring ...]"""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((4, 32, 4096, 128), device="cuda", generator=g).half() for _ in range(3))
dO = (torch.randn((4, 32, 4096, 128), device="cuda", generator=g) * 1e-3).half()
for rep in range(2):
    kt = bench.int8_kernel_times(q, k, v, dO, 10)
    sel = sys.argv[1:]
    print(" ".join(f"{n}={t * 1e3:.0f}us" for n, t in kt.items() if not sel or any(s in n for s in sel)), flush=True)
