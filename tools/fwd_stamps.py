"""Where an int8 forward workgroup's time goes (dev tool): the diagnostic build -DQA_FWD_STAMP=1
(tools/ab_build.sh int8_attn_fwd.hip fstamp -DQA_FWD_STAMP=1) stamps entry, end of prologue, end of
the tile loop and exit of every workgroup (s_memrealtime, 100 MHz); this runs the config-3 forward
(REPS launches, stamps of the last) and prints the phase durations.

    QATTN_AB=_ab/libqattn_fstamp.so [REPS=20] [CAUSAL=1] python tools/fwd_stamps.py

(The separate fixup launch of this entry would stamp over the fast pass: run with
QATTN_FWD_SKIP_FIXUP=1.)  CAUSAL=1 runs the causal forward and fits each workgroup's loop time against its key-tile count
(4 (b+1) for query block b: the sorted loop times matched to the sorted tile counts)."""
import ctypes, math, os, sys
os.environ.setdefault("QATTN_FWD_SKIP_FIXUP", "1")
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd._lib import SIGNATURES
torch.cuda.init()
lib = ctypes.CDLL(os.environ["QATTN_AB"], mode=ctypes.RTLD_GLOBAL)
fn = lib.qattn_int8_attn_fwd_ex; fn.argtypes = SIGNATURES["qattn_int8_attn_fwd_ex"]
B, H, S, D = 4, 32, 4096, 128
N = B * H * S
g = torch.Generator(device="cuda").manual_seed(0)
i8 = lambda: torch.randint(-127, 128, (N, D), device="cuda", generator=g, dtype=torch.int8)
sc = lambda: (torch.rand(N // 32, device="cuda", generator=g) * 0.01 + 0.01).half()
qi, ki, vt = i8(), i8(), i8(); sq, sk, sv = sc(), sc(), sc()
O = torch.empty((N, D), dtype=torch.float16, device="cuda"); lse = torch.empty((N,), dtype=torch.float16, device="cuda")
P = lambda t: ctypes.c_void_p(t.data_ptr()); st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
causal = int(os.environ.get("CAUSAL", "0"))
for _ in range(int(os.environ.get("REPS", "3"))):
    assert fn(P(qi), P(sq), P(ki), P(sk), P(vt), P(sv), P(O), P(lse), B * H, S, S, 1, causal, D, qks, st) == 0
torch.cuda.synchronize()
buf = np.zeros((8192, 4), dtype=np.uint64)
assert lib.qattn_fwd_stamps(ctypes.c_void_p(buf.ctypes.data)) == 0
t = buf[:4096].astype(np.int64); t -= t[:, 0].min(); us = t / 100.0
pro, loop, epi = us[:, 1] - us[:, 0], us[:, 2] - us[:, 1], us[:, 3] - us[:, 2]
print(f"span {us[:, 3].max():.1f} us")
for name, x in (("prologue", pro), ("loop", loop), ("epilogue", epi)):
    print(f"  {name:9s} min {x.min():7.1f} median {np.median(x):7.1f} max {x.max():7.1f}")
# gap between consecutive workgroups on the same slot is not known; show dispatch spread
starts = np.sort(us[:, 0]); print("  start quantiles", np.round(np.quantile(starts, [0, .125, .25, .5, .75, 1]), 1).tolist())
if causal:
    nqb = S // 128
    tiles = np.sort(np.repeat(4 * (np.arange(nqb) + 1), 4096 // nqb))
    lt = np.sort(loop)
    a, b = np.polyfit(tiles, lt, 1)
    print(f"  causal loop fit: {b:.2f} us + {a:.3f} us per key tile "
          f"(non-causal workgroups run 128 tiles)")
    for nt_ in (4, 32, 64, 128):
        sel = tiles == nt_
        if sel.any():
            print(f"    {nt_:3d} tiles: loop median {np.median(lt[sel]):.1f} us")
    busy = (us[:, 3] - us[:, 0]).sum()
    print(f"  sum of workgroup times {busy:.0f} us over 512 slots = {busy / 512:.1f} us per slot")
