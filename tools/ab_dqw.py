"""Time the dQ-from-records kernel of one library (A/B dev tool, QATTN_AB=variant .so)."""
import ctypes, math, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedattention_amd._lib import SIGNATURES  # noqa: E402
path = os.environ.get("QATTN_AB") or os.path.join(ROOT, "quantizedattention_amd", "libqattn.so")
torch.cuda.init()
lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
for n in ("qattn_int8_bwd_dq_ws", "qattn_int8_bwd_ws_bytes"):
    getattr(lib, n).argtypes = SIGNATURES[n]
lib.qattn_int8_bwd_ws_bytes.restype = ctypes.c_long
B, H, S, D = 4, 32, 4096, 128
N = B * H * S
ws = torch.randint(-127, 127, (lib.qattn_int8_bwd_ws_bytes(B * H, S, S),), dtype=torch.int8, device="cuda")
kb = torch.randn((N, D), device="cuda").bfloat16()
sk = torch.rand((N // 32,), device="cuda").half()
dq = torch.empty((N, D), device="cuda", dtype=torch.half)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
f = lambda: lib.qattn_int8_bwd_dq_ws(P(kb), P(sk), P(dq), P(ws), B * H, S, D, 0.088, st)  # noqa: E731
for _ in range(3):
    assert f() == 0
torch.cuda.synchronize()
ts = []
for _ in range(15):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); f(); b.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
t = sorted(ts)[7]
print(f"{os.path.basename(path)} dqw: {t * 1e3:.1f} us  records {ws.numel() / t / 1e9:.2f} TB/s")
