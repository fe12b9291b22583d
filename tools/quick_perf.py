"""Quick per-op timing (HIP events, median of N) for development."""
import sys, time, torch
sys.path.insert(0, '/root/repo')
from quantizedattention_amd import _lib
from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd, _int8_forward
from quantizedattention_amd.attention_bf16 import helion_atten_bf16_fwd_training

def timeit(fn, n=20, w=3):
    for _ in range(w): fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    ts.sort(); return ts[len(ts)//2]

B,H,S,D = 4,32,4096,128
g = torch.Generator(device='cuda').manual_seed(0)
q,k,v = [torch.randn((B,H,S,D), device='cuda', generator=g).half() for _ in range(3)]
ops = 4*B*H*S*S*D
t = timeit(lambda: helion_atten_int8_hl_dot_fwd(q,k,v))
print(f"int8 fwd full  (4,32,4096,128): {t*1e3:.1f} us  {ops/t/1e9:.1f} TOPS  ({ops/t/1e9/5033*100:.1f}% of 5.03 POPS)")
# attention kernel alone
O, lse, qi, kiT, vi, sq, sk, sv, _, _, _ = _int8_forward(q,k,v,False)
N = B*H*S
vdq = torch.empty((N,D), dtype=torch.float16, device='cuda')
st = _lib.stream_of(q)
_lib.call("qattn_int8_quant", _lib.ptr(v), _lib.ptr(vi), _lib.ptr(sv), _lib.ptr(vdq), None, N, S, D, st)
ki = kiT.t()
qks = float(torch.tensor(1/128**0.5*1.44269504, dtype=torch.float32))
def attn():
    _lib.call("qattn_int8_attn_fwd", _lib.ptr(qi), _lib.ptr(sq), _lib.ptr(ki), _lib.ptr(sk), _lib.ptr(vdq), _lib.ptr(O), _lib.ptr(lse), B*H, S, D, qks, st)
t2 = timeit(attn)
print(f"int8 attn kernel only: {t2*1e3:.1f} us  {ops/t2/1e9:.1f} TOPS ({ops/t2/1e9/5033*100:.1f}%)")
def quant():
    _lib.call("qattn_int8_quant", _lib.ptr(v), _lib.ptr(vi), _lib.ptr(sv), _lib.ptr(vdq), None, N, S, D, st)
t3 = timeit(quant)
print(f"int8 quant (V, with deq) : {t3*1e3:.1f} us  {(N*D*2 + N*D + N*D*2)/t3/1e6:.0f} GB/s")
vb = v.bfloat16()
for S2 in (2048, 4096):
    qq,kk,vv = q[:,:,:S2].contiguous(), k[:,:,:S2].contiguous(), vb[:,:,:S2].contiguous()
    for causal in (False, True):
        t4 = timeit(lambda: helion_atten_bf16_fwd_training(qq,kk,vv,causal))
        f = 4*B*H*S2*S2*D * (0.5 if causal else 1)
        print(f"bf16 fwd S={S2} causal={causal}: {t4*1e3:.1f} us  {f/t4/1e9:.1f} TFLOPS ({f/t4/1e9/2516*100:.1f}%)")
