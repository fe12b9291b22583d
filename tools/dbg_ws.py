import torch, sys
sys.path.insert(0, '.')
from quantizedattention_amd import _lib
from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
import quantizedattention_amd.attention_int8 as A
B,H,S,D = 1,2,128,128
g = torch.Generator().manual_seed(0)
q,k,v,dO = (torch.randn((B,H,S,D), generator=g).half().cuda() for _ in range(4))
O, lse, qi, kiT, vi, sq, sk, sv, _, _ = helion_atten_int8_hl_dot_fwd(q, k, v)
orig = torch.empty
cap = {}
def spy(*a, **kw):
    t = orig(*a, **kw)
    if kw.get('dtype') == torch.uint8 and len(a) == 1: t.fill_(7); cap['ws'] = t
    return t
A.torch.empty = spy
dq, dk, dv = A._int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, use_ws=True)
A.torch.empty = orig
torch.cuda.synchronize()
ws = cap['ws'].cpu()
n = B*H*(S//32)**2
print('ws bytes', ws.numel(), 'n rec', n)
print('records still 7:', (ws[:n*1024] == 7).float().mean().item())
print('scales', ws[n*1024:].view(torch.float32)[:8])
print('dq abs mean', dq.float().abs().mean().item())
