"""Launch one kernel of the int8 / bf16 paths N times at the headline shape (for rocprofv3 passes).

    python tools/kernel_runner.py <name> [reps]   name in: int8_fwd (f16 P.V), int8_fwd_i8 (default), int8_dkdv, int8_dv, int8_dk, int8_dq, int8_all, bf16_fwd,
                                                           bf16_bwd, jvp, quant
"""
import math
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from quantizedattention_amd import _lib  # noqa: E402
from quantizedattention_amd.attention_int8 import _int8_forward, helion_atten_int8_hl_dot_bwd  # noqa: E402
from quantizedattention_amd.attention_bf16 import (helion_atten_bf16_fwd_training,  # noqa: E402
                                                   helion_flash_atten_2_algo_4_bwd)
from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32  # noqa: E402

name = sys.argv[1]
if name == "int8_all":  # every int8 attention kernel once per rep, in step order
    names = ["int8_fwd_i8", "int8_fwd", "int8_dkdv_wsc", "int8_dqw_c", "int8_dkdv_ws", "int8_dqw",
             "int8_dkdv", "int8_dq"]
else:
    names = [name]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
B, H, S, D = 4, 32, 4096, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
dO = (torch.randn((B, H, S, D), device="cuda", generator=g) * 1e-3).half()
N = B * H * S
P = _lib.ptr
st = _lib.stream_of(q)
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
sms = float(torch.tensor(1 / math.sqrt(D), dtype=torch.float32))
O, lse, qi, kiT, vi, sq, sk, sv, km, _, _ = _int8_forward(q, k, v, False)
ki = kiT.t()
vt = torch.empty((N, D), dtype=torch.int8, device="cuda")
qi2, sq2 = torch.empty_like(qi), torch.empty_like(sq)
_lib.call("qattn_int8_quant_vt", P(v), P(vi), P(sv), P(vt), N, D, st)
dOi = torch.empty((N, D), dtype=torch.int8, device="cuda")
sdO = torch.empty((N // 32,), dtype=torch.float16, device="cuda")
LD = torch.empty((N, 2), dtype=torch.float32, device="cuda")
_lib.call("qattn_int8_bwd_prep", P(dO), P(O), P(lse), P(dOi), P(sdO), P(LD), None, B * H, S, D, st)
qb, kb, ob = (torch.empty((N, D), dtype=torch.bfloat16, device="cuda") for _ in range(3))
for a_, b_ in ((qi, qb), (ki, kb), (dOi, ob)):
    _lib.call("qattn_i8_to_bf16", P(a_), P(b_), N * D, st)
dq, dk, dv = (torch.empty_like(q) for _ in range(3))
ws = torch.empty((_lib.load().qattn_int8_bwd_ws_bytes(B * H, S, S),), dtype=torch.uint8, device="cuda")
vb = v.bfloat16()
from quantizedattention_amd.attention_int8 import _ws_chunk  # noqa: E402
CHUNK = _ws_chunk(None, False, B * H, S)   # heads per launch of the step's record backward
if name.startswith("bf16"):
    Ob, lseb = helion_atten_bf16_fwd_training(q, k, vb, False)
torch.cuda.synchronize()
for name in [n for _ in range(reps) for n in names]:
    if name == "int8_fwd":   # the forward the drop-ins run: q quantised in the kernel, with its fixup
        _lib.call("qattn_int8_attn_fwd_qf", P(q), P(qi2), P(sq2), None, P(ki), P(sk), P(vt), P(sv), P(O),
                  P(lse), B * H, S, S, 1, 0, D, qks, st)
    elif name == "int8_fwd_causal":
        _lib.call("qattn_int8_attn_fwd_qf", P(q), P(qi2), P(sq2), None, P(ki), P(sk), P(vt), P(sv), P(O),
                  P(lse), B * H, S, S, 1, 1, D, qks, st)
    elif name == "int8_bwd_causal":   # the causal record backward in one call (dK+dV, then dQ)
        _lib.call("qattn_int8_attn_bwd_ws", P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv),
                  P(LD), P(qb), P(kb), P(ob), P(dq), P(dk), P(dv), P(ws), B * H, S, S, 1, 1, D, qks, sms,
                  st)
    elif name == "int8_fwd_i8":
        _lib.call("qattn_int8_attn_fwd_ex", P(qi), P(sq), P(ki), P(sk), P(vt), P(sv), P(O), P(lse),
                  B * H, S, S, 1, 0, D, qks, st)
    elif name == "int8_dkdv":
        _lib.call("qattn_int8_bwd_dkdv", P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv), P(LD),
                  P(qb), P(ob), P(dk), P(dv), B * H, S, D, qks, sms, st)
    elif name in ("int8_dv", "int8_dk"):
        _lib.call("qattn_" + name.replace("int8_", "int8_bwd_"), P(dOi), P(sdO), P(qi), P(sq), P(ki),
                  P(sk), P(vi), P(sv), P(LD), P(qb), P(ob), P(dk), P(dv), B * H, S, D, qks, sms, st)
    elif name == "int8_dkdv_ws":
        _lib.call("qattn_int8_bwd_dkdv_ws", P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv),
                  P(LD), P(qb), P(ob), P(dk), P(dv), P(ws), B * H, S, D, qks, sms, st)
    elif name == "int8_dkdv_ws_2048":   # non-causal workgroups of 64 query tiles (the causal average at
        # S = 4096 is 68): the per-tile counters beside int8_bwd_causal's (operands re-used as S = 2048)
        _lib.call("qattn_int8_bwd_dkdv_ws", P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv),
                  P(LD), P(qb), P(ob), P(dk), P(dv), P(ws), B * H, 2048, D, qks, sms, st)
    elif name == "int8_dkdv_wsc":   # one launch of the step's chunked record backward (CHUNK heads)
        _lib.call("qattn_int8_bwd_dkdv_ws", P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv),
                  P(LD), P(qb), P(ob), P(dk), P(dv), P(ws), CHUNK, S, D, qks, sms, st)
    elif name == "int8_dqw_c":
        _lib.call("qattn_int8_bwd_dq_ws", P(kb), P(sk), P(dq), P(ws), CHUNK, S, D, sms, st)
    elif name == "int8_dqw":
        _lib.call("qattn_int8_bwd_dq_ws", P(kb), P(sk), P(dq), P(ws), B * H, S, D, sms, st)
    elif name == "int8_dq":
        _lib.call("qattn_int8_bwd_dq", P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv), P(LD),
                  P(kb), P(dq), B * H, S, D, qks, sms, st)
    elif name == "bf16_fwd":
        helion_atten_bf16_fwd_training(q, k, vb, False)
    elif name == "bf16_bwd":
        helion_flash_atten_2_algo_4_bwd(q, k, vb, Ob, lseb, False, dO.float())
    elif name == "jvp":
        qq = q[:2, :16, :2048].contiguous().bfloat16()
        helion_attention_jvp_forward_fp32(qq, qq, qq, qq, qq, qq)
    elif name == "quant":
        _lib.call("qattn_int8_quant", P(v), P(vi), P(sv), None, None, N, S, D, st)
torch.cuda.synchronize()
print("done", sys.argv[1], reps)
