"""int8 record backward: one pass vs head chunks (qattn_int8_attn_bwd_wsc), time + bit-identity (dev tool).

    python tools/time_bwd_chunk.py [chunks, comma-separated kv heads; 0 = one pass]"""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward
B, H, S, D = 4, 32, 4096, 128
chunks = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "0,8,16,24,32,64").split(",")]
for causal in (False, True):
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
    dO = (torch.randn((B, H, S, D), device="cuda", generator=g) * 1e-3).half()
    O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, _, q_bf, k_bf = _int8_forward(q, k, v, smooth=True, images=True, causal=causal)
    ref = None
    for c in chunks:
        ts = []
        for i in range(12):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            out = _int8_backward(dO, q_i8, sq, k_i8T, sk, v_i8, sv, O, lse, q_bf, k_bf, causal=causal,
                                 use_ws=True, ws_chunk=c)
            b.record()
            torch.cuda.synchronize()
            if i >= 2: ts.append(a.elapsed_time(b))
        if ref is None: ref = out
        same = all(torch.equal(x, y) for x, y in zip(out, ref))
        print(f"causal={causal} chunk={c}: bwd {sorted(ts)[len(ts)//2]:.3f} ms (min {min(ts):.3f}) bit-identical={same}", flush=True)
