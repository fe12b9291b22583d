"""Causal int8 record backward: time + output hash per head-chunk size, for A/B of dK+dV grid
variants (the paired grid of DESIGN.md §5 round 3 was measured with it and not kept; DESIGN.md
describes how it was built).  Run through tools/ab_run.sh; equal hashes across variants = bit-identical gradients.

    python tools/ab_pair.py            (env CHUNKS="0,32,64": key/value heads per chunk, 0 = one pass)"""
import hashlib, os, sys, torch
# the package loads QATTN_LIB: point it at the variant tools/ab_run.sh names in QATTN_AB
if os.environ.get("QATTN_AB"):
    os.environ["QATTN_LIB"] = os.environ["QATTN_AB"]
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward


def digest(ts):
    h = hashlib.sha256()
    for t in ts:
        h.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return h.hexdigest()[:12]


def run(shape, causal, chunks, reps, group=1):
    B, H, S, D = shape
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    k, v = (torch.randn((B, H // group, S, D), device="cuda", generator=g).half() for _ in range(2))
    dO = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, _, q_bf, k_bf = _int8_forward(q, k, v, smooth=True, images=True,
                                                                         causal=causal)
    for c in chunks:
        ts = []
        for i in range(reps + 2):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            out = _int8_backward(dO, q_i8, sq, k_i8T, sk, v_i8, sv, O, lse, q_bf, k_bf, causal=causal,
                                 kv_heads=H // group, use_ws=True, ws_chunk=c)
            b.record()
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(a.elapsed_time(b))
        ts.sort()
        print(f"{os.path.basename(os.environ.get('QATTN_AB', 'default'))} {shape} g{group} causal={causal} "
              f"chunk={c}: bwd {ts[len(ts) // 2]:.3f} ms (min {ts[0]:.3f}) hash {digest(out)}", flush=True)


chunks = [int(c) for c in os.environ.get("CHUNKS", "0,32,64").split(",")]
run((4, 32, 4096, 128), True, chunks, 10)
run((4, 32, 4096, 128), False, [0], 5)
run((2, 6, 3840, 64), True, [0, 4], 3)          # 15 key blocks: a lone middle block
run((2, 8, 1056, 128), True, [0], 3)            # ragged last key block
run((2, 8, 1024, 64), True, [0], 3, group=4)    # grouped heads: not paired
