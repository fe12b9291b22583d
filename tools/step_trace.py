"""Kernels of one int8 fwd+bwd step at config 3 in launch order, with durations and the idle gaps
between them (dev tool; run under rocprofv3 --kernel-trace --output-format csv, then
python tools/step_trace.py --report <kernel_trace.csv>); --causal for the causal step, --bf16 for the bf16 step."""
import csv
import os
import sys


def run(causal=False, bf16=False):
    import torch
    sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
    from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward
    g = torch.Generator(device="cuda").manual_seed(0)
    B, H, S, D = 4, 32, 4096, 128
    q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
    dO = (torch.randn((B, H, S, D), device="cuda", generator=g) * 1e-3).half()

    def step():
        O, lse, qi, kiT, vi, sq, sk, sv, km, qb_, kb_ = _int8_forward(q, k, v, smooth=True, images=True,
                                                                       causal=causal)
        _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb_, kb_, causal=causal)
    if bf16:   # the bench's bf16 step (k-mean marker launched first so --report finds the step)
        from quantizedattention_amd import _lib
        from quantizedattention_amd.attention_bf16 import (helion_atten_bf16_fwd_training,
                                                           helion_flash_atten_2_algo_4_bwd)
        vb, dOf = v.bfloat16(), dO.float()
        km = torch.empty((B, H, 1, D), dtype=torch.float16, device="cuda")

        def step():
            _lib.call("qattn_kmean", _lib.ptr(k), _lib.ptr(km), B * H, S, D, _lib.stream_of(k))
            O, lse = helion_atten_bf16_fwd_training(q, k, vb, causal)
            helion_flash_atten_2_algo_4_bwd(q, k, vb, O, lse, causal, dOf)
    for _ in range(6):
        step()
    torch.cuda.synchronize()
    print("done", flush=True)


def report(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    # the last step: from the last k-mean launch on
    first = max(i for i, k in enumerate(ks) if "kmean" in k[2])
    prev = None
    tot_k = 0.0
    for s, e, n in ks[first:]:
        gap = (s - prev) / 1e3 if prev else 0.0
        tot_k += (e - s) / 1e3
        print(f"{(e - s) / 1e3:9.1f} us  gap {gap:7.1f}  {n[:110]}")
        prev = e
    span = (ks[-1][1] - ks[first][0]) / 1e3
    print(f"step span {span:.1f} us, kernel time {tot_k:.1f} us, idle {span - tot_k:.1f} us")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run(causal="--causal" in sys.argv, bf16="--bf16" in sys.argv)
