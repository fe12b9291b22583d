"""Decoding-step time split into GPU kernel time and launch gaps (dev tool):
eager calls vs the same call captured once in a HIP graph and replayed.
    python tools/decode_breakdown.py"""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd.kv_cache import attention_int8_cached, quantize_kv  # noqa: E402


def timed(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for (B, Hq, Hkv, Sq, Sk) in [(8, 32, 8, 32, 8192), (8, 32, 32, 32, 8192), (1, 32, 8, 32, 32768)]:
    D = 128
    g = torch.Generator(device="cuda").manual_seed(0)
    k, v = (torch.randn((B, Hkv, Sk, D), device="cuda", generator=g).half() for _ in range(2))
    q = torch.randn((B, Hq, Sq, D), device="cuda", generator=g).half()
    kv = quantize_kv(k, v)
    kv.vt()
    f = lambda: attention_int8_cached(q, kv)  # noqa: E731
    t_eager = timed(f)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            f()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = f()
    t_graph = timed(graph.replay)
    ref = f()
    graph.replay()
    torch.cuda.synchronize()
    same = torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
    print(f"B={B} Hq={Hq} Hkv={Hkv} Sq={Sq} Sk={Sk}: eager {t_eager:.1f} us, graph replay "
          f"{t_graph:.1f} us (identical: {same})", flush=True)
