"""Key-split size sweep of the decoding forward (kv_cache._decode_split), dev tool."""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd import kv_cache  # noqa: E402
from quantizedattention_amd.kv_cache import attention_int8_cached, quantize_kv  # noqa: E402
orig = kv_cache._split_plan
for (B, Hq, Hkv, Sq, Sk) in [(8, 32, 8, 32, 8192), (8, 32, 32, 32, 8192), (1, 32, 8, 32, 32768), (1, 8, 8, 32, 32768)]:
    D = 128
    g = torch.Generator(device="cuda").manual_seed(0)
    k, v = (torch.randn((B, Hkv, Sk, D), device="cuda", generator=g).half() for _ in range(2))
    q = torch.randn((B, Hq, Sq, D), device="cuda", generator=g).half()
    kv = quantize_kv(k, v)
    res = []
    for ks in (256, 512, 1024, 2048, 4096, Sk):
        if ks > Sk:
            continue
        kv_cache._split_plan = lambda bhv, rows, sk, ks=ks: ks
        f = lambda: attention_int8_cached(q, kv)  # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            f()
        b.record()
        torch.cuda.synchronize()
        res.append(f"ks={ks}:{a.elapsed_time(b) / 20 * 1e3:.1f}us")
    kv_cache._split_plan = orig
    print(f"B={B} Hq={Hq} Hkv={Hkv} Sq={Sq} Sk={Sk} plan={orig(B * Hkv, Hq // Hkv * Sq, Sk)}: " + " ".join(res), flush=True)
