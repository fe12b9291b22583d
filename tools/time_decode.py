"""int8 KV-cache attention at decode shapes, HIP-event time and the HBM roofline of
the cache read (dev tool).   python tools/time_decode.py"""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd.kv_cache import attention_int8_cached, quantize_kv  # noqa: E402
for (B, Hq, Hkv, Sq, Sk) in [(8, 32, 8, 32, 8192), (8, 32, 32, 32, 8192), (1, 32, 8, 32, 32768)]:
    D = 128
    g = torch.Generator(device="cuda").manual_seed(0)
    k, v = (torch.randn((B, Hkv, Sk, D), device="cuda", generator=g).half() for _ in range(2))
    q = torch.randn((B, Hq, Sq, D), device="cuda", generator=g).half()
    kv = quantize_kv(k, v)
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
    t = a.elapsed_time(b) / 20 * 1e-3
    cache = 2 * B * Hkv * Sk * D + 2 * 2 * B * Hkv * Sk // 32
    print(f"B={B} Hq={Hq} Hkv={Hkv} Sq={Sq} Sk={Sk}: {t * 1e6:.1f} us, cache {cache / 1e6:.0f} MB -> "
          f"{cache / t / 1e12:.2f} TB/s ({cache / t / 8e12:.1%} of 8 TB/s); "
          f"{4 * B * Hq * Sq * Sk * D / t / 1e12:.0f} TOPS", flush=True)
