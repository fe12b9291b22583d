"""bf16 causal fwd+bwd step time at config 3 (dev tool; QATTN_LIB selects a library)."""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd.attention_bf16 import helion_atten_bf16_fwd_training, helion_flash_atten_2_algo_4_bwd
g = torch.Generator(device="cuda").manual_seed(0)
B, H, S, D = 4, 32, 4096, 128
q, k = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(2))
v = torch.randn((B, H, S, D), device="cuda", generator=g).bfloat16()
dO = torch.randn((B, H, S, D), device="cuda", generator=g)
def step():
    O, lse = helion_atten_bf16_fwd_training(q, k, v, True)
    helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, True, dO)
for _ in range(3): step()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10): step()
b.record(); torch.cuda.synchronize()
print(os.environ.get("QATTN_LIB", "new"), "bf16 causal fwd+bwd ms", round(a.elapsed_time(b) / 10, 3), flush=True)
