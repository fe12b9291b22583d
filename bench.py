"""Headline benchmark: fused-attention fwd+bwd at (B,H,S,D) = (4,32,4096,128), int8 vs bf16.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3|4]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (multi-GPU)

``--gpus N`` without a torchrun environment starts the N ranks itself (one process per GPU, RCCL),
before this process touches the GPU, and exits with their status.

A step = one training pass of the attention operator over one synthetic batch:
  int8 (the reported `value`): sage_attention_3_int8 forward (k-mean + q/k/v quantisation +
  int8 attention) and its backward (dO quantisation + D + dK/dV + dQ kernels);
  bf16 (reported beside it at N = 1): flash_atten_2_bf16 forward + backward.
Workloads (BASELINE.json):
  --config 3 (default at N = 1): each rank owns its own (4,32,4096,128) shard of a (4N,32,4096,128)
      batch (weak scaling);
  --config 4 (default at N > 1): the global (8,32,8192,128) problem; every rank generates the same
      seeded global tensors and slices its heads, then runs its (8/N,32,8192,128) shard
      (strong scaling).
With N > 1 the step also all-gathers O over RCCL, issued asynchronously after the forward so it
overlaps the backward.  Inputs are resident in HBM before timing starts.

Prints ONE JSON line (rank 0).  FLOP accounting: fwd 4*BH*S^2*D, bwd 10*BH*S^2*D.
"""
from __future__ import annotations

import argparse
import json
import hashlib
import math
import os
import socket
import statistics
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from quantizedattention_amd import _lib  # noqa: E402
from quantizedattention_amd.attention_bf16 import (  # noqa: E402
    helion_atten_bf16_fwd_training, helion_flash_atten_2_algo_4_bwd)
from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward  # noqa: E402
from quantizedattention_amd.sharded import local_slice, shard_for  # noqa: E402

PEAK_I8 = 256 * 8192 * 2.4e9          # ops/s, dense int8 MFMA (MI355X_MICROARCH: 2x bf16 per clock)
PEAK_BF16 = 256 * 4096 * 2.4e9        # flop/s, dense bf16/fp16 MFMA
PEAK_FP4 = 256 * 16384 * 2.4e9        # flop/s, dense MX-FP4 block-scaled MFMA (4x bf16 per clock)
PEAK_HBM = 8.0e12                     # B/s


def _f32(x):
    return float(torch.tensor(x, dtype=torch.float32))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", type=int, choices=(3, 4), default=None,
                   help="3: (4,32,4096,128) per rank (weak); 4: (8,32,8192,128) split over the ranks "
                        "(strong); default 3 at N = 1, 4 at N > 1")
    p.add_argument("--shape", type=str, default=None, help="per-rank (B,H,S,D) override of config 3")
    p.add_argument("--no-gather", action="store_true", help="skip the O all-gather for N>1")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--skip-bf16", action="store_true")
    p.add_argument("--no-configs", action="store_true",
                   help="skip the other-config timings (a profiled run whose kernels are all config 3)")
    return p.parse_args()


def timed(fn, steps, warmup, world):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = (time.perf_counter() - t0) / steps
    if world > 1:
        tt = torch.tensor([t], device="cuda", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = tt.item()
    return t


def event_time(fn, n):
    """Average device time of fn() on the current stream (HIP events), ms."""
    s = torch.cuda.current_stream()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(n):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def ws_chunk_heads(bh, S):
    """Heads per launch of the step's chunked record backward (attention_int8._ws_chunk)."""
    from quantizedattention_amd.attention_int8 import _ws_chunk
    return _ws_chunk(None, False, bh, S)


def int8_kernel_times(q, k, v, dO, n):
    """Per-kernel average durations (ms) of the int8 path, each launched alone on the stream."""
    B, H, S, D = q.shape
    N = B * H * S
    dev = q.device
    st = _lib.stream_of(q)
    P = _lib.ptr
    e = lambda *shape, dt: torch.empty(shape, dtype=dt, device=dev)  # noqa: E731
    qi, ki, vi, dOi = (e(N, D, dt=torch.int8) for _ in range(4))
    sq, sk, sv, sdO = (e(N // 32, dt=torch.float16) for _ in range(4))
    vt = e(N, D, dt=torch.int8)
    km = e(B * H, D, dt=torch.float16)
    O = e(B, H, S, D, dt=torch.float16)
    lse = e(N, dt=torch.float16)
    LD = e(N, 2, dt=torch.float32)
    qb, kb, ob = (e(N, D, dt=torch.bfloat16) for _ in range(3))
    dq, dk, dv = (e(B, H, S, D, dt=torch.float16) for _ in range(3))
    ws = e(_lib.load().qattn_int8_bwd_ws_bytes(B * H, S, S), dt=torch.uint8)
    chunk = ws_chunk_heads(B * H, S)
    qks, sms = _f32(1 / math.sqrt(D) * 1.44269504), _f32(1 / math.sqrt(D))
    calls = {
        "kmean_kernel": lambda: _lib.call("qattn_kmean", P(k), P(km), B * H, S, D, st),
        "quant_block32_kernel(k)": lambda: _lib.call("qattn_int8_quant_img", P(k), P(ki), P(sk), None,
                                                     P(kb), P(km), N, S, D, st),
        "quant_block32_kernel(q)": lambda: _lib.call("qattn_int8_quant_img", P(q), P(qi), P(sq), None,
                                                     P(qb), None, N, S, D, st),
        "quant_vt_kernel(v)": lambda: _lib.call("qattn_int8_quant_vt", P(v), P(vi), P(sv), P(vt), N, D,
                                                st),
        # the forward call's own quantiser launches (int8_fwd: no bf16 images)
        "quant_block32_kernel(k, fwd)": lambda: _lib.call("qattn_int8_quant", P(k), P(ki), P(sk), None,
                                                          P(km), N, S, D, st),
        # the forward the drop-ins run (q quantised in its prologue; P.V on the int8 MFMA, the
        # reference's hl.dot(P_i8, v_i8)), its fixup pass inline (int8_attn_fwd.hip)
        "int8_attn_fwd_kernel": lambda: _lib.call("qattn_int8_attn_fwd_qf", P(q), P(qi), P(sq), None,
                                                  P(ki), P(sk), P(vt), P(sv), P(O), P(lse), B * H, S,
                                                  S, 1, 0, D, qks, st),
        # the C-ABI form on a pre-quantised q (qattn_int8_attn_fwd_ex)
        "int8_attn_fwd_kernel<q_i8 in>": lambda: _lib.call("qattn_int8_attn_fwd_ex", P(qi), P(sq), P(ki),
                                                           P(sk), P(vt), P(sv), P(O), P(lse), B * H, S,
                                                           S, 1, 0, D, qks, st),
        "int8_bwd_prep": lambda: _lib.call("qattn_int8_bwd_prep", P(dO), P(O), P(lse), P(dOi), P(sdO),
                                           P(LD), P(ob), B * H, S, D, st),
        "int8_bwd_dkdv_kernel<dK+dV>": lambda: _lib.call("qattn_int8_bwd_dkdv", P(dOi), P(sdO), P(qi),
                                                         P(sq), P(ki), P(sk), P(vi), P(sv), P(LD),
                                                         P(qb), P(ob), P(dk), P(dv), B * H, S, D,
                                                         qks, sms, st),
        "int8_bwd_dkdv_kernel<dV>": lambda: _lib.call("qattn_int8_bwd_dv", P(dOi), P(sdO), P(qi), P(sq),
                                                  P(ki), P(sk), P(vi), P(sv), P(LD), P(qb), P(ob),
                                                  P(dk), P(dv), B * H, S, D, qks, sms, st),
        "int8_bwd_dkdv_kernel<dK>": lambda: _lib.call("qattn_int8_bwd_dk", P(dOi), P(sdO), P(qi), P(sq),
                                                  P(ki), P(sk), P(vi), P(sv), P(LD), P(qb), P(ob),
                                                  P(dk), P(dv), B * H, S, D, qks, sms, st),
        "int8_bwd_dq_kernel": lambda: _lib.call("qattn_int8_bwd_dq", P(dOi), P(sdO), P(qi), P(sq),
                                                P(ki), P(sk), P(vi), P(sv), P(LD), P(kb), P(dq),
                                                B * H, S, D, qks, sms, st),
        # the step's backward (qattn_int8_attn_bwd_wsc): per chunk of `chunk` heads, dK+dV writing
        # the dS workspace, then dQ from it -- timed as the step launches them (one chunk-sized launch)
        "int8_bwd_dkdv_kernel<dK+dV, dS out>": lambda: _lib.call(
            "qattn_int8_bwd_dkdv_ws", P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv), P(LD),
            P(qb), P(ob), P(dk), P(dv), P(ws), chunk, S, D, qks, sms, st),
        "int8_bwd_dqw_kernel": lambda: _lib.call("qattn_int8_bwd_dq_ws", P(kb), P(sk), P(dq), P(ws),
                                                 chunk, S, D, sms, st),
        # the same two kernels over all B*H heads in one launch each (qattn_int8_attn_bwd_ws)
        "int8_bwd_dkdv_kernel<dK+dV, dS out, one pass>": lambda: _lib.call(
            "qattn_int8_bwd_dkdv_ws", P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv), P(LD),
            P(qb), P(ob), P(dk), P(dv), P(ws), B * H, S, D, qks, sms, st),
        "int8_bwd_dqw_kernel<one pass>": lambda: _lib.call("qattn_int8_bwd_dq_ws", P(kb), P(sk), P(dq),
                                                           P(ws), B * H, S, D, sms, st),
    }
    order = list(calls)
    for name in order:  # populate every buffer once in dependency order
        calls[name]()
    return {name: event_time(calls[name], n) for name in order}


def mxfp4_fwd_times(q, k, v, n):
    """SURVEY §8f N4 beside the headline: the MX-FP4 inference forward at the same shape --
    the attention kernel alone (operands already quantised) and the whole call (k-mean,
    quantisers, attention)."""
    from quantizedattention_amd import _lib
    from quantizedattention_amd.attention_mxfp4 import _qk_scale, mxfp4_attn_fwd
    B, H, S, D = q.shape
    O, lse, ops = mxfp4_attn_fwd(q, k, v)
    st = _lib.stream_of(q)

    def kern():
        _lib.call("qattn_mxfp4_attn_fwd", *(_lib.ptr(t) for t in ops), _lib.ptr(O), _lib.ptr(lse),
                  B * H, S, S, 1, D, _qk_scale(D), st)
    tk = event_time(kern, n)
    te = event_time(lambda: mxfp4_attn_fwd(q, k, v), n)
    flop = 4.0 * B * H * S * S * D
    return {"kernel_ms": tk, "call_ms": te, "kernel_TFLOPs": flop / (tk * 1e-3) / 1e12,
            "frac_of_fp4_peak": flop / (tk * 1e-3) / PEAK_FP4}


def other_configs(n):
    """BASELINE.json's other GPU configs, each timed alone on this rank (HIP events, ms per call):
    config 2, bf16 fwd+bwd (4,32,2048,128); config 5, the JVP forward (2,16,2048,128) with bf16
    inputs and randn tangents; config 3 causal, int8 fwd+bwd; config 4's global (8,32,8192,128)
    int8 fwd+bwd on one GPU.  (Config 3 is the int8 forward reported as ``int8_fwd``; config 4 split
    over N GPUs is ``--gpus N``; config 1 is the CPU path, ``cpu_baseline``.)"""
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(7)
    out = {}
    B, H, S, D = 4, 32, 2048, 128
    q, k = (torch.randn((B, H, S, D), device=dev, generator=g).half() for _ in range(2))
    v = torch.randn((B, H, S, D), device=dev, generator=g).bfloat16()
    dO = torch.randn((B, H, S, D), device=dev, generator=g)

    def bf16_step():
        O, lse = helion_atten_bf16_fwd_training(q, k, v, False)
        helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, False, dO)
    t = event_time(bf16_step, n)
    tf = event_time(lambda: helion_atten_bf16_fwd_training(q, k, v, False), n)
    flop = 14.0 * B * H * S * S * D
    out["cfg2_bf16_fwd_bwd"] = {"shape": [B, H, S, D], "ms": t, "TFLOPs": flop / (t * 1e-3) / 1e12,
                                "frac_of_bf16_peak": flop / (t * 1e-3) / PEAK_BF16,
                                "fwd_ms": tf, "fwd_TFLOPs": 4 * B * H * S * S * D / (tf * 1e-3) / 1e12}

    # config 2 causal (causal=True secondary, credited half the flops); the forward
    # replaces the masked keys past each diagonal by per-head V suffix sums (bf16_fwd.hip)
    def bf16_causal_step():
        O, lse = helion_atten_bf16_fwd_training(q, k, v, True)
        helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, True, dO)
    t = event_time(bf16_causal_step, n)
    tf = event_time(lambda: helion_atten_bf16_fwd_training(q, k, v, True), n)
    out["cfg2_bf16_causal_fwd_bwd"] = {"shape": [B, H, S, D], "ms": t,
                                       "TFLOPs": 0.5 * flop / (t * 1e-3) / 1e12,
                                       "frac_of_bf16_peak": 0.5 * flop / (t * 1e-3) / PEAK_BF16,
                                       "fwd_ms": tf,
                                       "fwd_TFLOPs": 2 * B * H * S * S * D / (tf * 1e-3) / 1e12}
    del q, k, v, dO
    # config 3 causal (SURVEY §8f N2 extension): int8 fwd+bwd, credited 7·BH·S²·D (half the scores)
    B, H, S, D = 4, 32, 4096, 128
    q, k, v = (torch.randn((B, H, S, D), device=dev, generator=g).half() for _ in range(3))
    dO = (torch.randn((B, H, S, D), device=dev, generator=g) * 1e-3).half()

    def int8_causal_step():
        O, lse, qi, kiT, vi, sq, sk, sv, km, qb_, kb_ = _int8_forward(q, k, v, smooth=True, images=True,
                                                                      causal=True)
        _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb_, kb_, causal=True)
    t = event_time(int8_causal_step, n)
    flop = 7.0 * B * H * S * S * D
    out["cfg3_int8_causal_fwd_bwd"] = {"shape": [B, H, S, D], "ms": t,
                                       "TOPs": flop / (t * 1e-3) / 1e12,
                                       "frac_of_int8_peak": flop / (t * 1e-3) / PEAK_I8}
    del q, k, v, dO
    # config 4's global problem (8,32,8192,128) on this one GPU: the N = 1 point of its scaling
    # curve (bench.py --gpus N runs the same problem split over N ranks)
    B, H, S, D = 8, 32, 8192, 128
    q, k, v = (torch.randn((B, H, S, D), device=dev, generator=g).half() for _ in range(3))
    dO = (torch.randn((B, H, S, D), device=dev, generator=g) * 1e-3).half()

    def int8_cfg4_step():
        O, lse, qi, kiT, vi, sq, sk, sv, km, qb_, kb_ = _int8_forward(q, k, v, smooth=True, images=True)
        _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb_, kb_)
    t = event_time(int8_cfg4_step, max(2, n // 3))
    flop = 14.0 * B * H * S * S * D
    out["cfg4_int8_fwd_bwd_1gpu"] = {"shape": [B, H, S, D], "ms": t, "TOPs": flop / (t * 1e-3) / 1e12,
                                     "frac_of_int8_peak": flop / (t * 1e-3) / PEAK_I8}
    del q, k, v, dO
    # a decoding step against the int8 key/value cache -- 32 new queries per head,
    # 8 key/value heads shared by 32 query heads, 8192 cached tokens (kv_cache: grouped heads in
    # one workgroup, key splits merged); HBM-bound by the cache read
    from quantizedattention_amd.kv_cache import attention_int8_cached, quantize_kv
    B, Hq, Hkv, Sq, Sk, D = 8, 32, 8, 32, 8192, 128
    kc, vc = (torch.randn((B, Hkv, Sk, D), device=dev, generator=g).half() for _ in range(2))
    qd = torch.randn((B, Hq, Sq, D), device=dev, generator=g).half()
    kv = quantize_kv(kc, vc)
    t = event_time(lambda: attention_int8_cached(qd, kv), n)
    cache = 2 * B * Hkv * Sk * D + 2 * 2 * B * Hkv * Sk // 32
    out["n3_int8_kv_decode"] = {"shape": {"B": B, "Hq": Hq, "Hkv": Hkv, "Sq": Sq, "Sk": Sk, "D": D},
                                "ms": t, "cache_bytes": cache,
                                "cache_TBps": cache / (t * 1e-3) / 1e12,
                                "frac_of_hbm_peak": cache / (t * 1e-3) / PEAK_HBM,
                                "TOPs": 4.0 * B * Hq * Sq * Sk * D / (t * 1e-3) / 1e12}
    del kc, vc, qd, kv
    B, H, S, D = 2, 16, 2048, 128
    x = [torch.randn((B, H, S, D), device=dev, generator=g).bfloat16() for _ in range(6)]
    t = event_time(lambda: helion_attention_jvp_forward_fp32(*x), n)
    flop = 12.0 * B * H * S * S * D
    out["cfg5_jvp_fwd"] = {"shape": [B, H, S, D], "ms": t, "TFLOPs": flop / (t * 1e-3) / 1e12,
                           "frac_of_bf16_peak": flop / (t * 1e-3) / PEAK_BF16}
    return out


def _cgroup_cpus():
    """CPUs the cgroup quota allows this process (cgroup v2 cpu.max / v1 cfs), or None."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) / int(period)))
    except (OSError, ValueError):
        pass
    try:
        quota = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if quota > 0:
            return max(1, quota // period)
    except (OSError, ValueError):
        pass
    return None


def cpu_info():
    model, cores = None, set()
    phys = core = None
    try:
        for ln in open("/proc/cpuinfo"):
            k, _, v = ln.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
            elif not k and phys is not None:
                cores.add((phys, core))
                phys = core = None
    except OSError:
        pass
    if phys is not None:
        cores.add((phys, core))
    return {"cpu_model": model, "logical_cpus": os.cpu_count(), "physical_cores": len(cores) or None,
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": _cgroup_cpus()}


def cpu_baseline(S, D, seconds):
    """The reference's eager fp32 path (baseline_pytorch_attention fwd + autograd bwd, restated in
    oracle/restate.py) on the host cores, one (S, D) head at a time: one warm-up head, then heads
    until `seconds` elapse (at least 3); the median head time scales linearly in B*H (heads are
    independent).  Threads: os.cpu_count(), capped by the CPUs this process may
    actually use (affinity mask, cgroup quota: on a shared GPU box os.cpu_count() counts the whole
    machine while the quota grants a share)."""
    from oracle import restate as R
    info = cpu_info()
    threads = min(x for x in (info["logical_cpus"], info["affinity_cpus"], info["cgroup_quota_cpus"])
                  if x)
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    times = []
    t_total = 0.0
    for i in range(64):
        q, k, v, dO = (torch.randn((1, 1, S, D), generator=g) for _ in range(4))
        t0 = time.perf_counter()
        R.attention_grads_truth(q, k, v, dO, False)
        dt = time.perf_counter() - t0
        if i > 0:            # head 0 is the warm-up
            times.append(dt)
            t_total += dt
        if len(times) >= 3 and t_total >= seconds:
            break
    med = statistics.median(times)
    flop = 14.0 * S * S * D
    return {"value": flop / med / 1e12, "unit": "TFLOP/s", "cores": threads, "kind": "port",
            "torch_threads": torch.get_num_threads(), **info,
            "sample": f"{len(times)} heads of (S,D)=({S},{D}) fwd+bwd fp32 eager "
                      f"(baseline_pytorch_attention + autograd) after 1 warm-up head, median "
                      f"{med * 1e3:.0f} ms per head ({t_total:.1f} s timed); scales linearly in B*H"}


def source_hash():
    """sha256 of the kernel sources and the C-ABI header: ties a committed PMC traffic figure to
    the code it was measured on."""
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "quantizedattention_amd", "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h")))
    for f in files:
        h.update(f.encode())
        h.update(open(os.path.join(csrc, f), "rb").read())
    h.update(open(os.path.join(ROOT, "include", "qattn.h"), "rb").read())
    return h.hexdigest()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`bench.py --gpus N` outside torchrun: start N ranks (one process per GPU) and return their
    exit status.  Runs before this process touches the GPU (no exec after GPU initialisation)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__),
           *sys.argv[1:]]
    return subprocess.call(cmd)


def make_inputs(cfg, shape_arg, world, rank, dev):
    """(q, k, v, dO) of this rank, shapes (B, H, S, D) per rank, and the global FLOP per step."""
    if cfg == 4:
        GB, H, S, D = 8, 32, 8192, 128
        sh = shard_for(GB, H, world, rank)
        g = torch.Generator(device=dev).manual_seed(4321)   # same global tensors on every rank
        outs = []
        for scale in (1.0, 1.0, 1.0, 1e-3):
            full = torch.randn((GB, H, S, D), device=dev, generator=g).mul_(scale).half()
            outs.append(local_slice(full, sh).reshape(-1, H, S, D).clone())
            del full
        flop_global = 14.0 * GB * H * S * S * D
        return outs, flop_global
    B, H, S, D = (int(x) for x in (shape_arg or "4,32,4096,128").split(","))
    g = torch.Generator(device=dev).manual_seed(1234 + rank)   # this rank's batch slice
    q, k, v = (torch.randn((B, H, S, D), device=dev, generator=g).half() for _ in range(3))
    dO = (torch.randn((B, H, S, D), device=dev, generator=g) * 1e-3).half()
    return [q, k, v, dO], world * 14.0 * B * H * S * S * D


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus))
    world = int(env_world or "1")
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)          # before the process group: RCCL binds this device
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == a.gpus
    cfg = a.config or (3 if world == 1 else 4)
    (q, k, v, dO), flop_step = make_inputs(cfg, a.shape, world, rank, dev)
    B, H, S, D = q.shape
    gather = world > 1 and not a.no_gather
    O_full = torch.empty((world * B * H, S, D), dtype=torch.float16, device=dev) if gather else None
    comm = torch.cuda.Stream(device=dev) if gather else None

    def step_int8(with_gather=True):
        # the autograd path of sage_attention_3_int8: quantiser passes also write the bf16 images
        O, lse, qi, kiT, vi, sq, sk, sv, km, qb_, kb_ = _int8_forward(q, k, v, smooth=True, images=True)
        work = None
        if gather and with_gather:
            comm.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(comm):
                work = dist.all_gather_into_tensor(O_full, O.view(B * H, S, D), async_op=True)
        _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb_, kb_)
        if work is not None:
            work.wait()
            torch.cuda.current_stream().wait_stream(comm)

    flop_fb = 14.0 * B * H * S * S * D     # this rank's work per step
    t_i8 = timed(step_int8, a.steps, a.warmup, world)
    # N > 1 (SURVEY §8e "with and without the all-gather"): the same step without the O gather
    t_ng = timed(lambda: step_int8(False), a.steps, a.warmup, world) if gather else None
    extras = world == 1 and not a.skip_bf16
    res_bf = None
    if extras:
        qb, kb, vb = q, k, v.bfloat16()
        dOf = dO.float()

        def step_bf16():
            O, lse = helion_atten_bf16_fwd_training(qb, kb, vb, False)
            helion_flash_atten_2_algo_4_bwd(qb, kb, vb, O, lse, False, dOf)

        t_bf = timed(step_bf16, max(3, a.steps // 2), a.warmup, world)
        res_bf = {"value": flop_fb / t_bf / 1e12, "unit": "TFLOP/s", "ms_per_step": t_bf * 1e3,
                  "frac_of_bf16_peak": flop_fb / t_bf / PEAK_BF16}
        del qb, kb, vb, dOf

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    kt = int8_kernel_times(q, k, v, dO, max(3, a.steps // 2))
    chunk = ws_chunk_heads(B * H, S)
    launches = {"int8_attn_fwd_kernel": 1, "int8_bwd_dkdv_kernel<dK+dV, dS out>": -(-B * H // chunk),
                "int8_bwd_dqw_kernel": -(-B * H // chunk)}   # launches per step
    per_call = {  # algorithmic MFMA work per launch, the step's kernels
        "int8_attn_fwd_kernel": 4.0 * B * H * S * S * D,   # QK^T, PV
        "int8_bwd_dkdv_kernel<dK+dV, dS out>": 8.0 * chunk * S * S * D,   # S, dP, dV, dK
        "int8_bwd_dqw_kernel": 2.0 * chunk * S * S * D,    # dQ (S, dP, dS come from the workspace)
    }
    dom = max(per_call, key=lambda n: kt[n] * launches[n])   # most device time per step
    achieved = per_call[dom] / (kt[dom] * 1e-3) / 1e12
    # the inference forward as a caller sees it: sage_attention_3_int8 without autograd
    # (k-mean + q/k/v quantisation + attention, no bf16 images), one HIP-event-timed call
    fwd_ms = event_time(lambda: _int8_forward(q, k, v, smooth=True, images=False), max(3, a.steps // 2))
    fwd_flop = 4.0 * B * H * S * S * D
    shape_txt = "(8,32,8192,128) split over %d GPU(s), (%d,%d,%d,%d) per rank" % (world, B, H, S, D) \
        if cfg == 4 else "(%d,%d,%d,%d) per rank" % (B, H, S, D)
    out = {
        "metric": "fused-attn fwd+bwd TFLOP/s & us/call at (B,H,S,D)=(4,32,4096,128), int8 vs bf16",
        "value": flop_step / t_i8 / 1e12,
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": t_i8 * 1e3,
        "us_per_call": t_i8 * 1e6,
        "higher_is_better": True,
        "scaling": "strong" if cfg == 4 else "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic (seeded randn q,k,v fp16; dO = 1e-3*randn fp16)",
        "config": {"workload": f"config {cfg}: int8 SageAttention-3 fwd+bwd {shape_txt}, non-causal",
                   "shape_per_rank": [B, H, S, D],
                   "global_shape": [8, 32, 8192, 128] if cfg == 4 else [B * world, H, S, D],
                   "global_batch": 8 if cfg == 4 else B * world,
                   "parallelism": f"batch x head shard over {world} GPU(s)"
                                  + (" + async RCCL all-gather of O" if gather else "")},
        "bf16": res_bf,
        "int8_fwd": {"ms": fwd_ms, "TOPS": fwd_flop / (fwd_ms * 1e-3) / 1e12,
                     "frac_of_int8_peak": fwd_flop / (fwd_ms * 1e-3) / PEAK_I8,
                     "attention_kernel_ms": kt["int8_attn_fwd_kernel"],
                     "attention_kernel_frac_of_int8_peak":
                         fwd_flop / (kt["int8_attn_fwd_kernel"] * 1e-3) / PEAK_I8},
        "kernel_ms": kt,
        "mxfp4_fwd": mxfp4_fwd_times(q, k, v, max(3, a.steps // 2)) if extras and D == 128 else None,
        "configs": other_configs(max(3, a.steps // 2)) if extras and not a.no_configs else None,
        "per_gpu": {"TOPS": flop_fb / t_i8 / 1e12, "frac_of_int8_peak": flop_fb / t_i8 / PEAK_I8},
        "without_gather": None if t_ng is None else {
            "value": flop_step / t_ng / 1e12, "ms_per_step": t_ng * 1e3,
            "gather_cost_ms": (t_i8 - t_ng) * 1e3},
        # "bound": the roof the peak is taken from -- MFMA by arithmetic intensity (>> the ridge,
        # DESIGN.md §3); what limits the kernel in practice is "limiter" below (from the counters)
        "roofline": {"kernel": dom, "bound": "mfma", "achieved": achieved, "peak": PEAK_I8 / 1e12,
                     "unit": "TFLOP/s", "frac": achieved * 1e12 / PEAK_I8, "traffic": None,
                     "launch_ms": kt[dom], "work_per_launch": per_call[dom],
                     "launches_per_step": launches[dom],
                     "heads_per_launch": B * H if dom == "int8_attn_fwd_kernel" else chunk},
    }
    # HBM bytes per launch from the committed PMC passes (tools/profile_round.sh), only when they
    # were measured on these exact kernel sources and this shape
    tr_path = os.path.join(ROOT, "profiles", "traffic_latest.json")
    if os.path.exists(tr_path):
        try:
            tr = json.load(open(tr_path))
            if tr.get("source_sha256") == source_hash() and tr.get("shape") == [B, H, S, D]:
                out["roofline"]["traffic"] = tr["traffic"].get(dom)
                out["roofline"]["traffic_source"] = tr.get("tag")
                # effective shader clock of the kernel's profiled dispatch (GRBM_GUI_ACTIVE / 8 /
                # dispatch time); the peak above assumes 2.4 GHz
                if tr.get("clock_GHz", {}).get(dom):
                    out["roofline"]["clock_GHz_profiled"] = tr["clock_GHz"][dom]
                # SURVEY §8d "also report the VALU ceiling": the counters of the same PMC passes
                # (tools/profile_summary.py).  mfma_util: matrix-pipe busy share; valu_busy: share of
                # cycles a SIMD's vector issue is taken (SQ_ACTIVE_INST_VALU, MFMA issue included);
                # mfma_ceiling_frac: the kernel's attainable fraction of the int8 peak from its own
                # MFMA mix (its bf16 products run at half the int8 rate); limiter: the busier of the
                # two issue resources, i.e. what bounds the kernel in practice
                fwd_c = out["int8_fwd"].setdefault("attention_kernel_counters", {})
                for key, obj in ((dom, out["roofline"]), ("int8_attn_fwd_kernel", fwd_c)):
                    c = tr.get("counters", {}).get(key, {})
                    for f in ("mfma_util", "valu_busy", "mfma_ceiling_frac", "vector_insts_per_mfma"):
                        if f in c:
                            obj[f] = c[f]
                    if "clock_GHz" in c:
                        obj["clock_GHz_profiled"] = c["clock_GHz"]
                    if "mfma_util" in c and "valu_busy" in c:
                        obj["limiter"] = "valu_issue" if c["valu_busy"] > c["mfma_util"] else "mfma"
            else:
                out["roofline"]["traffic_note"] = "PMC traffic in profiles/ is from other sources: omitted"
        except Exception:
            pass
    if world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(S, D, a.cpu_seconds)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
