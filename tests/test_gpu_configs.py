"""Every BASELINE.json config on the HIP path, at its full size.

Where the CPU oracle would be too slow for the whole problem, the full-size run is checked through
size-independent properties (finite outputs, constant-V reproduces the constant, determinism) and
ONE or TWO heads of the full-length call are compared with the oracle / fp32 truth run on those heads
alone (heads are independent).  Tolerances are the ones DESIGN.md §4 states:

  cfg1 (1,4,128,64) bf16 fwd, non-causal: vs torch SDPA on CPU (BASELINE.json config 1): max-abs
       <= 3e-2 and at most 0.5 % of the elements past 1e-2 (the literal beta rule at KT=16 and the bf16
       P move O from the fp32 result: the oracle restatement of the same rule measures 2.2e-2 and
       0.36 % on these inputs, and the kernel must sit within 5e-3 of that distance), and vs the
       oracle at KT=16: max-abs <= 5e-3;
  cfg2 (4,32,2048,128) bf16 fwd+bwd: O vs oracle <= 5e-3 (heads checked); grads relL2 <= 2e-2 vs fp32
       autograd;
  cfg3 (4,32,4096,128) int8 fwd+bwd: grads of one head relL2 <= conftest.INT8_BWD_REL (0.015) vs the corrected oracle and
       <= 0.15 vs fp32 autograd (the forward's full-size test is test_gpu_int8.py);
  cfg4 per-rank shard (1,32,8192,128) of the head-sharded (8,32,8192,128) int8 fwd+bwd: O of one
       head <= 1e-2 vs the oracle, grads of one head <= 0.15 vs fp32 autograd, constant V;
  cfg5 (2,16,2048,128) JVP, bf16 inputs, randn tangents: O <= 1e-2 vs torch.func.jvp, tO <= 1e-2
       relative to max(1, max|tO| / 10) (test_gpu_jvp.py's bar).
"""
import pytest
import torch

from conftest import INT8_BWD_REL

from oracle import restate as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def _randn(shape, seed, dtype, scale=1.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(shape, device="cuda", generator=g) * scale).to(dtype)


# ------------------------------------------------------------------ config 1
def test_cfg1_bf16_fwd_vs_sdpa(lib):
    from quantizedattention_amd.attention_bf16 import helion_atten_bf16_fwd_training
    g = torch.Generator().manual_seed(1)
    q, k, v = (torch.randn((1, 4, 128, 64), generator=g) for _ in range(3))
    qh, kh, vb = q.half(), k.half(), v.bfloat16()
    O, lse = helion_atten_bf16_fwd_training(qh.cuda(), kh.cuda(), vb.cuda(), False)
    torch.cuda.synchronize()
    # BASELINE config 1: SDPA on CPU on the same (fp16 / bf16-representable) values
    sdpa = torch.nn.functional.scaled_dot_product_attention(qh.float(), kh.float(), vb.float())
    d = (O.cpu() - sdpa).abs()
    assert d.max().item() <= 3e-2, d.max().item()
    assert (d > 1e-2).float().mean().item() <= 5e-3
    O_ref, lse_ref = R.bf16_fwd(qh, kh, vb, False, kt=16)
    assert (O.cpu() - O_ref).abs().max().item() <= 5e-3
    assert (lse.cpu() - lse_ref).abs().max().item() <= 5e-3
    # the restatement of the same rule is as far from SDPA as the kernel is
    dr = (O_ref - sdpa).abs().max().item()
    assert abs(dr - d.max().item()) <= 5e-3


# ------------------------------------------------------------------ config 2
def test_cfg2_bf16_fwd_bwd_full_size(lib):
    from quantizedattention_amd.attention_bf16 import (helion_atten_bf16_fwd_training,
                                                       helion_flash_atten_2_algo_4_bwd)
    B, H, S, D = 4, 32, 2048, 128
    q = _randn((B, H, S, D), 21, torch.float16)
    k = _randn((B, H, S, D), 22, torch.float16)
    v = _randn((B, H, S, D), 23, torch.bfloat16)
    dO = _randn((B, H, S, D), 24, torch.float32)
    O1, _ = helion_atten_bf16_fwd_training(q, k, torch.ones_like(v), False)
    assert torch.isfinite(O1).all() and (O1 - 1).abs().max().item() <= 1e-2
    del O1
    O, lse = helion_atten_bf16_fwd_training(q, k, v, False)
    dq, dk, dv = helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, False, dO)
    torch.cuda.synchronize()
    for t in (O, lse, dq, dk, dv):
        assert torch.isfinite(t).all()
    for b, h in ((0, 0), (3, 31)):
        sl = lambda t: t[b:b + 1, h:h + 1].cpu()  # noqa: E731
        O_ref, _ = R.bf16_fwd(sl(q), sl(k), sl(v), False, kt=16)
        assert (sl(O) - O_ref).abs().max().item() <= 5e-3, (b, h)
        tq, tk, tv = R.attention_grads_truth(sl(q), sl(k), sl(v), sl(dO), False)
        for name, a, t in (("dq", dq, tq), ("dk", dk, tk), ("dv", dv, tv)):
            assert _rel(sl(a), t) <= 2e-2, (name, b, h, _rel(sl(a), t))


# ------------------------------------------------------------------ config 3 (backward)
def test_cfg3_int8_bwd_full_length_one_head(lib):
    from quantizedattention_amd.attention_int8 import (helion_atten_int8_hl_dot_bwd,
                                                       helion_atten_int8_hl_dot_fwd)
    B, H, S, D = 4, 32, 4096, 128
    q, k, v = (_randn((B, H, S, D), 30 + i, torch.float16) for i in range(3))
    dO = _randn((B, H, S, D), 33, torch.float16)
    O, lse, qi, kiT, vi, sq, sk, sv, Bq, Bkv = helion_atten_int8_hl_dot_fwd(q, k, v)
    dq, dk, dv = helion_atten_int8_hl_dot_bwd(dO, qi, sq, kiT, None, sk, vi, sv, O, lse, Bq, Bkv)
    torch.cuda.synchronize()
    for t in (dq, dk, dv):
        assert torch.isfinite(t).all()
    b, h = 2, 17
    sl = lambda t: t[b:b + 1, h:h + 1].cpu()  # noqa: E731
    rows = slice((b * H + h) * S, (b * H + h + 1) * S)
    blk = slice((b * H + h) * S // 32, (b * H + h + 1) * S // 32)
    rq, rk, rv = R.int8_bwd(sl(dO), qi[rows].cpu(), sq[blk].cpu(), kiT[:, rows].cpu(), None,
                            sk[blk].cpu(), vi[rows].cpu(), sv[blk].cpu(), sl(O), lse[rows].cpu())
    for name, a, r in (("dq", dq, rq), ("dk", dk, rk), ("dv", dv, rv)):
        rel = _rel(sl(a), r)
        print(f"RELL2 int8-bwd-vs-oracle {name} {rel:.5f}")
        assert rel <= INT8_BWD_REL, (name, rel)
    tq, tk, tv = R.attention_grads_truth(sl(q), sl(k), sl(v), sl(dO), False)
    for name, a, t in (("dq", dq, tq), ("dk", dk, tk), ("dv", dv, tv)):
        assert _rel(sl(a), t) <= 0.15, (name, _rel(sl(a), t))


# ------------------------------------------------------------------ config 4 (per-rank shard)
def test_cfg4_int8_shard_fwd_bwd(lib):
    """Rank r of the 8-GPU (8,32,8192,128) run owns batch r: a (1,32,8192,128) problem, the
    shape every rank of bench.py's config-4 mode runs at N = 8 (the sharding itself is covered by
    tests/test_sharded.py and tests/test_bench_host.py)."""
    from quantizedattention_amd.attention_int8 import sage_attention_3_int8
    B, H, S, D = 1, 32, 8192, 128
    q, k, v = (_randn((B, H, S, D), 40 + i, torch.float16) for i in range(3))
    dO = _randn((B, H, S, D), 43, torch.float16, 1e-3)
    O1 = sage_attention_3_int8(q, k, torch.ones_like(v))
    assert torch.isfinite(O1).all() and (O1.float() - 1).abs().max().item() < 0.05
    del O1
    qd, kd, vd = (t.clone().requires_grad_(True) for t in (q, k, v))
    O = sage_attention_3_int8(qd, kd, vd)
    O.backward(dO)
    torch.cuda.synchronize()
    for t in (O, qd.grad, kd.grad, vd.grad):
        assert torch.isfinite(t).all()
    h = 9
    sl = lambda t: t[:, h:h + 1].detach().cpu()  # noqa: E731
    ks, _ = R.k_smooth(sl(k))
    ref = R.int8_fwd(sl(q), ks, sl(v))
    assert (sl(O).float() - ref[0].float()).abs().max().item() <= 1e-2
    tq, tk, tv = R.attention_grads_truth(sl(q), sl(k), sl(v), sl(dO), False)
    for name, a, t in (("dq", qd.grad, tq), ("dk", kd.grad, tk), ("dv", vd.grad, tv)):
        assert _rel(sl(a), t) <= 0.15, (name, _rel(sl(a), t))


# ------------------------------------------------------------------ config 5
def test_cfg5_jvp_full_size(lib):
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    B, H, S, D = 2, 16, 2048, 128
    x = [_randn((B, H, S, D), 50 + i, torch.bfloat16) for i in range(6)]
    O, tO, lse = helion_attention_jvp_forward_fp32(*x)
    torch.cuda.synchronize()
    for t in (O, tO, lse):
        assert torch.isfinite(t).all()
    O2, tO2, _ = helion_attention_jvp_forward_fp32(*x)
    assert torch.equal(O, O2) and torch.equal(tO, tO2)
    for b, h in ((0, 3), (1, 15)):
        args = [t[b:b + 1, h:h + 1].float().cpu() for t in x]
        Ot, tOt = R.jvp_truth(*args)
        assert (O[b:b + 1, h:h + 1].cpu() - Ot).abs().max().item() <= 1e-2
        tol = 1e-2 * max(1.0, tOt.abs().max().item() / 10)
        assert (tO[b:b + 1, h:h + 1].cpu() - tOt).abs().max().item() <= tol
