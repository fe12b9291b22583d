"""The reference's eager fp32 attention (attention_bf16.py:450-478 == attention_int8.py:453-481;
attention_jvp.py:197-215 is its non-causal form), kept because the reference modules export it.

It is a user-facing utility of the API surface, not a fallback: no qattn op ever calls it.
"""
from __future__ import annotations

import math

import torch


def baseline_pytorch_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                               head_dim: int | None = None, causal: bool = False) -> torch.Tensor:
    """softmax(q k^T / sqrt(head_dim)) v in fp32; causal keeps strictly-lower entries and fills the
    rest with -128*ln(2) (bf16:461-476)."""
    if head_dim is None:
        head_dim = q.shape[-1]
    p = torch.matmul(q, k.transpose(2, 3)) / math.sqrt(head_dim)
    if causal:
        qn, kn = p.shape[-2], p.shape[-1]
        mask = (torch.arange(qn, device=q.device)[:, None]
                - torch.arange(kn, device=q.device)[None, :])[None, None]
        p = torch.where(mask > 0, p, -128 * torch.log(torch.tensor([2.0], device=q.device)))
    p = torch.softmax(p.to(torch.float32), dim=-1).to(torch.float32)
    return torch.matmul(p, v)
