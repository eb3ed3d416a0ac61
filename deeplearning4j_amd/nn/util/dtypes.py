"""Accumulation-dtype helper: fp32 math for bf16/fp16/fp32 tensors, fp64 stays fp64 (gradient checks)."""
import torch


def acc(t):
    return t if t.dtype == torch.float64 else t.float()


def acc_dtype(t_or_dtype):
    d = t_or_dtype if isinstance(t_or_dtype, torch.dtype) else t_or_dtype.dtype
    return torch.float64 if d == torch.float64 else torch.float32
