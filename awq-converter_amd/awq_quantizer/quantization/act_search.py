"""Activation-aware per-input-channel scale search (scale_method="awq").

No reference counterpart: the reference stores scale_method and never reads it
(awq.py:66,111-112) and collects no activations (SURVEY.md §8a, §8f row 4 — parity with
AutoAWQ unpinned).  The search and its canonical arithmetic are defined in
include/awq_hip.h (awq_act_*); every step below is one HIP launch through that ABI and
the CPU restatement is oracle/awq_oracle.c (oracle_act_*), used only by the tests.

For one layer group — linears W_j [R_j, K] that read the same input x [tokens, K]
(e.g. q/k/v projections) — candidate i scales input channel k by
s_i[k] ∝ x_mean[k]^r / (w_mean[k]^(1-r) + 1e-4) (r = i / n_grid; without duo scaling
x_mean[k]^r), quantizes W·diag(s_i), undoes s_i, and scores the result with
Σ_k E[x_k²] Σ_n (Ŵ - W)²_nk, the diagonal form of AutoAWQ's output MSE.  The winner's
W·diag(s) is quantized with the regular kernels and s is returned so the caller folds
1/s into whatever produces x (a norm's weight, the previous linear's rows).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .. import _hip

ACT_DTYPES = (torch.bfloat16, torch.float16, torch.float32)


def _check_group(weights: Dict[str, torch.Tensor], group_size: int):
    if not weights:
        raise ValueError("quantize_layer_group needs at least one weight")
    Ks = {tuple(w.shape[1:]) for w in weights.values()}
    dts = {w.dtype for w in weights.values()}
    for name, w in weights.items():
        if not isinstance(w, torch.Tensor) or w.dim() != 2:
            raise ValueError(f"{name}: activation-aware search takes 2-D [out_features, in_features] weights")
    if len(Ks) != 1:
        raise ValueError("all weights of a layer group must share in_features (they read the same input)")
    if len(dts) != 1 or next(iter(dts)) not in ACT_DTYPES:
        raise ValueError(f"weights of a layer group must share one dtype of {ACT_DTYPES}, got {sorted(map(str, dts))}")
    K = next(iter(Ks))[0]
    if group_size < 8 or group_size > 512 or group_size & (group_size - 1) or K % group_size:
        raise ValueError(f"activation-aware search needs a power-of-two group_size in [8, 512] dividing "
                         f"in_features (group_size={group_size}, in_features={K})")
    return K


def search_layer_group(weights: Dict[str, torch.Tensor], device: torch.device, *, group_size: int, bits: int,
                       symmetric: bool, n_grid: int, duo_scaling: bool,
                       activations: Optional[torch.Tensor] = None, x_mean: Optional[torch.Tensor] = None,
                       x_sq: Optional[torch.Tensor] = None, table: Optional[torch.Tensor] = None,
                       scale_weights: bool = True) -> dict:
    """Run the search on the device; returns device tensors
    {"x_mean", "x_sq", "w_mean", "table", "losses", "best", "input_scale", "weights": {name: W on
    the device}, "scaled": {name: W·diag(s)} (None with scale_weights=False: the caller
    quantizes W·diag(s) in one pass, awq_quantize_groups_scaled)}.
    `table` overrides the scale table (a caller's own table; since round 5 the kernel's table
    is bit-exact with the oracle's from the inputs alone, include/awq_hip.h awq_pow)."""
    K = _check_group(weights, group_size)
    if not 1 <= n_grid <= _hip.ACT_MAX_GRID:
        raise ValueError(f"search_grid must be in [1, {_hip.ACT_MAX_GRID}] for scale_method='awq': {n_grid}")
    ws = [w.detach().to(device).contiguous() for w in weights.values()]
    if activations is not None:
        if activations.dim() != 2 or activations.shape[1] != K or activations.dtype not in ACT_DTYPES:
            raise ValueError(f"activations must be [tokens, {K}] bf16/fp16/fp32, got {tuple(activations.shape)} "
                             f"{activations.dtype}")
        x_mean, x_sq = _hip.act_stats(activations.detach().to(device).contiguous())
    elif x_mean is None or x_sq is None:
        raise ValueError("scale_method='awq' needs calibration activations, or both x_mean and x_sq")
    else:
        if x_mean.numel() != K or x_sq.numel() != K:
            raise ValueError(f"x_mean / x_sq must have in_features = {K} elements")
        x_mean = x_mean.detach().to(device, torch.float32).contiguous().reshape(K)
        x_sq = x_sq.detach().to(device, torch.float32).contiguous().reshape(K)
    w_mean = _hip.weight_mean(ws, group_size) if duo_scaling else None
    if table is None:
        table = _hip.act_scale_table(x_mean, w_mean, n_grid)
    else:
        table = table.detach().to(device, torch.float32).contiguous()
        if tuple(table.shape) != (n_grid, K):
            raise ValueError(f"table must be [{n_grid}, {K}]")
    part = _hip.act_search_losses(ws, x_sq, table, group_size, bits, symmetric)
    losses, best, s_best = _hip.act_search_select(part, table)
    scaled = {name: _hip.apply_input_scale(w, s_best) for name, w in zip(weights, ws)} if scale_weights else None
    return {"x_mean": x_mean, "x_sq": x_sq, "w_mean": w_mean, "table": table, "losses": losses, "best": best,
            "input_scale": s_best, "weights": dict(zip(weights, ws)), "scaled": scaled}
