"""Tensor helpers with the reference's semantics (src/awq_quantizer/utils/tensor_utils.py).

File discovery (:207-314): every *.safetensors file under a directory (or the single
file given); files whose name contains "consolidated" are ignored when individual shard
files exist; more than one file -> sorted order.

Host-side helpers the reference exports (:10-204): dtype conversions, statistics and
the percentile lookup (2-argument signature: the reference's quantizer calls it with 3
and raises TypeError, which AWQQuantizer reproduces), fp16 dynamic scaling.  They are
not on the quantize path; the statistics are computed by torch on the tensor's own
device in fp32, like the reference.
"""
import os
from typing import Dict, List, Optional, Tuple

import torch

SAFETENSORS_DTYPES = {"BF16", "F16", "F32", "F64"}


def is_consolidated_file(file_path: str) -> bool:
    return file_path.endswith(".safetensors") and "consolidated" in os.path.basename(file_path).lower()


def filter_safetensor_files(file_paths: List[str]) -> List[str]:
    st = [p for p in file_paths if p.endswith(".safetensors")]
    individual = [p for p in st if not is_consolidated_file(p)]
    consolidated = [p for p in st if is_consolidated_file(p)]
    return individual if individual else consolidated


def get_model_files(model_path: str) -> List[str]:
    if os.path.isfile(model_path):
        return [model_path] if model_path.endswith(".safetensors") else []
    found = []
    for root, _, files in os.walk(model_path):
        found += [os.path.join(root, f) for f in files if f.endswith(".safetensors")]
    return filter_safetensor_files(found)


def filter_consolidated_files(files: List[str]) -> List[str]:
    if len(files) <= 1:
        return files
    individual = [f for f in files if not is_consolidated_file(f)]
    if individual:
        return sorted(individual)
    return [f for f in files if is_consolidated_file(f)]


_TYPE_NAMES = {torch.float32: "float32", torch.float16: "float16", torch.bfloat16: "bfloat16", torch.int32: "int32",
               torch.int8: "int8", torch.uint8: "uint8", torch.int16: "int16", torch.int64: "int64",
               torch.bool: "bool"}


def convert_bf16_to_fp16(tensor: torch.Tensor) -> torch.Tensor:
    """bf16 -> fp16 (:10-22); any other dtype is returned as is."""
    return tensor.to(torch.float16) if tensor.dtype == torch.bfloat16 else tensor


def convert_fp16_to_bf16(tensor: torch.Tensor) -> torch.Tensor:
    """fp16 -> bf16 (:25-37); any other dtype is returned as is."""
    return tensor.to(torch.bfloat16) if tensor.dtype == torch.float16 else tensor


def get_tensor_type(tensor: torch.Tensor) -> str:
    """Short dtype name (:40-61), str(dtype) for the ones outside the table."""
    return _TYPE_NAMES.get(tensor.dtype, str(tensor.dtype))


def _f32(tensor: torch.Tensor) -> torch.Tensor:
    return tensor if tensor.dtype == torch.float32 else tensor.to(torch.float32)


def get_tensor_stats(tensor: torch.Tensor) -> Dict[str, float]:
    """min / max / mean / std (unbiased) / abs_mean / sparsity (fraction of exact zeros),
    computed in fp32 (:64-84)."""
    x = _f32(tensor)
    return {"min": float(x.min()), "max": float(x.max()), "mean": float(x.mean()), "std": float(x.std()),
            "abs_mean": float(x.abs().mean()), "sparsity": float((x == 0).float().mean())}


def get_percentile_value(tensor: torch.Tensor, percentile: float) -> float:
    """Element of rank floor(percentile * (n - 1)) of the ascending fp32 values (:87-110);
    NaN sorts last, as in torch.sort."""
    flat = _f32(tensor).reshape(-1)
    k = int(percentile * (flat.numel() - 1))
    return float(torch.sort(flat).values[k])


def get_optimal_fp16_scale(tensor: torch.Tensor) -> float:
    """65504 / max|x| (1.0 for an all-zero tensor) (:113-135)."""
    m = float(_f32(tensor).abs().max())
    return 65504.0 / m if m > 0 else 1.0


def apply_dynamic_scale(tensor: torch.Tensor, scale: Optional[float] = None) -> Tuple[torch.Tensor, float]:
    """(fp32 tensor * scale, scale); scale defaults to get_optimal_fp16_scale (:138-161)."""
    x = _f32(tensor)
    if scale is None:
        scale = get_optimal_fp16_scale(x)
    return x * scale, scale


def revert_dynamic_scale(tensor: torch.Tensor, scale: float) -> torch.Tensor:
    """fp32 tensor / scale (:164-183)."""
    return _f32(tensor) / scale


def get_device_from_config(config: Dict) -> torch.device:
    """config["hardware"]["device"] (default "cuda"); "cuda" without a GPU -> cpu (:186-204)."""
    name = config.get("hardware", {}).get("device", "cuda")
    if name == "cuda" and not torch.cuda.is_available():
        return torch.device("cpu")
    if name == "mps" and not (hasattr(torch.backends, "mps") and torch.backends.mps.is_available()):
        return torch.device("cpu")
    return torch.device(name)
