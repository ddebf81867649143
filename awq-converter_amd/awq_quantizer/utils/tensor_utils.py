"""File-discovery helpers with the reference's semantics
(reference src/awq_quantizer/utils/tensor_utils.py:207-314): every *.safetensors file
under a directory (or the single file given); files whose name contains
"consolidated" are ignored when individual shard files exist; more than one file ->
sorted order."""
import os
from typing import List

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
