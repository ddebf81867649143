"""ctypes binding of libawq_hip.so (include/awq_hip.h) — the only compute path.

There is deliberately no CPU fallback: if the library is missing, or no gfx950 device
is present, every quantize call raises.  PyTorch provides device memory and the stream;
the arithmetic is the HIP kernels in awq-converter_amd/csrc.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libawq_hip.so")
ABI_VERSION = 3

AWQ_DTYPE = {torch.bfloat16: 0, torch.float16: 1, torch.float32: 2, torch.float64: 3}

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int


class TensorDesc(ctypes.Structure):
    """Mirror of awq_tensor_desc (include/awq_hip.h)."""
    _fields_ = [("w", _P), ("rows", _I64), ("K", _I64), ("qweight", _P), ("qzeros", _P),
                ("scales", _P), ("tensor_q", _P), ("zeros", _P), ("tile_begin", _I64),
                ("tile_count", _I64)]


assert ctypes.sizeof(TensorDesc) == 80

# symbol -> (restype, argtypes); the CPU test suite checks every one is exported.
SIGNATURES = {
    "awq_abi_version": (_I32, []),
    "awq_last_error": (ctypes.c_char_p, []),
    "awq_device_check": (_I32, [ctypes.c_char_p, _I32]),
    "awq_quantize_groups": (_I32, [_P, _I32, _I64, _I64, _I64, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "awq_quantize_search": (_I32, [_P, _I32, _I64, _I64, _I64, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "awq_ragged_eligible": (_I32, [_I32, _I64, _I64, _I64]),
    "awq_plan_ragged": (_I64, [ctypes.POINTER(TensorDesc), _I32, _I32]),
    "awq_stream_copy": (_I32, [_P, _P, _I64, _P]),
    "awq_export_autoawq_gemm": (_I32, [_P, _P, _P, _I64, _I64, _I64, _I32, _P, _P, _P, _P]),
    "awq_plan_block_tensor": (_I64, [ctypes.POINTER(TensorDesc), _I32, _I64, _P, _I64]),
    "awq_quantize_ragged": (_I32, [_P, _I32, _I64, _P, _I32, _I32, _I32, _P]),
    "awq_dequantize": (_I32, [_P, _P, _P, _I64, _I64, _I64, _P, _P]),
    "awq_dequantize_packed": (_I32, [_P, _P, _P, _I64, _I64, _I64, _I32, _I32, _P, _P]),
    "awq_pack_rows": (_I32, [_P, _I64, _I64, _I32, _I32, _P, _P]),
    "awq_selftest": (_I32, [_I32, _P, _P]),
}

_lib = None
_lock = threading.Lock()
_checked_devices = set()


class HipUnavailable(RuntimeError):
    """The HIP library or a gfx950 device is missing (no CPU fallback exists)."""


def load_library(path: str = LIB_PATH):
    """Load libawq_hip.so and bind every entry point (works without a GPU)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if path == LIB_PATH:   # tuning hook: run everything against another in-tree build
            path = os.environ.get("AWQ_HIP_LIB", path)
        if not os.path.exists(path):
            raise HipUnavailable(
                f"awq_quantizer: {path} is missing — build it with "
                f"`make -C awq-converter_amd/csrc` (hipcc --offload-arch=gfx950). "
                f"There is no CPU fallback.")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.awq_abi_version() != ABI_VERSION:
            raise HipUnavailable(f"libawq_hip.so ABI {lib.awq_abi_version()} != {ABI_VERSION}")
        _lib = lib
        return lib


def last_error() -> str:
    return (load_library().awq_last_error() or b"").decode(errors="replace")


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (code {rc}): {last_error()}")


def require_device(device: torch.device) -> None:
    """Fail loudly unless `device` is a HIP gfx950 GPU."""
    if device.type != "cuda" or not torch.cuda.is_available():
        raise HipUnavailable("awq_quantizer (MI355X build) needs a HIP gfx950 GPU; none is available "
                             "(there is no CPU fallback)")
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx in _checked_devices:
        return
    lib = load_library()
    buf = ctypes.create_string_buffer(64)
    with torch.cuda.device(idx):
        rc = lib.awq_device_check(buf, 64)
    if rc != 0:
        raise HipUnavailable(last_error())
    _checked_devices.add(idx)


def stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def quantize_groups(x: torch.Tensor, rows: int, K: int, L: int, bits: int, symmetric: bool, *,
                    qweight=None, qzeros=None, scales=None, tensor_q=None, zeros=None) -> None:
    """Launch awq_quantize_groups on x (device, contiguous) with caller-allocated outputs."""
    lib = load_library()
    rc = lib.awq_quantize_groups(ptr(x), AWQ_DTYPE[x.dtype], rows, K, L, bits, int(bool(symmetric)),
                                 ptr(qweight), ptr(qzeros), ptr(scales), ptr(tensor_q), ptr(zeros),
                                 ctypes.c_void_p(stream_ptr(x.device)))
    check(rc, "awq_quantize_groups")


def quantize_search(x: torch.Tensor, rows: int, K: int, L: int, bits: int, symmetric: bool, n_grid: int,
                    n_candidates: int, *, qweight=None, qzeros=None, scales=None, tensor_q=None,
                    zeros=None) -> None:
    """Launch awq_quantize_search (opt-in clip search, include/awq_hip.h)."""
    lib = load_library()
    rc = lib.awq_quantize_search(ptr(x), AWQ_DTYPE[x.dtype], rows, K, L, bits, int(bool(symmetric)),
                                 int(n_grid), int(n_candidates), ptr(qweight), ptr(qzeros), ptr(scales),
                                 ptr(tensor_q), ptr(zeros), ctypes.c_void_p(stream_ptr(x.device)))
    check(rc, "awq_quantize_search")


def ragged_eligible(dtype: torch.dtype, rows: int, K: int, L: int) -> bool:
    if dtype not in AWQ_DTYPE:
        return False
    return bool(load_library().awq_ragged_eligible(AWQ_DTYPE[dtype], rows, K, L))


def plan_ragged(descs, bits: int) -> int:
    lib = load_library()
    arr = (TensorDesc * len(descs))(*descs)
    total = lib.awq_plan_ragged(arr, len(descs), bits)
    if total < 0:
        raise RuntimeError(f"awq_plan_ragged failed: {last_error()}")
    for i in range(len(descs)):
        descs[i] = arr[i]
    return total


def descs_to_device(descs, device: torch.device) -> torch.Tensor:
    arr = (TensorDesc * len(descs))(*descs)
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.to(device)


def plan_block_tensor(descs, total_tiles: int, device: torch.device) -> torch.Tensor:
    """awq_plan_block_tensor: the tensor of every workgroup's first tile, as a device int32
    tensor (the kernel then skips the per-wave descriptor search)."""
    lib = load_library()
    arr = (TensorDesc * len(descs))(*descs)
    nblk = -(-int(total_tiles) // 4)
    host = torch.empty(max(nblk, 1), dtype=torch.int32)
    rc = lib.awq_plan_block_tensor(arr, len(descs), total_tiles, ctypes.c_void_p(host.data_ptr()), host.numel())
    if rc < 0:
        raise RuntimeError(f"awq_plan_block_tensor failed: {last_error()}")
    return host.to(device)


def quantize_ragged(descs_dev: torch.Tensor, n: int, total_tiles: int, bits: int, symmetric: bool,
                    stream: int, block_tensor: Optional[torch.Tensor] = None,
                    dtype: torch.dtype = torch.bfloat16) -> None:
    rc = load_library().awq_quantize_ragged(ptr(descs_dev), n, total_tiles, ptr(block_tensor), AWQ_DTYPE[dtype],
                                            bits, int(bool(symmetric)), ctypes.c_void_p(stream))
    check(rc, "awq_quantize_ragged")


def stream_copy(src: torch.Tensor, dst: torch.Tensor, stream: int) -> None:
    rc = load_library().awq_stream_copy(ptr(src), ptr(dst), src.numel() * src.element_size(), ctypes.c_void_p(stream))
    check(rc, "awq_stream_copy")


def export_autoawq_gemm(qweight, qzeros, scales, N: int, K: int, L: int, bits: int, qweight_t, qzeros_t,
                        scales_t) -> None:
    rc = load_library().awq_export_autoawq_gemm(ptr(qweight), ptr(qzeros), ptr(scales), N, K, L, bits,
                                                ptr(qweight_t), ptr(qzeros_t), ptr(scales_t),
                                                ctypes.c_void_p(stream_ptr(qweight.device)))
    check(rc, "awq_export_autoawq_gemm")


def dequantize(tensor_q, scales, zeros, rows, K, L, out) -> None:
    rc = load_library().awq_dequantize(ptr(tensor_q), ptr(scales), ptr(zeros), rows, K, L, ptr(out),
                                       ctypes.c_void_p(stream_ptr(out.device)))
    check(rc, "awq_dequantize")


def dequantize_packed(qweight, qzeros, scales, rows, K, L, bits, symmetric, out) -> None:
    rc = load_library().awq_dequantize_packed(ptr(qweight), ptr(qzeros), ptr(scales), rows, K, L, bits,
                                              int(bool(symmetric)), ptr(out),
                                              ctypes.c_void_p(stream_ptr(out.device)))
    check(rc, "awq_dequantize_packed")


def pack_rows(v, rows, n, bits, qmin, out) -> None:
    rc = load_library().awq_pack_rows(ptr(v), rows, n, bits, qmin, ptr(out),
                                      ctypes.c_void_p(stream_ptr(out.device)))
    check(rc, "awq_pack_rows")


def selftest(which: int, device: torch.device) -> int:
    """Run a device self-test (include/awq_hip.h awq_selftest); returns the mismatch count."""
    out = torch.zeros(1, dtype=torch.int64, device=device)
    check(load_library().awq_selftest(which, ptr(out), ctypes.c_void_p(stream_ptr(device))), "awq_selftest")
    return int(out.item())
