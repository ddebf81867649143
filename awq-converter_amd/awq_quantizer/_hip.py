"""ctypes binding of libawq_hip.so (include/awq_hip.h) — the only compute path.

There is deliberately no CPU fallback: if the library is missing, or no gfx950 device
is present, every quantize call raises.  PyTorch provides device memory and the stream;
the arithmetic is the HIP kernels in awq-converter_amd/csrc.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
from typing import Optional

import torch

from ._early import ABI_VERSION, LIB_DIR, LIB_PATH
# diagnostics build (`make -C awq-converter_amd/csrc diag`: -DAWQ_DIAG, awq_set_tuning + the A/B
# kernel variants): loaded only by tuning() below and by scripts/, never by the product path
DIAG_LIB_PATH = os.path.join(LIB_DIR, "libawq_hip_diag.so")
Q_SMALL_TENSOR = 1      # include/awq_hip.h AWQ_Q_SMALL_TENSOR

AWQ_DTYPE = {torch.bfloat16: 0, torch.float16: 1, torch.float32: 2, torch.float64: 3}
# awq_apply_params_ex tensor dtypes (AWQ_DTYPE_I32 .. AWQ_DTYPE_U64) and op dtypes (up to AWQ_DTYPE_U8)
APPLY_DTYPE = {**AWQ_DTYPE, torch.int32: 4, torch.int64: 5, torch.int16: 6, torch.int8: 7, torch.uint8: 8,
               torch.bool: 9, torch.uint16: 10, torch.uint32: 11, torch.uint64: 12}
APPLY_OP_DTYPE = {d: c for d, c in APPLY_DTYPE.items() if c <= 8}
APPLY_SCALE_ONE_ELEMENT, APPLY_ZERO_ONE_ELEMENT = 1, 2
APPLY_SCALE_INT, APPLY_ZERO_INT, APPLY_SCALE_UNSIGNED, APPLY_ZERO_UNSIGNED, APPLY_IEEE_CLAMP = 4, 8, 16, 32, 64

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int


class TensorDesc(ctypes.Structure):
    """Mirror of awq_tensor_desc (include/awq_hip.h)."""
    _fields_ = [("w", _P), ("rows", _I64), ("K", _I64), ("qweight", _P), ("qzeros", _P),
                ("scales", _P), ("tensor_q", _P), ("zeros", _P), ("tile_begin", _I64),
                ("tile_count", _I64)]


assert ctypes.sizeof(TensorDesc) == 80


class StreamItem(ctypes.Structure):
    """Mirror of awq_stream_item (include/awq_hip.h)."""
    _fields_ = [("fd", _I32), ("dtype", _I32), ("offset", _I64), ("rows", _I64), ("K", _I64), ("qweight", _P),
                ("qzeros", _P), ("scales", _P), ("tensor_q", _P), ("zeros", _P), ("dev_out", _P), ("host_out", _P),
                ("out_bytes", _I64), ("dev_out2", _P), ("host_out2", _P), ("out_bytes2", _I64),
                ("dev_gate", _I32), ("host_gate", _I32)]


class StreamConfig(ctypes.Structure):
    """Mirror of awq_stream_config (include/awq_hip.h)."""
    _fields_ = [("bits", _I32), ("symmetric", _I32), ("group_size", _I32), ("readers", _I32), ("nslots", _I32),
                ("trace_batches", _I32), ("search_grid", _I32), ("search_candidates", _I32), ("slot_bytes", _I64), ("first_batch_bytes", _I64), ("host_staging", _P),
                ("dev_staging", _P), ("compute_stream", _P),
                ("h2d_stream", _P), ("d2h_stream", _P), ("trace", _P)]


STREAM_TRACE_FIELDS = 14   # AWQ_STREAM_TRACE_FIELDS
STREAM_TRACE_NAMES = ("read_first", "read_last", "h2d_enq", "kern_enq", "d2h_enq", "h2d_done", "kern_done",
                      "d2h_done", "h2d_call", "d2h_call", "plan", "wait_slot", "ragged_launch", "other_launch")


class StreamStats(ctypes.Structure):
    """Mirror of awq_stream_stats (include/awq_hip.h)."""
    _fields_ = [("batches", _I64), ("pieces", _I64), ("bytes_read", _I64), ("wall_s", ctypes.c_double),
                ("read_busy_s", ctypes.c_double), ("wait_read_s", ctypes.c_double), ("wait_slot_s", ctypes.c_double),
                ("wait_release_s", ctypes.c_double), ("prepare_s", ctypes.c_double)]


assert ctypes.sizeof(StreamItem) == 128 and ctypes.sizeof(StreamConfig) == 96


class Tuning(ctypes.Structure):
    """Mirror of awq_tuning (csrc/awq_diag.h, diagnostics build): diagnostics / A-B controls only."""
    _fields_ = [("max_blocks", _I32), ("tiles_per_wave", _I32), ("no_rowgroup", _I32), ("rg_waves", _I32),
                ("rg_gpt", _I32), ("gen_noreg", _I32), ("dq_words_v1", _I32),
                ("rg_p1", _I32), ("rg_lds_full", _I32), ("rg_ldsdma", _I32), ("rg_p2reg", _I32),
                ("rg_p1u", _I32)]

# symbol -> (restype, argtypes); the CPU test suite checks every one is exported.
SIGNATURES = {
    "awq_abi_version": (_I32, []),
    # chunk-file writer (include/awq_ptfile.h; awq_quantizer/ptfile.py)
    "awq_crc32": (ctypes.c_uint32, [ctypes.c_uint32, _P, _I64, _I32]),
    "awq_write_pt": (_I32, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, _I64, _I32, ctypes.POINTER(ctypes.c_void_p),
                            ctypes.POINTER(ctypes.c_int64), ctypes.c_char_p]),
    "awq_last_error": (ctypes.c_char_p, []),
    "awq_device_check": (_I32, [ctypes.c_char_p, _I32]),
    "awq_quantize_groups": (_I32, [_P, _I32, _I64, _I64, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "awq_quantize_search": (_I32, [_P, _I32, _I64, _I64, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "awq_quantize_groups_ex": (_I32, [_P, _I32, _I64, _I64, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "awq_quantize_search_ex": (_I32, [_P, _I32, _I64, _I64, _I32, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P,
                                      _P]),
    "awq_group_params": (_I32, [_P, _I32, _I64, _I64, _I64, _I32, _I32, _P, _P, _P]),
    "awq_group_params_ex": (_I32, [_P, _I32, _I64, _I64, _I64, _I32, _I32, _I32, _P, _P, _P]),
    "awq_apply_params": (_I32, [_P, _I32, _I64, _I64, _I64, _P, _P, _I32, _I32, _I32, _P, _P]),
    "awq_apply_params_ex": (_I32, [_P, _I32, _I64, _I64, _I64, _P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _P, _P]),
    "awq_packs_directly": (_I32, [_I32, _I64, _I64, _I64]),
    "awq_ragged_eligible": (_I32, [_I32, _I64, _I64, _I64]),
    "awq_plan_ragged": (_I64, [ctypes.POINTER(TensorDesc), _I32, _I32, _I64]),
    "awq_stream_copy": (_I32, [_P, _P, _I64, _P]),
    "awq_stream_ceiling": (_I32, [_P, _P, _I64, _P]),
    "awq_dequant_ceiling": (_I32, [_P, _P, _I64, _P]),
    "awq_export_autoawq_gemm": (_I32, [_P, _P, _P, _I64, _I64, _I64, _I32, _P, _P, _P, _P]),
    "awq_plan_block_tensor": (_I64, [ctypes.POINTER(TensorDesc), _I32, _I64, _P, _I64]),
    "awq_ragged_flags": (_I32, [ctypes.POINTER(TensorDesc), _I32, _I64]),
    "awq_quantize_ragged": (_I32, [_P, _I32, _I64, _P, _I32, _I32, _I32, _I64, _I32, _P]),
    "awq_quantize_ragged_search": (_I32, [_P, _I32, _I64, _P, _I32, _I32, _I32, _I64, _I32, _I32, _I32, _P]),
    "awq_dequantize": (_I32, [_P, _P, _P, _I64, _I64, _I64, _P, _P]),
    "awq_dequantize_packed": (_I32, [_P, _P, _P, _I64, _I64, _I64, _I32, _I32, _P, _P]),
    "awq_pack_rows": (_I32, [_P, _I64, _I64, _I32, _I32, _P, _P]),
    "awq_selftest": (_I32, [_I32, _P, _P]),
    "awq_stream_table_bytes": (_I64, [_I64]),
    "awq_stream_start": (_I32, [ctypes.POINTER(StreamItem), _I32, ctypes.POINTER(StreamConfig),
                                ctypes.POINTER(ctypes.c_void_p)]),
    "awq_stream_batches": (_I64, [_P]),
    "awq_stream_plan": (_I64, [ctypes.POINTER(StreamItem), _I32, ctypes.POINTER(StreamConfig),
                               ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
    "awq_stream_release": (_I32, [_P, _I32]),
    "awq_runtime_warmup": (_I32, [_I32]),
    "awq_runtime_warmup_wait": (_I32, [_I32, ctypes.POINTER(ctypes.c_double)]),
    "awq_stream_wait": (_I32, [_P, _I64, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
    "awq_stream_end": (_I32, [_P, ctypes.POINTER(StreamStats)]),
    "awq_act_stats": (_I32, [_P, _I32, _I64, _I64, _P, _P, _P, _P]),
    "awq_weight_colsum": (_I32, [_P, _I32, _I64, _I64, _I64, _P, _P, _P]),
    "awq_column_mean": (_I32, [_P, _I64, _I64, ctypes.c_double, _P, _P]),
    "awq_act_scale_table": (_I32, [_P, _P, _I64, _I32, _P, _P]),
    "awq_act_scale_table_ws": (_I32, [_P, _P, _I64, _I32, _P, _P, _P]),
    "awq_quantize_groups_scaled": (_I32, [_P, _I32, _I64, _I64, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    "awq_act_recip_table": (_I32, [_P, _I32, _I64, _P, _P]),
    "awq_act_search_losses": (_I32, [_P, _I32, _I64, _I64, _I64, _I32, _I32, _P, _P, _I32, _P, _P, _I64, _P]),
    "awq_act_search_select": (_I32, [_P, _I32, _I64, _P, _I64, _P, _P, _P, _P, _P]),
    "awq_apply_input_scale": (_I32, [_P, _I32, _I64, _I64, _P, _P, _P]),
}

_lib = None
_lock = threading.Lock()
_checked_devices = set()


class HipUnavailable(RuntimeError):
    """The HIP library or a gfx950 device is missing (no CPU fallback exists)."""


def load_library(path: str = LIB_PATH):
    """Load libawq_hip.so and bind every entry point (works without a GPU).  The first call
    decides the library (diagnostics scripts pass another in-tree build explicitly; nothing
    in the environment redirects it)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
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
                    qweight=None, qzeros=None, scales=None, tensor_q=None, zeros=None, small: bool = False) -> None:
    """Launch awq_quantize_groups_ex on x (device, contiguous) with caller-allocated outputs.
    small: the reference's small-tensor path (awq.py:130-171, L = K; AWQ_Q_SMALL_TENSOR)."""
    lib = load_library()
    rc = lib.awq_quantize_groups_ex(ptr(x), AWQ_DTYPE[x.dtype], rows, K, L, bits, int(bool(symmetric)),
                                    Q_SMALL_TENSOR if small else 0, ptr(qweight), ptr(qzeros), ptr(scales),
                                    ptr(tensor_q), ptr(zeros), ctypes.c_void_p(stream_ptr(x.device)))
    check(rc, "awq_quantize_groups")


def quantize_search(x: torch.Tensor, rows: int, K: int, L: int, bits: int, symmetric: bool, n_grid: int,
                    n_candidates: int, *, qweight=None, qzeros=None, scales=None, tensor_q=None,
                    zeros=None, small: bool = False) -> None:
    """Launch awq_quantize_search_ex (opt-in clip search, include/awq_hip.h)."""
    lib = load_library()
    rc = lib.awq_quantize_search_ex(ptr(x), AWQ_DTYPE[x.dtype], rows, K, L, bits, int(bool(symmetric)),
                                    Q_SMALL_TENSOR if small else 0, int(n_grid), int(n_candidates), ptr(qweight),
                                    ptr(qzeros), ptr(scales), ptr(tensor_q), ptr(zeros),
                                    ctypes.c_void_p(stream_ptr(x.device)))
    check(rc, "awq_quantize_search")


GP_TORCH_GPU = 1        # include/awq_hip.h AWQ_GP_TORCH_GPU


def group_params(x: torch.Tensor, rows: int, K: int, L: int, bits: int, symmetric: bool, torch_gpu: bool = False):
    """awq_group_params_ex: the reference's per-group (scale, zero point) in x's own arithmetic,
    as exact float64 device tensors [rows, ceil(K / L)]; torch_gpu: as torch's GPU kernels
    evaluate awq.py:202-211 (AWQ_GP_TORCH_GPU)."""
    G = -(-K // L) if K else 0
    s = torch.empty((rows, G), dtype=torch.float64, device=x.device)
    z = torch.empty((rows, G), dtype=torch.float64, device=x.device)
    check(load_library().awq_group_params_ex(ptr(x), AWQ_DTYPE[x.dtype], rows, K, L, bits, int(bool(symmetric)),
                                             GP_TORCH_GPU if torch_gpu else 0, ptr(s), ptr(z), _stream(x)),
          "awq_group_params_ex")
    return s, z


def apply_params(x: torch.Tensor, rows: int, K: int, L: int, scales: torch.Tensor, zeros: torch.Tensor, qmin: int,
                 qmax: int, mode: int, op1_dtype: torch.dtype, op2_dtype: torch.dtype, flags: int) -> torch.Tensor:
    """awq_apply_params_ex: mode 0 quantize / mode 1 dequantize x (device, contiguous) with
    per-group parameters (8-byte words: float64 values, or int64 / uint64 under the *_INT /
    *_UNSIGNED flags), the first op in op1_dtype and the second in op2_dtype (torch's result
    dtypes); result of op2_dtype, x's shape."""
    out = torch.empty(x.shape, dtype=op2_dtype, device=x.device)
    check(load_library().awq_apply_params_ex(ptr(x), APPLY_DTYPE[x.dtype], rows, K, L, ptr(scales), ptr(zeros),
                                             int(qmin), int(qmax), int(mode), APPLY_OP_DTYPE[op1_dtype],
                                             APPLY_OP_DTYPE[op2_dtype], int(flags), ptr(out), _stream(x)),
          "awq_apply_params_ex")
    return out


def packs_directly(dtype: torch.dtype, rows: int, K: int, L: int) -> bool:
    """awq_quantize_groups writes packed outputs without int32 staging buffers."""
    if dtype not in AWQ_DTYPE:
        return False
    return bool(load_library().awq_packs_directly(AWQ_DTYPE[dtype], rows, K, L))


def ragged_eligible(dtype: torch.dtype, rows: int, K: int, L: int) -> bool:
    if dtype not in AWQ_DTYPE:
        return False
    return bool(load_library().awq_ragged_eligible(AWQ_DTYPE[dtype], rows, K, L))


def ragged_flags(descs, group_size: int = 128) -> int:
    arr = (TensorDesc * len(descs))(*descs)
    return int(load_library().awq_ragged_flags(arr, len(descs), group_size))


def plan_ragged(descs, bits: int, group_size: int = 128) -> int:
    lib = load_library()
    arr = (TensorDesc * len(descs))(*descs)
    total = lib.awq_plan_ragged(arr, len(descs), bits, group_size)
    if total < 0:
        raise RuntimeError(f"awq_plan_ragged failed: {last_error()}")
    for i in range(len(descs)):
        descs[i] = arr[i]
    return total


_diag = None


def load_diag_library(path: str = DIAG_LIB_PATH):
    """The diagnostics build, bound like load_library() plus awq_set_tuning."""
    global _diag
    with _lock:
        if _diag is None:
            if not os.path.exists(path):
                raise HipUnavailable(f"{path} is missing — build it with `make -C awq-converter_amd/csrc diag`")
            lib = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype, fn.argtypes = res, args
            lib.awq_set_tuning.restype = _I32
            lib.awq_set_tuning.argtypes = [ctypes.POINTER(Tuning)]
            if lib.awq_abi_version() != ABI_VERSION:
                raise HipUnavailable(f"libawq_hip_diag.so ABI {lib.awq_abi_version()} != {ABI_VERSION}")
            _diag = lib
        return _diag


@contextlib.contextmanager
def tuning(**kw):
    """Diagnostics / A-B only (awq-converter_amd/csrc/awq_diag.h).  PROCESS-WIDE: inside the
    block every entry point of this module, on every thread, calls the DIAGNOSTICS build (the
    shipped libawq_hip.so has no tuning and no variant kernels).  The overrides (max_blocks,
    tiles_per_wave, no_rowgroup, rg_waves, rg_gpt, gen_noreg, dq_words_v1, rg_p1, rg_lds_full)
    are thread-local inside that library: they apply to launches from the calling thread only
    (not, e.g., to the native stream's submitter thread).  Same results, other speed.  Restores
    the product library on exit; meant for single-threaded scripts."""
    global _lib
    diag = load_diag_library()
    prev = load_library()
    t = Tuning(**{k: int(v) for k, v in kw.items()})
    if diag.awq_set_tuning(ctypes.byref(t)) != 0:
        raise RuntimeError(f"awq_set_tuning failed: {(diag.awq_last_error() or b'').decode()}")
    with _lock:
        _lib = diag
    try:
        yield diag
    finally:
        diag.awq_set_tuning(None)
        with _lock:
            _lib = prev



def _upload(host: torch.Tensor, device: torch.device) -> torch.Tensor:
    """Host table -> device on the current stream.  From page-locked memory the copy is
    asynchronous (the CLI pipeline keeps running); torch's caching host allocator holds the
    staging block until the copy has completed, so it may be dropped right away."""
    pinned = torch.empty(host.shape, dtype=host.dtype, pin_memory=True)
    pinned.copy_(host)
    return pinned.to(device, non_blocking=True)


def descs_to_device(descs, device: torch.device) -> torch.Tensor:
    arr = (TensorDesc * len(descs))(*descs)
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return _upload(host, device)


def plan_block_tensor(descs, total_tiles: int, device: torch.device) -> torch.Tensor:
    """awq_plan_block_tensor: the tensor of every workgroup's first tile, as a device int32
    tensor (the kernel then skips the per-wave descriptor search)."""
    lib = load_library()
    arr = (TensorDesc * len(descs))(*descs)
    nblk = lib.awq_plan_block_tensor(arr, len(descs), total_tiles, None, 0)   # size query
    if nblk < 0:
        raise RuntimeError(f"awq_plan_block_tensor failed: {last_error()}")
    host = torch.empty(max(nblk, 1), dtype=torch.int32)
    rc = lib.awq_plan_block_tensor(arr, len(descs), total_tiles, ctypes.c_void_p(host.data_ptr()), host.numel())
    if rc < 0:
        raise RuntimeError(f"awq_plan_block_tensor failed: {last_error()}")
    return _upload(host, device)


def quantize_ragged(descs_dev: torch.Tensor, n: int, total_tiles: int, bits: int, symmetric: bool,
                    stream: int, block_tensor: Optional[torch.Tensor] = None,
                    dtype: torch.dtype = torch.bfloat16, group_size: int = 128, flags: int = 0,
                    search: Optional[tuple] = None) -> None:
    """One ragged launch; search = (n_grid, n_candidates): the clip search (scale_method="search")."""
    if search is not None and search[1] > 1:
        rc = load_library().awq_quantize_ragged_search(ptr(descs_dev), n, total_tiles, ptr(block_tensor),
                                                       AWQ_DTYPE[dtype], bits, int(bool(symmetric)), group_size,
                                                       flags, int(search[0]), int(search[1]), ctypes.c_void_p(stream))
        check(rc, "awq_quantize_ragged_search")
        return
    rc = load_library().awq_quantize_ragged(ptr(descs_dev), n, total_tiles, ptr(block_tensor), AWQ_DTYPE[dtype],
                                            bits, int(bool(symmetric)), group_size, flags, ctypes.c_void_p(stream))
    check(rc, "awq_quantize_ragged")


def stream_copy(src: torch.Tensor, dst: torch.Tensor, stream: int) -> None:
    rc = load_library().awq_stream_copy(ptr(src), ptr(dst), src.numel() * src.element_size(), ctypes.c_void_p(stream))
    check(rc, "awq_stream_copy")


def stream_ceiling(src: torch.Tensor, dst: torch.Tensor, stream: int) -> None:
    """Read `src` whole, write len(src) / 4 bytes of dst (bench.py's read-dominant ceiling)."""
    n = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < n // 4:
        raise ValueError("stream_ceiling: dst must hold a quarter of src's bytes")
    rc = load_library().awq_stream_ceiling(ptr(src), ptr(dst), n, ctypes.c_void_p(stream))
    check(rc, "awq_stream_ceiling")


def dequant_ceiling(words: torch.Tensor, out: torch.Tensor, stream: int) -> None:
    """awq_dequant_ceiling: read out.nbytes / 8 of words, write out whole (dequantize's structure)."""
    n = out.numel() * out.element_size()
    if words.numel() * words.element_size() < n // 8:
        raise ValueError("dequant_ceiling: words must hold an eighth of out's bytes")
    check(load_library().awq_dequant_ceiling(ptr(words), ptr(out), n, ctypes.c_void_p(stream)), "awq_dequant_ceiling")


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


# ---- activation-aware scale search (include/awq_hip.h awq_act_*) ----
ACT_ROW_BLOCK = 256      # canonical fp64 column-sum block (rows / tokens)
ACT_GROUP_BLOCK = 1024   # canonical fp64 loss block (groups)
ACT_MAX_GRID = 256


def _stream(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(stream_ptr(t.device))


def act_stats(x: torch.Tensor):
    """x [tokens, K] on the device -> (x_mean, x_sq) fp32 [K]."""
    T, K = x.shape
    work = torch.empty(2 * (-(-T // ACT_ROW_BLOCK)) * K, dtype=torch.float64, device=x.device)
    xm = torch.empty(K, dtype=torch.float32, device=x.device)
    xs = torch.empty(K, dtype=torch.float32, device=x.device)
    check(load_library().awq_act_stats(ptr(x), AWQ_DTYPE[x.dtype], T, K, ptr(work), ptr(xm), ptr(xs), _stream(x)),
          "awq_act_stats")
    return xm, xs


def weight_mean(weights, group_size: int) -> torch.Tensor:
    """Duo-scaling w_mean [K] of linears sharing an input (rows concatenated in list order)."""
    lib = load_library()
    K = weights[0].shape[1]
    dev = weights[0].device
    nblk = [-(-w.shape[0] // ACT_ROW_BLOCK) for w in weights]
    part = torch.empty((sum(nblk), K), dtype=torch.float64, device=dev)
    b0 = 0
    for w, nb in zip(weights, nblk):
        gmax = torch.empty(w.shape[0] * (K // group_size), dtype=torch.float32, device=dev)
        check(lib.awq_weight_colsum(ptr(w), AWQ_DTYPE[w.dtype], w.shape[0], K, group_size, ptr(gmax),
                                    ctypes.c_void_p(part[b0].data_ptr()), _stream(w)), "awq_weight_colsum")
        b0 += nb
    out = torch.empty(K, dtype=torch.float32, device=dev)
    check(lib.awq_column_mean(ptr(part), part.shape[0], K, float(sum(w.shape[0] for w in weights)), ptr(out),
                              _stream(out)), "awq_column_mean")
    return out


def act_scale_table(x_mean: torch.Tensor, w_mean: Optional[torch.Tensor], n_grid: int,
                    workspace: bool = True) -> torch.Tensor:
    """table fp32 [n_grid, K] (awq_act_scale_table_ws; workspace=False: the workspace-free
    awq_act_scale_table, same bits)."""
    K = x_mean.numel()
    table = torch.empty((n_grid, K), dtype=torch.float32, device=x_mean.device)
    lib = load_library()
    if workspace:
        work = torch.empty(n_grid * (K + 3 * (-(-K // 256))), dtype=torch.float64, device=x_mean.device)
        check(lib.awq_act_scale_table_ws(ptr(x_mean), ptr(w_mean), K, n_grid, ptr(work), ptr(table), _stream(table)),
              "awq_act_scale_table_ws")
    else:
        check(lib.awq_act_scale_table(ptr(x_mean), ptr(w_mean), K, n_grid, ptr(table), _stream(table)),
              "awq_act_scale_table")
    return table


def act_recip_table(table: torch.Tensor) -> torch.Tensor:
    """RN(1 / table) where the loss kernel's Markstein quotient is proven exact, else 0."""
    n_grid, K = table.shape
    rtable = torch.empty_like(table)
    check(load_library().awq_act_recip_table(ptr(table), n_grid, K, ptr(rtable), _stream(table)),
          "awq_act_recip_table")
    return rtable


def act_search_losses(weights, x_sq: torch.Tensor, table: torch.Tensor, group_size: int, bits: int,
                      symmetric: bool, rtable: Optional[torch.Tensor] = None, use_rtable: bool = True) -> torch.Tensor:
    """Per-group losses of every candidate: part fp32 [n_grid, total groups of all linears].
    rtable: act_recip_table(table) (computed here unless given; use_rtable=False: IEEE
    divisions, same results)."""
    lib = load_library()
    n_grid, K = table.shape
    if use_rtable and rtable is None:
        rtable = act_recip_table(table)
    if not use_rtable:
        rtable = None
    groups = [w.shape[0] * (K // group_size) for w in weights]
    stride = sum(groups)
    part = torch.empty((n_grid, stride), dtype=torch.float32, device=table.device)
    off = 0
    for w, g in zip(weights, groups):
        check(lib.awq_act_search_losses(ptr(w), AWQ_DTYPE[w.dtype], w.shape[0], K, group_size, bits,
                                        int(bool(symmetric)), ptr(table), ptr(rtable), n_grid, ptr(x_sq),
                                        ctypes.c_void_p(part.data_ptr() + 4 * off), stride, _stream(w)),
              "awq_act_search_losses")
        off += g
    return part


def act_search_select(part: torch.Tensor, table: torch.Tensor):
    """-> (losses fp64 [n_grid], best int32 [1], s_best fp32 [K]) on the device."""
    n_grid, stride = part.shape
    K = table.shape[1]
    dev = part.device
    work = torch.empty(n_grid * (-(-stride // ACT_GROUP_BLOCK)), dtype=torch.float64, device=dev)
    losses = torch.empty(n_grid, dtype=torch.float64, device=dev)
    best = torch.empty(1, dtype=torch.int32, device=dev)
    s_best = torch.empty(K, dtype=torch.float32, device=dev)
    check(load_library().awq_act_search_select(ptr(part), n_grid, stride, ptr(table), K, ptr(work), ptr(losses),
                                               ptr(best), ptr(s_best), _stream(part)), "awq_act_search_select")
    return losses, best, s_best


def scaled_eligible(dtype: torch.dtype, rows: int, K: int, L: int) -> bool:
    """awq_quantize_groups_scaled takes this shape (one pass over W for W * diag(s))."""
    return dtype in (torch.bfloat16, torch.float16, torch.float32) and L in (32, 64, 128, 256) and K % L == 0 \
        and K % 8 == 0 and ragged_eligible(dtype, rows, K, L)


def quantize_groups_scaled(w: torch.Tensor, s: torch.Tensor, L: int, bits: int, symmetric: bool, *,
                           qweight=None, qzeros=None, scales=None) -> None:
    """Packed RTN of w * diag(s) (w [rows, K] device, contiguous; s fp32 [K]) in one pass."""
    rows, K = w.shape
    check(load_library().awq_quantize_groups_scaled(ptr(w), AWQ_DTYPE[w.dtype], rows, K, L, bits, int(bool(symmetric)),
                                                    ptr(s), ptr(qweight), ptr(qzeros), ptr(scales), _stream(w)),
          "awq_quantize_groups_scaled")


def apply_input_scale(w: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(w)
    check(load_library().awq_apply_input_scale(ptr(w), AWQ_DTYPE[w.dtype], w.shape[0], w.shape[1], ptr(s), ptr(out),
                                               _stream(w)), "awq_apply_input_scale")
    return out
