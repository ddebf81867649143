"""torch.save for the CLI's chunk objects without the GIL.

The chunk files (model_chunk_NNNN.pt, reference main.py:430-512) are dicts of per-tensor
result dicts of CPU tensors.  torch.save pickles them with a Python persistent_id callback
per object and then holds the GIL through the zip writer's CRC-32 and copies, so the CLI's
writer threads ran one at a time (0.67 GB/s for a 5.4 MB packed chunk with 1 to 8 threads).
Here the pickle stream is built directly (the opcodes torch.save's pickler emits for these
objects: protocol 2, torch._utils._rebuild_tensor_v2 over persistent storage ids
('storage', torch.<T>Storage, key, 'cpu', numel), collections.OrderedDict hooks) and the
archive is written by libawq_hip.so's awq_write_pt (csrc/awq_ptfile.hip) through ctypes,
which releases the GIL: same record names, order, 64-byte data alignment and CRC-32 as
torch.save, read back by torch.load (weights_only=True included) into equal objects.
Anything else (other value types, archives needing ZIP64) goes to torch.save."""
import ctypes
import functools
import os
import random
import struct
from typing import Any, List

import torch

_SYSRAND = random.SystemRandom()

_STORAGE = {
    torch.float32: b"FloatStorage", torch.float64: b"DoubleStorage", torch.float16: b"HalfStorage",
    torch.bfloat16: b"BFloat16Storage", torch.int64: b"LongStorage", torch.int32: b"IntStorage",
    torch.int16: b"ShortStorage", torch.int8: b"CharStorage", torch.uint8: b"ByteStorage",
    torch.bool: b"BoolStorage",
}
_REBUILD = b"ctorch._utils\n_rebuild_tensor_v2\n"
_HOOKS = b"ccollections\nOrderedDict\n)R"


class _Unsupported(Exception):
    pass


@functools.lru_cache(maxsize=4096)
def _uni(s: str) -> bytes:
    b = s.encode("utf-8")
    return b"X" + struct.pack("<I", len(b)) + b


def _int(n: int) -> bytes:
    if 0 <= n < 256:
        return _SMALL[n]
    if 0 <= n < 65536:
        return b"M" + struct.pack("<H", n)
    if -(1 << 31) <= n < (1 << 31):
        return b"J" + struct.pack("<i", n)
    b = n.to_bytes((n.bit_length() + 8) // 8, "little", signed=True)
    return b"\x8a" + bytes((len(b),)) + b


_SMALL = [b"K" + bytes((n,)) for n in range(256)]


@functools.lru_cache(maxsize=4096)
def _tuple(xs: tuple) -> bytes:
    body = b"".join(_int(int(x)) for x in xs)
    n = len(xs)
    if n == 0:
        return b")"
    if n <= 3:
        return body + (b"\x85", b"\x86", b"\x87")[n - 1]
    return b"(" + body + b"t"


# per storage type: everything of a tensor's record before its storage key
_HEAD = {dt: _REBUILD + b"((" + _uni("storage") + b"ctorch\n" + st + b"\n" for dt, st in _STORAGE.items()}
_CPU = _uni("cpu")
_MID = b"tQ" + _int(0)
_TAIL = b"\x89" + _HOOKS + b"tR"


def _pickle(obj: Any, tensors: List[torch.Tensor], out: List[bytes]) -> None:
    # (the hot loop of a chunk write: every fragment that repeats is precomputed or cached —
    #  the Python work here holds the GIL, which the writer threads share)
    if type(obj) is torch.Tensor:
        head = _HEAD.get(obj.dtype)
        if head is None or obj.device.type != "cpu" or obj.requires_grad or not obj.is_contiguous():
            raise _Unsupported
        out.append(head + _uni(str(len(tensors))) + _CPU + _int(obj.numel()) + _MID + _tuple(tuple(obj.shape))
                   + _tuple(obj.stride()) + _TAIL)
        tensors.append(obj)
    elif type(obj) is dict:
        out.append(b"}")
        if obj:
            out.append(b"(")
            for k, v in obj.items():
                if type(k) is not str:
                    raise _Unsupported
                out.append(_uni(k))
                _pickle(v, tensors, out)
            out.append(b"u")
    else:
        raise _Unsupported


def _library():
    from . import _hip                 # (signatures: _hip.SIGNATURES)
    return _hip.load_library()


def save(obj: Any, path: str) -> None:
    """torch.save(obj, path) for dicts (str keys) of dicts / CPU tensors."""
    tensors: List[torch.Tensor] = []
    parts: List[bytes] = [b"\x80\x02"]
    try:
        _pickle(obj, tensors, parts)
    except _Unsupported:
        torch.save(obj, path)
        return
    parts.append(b".")
    pkl = b"".join(parts)
    n = len(tensors)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[t.data_ptr() for t in tensors])
    sizes = (ctypes.c_int64 * max(n, 1))(*[t.numel() * t.element_size() for t in tensors])
    archive = os.path.splitext(os.path.basename(path))[0]
    sid = "%040d" % _SYSRAND.randrange(10 ** 40)   # 40 uniform digits; leaves the caller's RNG alone
    rc = _library().awq_write_pt(path.encode(), archive.encode(), pkl, len(pkl), n, ptrs, sizes, sid.encode())
    if rc in (1, 2):      # 2: would need ZIP64; 1: I/O error — torch.save raises it with its errno
        torch.save(obj, path)
    elif rc != 0:
        raise ValueError(f"awq_write_pt({path}) rejected its arguments (rc {rc})")
