"""The ctypes stub a maintainer of the reference (shanefitch/AWQ-Converter) adds to
`src/awq_quantizer/quantization/` to run `AWQQuantizer._quantize_per_group`
(awq.py:286-374) on libawq_hip.so.  INTEGRATION.md §2 shows the two-line change in awq.py.

It binds only the C ABI (include/awq_hip.h) with ctypes and keeps the reference's return
contract: `(tensor_q int32 [input shape], scales fp32 [rows, G], zero_points fp32 [rows, G])`
on the quantizer's device (awq.py:327-329), and the reference's small-tensor branch
(awq.py:297-300, unchanged: it calls the quantizer's own _calculate_scale_zp /
_quantize_tensor).  The fp32 scales are the input dtype's scale values (awq_group_params:
exact, RN_f32 for fp64 — what awq.py:352 stores); a NaN scale is stored as the fp32 NaN
whose fp16 conversion (awq.py:411) gives the reference's fp16 bits (the kernel's own fp16
scale output), so quantize()'s result dict is bit-identical to the unmodified reference.
(The intermediate fp32 NaN payload itself is not the reference's: e.g. 0x7FFFE000 where the
reference's fp16 -> fp32 store leaves 0x7FFFFFFF; nothing downstream can tell.)

Exercised by tests/test_gpu_integration_stub.py against the reference's golden outputs.
"""
import ctypes
import math
import os

import torch

_P, _I, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_DT = {torch.bfloat16: 0, torch.float16: 1, torch.float32: 2, torch.float64: 3}
_lib = None


def load(path=None):
    """Bind libawq_hip.so (default: next to this file, where the maintainer drops it)."""
    global _lib
    if _lib is None:
        lib = ctypes.CDLL(path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libawq_hip.so"))
        lib.awq_quantize_groups.argtypes = [_P, _I, _L, _L, _I, _I, _I, _P, _P, _P, _P, _P, _P]   # group_size int32
        lib.awq_group_params.argtypes = [_P, _I, _L, _L, _L, _I, _I, _P, _P, _P]
        lib.awq_last_error.restype = ctypes.c_char_p
        _lib = lib
    return _lib


def _check(rc):
    if rc:
        raise RuntimeError(_lib.awq_last_error().decode())


def quantize_per_group(self, tensor):
    """Drop-in body of AWQQuantizer._quantize_per_group(self, tensor) (awq.py:286-374)."""
    if tensor.numel() < self.group_size:                       # awq.py:297-300, the reference's own path
        scale, zero_point = self._calculate_scale_zp(tensor)
        tensor_q = self._quantize_tensor(tensor, scale, zero_point)
        return tensor_q, scale, zero_point
    lib = load()
    dev = torch.device("cuda", torch.cuda.current_device())
    x = tensor.detach().to(dev).contiguous()
    if x.data_ptr() % 16:                                      # the kernels' 16-B vector loads
        x = x.clone()
    rows = 1 if x.dim() <= 1 else x.shape[0]                   # awq.py:306-320: rows = dim 0
    K = x.numel() // rows
    G = math.ceil(K / self.group_size)                         # awq.py:323
    tq = torch.empty(rows * K, dtype=torch.int32, device=dev)
    sc16 = torch.empty(rows, G, dtype=torch.float16, device=dev)
    s64 = torch.empty(rows, G, dtype=torch.float64, device=dev)
    z64 = torch.empty(rows, G, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _check(lib.awq_quantize_groups(x.data_ptr(), _DT[x.dtype], rows, K, self.group_size, self.bits,
                                   int(self.symmetric), None, None, sc16.data_ptr(), tq.data_ptr(), None, stream))
    _check(lib.awq_group_params(x.data_ptr(), _DT[x.dtype], rows, K, self.group_size, self.bits,
                                int(self.symmetric), s64.data_ptr(), z64.data_ptr(), stream))
    scales = s64.to(torch.float32)                             # awq.py:327, 352: fp32 [rows, G]
    nan = torch.isnan(scales)
    if bool(nan.any()):                                        # the fp32 NaN whose fp16 is the reference's
        h = sc16.view(torch.int16).to(torch.int32) & 0xFFFF
        wide = ((h & 0x8000) << 16) | 0x7F800000 | ((h & 0x3FF) << 13)
        scales = torch.where(nan, wide.view(torch.float32), scales)
    zero_points = z64.to(torch.float32)                        # awq.py:328, 353
    home = torch.device(self.device) if str(self.device).startswith("cuda") else torch.device("cpu")
    return tq.reshape(tensor.shape).to(home), scales.to(home), zero_points.to(home)
