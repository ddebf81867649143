"""
AWQ group quantizer — drop-in for the reference's AWQQuantizer, computed on MI355X.

Reference: shanefitch/AWQ-Converter src/awq_quantizer/quantization/awq.py.
Same constructor signature and defaults (awq.py:29-43), same validation errors
(awq.py:95-112), same result dict (awq.py:409-416, CPU tensors owned by the caller),
same quantize_model skip-and-log behaviour (awq.py:435-457) and dequantize
(awq.py:459-539).  The per-group Python double loop (awq.py:286-374) is replaced by
one launch of the HIP kernels behind include/awq_hip.h; results are bit-identical to
the reference CPU path (tests/test_gpu_parity.py against the oracle and the golden
fixtures).

Extensions (no reference counterpart): quantize_packed / quantize_model_packed keep the
packed int4/int8 words (qweight/qzeros) and fp16 scales on the device for throughput;
scale_method="search" (new value, opt-in) runs the per-group clip search of
include/awq_hip.h awq_quantize_search instead of plain RTN ("mse"/"minmax" stay RTN);
scale_method="awq" (new value, opt-in) adds quantize_layer_group, the activation-aware
per-input-channel scale search of include/awq_hip.h awq_act_* (act_search.py).
"""

import math
from typing import Dict, List, Optional, Tuple

import torch

from .. import _hip
from ..utils.logger import get_logger


def _aligned(x: torch.Tensor) -> torch.Tensor:
    """The streaming kernel's 16-B vector loads need a 16-B aligned base: a misaligned
    device view (e.g. flat[4:4100]) is copied into fresh (aligned) storage."""
    return x if x.data_ptr() % 16 == 0 else x.clone()


def _device_input(v: torch.Tensor, dev: torch.device) -> torch.Tensor:
    if v.device == dev and v.is_contiguous():
        return _aligned(v)
    return v.detach().to(dev).contiguous()


class AWQQuantizer:
    """
    AWQ Quantizer (group-wise min/max RTN quantization, HIP backend).
    """

    def __init__(
        self,
        bits: int = 4,
        group_size: int = 128,
        symmetric: bool = True,
        zero_point: str = "minmax",
        percentile: float = 0.99,
        scale_method: str = "mse",
        per_channel: bool = True,
        device: Optional[str] = None,
        logger_name: str = "awq_quantizer",
        logger_level: str = "INFO",
        logger_to_file: bool = False,
        logger_file_path: Optional[str] = None,
        search_grid: int = 20,
        search_max_shrink: float = 0.5,
        duo_scaling: bool = True,
    ):
        self.bits = bits
        self.group_size = group_size
        self.symmetric = symmetric
        self.zero_point = zero_point
        self.percentile = percentile
        # accepted and validated like the reference; "mse" and "minmax" both give the
        # reference's round-to-nearest scales (awq.py:66 stores it, nothing reads it)
        self.scale_method = scale_method
        self.per_channel = per_channel
        # scale_method="search" only: candidates alpha = 1 - i/search_grid,
        # i < int(search_max_shrink * search_grid) (alpha = 1 first: RTN wins ties)
        self.search_grid = search_grid
        self.search_max_shrink = search_max_shrink
        # scale_method="awq" only (quantize_layer_group): search_grid ratios r = i/search_grid,
        # channel scales x_mean^r [/ w_mean^(1-r)] (duo_scaling, AutoAWQ's default)
        self.duo_scaling = duo_scaling

        # device string semantics of awq.py:70-77
        if device is None:
            self.device = "cuda" if torch.cuda.is_available() else "cpu"
        else:
            self.device = device
        if self.device.startswith("cuda") and not torch.cuda.is_available():
            self.device = "cpu"

        self.logger = get_logger(name=logger_name, level=logger_level, to_file=logger_to_file,
                                 file_path=logger_file_path)
        self._validate_parameters()
        self.qmin, self.qmax = self._calculate_qmin_qmax()
        self.logger.info(f"Initialized AWQ Quantizer with bits={bits}, group_size={group_size}, symmetric={symmetric}")
        self.logger.info(f"Quantization range: [{self.qmin}, {self.qmax}]")
        if self.device == "cpu" and torch.cuda.is_available():
            self.logger.info("device='cpu': this build has no CPU path; the HIP kernels run on the current GPU "
                             "and results are returned on the CPU (bit-identical to the reference's CPU results)")
        if self.scale_method == "awq":
            self.logger.info("scale_method='awq': the activation-aware search runs in quantize_layer_group(); "
                             "tensors quantized without activations (quantize, quantize_model) are RTN")

    # ------------------------------------------------------------------ validation
    def _validate_parameters(self) -> None:
        """awq.py:95-112 (same exception types and messages)."""
        if self.bits not in [4, 8]:
            raise ValueError(f"Unsupported bit width: {self.bits}. Supported: 4, 8.")
        if self.group_size <= 0 or not isinstance(self.group_size, int):
            raise ValueError(f"Group size must be a positive integer: {self.group_size}")
        if self.zero_point not in ["none", "minmax", "percentile"]:
            raise ValueError(f"Unsupported zero point calibration method: {self.zero_point}")
        if self.zero_point == "percentile" and (self.percentile <= 0 or self.percentile >= 1):
            raise ValueError(f"Percentile must be in range (0, 1): {self.percentile}")
        if self.scale_method not in ["minmax", "mse", "search", "awq"]:
            raise ValueError(f"Unsupported scale calibration method: {self.scale_method}")
        if self.scale_method in ("search", "awq"):
            if not isinstance(self.search_grid, int) or self.search_grid < 1:
                raise ValueError(f"search_grid must be a positive integer: {self.search_grid}")
        if self.scale_method == "awq" and self.search_grid > _hip.ACT_MAX_GRID:
            raise ValueError(f"search_grid must be <= {_hip.ACT_MAX_GRID} for scale_method='awq': {self.search_grid}")
        if self.scale_method == "search":
            if not (0 < self.search_max_shrink <= 1):
                raise ValueError(f"search_max_shrink must be in (0, 1]: {self.search_max_shrink}")

    @property
    def search_candidates(self) -> int:
        """Number of clip candidates of scale_method="search" (0 = plain RTN)."""
        if self.scale_method != "search":
            return 0
        return min(self.search_grid, max(1, int(self.search_max_shrink * self.search_grid)))

    def _search_args(self):
        """(n_grid, n_candidates) of scale_method="search" for ragged launches, else None."""
        return (self.search_grid, self.search_candidates) if self.search_candidates > 1 else None

    def _launch(self, x, rows, K, L, small: bool = False, **outs) -> None:
        if self.scale_method == "search":
            _hip.quantize_search(x, rows, K, L, self.bits, self.symmetric, self.search_grid,
                                 self.search_candidates, small=small, **outs)
        else:
            _hip.quantize_groups(x, rows, K, L, self.bits, self.symmetric, small=small, **outs)

    def _calculate_qmin_qmax(self) -> Tuple[int, int]:
        """awq.py:114-128."""
        if self.symmetric:
            return -(2 ** (self.bits - 1)), 2 ** (self.bits - 1) - 1
        return 0, 2 ** self.bits - 1

    # ------------------------------------------------------------------ helpers
    def compute_device(self) -> torch.device:
        """The GPU the kernels run on.  `self.device` keeps the reference's string
        semantics; a "cpu" quantizer still computes on the current GPU (results are
        identical and returned on the CPU), because this build has no CPU path."""
        if self.device.startswith("cuda"):
            dev = torch.device(self.device)
            if dev.index is None and torch.cuda.is_available():
                dev = torch.device("cuda", torch.cuda.current_device())
        elif torch.cuda.is_available():
            dev = torch.device("cuda", torch.cuda.current_device())
        else:
            dev = torch.device("cpu")
        _hip.require_device(dev)
        return dev

    def _check_mode(self) -> None:
        if self.zero_point == "percentile":
            # The reference's percentile branch (awq.py:187-190) calls
            # get_percentile_value(tensor, p, stats) against a 2-argument helper
            # (utils/tensor_utils.py:87) and therefore always raises this TypeError;
            # quantize_model() then skips every tensor.  Reproduced as behaviour.
            raise TypeError("get_percentile_value() takes 2 positional arguments but 3 were given")

    @staticmethod
    def _check_input(tensor) -> None:
        if not isinstance(tensor, torch.Tensor):
            raise ValueError(f"Expected torch.Tensor, got {type(tensor)}")
        if not tensor.is_floating_point():
            raise ValueError(f"Expected floating point tensor, got {tensor.dtype}")
        if tensor.dtype not in _hip.AWQ_DTYPE:
            raise RuntimeError(f"\"min_all\" not implemented for '{tensor.dtype}'")

    def _layout(self, tensor: torch.Tensor):
        """(rows, K, L, small) following awq.py:297-320 and :130-171."""
        n = tensor.numel()
        if n < self.group_size:
            if n == 0:
                raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0. "
                                   "Specify the reduction dim with the 'dim' argument.")
            if tensor.dim() <= 1 or not self.per_channel:
                return 1, n, n, "tensor"
            rows = tensor.shape[0]
            return rows, n // rows, n // rows, "row"
        rows = 1 if tensor.dim() <= 1 else tensor.shape[0]
        return rows, n // rows, self.group_size, None

    # ------------------------------------------------------------------ reference API
    def quantize(self, tensor: torch.Tensor) -> Dict[str, torch.Tensor]:
        """
        Quantize a single tensor (awq.py:376-433).

        Returns a dict of CPU tensors: tensor_q (int32, input shape), scales (float16,
        [rows, groups]; 0-d or [rows] for tensors smaller than one group), zero_points
        (int32, same shape as scales), bits / group_size (int32 0-d), symmetric (bool 0-d).
        """
        return {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in self._quantize_device(tensor).items()}

    def _quantize_device(self, tensor: torch.Tensor) -> Dict[str, torch.Tensor]:
        """quantize() with the result tensors left on the device."""
        self._check_input(tensor)
        rows, K, L, small = self._layout(tensor)
        self._check_mode()
        dev = self.compute_device()
        x = _aligned(tensor.detach().to(dev).contiguous())
        G = -(-K // L)
        tensor_q = torch.empty(rows * K, dtype=torch.int32, device=dev)
        scales = torch.empty((rows, G), dtype=torch.float16, device=dev)
        zeros = torch.empty((rows, G), dtype=torch.int32, device=dev)
        # (small-tensor path: its scales reach fp16 straight from the input dtype, awq.py:130-171
        #  -> 411, not through the fp32 buffer of awq.py:327 — only NaN scale bits differ)
        self._launch(x, rows, K, L, small=small is not None, scales=scales, tensor_q=tensor_q, zeros=zeros)
        if small == "tensor":
            scales, zeros = scales.reshape(()), zeros.reshape(())
        elif small == "row":
            scales, zeros = scales.reshape(rows), zeros.reshape(rows)
        return {
            "tensor_q": tensor_q.reshape(tensor.shape),
            "scales": scales,
            "zero_points": zeros,
            "bits": torch.tensor(self.bits, dtype=torch.int32),
            "group_size": torch.tensor(self.group_size, dtype=torch.int32),
            "symmetric": torch.tensor(self.symmetric, dtype=torch.bool),
        }

    def quantize_model(self, tensors: Dict[str, torch.Tensor]) -> Dict[str, Dict[str, torch.Tensor]]:
        """awq.py:435-457: quantize every tensor; failures are logged and skipped."""
        out = {}
        for name, tensor in tensors.items():
            try:
                self.logger.info(f"Quantizing tensor: {name}")
                out[name] = self.quantize(tensor)
                self.logger.info(f"Successfully quantized tensor: {name}")
            except Exception as e:  # reference semantics: skip and continue
                self.logger.error(f"Error quantizing tensor: {name}, error: {e}")
                continue
        return out

    def dequantize(self, quantized_tensor: Dict[str, torch.Tensor]) -> torch.Tensor:
        """
        awq.py:459-539: (tensor_q - zero_points) * fp16 scale, evaluated in fp16 like the
        reference, returned as float32 on the CPU.  Uses the dict's own group_size.
        """
        tq = quantized_tensor["tensor_q"]
        scales = quantized_tensor["scales"]
        zeros = quantized_tensor["zero_points"]
        L = int(quantized_tensor["group_size"].item())
        rows = 1 if tq.dim() <= 1 else tq.shape[0]
        K = tq.numel() // max(rows, 1)
        G = -(-K // L) if K else 0
        if scales.dim() != 2 or zeros.dim() != 2:
            raise IndexError(f"too many indices for tensor of dimension {scales.dim()}")
        if tuple(scales.shape) != (rows, G) or tuple(zeros.shape) != (rows, G):
            raise IndexError(f"scales/zero_points shape {tuple(scales.shape)} does not match "
                             f"{rows} rows x {G} groups")
        dev = self.compute_device()
        out = torch.empty(tq.shape, dtype=torch.float32, device=dev)
        if tq.numel():
            _hip.dequantize(tq.to(dev, torch.int32).contiguous(), scales.to(dev, torch.float16).contiguous(),
                            zeros.to(dev, torch.int32).contiguous(), rows, K, L, out)
        return out.cpu()

    # ------------------------------------------------------------------ reference private methods
    # awq.py:130-374.  Subclasses and callers of the reference reach into these; they keep the
    # reference's signatures, result dtypes and shapes (pinned bit for bit by
    # tests/test_private_methods.py against 1 024 + 2 668 + 4 484 calls of the reference) and
    # run on the HIP kernels: awq_group_params_ex (scale / zero point of every group in the
    # input dtype's own arithmetic), awq_apply_params_ex (element-wise quantize / dequantize with
    # given parameters) and awq_quantize_groups.  They are the reference's round-to-nearest
    # whatever scale_method says (the clip search is reached through quantize / quantize_packed).
    # Results are placed where the reference places them (self.device; _compute_scale_zp_for_group:
    # the input's device), and computed the way torch computes them THERE: the reference moves its
    # tensors to self.device, whose torch kernels differ from the CPU's in four places — a GPU
    # divides by a Python int as a product with its reciprocal (the scale, awq.py:202), clamps -0
    # to +0 (awq.py:211, 248), converts a one-element device parameter to the op dtype first
    # (awq.py:245, 282) and converts a NaN to int32 as 0 (awq.py:367).  The public API (quantize,
    # quantize_packed, dequantize, ...) always gives the reference CPU awq.py's bits (north_star).

    def _home(self, t: torch.Tensor) -> torch.Tensor:
        return t.to(self.device) if self.device.startswith("cuda") else t.cpu()

    def _torch_gpu(self) -> bool:
        """The reference would evaluate on a GPU (self.device is a CUDA device)."""
        return self.device.startswith("cuda")

    def _on_gpu(self, tensor: torch.Tensor) -> torch.Tensor:
        self._check_input(tensor)
        return tensor.detach().to(self.compute_device()).contiguous()

    def _compute_scale_zp_for_group(self, tensor: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """awq.py:173-213: (scale, zero_point) of the whole tensor as one group, 0-d tensors
        of its dtype (zero_point = 0 when symmetric), on the input's device and computed the way
        torch computes there (the reference does not move this method's input)."""
        self._check_mode()
        x = self._on_gpu(tensor)
        n = x.numel()
        if n == 0:
            raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0. "
                               "Specify the reduction dim with the 'dim' argument.")
        s, z = _hip.group_params(x, 1, n, n, self.bits, self.symmetric, torch_gpu=tensor.is_cuda)
        return s.reshape(()).to(tensor.device, tensor.dtype), z.reshape(()).to(tensor.device, tensor.dtype)

    def _calculate_scale_zp(self, tensor: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """awq.py:130-171: one group for the whole tensor (dim <= 1 or per_channel=False),
        else one per dim-0 channel ([C] tensors of the input dtype)."""
        if tensor.dim() <= 1 or not self.per_channel:
            s, z = self._compute_scale_zp_for_group(tensor.to(self._home_device()))   # awq.py:141
            return s, z
        self._check_mode()
        C = tensor.size(0)
        if C == 0:
            raise RuntimeError("stack expects a non-empty TensorList")
        x = self._on_gpu(tensor)
        K = x.numel() // C
        if K == 0:
            raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0. "
                               "Specify the reduction dim with the 'dim' argument.")
        s, z = _hip.group_params(x, C, K, K, self.bits, self.symmetric, torch_gpu=self._torch_gpu())
        return self._home(s.reshape(C).to(tensor.dtype)), self._home(z.reshape(C).to(tensor.dtype))

    def _home_device(self) -> torch.device:
        """Where the reference's tensor.to(self.device) puts a tensor (awq.py:141, 233, 303)."""
        return self.compute_device() if self._torch_gpu() else torch.device("cpu")

    @staticmethod
    def _sub_check(a: torch.dtype, b: torch.dtype) -> None:
        """ATen's sub_check: `-` with a bool operand raises (the meta ops below skip it)."""
        if a == torch.bool and b == torch.bool:
            raise RuntimeError("Subtraction, the `-` operator, with two bool tensors is not supported. "
                               "Use the `^` or `logical_xor()` operator instead.")
        if a == torch.bool or b == torch.bool:
            raise RuntimeError("Subtraction, the `-` operator, with a bool tensor is not supported. "
                               "If you are trying to invert a mask, use the `~` or `logical_not()` operator "
                               "instead.")

    @staticmethod
    def _param_words(p: torch.Tensor, dev: torch.device) -> Tuple[torch.Tensor, int]:
        """A parameter on the device as 8-byte words and its awq_apply_params_ex flag bits:
        float64 values (exact for every float dtype), or int64 values for integer / bool
        parameters (uint64: their bits) — exact whatever their magnitude."""
        if p.is_floating_point():
            return p.detach().to(dev, torch.float64), 0
        if p.dtype == torch.uint64:
            return p.detach().to(dev).view(torch.int64).view(torch.float64), 2
        return p.detach().to(dev, torch.int64).view(torch.float64), 1

    _UNSIGNED_NAMES = {torch.uint16: "UInt16", torch.uint32: "UInt32", torch.uint64: "UInt64"}

    def _apply(self, tensor: torch.Tensor, scale, zero_point, mode: int) -> torch.Tensor:
        """_quantize_tensor (mode 0) / _dequantize_tensor (mode 1) as the reference evaluates
        awq.py:245 / awq.py:282: the per-channel reshape of awq.py:237-242 / 274-279, then
        torch's broadcasting and type promotion, for tensors and parameters of any float,
        integer or bool dtype.  The two ops' result dtypes come from torch's own promotion
        (meta tensors: no data, no compute; torch.result_type for the promotion errors the meta
        ops skip); the arithmetic runs in awq_apply_params_ex in those dtypes.  A one-element
        parameter of a bf16 / fp16 op enters at its own value when the reference would evaluate
        on the CPU (device="cpu": ATen's CPU kernels read its original value) and converted to
        the op dtype first when it would evaluate on the GPU (device="cuda": a device tensor,
        cast like any operand; and there clamp(-0, 0, qmax) is +0, the GPU clamp's IEEE maximum).  Pinned by tests/golden/golden_promote.* and
        golden_promote_int.* (reference calls on the CPU: float / int32 tensors with promoting
        parameters; int64 / int16 / int8 / uint8 / bool / uint16 / uint32 / uint64 tensors with
        float, integer and bool parameters) and, for device="cuda", by torch's own CUDA
        evaluation of the same expressions (tests/test_private_methods.py)."""
        scale, zero_point = torch.as_tensor(scale), torch.as_tensor(zero_point)
        if scale.is_complex() or zero_point.is_complex() or tensor.is_complex():
            raise NotImplementedError("complex tensors or parameters")
        per_ch = self.per_channel and tensor.dim() > 1 and scale.dim() == 1
        if per_ch:                                   # awq.py:238-242 (same errors as the reference)
            shp = [scale.size(0)] + [1] * (tensor.dim() - 1)
            scale, zero_point = scale.reshape(shp), zero_point.reshape(shp)
        meta = lambda t: torch.empty(t.shape, dtype=t.dtype, device="meta")
        x_m, s_m, z_m = meta(tensor), meta(scale), meta(zero_point)
        if mode == 1:
            self._sub_check(tensor.dtype, zero_point.dtype)
        torch.result_type(x_m, s_m if mode == 0 else z_m)       # torch's promotion errors
        first = (x_m / s_m) if mode == 0 else (x_m - z_m)       # torch's broadcasting / promotion
        torch.result_type(first, z_m if mode == 0 else s_m)
        res = (first + z_m) if mode == 0 else (first * s_m)
        d1, d2, shape = first.dtype, res.dtype, tuple(res.shape)
        for dt in (d1, d2):
            if dt not in _hip.APPLY_OP_DTYPE:                    # torch has no such kernel either
                raise NotImplementedError(f"\"add_stub\" not implemented for '{self._UNSIGNED_NAMES.get(dt, dt)}'")
        if tensor.dtype not in _hip.APPLY_DTYPE:
            raise NotImplementedError(f"tensor dtype {tensor.dtype}")
        dev = self.compute_device()
        if math.prod(shape) == 0:
            return self._home(torch.empty(shape, dtype=d2, device=dev))
        x = tensor.detach().to(dev).contiguous()
        s64, s_kind = self._param_words(scale, dev)
        z64, z_kind = self._param_words(zero_point, dev)
        n = x.numel()
        if shape == tuple(tensor.shape) and scale.numel() == 1 and zero_point.numel() == 1:
            rows, K, L = 1, n, n                     # one parameter pair for the whole tensor
            s64, z64 = s64.reshape(1), z64.reshape(1)
        elif shape == tuple(tensor.shape) and per_ch:
            rows = tensor.size(0)                    # one pair per dim-0 channel
            K = n // rows
            L = max(K, 1)
            s64, z64 = s64.reshape(rows), z64.reshape(rows)
        else:                                        # any other broadcast: one pair per element
            x = x.expand(shape).contiguous()
            s64, z64 = s64.expand(shape).reshape(-1), z64.expand(shape).reshape(-1)
            rows, K, L = 1, x.numel(), 1
        cpu_scalars = not self._torch_gpu()
        flags = ((_hip.APPLY_SCALE_ONE_ELEMENT if cpu_scalars and scale.numel() == 1 else 0) |
                 (0 if cpu_scalars else _hip.APPLY_IEEE_CLAMP) |
                 (_hip.APPLY_ZERO_ONE_ELEMENT if cpu_scalars and zero_point.numel() == 1 else 0) |
                 (_hip.APPLY_SCALE_INT if s_kind else 0) | (_hip.APPLY_ZERO_INT if z_kind else 0) |
                 (_hip.APPLY_SCALE_UNSIGNED if s_kind == 2 else 0) | (_hip.APPLY_ZERO_UNSIGNED if z_kind == 2 else 0))
        out = _hip.apply_params(x, rows, K, L, s64.contiguous(), z64.contiguous(), self.qmin, self.qmax, mode, d1, d2,
                                flags)
        return self._home(out.reshape(shape))

    def _quantize_tensor(self, tensor: torch.Tensor, scale: torch.Tensor, zero_point: torch.Tensor) -> torch.Tensor:
        """awq.py:215-250: clamp(round(tensor / scale + zero_point), qmin, qmax), a float
        tensor of the input dtype (NaN stays NaN)."""
        return self._apply(tensor, scale, zero_point, 0)

    def _dequantize_tensor(self, tensor_q: torch.Tensor, scale: torch.Tensor, zero_point: torch.Tensor) -> torch.Tensor:
        """awq.py:252-284: (tensor_q - zero_point) * scale in the tensors' dtype."""
        return self._apply(tensor_q, scale, zero_point, 1)

    def _quantize_per_group(self, tensor: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """awq.py:286-374: (tensor_q int32 of the input shape, scales fp32 [rows, G],
        zero_points fp32 [rows, G]); tensors smaller than one group take
        _calculate_scale_zp + _quantize_tensor (awq.py:297-300)."""
        if tensor.numel() < self.group_size:
            scale, zero_point = self._calculate_scale_zp(tensor)
            return self._quantize_tensor(tensor, scale, zero_point), scale, zero_point
        self._check_mode()
        x = self._on_gpu(tensor)
        rows = 1 if x.dim() <= 1 else x.shape[0]
        K = x.numel() // rows
        L = self.group_size
        gpu = self._torch_gpu()
        s, z = _hip.group_params(x, rows, K, L, self.bits, self.symmetric, torch_gpu=gpu)
        if not gpu:
            tq = torch.empty(rows * K, dtype=torch.int32, device=x.device)
            _hip.quantize_groups(x, rows, K, L, self.bits, self.symmetric, tensor_q=tq)
        else:
            # awq.py:356-367 as the GPU evaluates it: each group quantized with its own 0-d
            # parameters (awq_apply_params_ex, GPU clamp), the float result stored into the
            # int32 tensor_q by torch's own GPU conversion (NaN -> 0; the reference's setitem)
            tqf = _hip.apply_params(x.reshape(-1), rows, K, L, s.reshape(-1).contiguous(), z.reshape(-1).contiguous(),
                                    self.qmin, self.qmax, 0, x.dtype, x.dtype, _hip.APPLY_IEEE_CLAMP)
            tq = tqf.to(torch.int32)
        return self._home(tq.reshape(tensor.shape)), self._home(s.float()), self._home(z.float())

    # ------------------------------------------------------------------ packed extension
    def packed_shapes(self, shape) -> dict:
        """Shapes of the packed outputs for an input of `shape` (group path only)."""
        n = math.prod(shape) if len(shape) else 1
        rows = 1 if len(shape) <= 1 else shape[0]
        K = n // rows
        G = -(-K // self.group_size)
        per = 32 // self.bits
        return {"qweight": (rows, -(-K // per)), "qzeros": (rows, -(-G // per)), "scales": (rows, G),
                "rows": rows, "K": K, "G": G}

    def quantize_packed(self, tensor: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Quantize into packed device tensors: qweight int32 [rows, ceil(K*bits/32)],
        qzeros int32 [rows, ceil(G*bits/32)], scales fp16 [rows, G] (nibble/byte j of a word
        = element j of its run of 32/bits, value q - qmin).  Values are those of quantize()."""
        self._check_input(tensor)
        self._check_mode()
        if tensor.numel() < self.group_size:
            raise ValueError("quantize_packed needs at least one full group (numel >= group_size)")
        dev = self.compute_device()
        x = _aligned(tensor.detach().to(dev).contiguous())
        sh = self.packed_shapes(tuple(tensor.shape))
        qweight = torch.empty(sh["qweight"], dtype=torch.int32, device=dev)
        qzeros = torch.empty(sh["qzeros"], dtype=torch.int32, device=dev)
        scales = torch.empty(sh["scales"], dtype=torch.float16, device=dev)
        kw = {}
        if self.search_candidates or not _hip.packs_directly(x.dtype, sh["rows"], sh["K"], self.group_size):
            kw = dict(tensor_q=torch.empty(sh["rows"] * sh["K"], dtype=torch.int32, device=dev),
                      zeros=torch.empty(sh["scales"], dtype=torch.int32, device=dev))
        self._launch(x, sh["rows"], sh["K"], self.group_size, qweight=qweight, qzeros=qzeros, scales=scales,
                     **kw)
        return {"qweight": qweight, "qzeros": qzeros, "scales": scales,
                "bits": torch.tensor(self.bits, dtype=torch.int32),
                "group_size": torch.tensor(self.group_size, dtype=torch.int32),
                "symmetric": torch.tensor(self.symmetric, dtype=torch.bool),
                "shape": torch.tensor(list(tensor.shape), dtype=torch.int64)}

    def _packed_outputs(self, tensor: torch.Tensor) -> Dict[str, torch.Tensor]:
        """quantize_packed()'s result dict for `tensor`'s shape, outputs allocated on the
        compute device and not yet written."""
        dev = self.compute_device()
        sh = self.packed_shapes(tuple(tensor.shape))
        return {"qweight": torch.empty(sh["qweight"], dtype=torch.int32, device=dev),
                "qzeros": torch.empty(sh["qzeros"], dtype=torch.int32, device=dev),
                "scales": torch.empty(sh["scales"], dtype=torch.float16, device=dev),
                "bits": torch.tensor(self.bits, dtype=torch.int32),
                "group_size": torch.tensor(self.group_size, dtype=torch.int32),
                "symmetric": torch.tensor(self.symmetric, dtype=torch.bool),
                "shape": torch.tensor(list(tensor.shape), dtype=torch.int64)}

    def quantize_model_packed(self, tensors: Dict[str, torch.Tensor]) -> Dict[str, Dict[str, torch.Tensor]]:
        """Packed quantization of many tensors: the fast-path-eligible tensors (bf16, fp16 or fp32,
        group_size 32/64/128/256, K % group_size == 0) go into one ragged launch per dtype (with the
        clip search when scale_method="search"); the rest are quantized one by one.  Outputs stay
        on the device.  Failures are logged and skipped."""
        from .batch import PackedBatch
        self._check_mode()
        eligible, rest = {}, {}
        for name, t in tensors.items():
            try:
                self._check_input(t)
            except Exception as e:
                self.logger.error(f"Error quantizing tensor: {name}, error: {e}")
                continue
            if t.numel() < self.group_size:
                self.logger.error(f"Error quantizing tensor: {name}, error: numel < group_size")
                continue
            rows = 1 if t.dim() <= 1 else t.shape[0]
            if _hip.ragged_eligible(t.dtype, rows, t.numel() // rows, self.group_size):
                eligible[name] = t
            else:
                rest[name] = t
        out = {}
        if eligible:
            dev = self.compute_device()
            for dt in (torch.bfloat16, torch.float16, torch.float32):   # one ragged launch per input dtype
                part = {k: _device_input(v, dev) for k, v in eligible.items() if v.dtype == dt}
                if part:
                    try:
                        batch = PackedBatch(part, bits=self.bits, symmetric=self.symmetric, group_size=self.group_size,
                                            search=self._search_args())
                        batch.run()
                        out.update(batch.results())
                    except Exception as e:   # the batch as a whole failed: every tensor on its own
                        self.logger.error(f"ragged launch of {len(part)} tensors failed ({e}); quantizing them "
                                          f"one by one")
                        rest.update(part)
        for name, t in rest.items():
            try:
                out[name] = self.quantize_packed(t)
            except Exception as e:
                self.logger.error(f"Error quantizing tensor: {name}, error: {e}")
        return {k: out[k] for k in tensors if k in out}

    def quantize_model_device(self, tensors: Dict[str, torch.Tensor], packed: bool = True
                              ) -> Dict[str, Dict[str, torch.Tensor]]:
        """Many tensors at once, results left on the device: packed outputs
        (quantize_model_packed) or the reference's result dicts (quantize(), unpacked int32),
        the latter also from one ragged launch per dtype for the streaming-eligible tensors.
        Failures are logged and skipped (awq.py:453-455)."""
        if packed:
            return self.quantize_model_packed(tensors)
        from .batch import PackedBatch
        out, eligible = {}, {}
        for name, t in tensors.items():
            try:
                self._check_input(t)
                self._check_mode()
            except Exception as e:  # reference semantics: skip and continue
                self.logger.error(f"Error quantizing tensor: {name}, error: {e}")
                continue
            rows = 1 if t.dim() <= 1 else t.shape[0]
            if (t.numel() >= self.group_size
                    and _hip.ragged_eligible(t.dtype, rows, t.numel() // rows, self.group_size)):
                eligible[name] = t
            else:
                try:
                    out[name] = self._quantize_device(t)
                except Exception as e:
                    self.logger.error(f"Error quantizing tensor: {name}, error: {e}")
        if eligible:
            dev = self.compute_device()
            for dt in (torch.bfloat16, torch.float16, torch.float32):
                part = {k: _device_input(v, dev) for k, v in eligible.items() if v.dtype == dt}
                if not part:
                    continue
                try:
                    batch = PackedBatch(part, bits=self.bits, symmetric=self.symmetric, parity=True, packed=False,
                                        group_size=self.group_size, search=self._search_args())
                    batch.run()
                    res = batch.results()
                except Exception as e:   # the batch as a whole failed: every tensor on its own
                    self.logger.error(f"ragged launch of {len(part)} tensors failed ({e}); quantizing them one by one")
                    for name, t in part.items():
                        try:
                            out[name] = self._quantize_device(t)
                        except Exception as e2:
                            self.logger.error(f"Error quantizing tensor: {name}, error: {e2}")
                    continue
                for name, r in res.items():
                    out[name] = {"tensor_q": r["tensor_q"], "scales": r["scales"],
                                 "zero_points": r["zero_points"], "bits": r["bits"],
                                 "group_size": r["group_size"], "symmetric": r["symmetric"]}
        return {k: out[k] for k in tensors if k in out}

    def quantize_layer_group(self, weights: Dict[str, torch.Tensor], activations: Optional[torch.Tensor] = None,
                             *, x_mean: Optional[torch.Tensor] = None, x_sq: Optional[torch.Tensor] = None,
                             packed: bool = True, table: Optional[torch.Tensor] = None) -> dict:
        """Activation-aware scale search + quantization of linears that read one input
        (scale_method="awq"; include/awq_hip.h awq_act_*, act_search.py).

        weights: name -> [out_features, in_features] (one dtype: bf16 / fp16 / fp32);
        activations: calibration inputs [tokens, in_features], or the per-channel statistics
        x_mean = mean |x|, x_sq = mean x^2 directly.  Each weight is quantized as
        W * diag(input_scale) (quantize_packed() result dicts if packed, else quantize()'s,
        device tensors, each with "input_scale"); the caller folds 1 / input_scale into the
        op producing x.  Returns {"results", "input_scale" fp32 [in], "ratio", "best",
        "losses" fp64 [search_grid] (the candidates' diagonal-MSE losses)}."""
        from .act_search import _check_group, search_layer_group
        if self.scale_method != "awq":
            raise ValueError("quantize_layer_group needs scale_method='awq'")
        _check_group(weights, self.group_size)
        self._check_mode()
        dev = self.compute_device()
        # packed outputs of eligible shapes: W * diag(s) quantized in one pass (the scaled copy
        # is never written: awq_quantize_groups_scaled); otherwise the copy, then quantize
        one_pass = packed and all(
            _hip.scaled_eligible(w.dtype, w.shape[0], w.shape[1], self.group_size) for w in weights.values())
        sr = search_layer_group(weights, dev, group_size=self.group_size, bits=self.bits, symmetric=self.symmetric,
                                n_grid=self.search_grid, duo_scaling=self.duo_scaling, activations=activations,
                                x_mean=x_mean, x_sq=x_sq, table=table, scale_weights=not one_pass)
        results = {}
        for name in weights:
            w = sr["weights"][name]
            if one_pass and w.data_ptr() % 16 == 0:
                r = self._packed_outputs(w)
                _hip.quantize_groups_scaled(w, sr["input_scale"], self.group_size, self.bits, self.symmetric,
                                            qweight=r["qweight"], qzeros=r["qzeros"], scales=r["scales"])
            else:
                sw = sr["scaled"][name] if sr["scaled"] is not None else _hip.apply_input_scale(w, sr["input_scale"])
                r = self.quantize_packed(sw) if packed else self._quantize_device(sw)   # RTN of W * diag(s)
            r["input_scale"] = sr["input_scale"]
            results[name] = r
        best = int(sr["best"].item())
        self.logger.info(f"awq search over {list(weights)}: ratio {best}/{self.search_grid}")
        return {"results": results, "input_scale": sr["input_scale"], "best": best,
                "ratio": best / self.search_grid, "losses": sr["losses"], "table": sr["table"]}

    def export_autoawq(self, packed: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """A quantize_packed() result of a 2-D [out_features, in_features] weight in the
        AutoAWQ "GEMM" layout (include/awq_hip.h awq_export_autoawq_gemm): qweight int32
        [in, out/8], qzeros int32 [in/group_size, out/8], scales fp16 [in/group_size, out],
        packed along out_features with AWQ_ORDER.  Device tensors; 4-bit only."""
        shape = tuple(int(v) for v in packed["shape"].tolist())
        if len(shape) != 2:
            raise ValueError(f"AutoAWQ GEMM layout is for 2-D linear weights, got shape {shape}")
        N, K = shape
        L = int(packed["group_size"].item())
        bits = int(packed["bits"].item())
        dev = packed["qweight"].device
        G = K // L
        out = {"qweight": torch.empty((K, N // 8), dtype=torch.int32, device=dev),
               "qzeros": torch.empty((G, N // 8), dtype=torch.int32, device=dev),
               "scales": torch.empty((G, N), dtype=torch.float16, device=dev)}
        _hip.export_autoawq_gemm(packed["qweight"].contiguous(), packed["qzeros"].contiguous(),
                                 packed["scales"].contiguous(), N, K, L, bits, out["qweight"], out["qzeros"],
                                 out["scales"])
        return out

    def dequantize_packed(self, packed: Dict[str, torch.Tensor], dtype: torch.dtype = torch.float32) -> torch.Tensor:
        """Inverse of quantize_packed with the reference's dequantize arithmetic (fp16 math)."""
        shape = tuple(int(v) for v in packed["shape"].tolist())
        L = int(packed["group_size"].item())
        bits = int(packed["bits"].item())
        sym = bool(packed["symmetric"].item())
        n = math.prod(shape) if shape else 1
        rows = 1 if len(shape) <= 1 else shape[0]
        K = n // rows
        dev = packed["qweight"].device
        out = torch.empty(shape, dtype=torch.float32, device=dev)
        _hip.dequantize_packed(packed["qweight"], packed["qzeros"], packed["scales"], rows, K, L, bits, sym, out)
        return out if dtype == torch.float32 else out.to(dtype)
