"""Ragged multi-tensor launch: many tensors, one kernel (include/awq_hip.h
awq_plan_ragged / awq_quantize_ragged).

A model's tensor set (e.g. opt-125m: 196 tensors, 110 of them 768-element biases) is
quantized by ONE launch of the streaming kernel over all tensors' tiles instead of one
launch (or, in the reference, ~20 ATen dispatches per 128-element group,
awq.py:345-368) per tensor.  The descriptor table is planned once on the host,
uploaded once, and can be re-launched any number of times (bench.py does).
"""
from typing import Dict, Optional

import torch

from .. import _hip


class PackedBatch:
    """Device-resident inputs + packed outputs of one ragged launch.

    inputs: name -> contiguous device tensor ([rows, ...] or 1-D), K % group_size == 0, all
    bf16, all fp16 or all fp32; group_size 32, 64, 128 or 256 (one per batch).
    parity=True additionally produces the reference's unpacked int32 tensor_q and
    zero_points (6.05 B/element of output traffic instead of 0.52).
    use_block_table: upload the per-workgroup tensor table (awq_plan_block_tensor; 4 B per
    4 tiles) so no wave has to search the descriptors.
    search: (n_grid, n_candidates) runs the clip search of scale_method="search" in the same
    one launch (awq_quantize_ragged_search; the bits of awq_quantize_search per tensor).
    """

    def __init__(self, inputs: Dict[str, torch.Tensor], bits: int = 4, symmetric: bool = False,
                 parity: bool = False, packed: bool = True, use_block_table: bool = True, group_size: int = 128,
                 search: Optional[tuple] = None):
        if not inputs:
            raise ValueError("PackedBatch needs at least one tensor")
        self.bits, self.symmetric, self.parity = bits, bool(symmetric), parity
        self.group_size = gs = int(group_size)
        self.search = tuple(search) if search is not None and search[1] > 1 else None
        self.names = list(inputs)
        first = next(iter(inputs.values()))
        dev, self.dtype = first.device, first.dtype
        if self.dtype not in (torch.bfloat16, torch.float16, torch.float32):
            raise ValueError(f"PackedBatch takes bf16, fp16 or fp32 tensors, got {self.dtype}")
        _hip.require_device(dev)
        self.device = dev
        self.inputs = inputs
        per = 32 // bits
        self.out = {}
        descs = []
        for name in self.names:
            x = inputs[name]
            if x.device != dev or x.dtype != self.dtype or not x.is_contiguous():
                raise ValueError(f"{name}: inputs must be contiguous {self.dtype} tensors on {dev} (one dtype "
                                 f"per batch)")
            rows = 1 if x.dim() <= 1 else x.shape[0]
            K = x.numel() // rows
            if not _hip.ragged_eligible(x.dtype, rows, K, gs):
                raise ValueError(f"{name}: shape {tuple(x.shape)} is not eligible for a ragged launch "
                                 f"(group_size {gs})")
            G = -(-K // gs)          # padded rows: the tail group counts (awq.py:337-339)
            o = {"scales": torch.empty((rows, G), dtype=torch.float16, device=dev)}
            if packed:
                o["qweight"] = torch.empty((rows, -(-K // per)), dtype=torch.int32, device=dev)
                o["qzeros"] = torch.empty((rows, -(-G // per)), dtype=torch.int32, device=dev)
            if parity:
                o["tensor_q"] = torch.empty(x.shape, dtype=torch.int32, device=dev)
                o["zero_points"] = torch.empty((rows, G), dtype=torch.int32, device=dev)
            self.out[name] = o
            p = lambda k: o[k].data_ptr() if k in o else None
            descs.append(_hip.TensorDesc(x.data_ptr(), rows, K, p("qweight"), p("qzeros"), p("scales"),
                                         p("tensor_q"), p("zero_points"), 0, 0))
        self.total_tiles = _hip.plan_ragged(descs, bits, gs)
        self.flags = _hip.ragged_flags(descs, gs)       # padded rows -> the row-tile kernel instance
        self.descs = descs
        # the tables go up asynchronously on the construction stream (pinned H2D); `ready`
        # orders any other stream run() is given after them
        self._stream0 = torch.cuda.current_stream(dev)
        self.descs_dev = _hip.descs_to_device(descs, dev)
        self.block_tensor = _hip.plan_block_tensor(descs, self.total_tiles, dev) if use_block_table else None
        self._ready = torch.cuda.Event()
        self._ready.record(self._stream0)
        self.elements = sum(inputs[n].numel() for n in self.names)

    def run(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if s != self._stream0:       # the kernel reads the uploaded tables (raw output pointers)
            s.wait_event(self._ready)
        _hip.quantize_ragged(self.descs_dev, len(self.descs), self.total_tiles, self.bits, self.symmetric,
                             s.cuda_stream, self.block_tensor, self.dtype, self.group_size, self.flags,
                             search=self.search)

    def results(self) -> Dict[str, Dict[str, torch.Tensor]]:
        res = {}
        for name in self.names:
            o = dict(self.out[name])
            o["bits"] = torch.tensor(self.bits, dtype=torch.int32)
            o["group_size"] = torch.tensor(self.group_size, dtype=torch.int32)
            o["symmetric"] = torch.tensor(self.symmetric, dtype=torch.bool)
            o["shape"] = torch.tensor(list(self.inputs[name].shape), dtype=torch.int64)
            res[name] = o
        return res

    def algorithmic_bytes(self) -> int:
        """HBM bytes one launch must move: bf16 in + packed out (+ parity outputs)."""
        b = 0
        for name in self.names:
            b += self.inputs[name].numel() * self.inputs[name].element_size()
            for t in self.out[name].values():
                b += t.numel() * t.element_size()
        return b
