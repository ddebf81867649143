"""
awq_quantizer command line — drop-in for the reference CLI (src/awq_quantizer/main.py).

Same flags and defaults (reference main.py:22-159), same tensor filter (floating point,
numel >= 128, main.py:244-253), same processing / output order (bytes descending,
stable, main.py:259), same output layout (model_chunk_NNNN.pt holding nested result
dicts + metadata.json, main.py:430-512) and exit codes (0 ok; 1 on load failure, no
tensor quantized, or save failure).

What changes underneath, MI355X-first:
  * weights are streamed: headers are read first, then batches of tensors are read by
    reader threads into pinned host memory, copied to the GPU on a copy stream while the
    previous batch is quantized (one ragged launch per batch), and the results copied
    back asynchronously (the reference loads every file whole, then copies every tensor
    to the device eagerly, main.py:296-307, and quantizes tensor by tensor);
  * --multi_gpu / --device all really shards: the tensor list is LPT-partitioned over
    the GPUs (the reference's own partition_tensors, main.py:395-427, which it never
    calls; instead every device re-quantizes every tensor, main.py:596-606), one host
    thread per GPU;
  * the arithmetic is the HIP kernels behind include/awq_hip.h;
  * --save_safetensors works (the reference passes nested dicts to save_file and
    always fails, main.py:488-490): result dicts are flattened to "<name>.<field>";
  * --output_format packed writes qweight/qzeros/scales (int4/int8 packed) instead of
    the reference's unpacked int32 tensor_q (8x smaller on disk at 4 bits).
"""

import argparse
import ctypes
import json
import logging
import math
import os
import sys
import threading
import time
from collections import deque
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, List, Optional, Tuple

_T_MODULE = time.time()
if __name__ == "__main__":
    # the program itself (`python -m awq_quantizer.main`): HIP's first-use work starts on a
    # native thread now and overlaps `import torch` (~1.5 s); see _early.py
    from awq_quantizer import _early
    _early.start(sys.argv[1:])

import torch

_IMPORT_TORCH_S = time.time() - _T_MODULE

from . import ptfile
from .stream import device_name, start_warmup
from .model_loading import TensorInfo, load_model_from_hub
from .quantization.awq import AWQQuantizer
from .utils.logger import get_logger


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="AWQ Quantizer CLI")
    p.add_argument("--model_id", type=str, required=True, help="Model ID on HuggingFace Hub or path to local model")
    p.add_argument("--output_dir", type=str, required=True, help="Directory to save quantized model")
    p.add_argument("--bits", type=int, default=4, choices=[4, 8], help="Number of bits for quantization")
    p.add_argument("--group_size", type=int, default=128, help="Group size for quantization")
    p.add_argument("--symmetric", action="store_true", help="Use symmetric quantization")
    p.add_argument("--zero_point", type=str, default="minmax", choices=["none", "minmax", "percentile"],
                   help="Zero point calibration method")
    p.add_argument("--percentile", type=float, default=0.99, help="Percentile for zero point calibration")
    p.add_argument("--scale_method", type=str, default="mse", choices=["minmax", "mse", "search", "awq"],
                   help="Scale calibration method (minmax/mse: round-to-nearest as the reference; "
                        "search: per-group clip search, opt-in extension)")
    p.add_argument("--search_grid", type=int, default=20, help="scale_method=search / awq: grid size")
    p.add_argument("--act_stats", type=str, default=None,
                   help="scale_method=awq: safetensors file of per-input-channel activation statistics, "
                        "'<weight name>.x_mean' (mean |x|) and '<weight name>.x_sq' (mean x^2), fp32 [in_features]; "
                        "weights without statistics are quantized RTN")
    p.add_argument("--no_duo_scaling", action="store_true",
                   help="scale_method=awq: channel scales x_mean^r instead of x_mean^r / w_mean^(1-r)")
    p.add_argument("--search_max_shrink", type=float, default=0.5,
                   help="scale_method=search: largest shrink of the group range tried")
    p.add_argument("--per_channel", action="store_true", help="Use per-channel quantization")
    p.add_argument("--device", type=str, default="cuda" if torch.cuda.is_available() else "cpu",
                   help="Device to use for quantization (cuda, cuda:0, cuda:1, cpu, or 'all' for all GPUs)")
    p.add_argument("--num_workers", type=int, default=4,
                   help="Number of host threads reading weights ahead of the GPU (per GPU)")
    p.add_argument("--max_memory", type=float, default=0.8,
                   help="Maximum fraction of GPU memory to use (0.0-1.0)")
    p.add_argument("--multi_gpu", action="store_true", help="Use all available GPUs for processing (overrides --device)")
    p.add_argument("--batch_size", type=int, default=10, help="Number of tensors to process in each batch")
    p.add_argument("--prefetch_factor", type=int, default=2,
                   help="Batches of tensors read ahead of the GPU (higher values use more host memory)")
    p.add_argument("--memory_efficient", action="store_true",
                   help="Enable memory-efficient mode (release cached GPU memory after every batch)")
    p.add_argument("--log_level", type=str, default="INFO", choices=["DEBUG", "INFO", "WARNING", "ERROR", "CRITICAL"],
                   help="Logging level")
    p.add_argument("--log_file", type=str, help="Log file path")
    p.add_argument("--save_safetensors", action="store_true", help="Save in safetensors format instead of pytorch format")
    p.add_argument("--chunk_size", type=int, default=10, help="Number of tensors to save in each chunk (for large models)")
    # extension (not in the reference)
    p.add_argument("--output_format", type=str, default="reference", choices=["reference", "packed", "autoawq"],
                   help="reference: int32 tensor_q/zero_points + fp16 scales per tensor (reference layout); "
                        "packed: int32 qweight/qzeros (bits-packed) + fp16 scales; "
                        "autoawq: a 4-bit checkpoint in AutoAWQ's GEMM layout (linear weights quantized, "
                        "everything else copied) + quant_config.json")
    p.add_argument("--dist_output", type=str, default="per_rank", choices=["per_rank", "gather"],
                   help="torchrun mode: per_rank = every rank writes its own chunk files (rank 0 adds "
                        "metadata.json over all of them); gather = results sent to rank 0, which writes everything")
    p.add_argument("--stream_engine", type=str, default="native", choices=["native", "python"],
                   help="native: the C++ read -> H2D -> quantize -> D2H pipeline of libawq_hip.so (awq_stream_*); "
                        "python: the same pipeline driven from Python (the round-2 path; also used for "
                        "--act_stats and --output_format autoawq)")
    return p


def parse_args(argv: Optional[List[str]] = None) -> argparse.Namespace:
    """Command-line arguments (reference main.py:22-159)."""
    return build_parser().parse_args(argv)


def get_available_gpus(logger=None) -> List[str]:
    """["cuda:0", ...] for every visible GPU (reference main.py:162-186)."""
    if not torch.cuda.is_available():
        if logger:
            logger.warning("No CUDA devices available")
        return []
    devs = []
    for i in range(torch.cuda.device_count()):
        if logger:
            logger.info(f"Found CUDA device {i}: {device_name(i)}")
        devs.append(f"cuda:{i}")
    return devs


def get_device_memory_info(device_idx: int) -> Tuple[float, float]:
    """(total GB, free GB) of a device (reference main.py:189-213)."""
    if not torch.cuda.is_available():
        return 0.0, 0.0
    try:
        free, total = torch.cuda.mem_get_info(device_idx)
        return total / 1024 ** 3, free / 1024 ** 3
    except Exception:  # noqa: BLE001
        return 0.0, 0.0


def select_tensors(index: List[TensorInfo], logger=None) -> List[TensorInfo]:
    """Filter + order of reference main.py:241-259, on header information only."""
    keep = []
    for info in index:
        if info.dtype is None or not info.dtype.is_floating_point or info.numel == 0:
            if logger:
                logger.warning(f"Skipping invalid tensor: {info.name}")
            continue
        if info.numel < 128:
            if logger:
                logger.warning(f"Skipping tensor too small for grouping: {info.name}")
            continue
        keep.append(info)
    keep.sort(key=lambda i: i.nbytes, reverse=True)   # stable
    return keep


def prepare_tensors_for_quantization(tensors: Dict[str, torch.Tensor], device: str, max_memory_fraction: float = 0.8,
                                     batch_size: int = 10, logger=None) -> List[Dict[str, torch.Tensor]]:
    """In-memory API of reference main.py:216-330: filtered, size-ordered batches of at most
    batch_size tensors.  Tensors stay where they are (they are moved to the GPU one at a
    time when quantized, not all at once)."""
    infos = []
    for name, t in tensors.items():
        if not isinstance(t, torch.Tensor):
            if logger:
                logger.warning(f"Skipping invalid tensor: {name}")
            continue
        infos.append(TensorInfo(name, None, t.dtype, t.shape))
    ordered = select_tensors(infos, logger)
    batches, cur = [], {}
    for info in ordered:
        if len(cur) >= batch_size:
            batches.append(cur)
            cur = {}
        cur[info.name] = tensors[info.name]
    if cur:
        batches.append(cur)
    if logger:
        logger.info(f"Created {len(batches)} batches with {sum(len(b) for b in batches)} total tensors")
    return batches


def partition_tensors(items, num_partitions: int):
    """Greedy LPT by bytes (reference main.py:395-427).  `items` is a dict name->tensor or a
    list of TensorInfo; returns num_partitions collections of the same kind."""
    if num_partitions <= 1:
        return [items]
    if isinstance(items, dict):
        sizes = [(n, t.numel() * t.element_size()) for n, t in items.items()]
    else:
        sizes = [(i, i.nbytes) for i in items]
    sizes.sort(key=lambda x: x[1], reverse=True)
    parts = [dict() if isinstance(items, dict) else [] for _ in range(num_partitions)]
    load = [0] * num_partitions
    for key, size in sizes:
        k = load.index(min(load))
        if isinstance(items, dict):
            parts[k][key] = items[key]
        else:
            parts[k].append(key)
        load[k] += size
    return parts


def _flatten(tensors: Dict[str, Dict[str, torch.Tensor]]) -> Dict[str, torch.Tensor]:
    flat = {}
    for name, d in tensors.items():
        for k, v in d.items():
            flat[f"{name}.{k}"] = v.contiguous()
    return flat


def save_model_in_chunks(tensors: Dict[str, Dict[str, torch.Tensor]], output_dir: str, chunk_size: int = 10,
                         use_safetensors: bool = False, logger=None) -> None:
    """model_chunk_NNNN.{pt|safetensors} + metadata.json (reference main.py:430-512)."""
    os.makedirs(output_dir, exist_ok=True)
    names = list(tensors)
    num_chunks = (len(names) + chunk_size - 1) // chunk_size
    if logger:
        logger.info(f"Saving model in {num_chunks} chunks with {chunk_size} tensors per chunk")
    first = next(iter(tensors.values()))
    qparams = {k: (first[k].item() if k in first else None) for k in ("bits", "group_size", "symmetric")}
    tensor_to_chunk = {}
    # chunk files are independent: written by a small thread pool (ptfile.save: the archive is
    # written by native code that releases the GIL)
    with ThreadPoolExecutor(max_workers=min(8, max(2, cpu_share() // 2))) as pool:
        futs = []
        for c in range(num_chunks):
            chunk_names = names[c * chunk_size:(c + 1) * chunk_size]
            for n in chunk_names:
                tensor_to_chunk[n] = c
            futs.append(pool.submit(_write_chunk, {n: tensors[n] for n in chunk_names}, output_dir, c,
                                    use_safetensors, logger, f"{c + 1}/{num_chunks}"))
        for f in futs:
            f.result()
    _write_metadata(output_dir, num_chunks, chunk_size, tensor_to_chunk, use_safetensors, len(names), qparams,
                    logger)


CHUNK_STEM = "model_chunk_{:04d}"   # reference main.py:485


def _chunk_path(output_dir: str, c: int, use_safetensors: bool, stem: str = CHUNK_STEM) -> str:
    return os.path.join(output_dir, stem.format(c) + (".safetensors" if use_safetensors else ".pt"))


_ST_DTYPE = {torch.int32: "I32", torch.int64: "I64", torch.int16: "I16", torch.int8: "I8", torch.uint8: "U8",
             torch.bool: "BOOL", torch.float16: "F16", torch.bfloat16: "BF16", torch.float32: "F32",
             torch.float64: "F64"}


def save_safetensors(flat: Dict[str, torch.Tensor], path: str) -> None:
    """A safetensors file (8-byte header length, JSON header, the tensors' bytes back to back)
    written straight from the tensors' memory: tensors may be views of one buffer (the native
    pipeline's chunk buffers), which safetensors.torch.save_file refuses to write."""
    import numpy as np
    header, off, parts = {}, 0, []
    for name in sorted(flat):
        t = flat[name].detach().cpu().contiguous()
        nb = t.numel() * t.element_size()
        header[name] = {"dtype": _ST_DTYPE[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + nb]}
        parts.append(t)
        off += nb
    header["__metadata__"] = {"format": "pt"}
    h = json.dumps(header, separators=(",", ":")).encode()
    h += b" " * (-len(h) % 8)
    with open(path, "wb") as f:
        f.write(len(h).to_bytes(8, "little"))
        f.write(h)
        for t in parts:
            if t.numel():
                raw = t.reshape(-1).view(torch.uint8) if t.dtype != torch.bool else t.reshape(-1).to(torch.uint8)
                f.write(memoryview(np.ascontiguousarray(raw.numpy())))


def _write_chunk(chunk: Dict[str, Dict[str, torch.Tensor]], output_dir: str, c: int, use_safetensors: bool,
                 logger=None, label: str = "", stem: str = CHUNK_STEM) -> None:
    path = os.path.join(output_dir, stem.format(c))
    if use_safetensors:
        save_safetensors(_flatten(chunk), path + ".safetensors")
        if logger:
            logger.info(f"Saved chunk {label or c + 1} with {len(chunk)} tensors in safetensors format")
    else:
        ptfile.save(chunk, path + ".pt")        # torch.save's archive, written without the GIL
        if logger:
            logger.info(f"Saved chunk {label or c + 1} with {len(chunk)} tensors in PyTorch format")


def _write_metadata(output_dir, num_chunks, chunk_size, tensor_to_chunk, use_safetensors, num_tensors, qparams,
                    logger=None) -> None:
    meta = {"num_chunks": num_chunks, "chunk_size": chunk_size, "tensor_to_chunk": tensor_to_chunk,
            "format": "safetensors" if use_safetensors else "pytorch", "num_tensors": num_tensors,
            "quantization_params": qparams}
    with open(os.path.join(output_dir, "metadata.json"), "w") as f:
        json.dump(meta, f, indent=2)
    if logger:
        logger.info("Saved metadata file with tensor mapping")


class ChunkWriter:
    """save_model_in_chunks while the GPU pipeline is still running: a writer thread walks the
    tensors in processing order (bytes descending, main.py:259) and writes chunk c as soon as
    its chunk_size successful tensors are on the host, so disk writes overlap the reads and
    kernels of later batches.  Output files and metadata.json are identical to
    save_model_in_chunks on the finished dict (failed tensors are skipped in the same order;
    chunk numbers are only known once every earlier tensor has finished).  Complete chunks
    are written by a small thread pool: ptfile.save builds the pickle stream in Python and
    writes the archive natively without the GIL, so chunks serialise in parallel (5.4 MB
    packed chunks in the build container: torch.save 0.72 / 1.2 GB/s on 1 / 8 threads,
    ptfile 1.5 / 5.1 GB/s).

    stem / metadata: torchrun's per-rank mode writes under a rank-private file stem and no
    metadata.json; after close(), `t2c` (name -> local chunk), `n_chunks`, `n_ok` and
    `qparams` describe what was written (_commit_rank_chunks renumbers the files)."""

    def __init__(self, order: List[str], output_dir: str, chunk_size: int, use_safetensors: bool, logger=None,
                 writers: int = 0, stem: str = CHUNK_STEM, metadata: bool = True):
        self.order, self.dir, self.size, self.st, self.logger = order, output_dir, chunk_size, use_safetensors, logger
        self.writers = writers or min(8, max(2, cpu_share() // 2))
        # while producers run, at most `writers` chunk writes at once (more stalled the GPU
        # pipeline's HIP calls); once close() is called the backlog drains with tail_writers
        self.tail_writers = max(self.writers, min(8, max(2, cpu_share() // 2)))
        self.gate = threading.Semaphore(self.writers)
        self.stem, self.metadata = stem, metadata
        self.t2c: Dict[str, int] = {}
        self.n_chunks = self.n_ok = 0
        self.qparams: Optional[Dict] = None
        self.status: Dict[str, Optional[Dict[str, torch.Tensor]]] = {}
        self.closed = False
        self.error: Optional[BaseException] = None
        self.cv = threading.Condition()
        self.times: List[Tuple[float, float, float]] = []   # per chunk: submitted, started, ended (time.time)
        self.failed: set = set()
        self.hooks: List[Callable[[List[str]], None]] = []
        self.n_reported = 0
        self.widened = False
        os.makedirs(output_dir, exist_ok=True)
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def done(self, name: str, result: Optional[Dict[str, torch.Tensor]]) -> None:
        """A tensor finished: its host result dict, or None if it failed.  Once every tensor
        has reported, the producers' HIP work is over: the pool widens for the tail.  Raises
        once a chunk write has failed, so the producer stops (the native pipeline then cancels
        its remaining batches) instead of quantizing into a run that cannot be saved."""
        with self.cv:
            if self.error is not None:
                raise RuntimeError(f"chunk writer failed: {self.error}") from self.error
            self.status[name] = result
            if result is None:
                self.failed.add(name)
            self.n_reported += 1
            last = self.n_reported == len(self.order)
            self.cv.notify()
        if last:
            self._widen()

    def _widen(self) -> None:
        with self.cv:
            if self.widened:
                return
            self.widened = True
        for _ in range(self.tail_writers - self.writers):
            self.gate.release()

    def add_written_hook(self, fn: Callable[[List[str]], None]) -> None:
        """fn(names) after each chunk file is written: its results are no longer read."""
        with self.cv:
            self.hooks.append(fn)

    def predict_groups(self) -> Dict[str, int]:
        """The chunk every tensor not yet known to have failed lands in, if it succeeds."""
        with self.cv:
            failed = set(self.failed)
        out, k = {}, 0
        for name in self.order:
            if name not in failed:
                out[name] = k // self.size
                k += 1
        return out

    def _run(self) -> None:
        try:
            with ThreadPoolExecutor(max_workers=self.tail_writers) as pool:
                futs = []
                chunk, c, t2c, qparams, n_ok = {}, 0, {}, None, 0
                for name in self.order:
                    with self.cv:
                        while name not in self.status and not self.closed:
                            self.cv.wait()
                        res = self.status.pop(name, None)
                    if res is None:
                        continue
                    if qparams is None:
                        qparams = {k: (res[k].item() if k in res else None) for k in ("bits", "group_size", "symmetric")}
                    chunk[name] = res
                    t2c[name] = c
                    n_ok += 1
                    if len(chunk) == self.size:
                        futs.append(pool.submit(self._timed_write, chunk, c, time.time()))
                        chunk, c = {}, c + 1
                if chunk:
                    futs.append(pool.submit(self._timed_write, chunk, c, time.time()))
                    c += 1
                for f in futs:
                    f.result()
            self.t2c, self.n_chunks, self.n_ok, self.qparams = t2c, c, n_ok, qparams
            if n_ok and self.metadata:
                _write_metadata(self.dir, c, self.size, t2c, self.st, n_ok, qparams, self.logger)
        except BaseException as e:  # noqa: BLE001  (reported by close())
            with self.cv:
                if self.error is None:
                    self.error = e
            # nothing more will be written: release every result, so a producer blocked on a
            # wrapping host ring (awq_stream_release) is never left waiting for this thread
            self._report_written(list(self.order))

    def _report_written(self, names: List[str]) -> None:
        with self.cv:
            hooks = list(self.hooks)
        for fn in hooks:
            fn(names)

    def _timed_write(self, chunk, c: int, t_submit: float) -> None:
        names = list(chunk)
        try:
            with self.gate:
                t0 = time.time()
                _write_chunk(chunk, self.dir, c, self.st, self.logger, stem=self.stem)
                self.times.append((t_submit, t0, time.time()))
        except BaseException as e:  # noqa: BLE001  (first error wins; done() and close() report it)
            with self.cv:
                if self.error is None:
                    self.error = e
            raise
        finally:
            # written or failed, these results are never read again: the pipeline may reuse
            # their ring range (a failed write must not leave it blocked)
            chunk.clear()
            self._report_written(names)

    def close(self) -> None:
        """Every producer has finished: unfinished tensors count as failed; wait for the writes."""
        with self.cv:
            self.closed = True
            self.cv.notify()
        self._widen()                                       # the producers are done: widen the pool
        self.thread.join()
        if self.error is not None:
            raise self.error


def _to_cpu(d: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in d.items()}


_NOT_LINEAR = ("embed", "lm_head", "norm", "wte", "wpe", "ln_", "router")
# model types whose projection weights are transformers Conv1D modules, stored [in, out]
# (quantizing them as [out, in] would group along the wrong axis): copied, not quantized
CONV1D_MODEL_TYPES = ("gpt2", "openai-gpt", "imagegpt", "decision_transformer")


def is_linear_weight(info: TensorInfo, group_size: int, model_type: Optional[str] = None) -> bool:
    """The tensors an AutoAWQ checkpoint quantizes: 2-D `*.weight` of nn.Linear layers whose
    shape the GEMM layout can hold.  Heuristic on names (no module graph in a checkpoint):
    not embeddings, the LM head, norms, MoE routers (`*.router.*`, and `*.gate.weight` —
    Mixtral's block_sparse_moe.gate / Qwen-MoE's mlp.gate; `gate_proj` is a linear) which
    AutoAWQ keeps in fp16, nor any weight of a Conv1D model (CONV1D_MODEL_TYPES)."""
    if len(info.shape) != 2 or not info.name.endswith(".weight") or not info.dtype.is_floating_point:
        return False
    if model_type in CONV1D_MODEL_TYPES:
        return False
    if any(s in info.name for s in _NOT_LINEAR) or info.name.endswith(".gate.weight"):
        return False
    n, k = info.shape
    return n % 8 == 0 and k % group_size == 0


def model_type_of(loader) -> Optional[str]:
    """config.json's model_type next to the weights, if any."""
    path = os.path.join(getattr(loader, "model_path", "") or "", "config.json")
    try:
        with open(path) as f:
            return json.load(f).get("model_type")
    except (OSError, ValueError):
        return None


def autoawq_tensors(quantized: Dict[str, Dict[str, torch.Tensor]], loader, passthrough: List[TensorInfo],
                    failed: List[TensorInfo] = ()) -> Dict[str, torch.Tensor]:
    """The tensors of an AutoAWQ checkpoint (or one shard of it): `<layer>.qweight/.qzeros/
    .scales` per quantized linear weight; every passthrough tensor and every linear weight
    that failed to quantize copied unchanged (those layers stay unquantized:
    modules_to_not_convert)."""
    tensors = {}
    for name, r in quantized.items():
        prefix = name[: -len(".weight")]
        for f in ("qweight", "qzeros", "scales"):
            tensors[f"{prefix}.{f}"] = r[f].contiguous()
    for info in list(passthrough) + list(failed):
        tensors[info.name] = loader.read(info).contiguous()
    return tensors


def write_autoawq_configs(output_dir: str, args, loader, not_converted: List[str], logger=None) -> None:
    """quant_config.json (AutoAWQ) and, when the source has one, config.json with a
    transformers `quantization_config`; `not_converted` = module names of linear weights
    left unquantized (their quantization failed and they were copied through)."""
    qcfg = {"zero_point": not args.symmetric, "q_group_size": args.group_size, "w_bit": 4, "version": "GEMM"}
    if not_converted:
        qcfg["modules_to_not_convert"] = list(not_converted)
    with open(os.path.join(output_dir, "quant_config.json"), "w") as f:
        json.dump(qcfg, f, indent=2)
    src = os.path.join(getattr(loader, "model_path", "") or "", "config.json")
    if os.path.isfile(src):
        with open(src) as f:
            cfg = json.load(f)
        cfg["quantization_config"] = {"quant_method": "awq", "bits": 4, "group_size": args.group_size,
                                      "zero_point": not args.symmetric, "version": "gemm"}
        if not_converted:
            cfg["quantization_config"]["modules_to_not_convert"] = list(not_converted)
        with open(os.path.join(output_dir, "config.json"), "w") as f:
            json.dump(cfg, f, indent=2)
    if not_converted and logger:
        logger.warning(f"{len(not_converted)} linear weight(s) failed to quantize and were copied unquantized "
                       f"(modules_to_not_convert): {not_converted}")


def save_autoawq(quantized: Dict[str, Dict[str, torch.Tensor]], loader, passthrough: List[TensorInfo],
                 output_dir: str, args, logger=None, failed: List[TensorInfo] = ()) -> None:
    """model.safetensors with `<layer>.qweight/.qzeros/.scales` for every quantized linear
    weight and every other tensor copied unchanged (linear weights that failed to quantize
    included, listed in modules_to_not_convert so the checkpoint still loads), plus the
    configs of write_autoawq_configs."""
    from safetensors.torch import save_file
    tensors = autoawq_tensors(quantized, loader, passthrough, failed)
    save_file(tensors, os.path.join(output_dir, "model.safetensors"), metadata={"format": "pt"})
    write_autoawq_configs(output_dir, args, loader, [i.name[: -len(".weight")] for i in failed], logger)
    if logger:
        logger.info(f"Saved AutoAWQ checkpoint: {len(quantized)} quantized linear weights, "
                    f"{len(passthrough) + len(failed)} tensors copied")


def cpu_share() -> int:
    """CPUs this process may actually use: its affinity set, capped by a cgroup v2 CPU quota
    (`cpu.max`) — os.cpu_count() reports the whole machine, which on a shared GPU node is
    many times the process's share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def writer_threads(infos: List[TensorInfo], packed: bool) -> int:
    """Chunk-writer threads for an output of this size: more writers only pay when the
    files are large — below ~2 GB of output, 8 concurrent writers stalled the pipeline's
    HIP calls for 8-12 ms at a time while 3-4 did not (opt-350m, profiles/round3/r3o: 0.057 s
    vs 0.066-0.072 s warm), and above it the writes are the bound (Llama-3-8B packed 0.36 s
    at 8 writers vs 0.42-0.46 at 4).  STREAM_OPTS["writers"] overrides."""
    forced = STREAM_OPTS.get("writers")
    if forced:
        return int(forced)
    in_bytes = sum(i.nbytes for i in infos)
    out_bytes = in_bytes * (0.26 if packed else 2.05)   # 4-bit packed ~ in / 4; reference ~ 2 x in
    share = cpu_share()
    return min(4, max(2, share // 4)) if out_bytes < (2 << 30) else min(8, max(2, share // 2))


def _batches(infos: List[TensorInfo], budget: int) -> List[List[TensorInfo]]:
    """Consecutive runs of tensors (processing order kept) of at most `budget` input bytes
    (a larger tensor forms a batch of its own)."""
    out, cur, size = [], [], 0
    for info in infos:
        if cur and size + info.nbytes > budget:
            out.append(cur)
            cur, size = [], 0
        cur.append(info)
        size += info.nbytes
    if cur:
        out.append(cur)
    return out


def _batch_budget(total: int, batch_bytes: int) -> int:
    """Input bytes per batch: small enough that a small model still pipelines (read / H2D /
    kernel / D2H of neighbouring batches overlap) — about 8 batches per device, 32 MiB ..
    batch_bytes each."""
    return max(32 << 20, min(batch_bytes, total // 8))


def _pinned_copy(t: torch.Tensor) -> torch.Tensor:
    """Host copy in page-locked memory (torch's caching host allocator), so the H2D / D2H
    copies run asynchronously on the copy stream."""
    p = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    p.copy_(t)
    return p


def quantize_stream_native(loader, infos: List[TensorInfo], quantizer: AWQQuantizer, device: str, readers: int,
                           packed: bool, out: Dict, lock: threading.Lock, logger, keep_on_device: bool = False,
                           on_done: Optional[Callable[[str, Optional[Dict[str, torch.Tensor]]], None]] = None,
                           writer: Optional["ChunkWriter"] = None, slot_bytes: int = 0, host_ring_bytes: int = 0,
                           dev_ring_bytes: int = 0) -> None:
    """The CLI's read -> quantize -> collect loop on the native pipeline with bounded output
    memory (awq_quantizer/stream.py).  With `writer` (the ChunkWriter that consumes
    `on_done`'s results) the host ring may wrap: results are released once their chunk is
    written; without it the host ring holds the whole output."""
    from .stream import quantize_stream_native as run
    hook = groups = None
    if writer is not None and not keep_on_device:
        hook = writer.add_written_hook
        groups = writer.predict_groups
    run(loader, infos, quantizer, device, readers, packed, out, lock, logger, keep_on_device=keep_on_device,
        on_done=on_done, release_hook=hook, group_of=groups, slot_bytes=slot_bytes,
        host_ring_bytes=host_ring_bytes or int(STREAM_OPTS.get("host_ring_bytes", 0)),
        dev_ring_bytes=dev_ring_bytes or int(STREAM_OPTS.get("dev_ring_bytes", 0)),
        opts=STREAM_OPTS, timings=TIMINGS)


def quantize_stream(loader, infos: List[TensorInfo], quantizer: AWQQuantizer, device: str, readers: int,
                    lookahead: int, packed: bool, out: Dict, lock: threading.Lock, logger,
                    memory_efficient: bool = False, keep_on_device: bool = False,
                    batch_bytes: int = 1 << 30, export_autoawq: bool = False,
                    act_stats: Optional[Dict[str, Tuple[torch.Tensor, torch.Tensor]]] = None,
                    on_done: Optional[Callable[[str, Optional[Dict[str, torch.Tensor]]], None]] = None,
                    writer: Optional["ChunkWriter"] = None, engine: str = "native") -> None:
    """Quantize `infos` on one GPU.  RTN and the per-group clip search (scale_method
    "search") to the packed or reference format run on the native pipeline
    (quantize_stream_native; `writer`: the ChunkWriter consuming on_done, whose written
    chunks release the pipeline's host ring — only when it serves this device alone); the
    activation-aware search (`act_stats`), the AutoAWQ export and `engine="python"` on the
    Python pipeline below."""
    if engine == "native" and not act_stats and not export_autoawq and hasattr(loader, "data_location"):
        return quantize_stream_native(loader, infos, quantizer, device, readers, packed, out, lock, logger,
                                      keep_on_device=keep_on_device, on_done=on_done, writer=writer)
    return quantize_stream_python(loader, infos, quantizer, device, readers, lookahead, packed, out, lock, logger,
                                  memory_efficient, keep_on_device, batch_bytes, export_autoawq, act_stats, on_done)


def quantize_stream_python(loader, infos: List[TensorInfo], quantizer: AWQQuantizer, device: str, readers: int,
                           lookahead: int, packed: bool, out: Dict, lock: threading.Lock, logger,
                           memory_efficient: bool = False, keep_on_device: bool = False,
                           batch_bytes: int = 1 << 30, export_autoawq: bool = False,
                           act_stats: Optional[Dict[str, Tuple[torch.Tensor, torch.Tensor]]] = None,
                           on_done: Optional[Callable[[str, Optional[Dict[str, torch.Tensor]]], None]] = None) -> None:
    """Quantize `infos` on one GPU as a pipeline over batches of tensors (<= batch_bytes of
    input each):

      reader threads: safetensors read -> pinned host copy      (batch k+1 .. k+lookahead)
      copy stream:    H2D of batch k                            (overlaps batch k-1's kernels)
      compute stream: one ragged launch per dtype for batch k   (awq_quantize_ragged)
      copy stream:    D2H of batch k's results into pinned host memory

    The reference instead loads every file whole and copies every tensor to the device
    eagerly (main.py:296-307), then quantizes tensor by tensor.  Per-tensor failures are
    logged and skipped (main.py:387-390).

    act_stats (scale_method="awq"): name -> (x_mean, x_sq); those weights take the
    activation-aware search (AWQQuantizer.quantize_layer_group, one weight per layer group)
    and carry its "input_scale" in their results."""
    t_enter = time.perf_counter()
    if not (device.startswith("cuda") and torch.cuda.is_available()):
        quantizer.compute_device()   # raises HipUnavailable: no CPU path
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    torch.cuda.set_device(dev)
    copy_stream = torch.cuda.Stream(dev)
    compute = torch.cuda.current_stream(dev)
    budget = _batch_budget(sum(i.nbytes for i in infos), batch_bytes)
    batches = _batches(infos, budget)
    depth = max(1, lookahead // max(1, max(len(b) for b in batches) if batches else 1))
    clock = time.perf_counter
    t_read = t_submit = t_finish = 0.0

    direct = hasattr(loader, "read_pinned")

    def read(info, dst=None):
        # straight from the file into pinned memory (one copy) — into the batch's staging
        # buffer when one is given (a loader without direct reads: its read + a pinned copy)
        if dst is not None:
            return loader.read_into(info, dst)
        return loader.read_pinned(info) if direct else _pinned_copy(loader.read(info))

    staging = {}   # batch -> (pinned uint8 buffer, name -> byte offset): one H2D per batch

    def stage(k):
        offs, pos = {}, 0
        for info in batches[k]:
            if info.dtype is None:
                continue
            offs[info.name] = pos
            pos += (info.nbytes + 255) // 256 * 256      # 256-B aligned slices (16-B vector loads)
        buf = torch.empty(max(pos, 1), dtype=torch.uint8, pin_memory=True)
        staging[k] = (buf, offs)
        return buf, offs

    def view(buf, off, info):
        return buf[off:off + info.nbytes].view(info.dtype).view(info.shape)

    inflight = deque()

    def finish(entry):
        nonlocal t_finish
        results, ev, _keep = entry
        t0 = clock()
        ev.synchronize()
        t_finish += clock() - t0
        with lock:
            out.update(results)
        for name in results:
            if logger:
                logger.info(f"Successfully quantized tensor: {name} on {device}")
            if on_done:
                on_done(name, results[name])

    with ThreadPoolExecutor(max_workers=max(1, readers)) as pool:
        futs = {}

        def submit(k):
            if k < len(batches) and k not in futs:
                if direct:
                    buf, offs = stage(k)
                    futs[k] = [(info, pool.submit(read, info, view(buf, offs[info.name], info) if info.name in offs
                                                  else None)) for info in batches[k]]
                else:
                    futs[k] = [(info, pool.submit(read, info)) for info in batches[k]]

        for k in range(min(len(batches), depth + 1)):
            submit(k)
        for k in range(len(batches)):
            submit(k + depth)
            host = {}
            t0 = clock()
            for info, fut in futs.pop(k):
                try:
                    host[info.name] = fut.result()
                except Exception as e:  # noqa: BLE001
                    if logger:
                        logger.error(f"Failed to quantize tensor {info.name} on {device}: {e}")
                    if on_done:
                        on_done(info.name, None)
            t1 = clock()
            t_read += t1 - t0
            if not host:
                continue
            if logger:
                for name in host:
                    logger.info(f"Quantizing tensor: {name} on {device}")
            staged = None
            with torch.cuda.stream(copy_stream):
                if k in staging:     # the whole staging buffer in one copy; device views of it
                    buf, offs = staging.pop(k)
                    dbuf = torch.empty(buf.numel(), dtype=torch.uint8, device=dev)
                    dbuf.copy_(buf, non_blocking=True)
                    by_name = {i.name: i for i in batches[k]}
                    dev_in = {n: view(dbuf, offs[n], by_name[n]) for n in host}
                    staged = buf                      # kept alive until the copy is done
                else:
                    dev_in = {n: t.to(dev, non_blocking=True) for n, t in host.items()}
                ev_in = torch.cuda.Event()
                ev_in.record(copy_stream)
            compute.wait_event(ev_in)
            with torch.cuda.stream(compute):
                searched = {}
                for name in [n for n in dev_in if act_stats and n in act_stats]:
                    try:
                        xm, xs = act_stats[name]
                        searched[name] = quantizer.quantize_layer_group(
                            {name: dev_in[name]}, x_mean=xm, x_sq=xs, packed=packed)["results"][name]
                    except Exception as e:  # noqa: BLE001  (reference semantics: skip and continue)
                        if logger:
                            logger.error(f"Error quantizing tensor: {name}, error: {e}")
                res = quantizer.quantize_model_device({n: t for n, t in dev_in.items()
                                                       if not (act_stats and n in act_stats)}, packed=packed)
                res.update(searched)
                if export_autoawq:
                    res = {n: _with_input_scale(quantizer.export_autoawq(r), r) for n, r in res.items()}
                ev_k = torch.cuda.Event()
                ev_k.record(compute)
            for name in host:
                if name not in res:
                    if logger:
                        logger.error(f"Failed to quantize tensor {name} on {device}")
                    if on_done:
                        on_done(name, None)
            if keep_on_device:
                ev_k.synchronize()
                with lock:
                    out.update(res)
                continue
            copy_stream.wait_event(ev_k)
            with torch.cuda.stream(copy_stream):
                host_res = {}
                for name, r in res.items():
                    hr = {}
                    for f, v in r.items():
                        if isinstance(v, torch.Tensor) and v.is_cuda:
                            h = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
                            h.copy_(v, non_blocking=True)
                            hr[f] = h
                        else:
                            hr[f] = v
                    host_res[name] = hr
                ev_out = torch.cuda.Event()
                ev_out.record(copy_stream)
            t_submit += clock() - t1
            # inputs and device results stay referenced until their copies are done
            inflight.append((host_res, ev_out, (host, dev_in, res, staged)))
            while len(inflight) > 1:
                finish(inflight.popleft())
            if memory_efficient:
                torch.cuda.empty_cache()
        while inflight:
            finish(inflight.popleft())
    # host-side phase times of this device's pipeline (scripts/cli_bench.py prints them)
    TIMINGS.update({f"stream_{device}": {"wall_s": round(time.perf_counter() - t_enter, 4),
                                          "batches": len(batches), "batch_MB": budget >> 20,
                                          "read_wait_s": round(t_read, 4), "submit_s": round(t_submit, 4),
                                          "finish_wait_s": round(t_finish, 4)}})


def _with_input_scale(exported: Dict[str, torch.Tensor], packed: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    if "input_scale" in packed:
        exported["input_scale"] = packed["input_scale"]
    return exported


def load_act_stats(path: str, logger=None) -> Dict[str, Tuple[torch.Tensor, torch.Tensor]]:
    """--act_stats: '<weight name>.x_mean' / '<weight name>.x_sq' fp32 vectors (safetensors)."""
    from safetensors.torch import load_file
    flat = load_file(path)
    out = {}
    for key, t in flat.items():
        if key.endswith(".x_mean"):
            name = key[: -len(".x_mean")]
            sq = flat.get(name + ".x_sq")
            if sq is None:
                raise ValueError(f"--act_stats: {key} has no matching {name}.x_sq")
            out[name] = (t.float().reshape(-1), sq.float().reshape(-1))
    if logger:
        logger.info(f"Loaded activation statistics for {len(out)} weights from {path}")
    return out


def _device_worker(*args, **kwargs) -> None:
    """Thread body of one device: a failure of the whole device (no GPU, no library) is
    logged; its tensors then count as not quantized."""
    logger, device = args[9], args[3]
    try:
        quantize_stream(*args, **kwargs)
    except Exception as e:  # noqa: BLE001
        if logger:
            logger.error(f"Quantization on {device} failed: {e}")


def main(argv: Optional[List[str]] = None) -> int:
    logger = None
    t_main = time.time()
    try:
        args = parse_args(argv)
        logger = get_logger(name="awq_quantizer", level=args.log_level, to_file=args.log_file is not None,
                            file_path=args.log_file)
        os.makedirs(args.output_dir, exist_ok=True)

        if args.multi_gpu or args.device.lower() == "all":
            devices = get_available_gpus(logger)
            if not devices:
                logger.warning("No CUDA devices available, falling back to CPU")
                devices = ["cpu"]
            else:
                logger.info(f"Using {len(devices)} GPU(s) for processing")
        else:
            devices = [args.device]
        for d in devices:
            if d.startswith("cuda") and torch.cuda.is_available():
                idx = int(d.split(":")[1]) if ":" in d else 0
                total, free = get_device_memory_info(idx)
                logger.info(f"Using GPU {d}: {device_name(idx)}")
                logger.info(f"  Total memory: {total:.2f} GB")
                logger.info(f"  Free memory: {free:.2f} GB")
            elif d.startswith("cuda"):
                logger.warning(f"CUDA device {d} requested but not available, falling back to CPU")
                devices = ["cpu"]
            elif d == "cpu":
                logger.info("Using CPU for quantization")

        from . import distributed as D
        if len(devices) == 1 and D.env_world()[2] <= 1:
            start_warmup(devices[0])    # HIP's first-use costs overlap the index and planning below
        TIMINGS["devices_s"] = round(time.time() - t_main, 4)
        TIMINGS["module_import_torch_s"] = round(_IMPORT_TORCH_S, 4)
        logger.info(f"Loading model from {args.model_id}")
        try:
            loader = load_model_from_hub(args.model_id, logger_level=args.log_level)
            index = loader.tensor_index()
        except Exception as e:  # noqa: BLE001
            logger.error(f"Failed to load model: {e}")
            return 1

        TIMINGS["index_s"] = round(time.time() - t_main - TIMINGS["devices_s"], 4)
        logger.info("Preparing tensors for quantization")
        start = time.time()
        ordered = select_tensors(index, logger)
        autoawq = args.output_format == "autoawq"
        passthrough: List[TensorInfo] = []
        if autoawq:
            if args.bits != 4:
                logger.error("--output_format autoawq writes 4-bit checkpoints (AutoAWQ GEMM layout)")
                return 1
            mtype = model_type_of(loader)
            if mtype in CONV1D_MODEL_TYPES:
                logger.warning(f"model_type {mtype}: Conv1D projection weights ([in, out]) are copied unquantized")
            linear = {i.name for i in ordered if is_linear_weight(i, args.group_size, mtype)}
            passthrough = [i for i in index if i.name not in linear]
            ordered = [i for i in ordered if i.name in linear]
            logger.info(f"AutoAWQ export: {len(ordered)} linear weights quantized, {len(passthrough)} copied")
        act_stats = None
        if args.act_stats:
            if args.scale_method != "awq":
                logger.error("--act_stats needs --scale_method awq")
                return 1
            if autoawq:
                logger.error("--act_stats with --output_format autoawq: the searched input scales must be folded "
                             "into the ops producing each input first; use --output_format packed or reference "
                             "(results carry 'input_scale')")
                return 1
            act_stats = load_act_stats(args.act_stats, logger)
        elif args.scale_method == "awq":
            logger.warning("--scale_method awq without --act_stats: every weight is quantized RTN")
        from . import distributed as D
        rank, local, world = D.env_world()
        if world > 1:   # torchrun: one process per GPU, LPT shard, RCCL gather to rank 0
            return _main_distributed(args, loader, ordered, logger, start, passthrough, act_stats)
        parts = partition_tensors(ordered, len(devices))
        quantizers = {d: AWQQuantizer(bits=args.bits, group_size=args.group_size, symmetric=args.symmetric,
                                      zero_point=args.zero_point, percentile=args.percentile,
                                      scale_method=args.scale_method, per_channel=args.per_channel, device=d,
                                      search_grid=args.search_grid, search_max_shrink=args.search_max_shrink,
                                      duo_scaling=not args.no_duo_scaling, logger_name=f"awq_quantizer_{d}", logger_level=args.log_level,
                                      logger_to_file=args.log_file is not None, logger_file_path=args.log_file)
                      for d in devices}
        results: Dict[str, Dict[str, torch.Tensor]] = {}
        lock = threading.Lock()
        lookahead = max(1, args.prefetch_factor * args.batch_size)
        packed = args.output_format in ("packed", "autoawq")
        # chunked output written while later batches are still being read and quantized
        writer = None
        if not autoawq:
            writer = ChunkWriter([i.name for i in ordered], args.output_dir, args.chunk_size, args.save_safetensors,
                                 logger, writers=writer_threads(ordered, packed))
        if writer is not None:
            # the writer owns every result until its chunk is on disk; a device's pipeline may
            # then reuse (wrap) its host output ring — only when it is the writer's only producer
            results = _NullSink()
        threads = []
        TIMINGS["pre_stream_s"] = time.time() - start
        for d, part in zip(devices, parts):
            logger.info(f"Processing {len(part)} tensors on {d}")
            th = threading.Thread(target=_device_worker, args=(loader, part, quantizers[d], d, args.num_workers,
                                                               lookahead, packed, results, lock, logger,
                                                               args.memory_efficient, False, 1 << 30, autoawq),
                                  kwargs={"act_stats": act_stats, "on_done": writer.done if writer else None,
                                          "writer": writer if len(devices) == 1 else None,
                                          "engine": args.stream_engine})
            th.start()
            threads.append(th)
        for th in threads:
            th.join()
        TIMINGS["quantize_s"] = time.time() - start

        quantized = {i.name: results[i.name] for i in ordered if i.name in results}   # size-descending
        if not quantized:
            if writer is not None:
                writer.close()
            logger.error("No tensors were successfully quantized")
            return 1
        logger.info(f"Successfully quantized {len(quantized)} tensors")
        logger.info(f"Saving quantized model to {args.output_dir}")
        try:
            if autoawq:
                save_autoawq(quantized, loader, passthrough, args.output_dir, args, logger,
                             failed=[i for i in ordered if i.name not in quantized])
            elif writer is not None:
                t_close = time.time()
                writer.close()
                if writer.times:
                    TIMINGS["writer"] = {"chunks": len(writer.times), "close_wait_s": round(time.time() - t_close, 4),
                                         "write_s_sum": round(sum(e - b for _, b, e in writer.times), 4),
                                         "write_s_max": round(max(e - b for _, b, e in writer.times), 4),
                                         "last_submit_to_end_s": round(max(e for _, _, e in writer.times)
                                                                       - max(a for a, _, _ in writer.times), 4)}
                    if STREAM_OPTS.get("trace"):   # per chunk: submitted, started, ended (s after `start`)
                        TIMINGS["writer"]["trace"] = [tuple(round(v - start, 4) for v in t) for t in writer.times]
            else:
                save_model_in_chunks(quantized, args.output_dir, chunk_size=args.chunk_size,
                                     use_safetensors=args.save_safetensors, logger=logger)
        except Exception as e:  # noqa: BLE001
            logger.error(f"Failed to save quantized model: {e}")
            return 1
        TIMINGS["total_s"] = time.time() - start
        logger.info(f"Quantization complete in {time.time() - start:.2f} seconds")
        logger.info("metrics " + json.dumps(run_metrics(ordered, quantized, TIMINGS)))
        return 0
    except SystemExit:
        raise
    except Exception as e:  # noqa: BLE001
        if logger is None:
            logging.getLogger("awq_quantizer").error(f"Error during quantization: {e}")
        else:
            logger.error(f"Error during quantization: {e}")
        return 1


def run_metrics(ordered, quantized, timings) -> Dict[str, float]:
    """One JSON line per run (SURVEY.md §5 metrics): tensors quantized, their input bytes, the
    quantize phase (read + H2D + kernels + D2H, overlapped) and the whole run incl. the final
    writes, and the end-to-end rate over the input bytes.  (Not the kernel's roofline: that is
    bench.py's, with inputs resident in HBM.)"""
    nbytes = sum(i.nbytes for i in ordered if i.name in quantized)
    total = max(float(timings.get("total_s", 0.0)), 1e-9)
    return {"tensors": len(quantized), "input_bytes": int(nbytes),
            "quantize_s": round(float(timings.get("quantize_s", 0.0)), 4), "total_s": round(total, 4),
            "input_GB_per_s": round(nbytes / total / 1e9, 3)}


_SCALARS = ("bits", "group_size", "symmetric", "shape")
TIMINGS: Dict[str, float] = {}   # phase times of the last main() call (scripts/cli_bench.py)
# native pipeline overrides for measurement scripts (scripts/cli_profile.py --stream-opts):
# slot_bytes, nslots, copy_streams (1: H2D and D2H share one stream), trace (1: per-batch
# timestamps, include/awq_hip.h awq_stream_config.trace), readers (pread threads), writers
# (ChunkWriter threads), host_arena (0: one pinned buffer per output chunk)
STREAM_OPTS: Dict[str, int] = {}


def _main_distributed(args, loader, ordered: List[TensorInfo], logger, start: float,
                      passthrough: Optional[List[TensorInfo]] = None, act_stats=None) -> int:
    """torchrun mode: one process per GPU; rank r quantizes the tensors an LPT partition by
    bytes assigns it (identical on every rank, derived from the header index with no
    exchange; the reference's own partition_tensors, main.py:395-427).  Output
    (--dist_output):

      per_rank (default): every rank writes its own results as they come off its GPU
        (ChunkWriter under a rank-private file stem, disk writes overlapping its later
        batches); one all_gather_object of the per-rank chunk tables, then each rank renames
        its files to global chunk numbers (rank r's chunks follow rank r-1's) and rank 0
        writes metadata.json over every tensor in processing order (reference main.py:
        430-512).  No result bytes cross the fabric.  AutoAWQ: one safetensors shard per rank
        + model.safetensors.index.json.
      gather: every result is sent to rank 0 in one batched point-to-point round over RCCL
        (xGMI) and rank 0 writes the single-process layout.

    A rank whose pipeline fails as a whole (no device, no library, a batch error) still
    joins every collective, with no results; the failure is agreed (MAX over ranks), nothing
    is published and every rank exits 1.  Per-tensor failures are skipped and logged as in
    the single-process CLI."""
    from . import distributed as D
    import torch.distributed as dist
    backend = os.environ.get("AWQ_DIST_BACKEND", "nccl")      # gloo: tests with 2 ranks on one GPU
    if backend != "nccl":
        D.init(backend)
    rank, local, world = D.init("nccl") if backend == "nccl" else D.env_world()
    device = f"cuda:{local % max(1, torch.cuda.device_count())}"
    comm = torch.device(device) if backend == "nccl" else torch.device("cpu")
    owner = dict(zip((i.name for i in ordered), D.shard([i.nbytes for i in ordered], world)))
    mine = [i for i in ordered if owner[i.name] == rank]
    autoawq = args.output_format == "autoawq"
    per_rank = args.dist_output == "per_rank"
    if per_rank and not _shared_output_dir(args.output_dir, rank, world, logger):
        # node-local disks (multi-node torchrun): rank 0's metadata.json could not reach the
        # other ranks' chunk files, so every result goes to rank 0 instead
        if rank == 0:
            logger.warning(f"{args.output_dir} is not one shared directory for all {world} ranks; "
                           f"falling back to --dist_output gather")
        per_rank = False
    results: Dict[str, Dict[str, torch.Tensor]] = {}
    writer, failed = None, 0
    t0 = time.time()
    try:
        q = AWQQuantizer(bits=args.bits, group_size=args.group_size, symmetric=args.symmetric,
                         zero_point=args.zero_point, percentile=args.percentile, scale_method=args.scale_method,
                         per_channel=args.per_channel, search_grid=args.search_grid,
                         search_max_shrink=args.search_max_shrink, duo_scaling=not args.no_duo_scaling, device=device,
                         logger_name=f"awq_quantizer_{device}", logger_level=args.log_level,
                         logger_to_file=args.log_file is not None, logger_file_path=args.log_file)
        logger.info(f"rank {rank}/{world}: {len(mine)} of {len(ordered)} tensors on {device}")
        if per_rank and not autoawq:
            writer = ChunkWriter([i.name for i in mine], args.output_dir, args.chunk_size, args.save_safetensors,
                                 logger, stem=_rank_stem(rank), metadata=False,
                                 writers=writer_threads(mine, args.output_format in ("packed", "autoawq")))
        # per-rank chunks: the writer holds each result until its chunk is on disk, nothing else does
        sink = _NullSink() if writer is not None else results
        quantize_stream(loader, mine, q, device, args.num_workers, max(1, args.prefetch_factor * args.batch_size),
                        args.output_format in ("packed", "autoawq"), sink, threading.Lock(), logger,
                        args.memory_efficient, keep_on_device=not per_rank, export_autoawq=autoawq,
                        act_stats=act_stats, on_done=writer.done if writer else None, writer=writer,
                        engine=args.stream_engine)
    except Exception as e:  # noqa: BLE001  (agreed below: every rank exits 1)
        logger.error(f"rank {rank}: quantization failed: {e}")
        failed = 1
    if writer is not None:
        try:
            writer.close()
        except Exception as e:  # noqa: BLE001
            logger.error(f"rank {rank}: writing chunks failed: {e}")
            failed = 1
    if failed:
        results = {}
    TIMINGS[f"rank{rank}_quantize_write_s"] = round(time.time() - t0, 4)
    try:
        if per_rank and autoawq:
            rc = _commit_rank_autoawq(args, loader, ordered, mine, results, passthrough or [], rank, world, failed,
                                      comm, logger)
        elif per_rank:
            rc = _commit_rank_chunks(args, ordered, writer, rank, world, failed, comm, logger)
        else:
            rc = _gather_and_write(args, loader, ordered, results, passthrough or [], rank, world, failed, comm,
                                   logger)
    finally:
        dist.destroy_process_group()
    if rank == 0 and rc == 0:
        logger.info(f"Quantization complete in {time.time() - start:.2f} seconds")
        TIMINGS["total_s"] = time.time() - start
        logger.info("metrics " + json.dumps(dict(run_metrics(ordered, {i.name for i in ordered}, TIMINGS), world=world)))
    return rc


def _shared_output_dir(output_dir: str, rank: int, world: int, logger) -> bool:
    """True if every rank sees the same output directory (per-rank chunk files are only a
    checkpoint when rank 0's metadata.json and every rank's chunks land in one directory):
    rank 0 creates a sentinel file with a random name, every rank looks for it."""
    import secrets
    import torch.distributed as dist
    token = [secrets.token_hex(8) if rank == 0 else None]
    dist.broadcast_object_list(token, src=0)
    path = os.path.join(output_dir, f".awq_shared_{token[0]}")
    made = 1
    if rank == 0:
        try:
            os.makedirs(output_dir, exist_ok=True)
            with open(path, "w") as f:
                f.write("awq_quantizer per-rank output check\n")
        except OSError as e:
            logger.error(f"cannot write to {output_dir}: {e}")
            made = 0
    dist.barrier()
    seen = [None] * world
    dist.all_gather_object(seen, bool(made) and os.path.exists(path))
    dist.barrier()
    if rank == 0 and made:
        try:
            os.remove(path)
        except OSError:
            pass
    return all(seen)


class _NullSink(dict):
    """quantize_stream's result dict when a ChunkWriter already owns every result: it keeps
    the names only (the results may be views of a ring the pipeline reuses once written)."""

    def __setitem__(self, name, value) -> None:
        super().__setitem__(name, None)

    def update(self, *a, **k) -> None:
        for d in a + (k,):
            for name in d:
                super().__setitem__(name, None)


def _rank_stem(rank: int) -> str:
    """Rank-private chunk file stem (renamed to CHUNK_STEM numbers once all ranks agree)."""
    return f".rank{rank:05d}_chunk_{{:04d}}"


def _agree(flag: int, comm: torch.device) -> int:
    """MAX of a per-rank int over all ranks (a failure anywhere fails everyone)."""
    from . import distributed as D
    return int(D.max_over_ranks(float(flag), comm))


def _commit_rank_chunks(args, ordered: List[TensorInfo], writer: Optional["ChunkWriter"], rank: int, world: int,
                        failed: int, comm: torch.device, logger) -> int:
    """Per-rank chunk files -> the reference layout: global chunk numbers in rank order,
    metadata.json (rank 0) whose tensor_to_chunk lists every tensor in processing order.
    Loading the chunks through metadata.json gives exactly the single-process result dicts
    (tests/test_dist_output.py)."""
    import torch.distributed as dist
    st = args.save_safetensors
    mine = {"failed": failed, "t2c": dict(writer.t2c) if writer and not failed else {},
            "n_chunks": writer.n_chunks if writer and not failed else 0,
            "qparams": writer.qparams if writer and not failed else None}
    infos = [None] * world
    dist.all_gather_object(infos, mine)
    n_own = mine["n_chunks"]
    if any(i["failed"] for i in infos):
        tmp = _rank_stem(rank).split("{")[0]        # every chunk this rank wrote, whatever its state
        for f in os.listdir(args.output_dir):
            if f.startswith(tmp):
                try:
                    os.remove(os.path.join(args.output_dir, f))
                except OSError:
                    pass
        if rank == 0:
            logger.error("A rank failed; no output was published")
        return 1
    offs = [0] * world
    for r in range(1, world):
        offs[r] = offs[r - 1] + infos[r - 1]["n_chunks"]
    bad = 0
    renamed = []
    try:
        for c in range(n_own):
            dst = _chunk_path(args.output_dir, offs[rank] + c, st)
            os.replace(_chunk_path(args.output_dir, c, st, _rank_stem(rank)), dst)
            renamed.append(dst)
    except OSError as e:
        logger.error(f"rank {rank}: renaming chunk files failed: {e}")
        bad = 1
    rc = _agree(bad, comm)
    if rank == 0 and rc == 0:
        t2c = {}
        for info in ordered:           # processing order = bytes descending (main.py:259)
            for r, i in enumerate(infos):
                if info.name in i["t2c"]:
                    t2c[info.name] = offs[r] + i["t2c"][info.name]
                    break
        total = offs[-1] + infos[-1]["n_chunks"]
        if not t2c:
            logger.error("No tensors were successfully quantized")
            rc = 1
        else:
            qparams = next(i["qparams"] for i in infos if i["qparams"] is not None)
            try:
                _write_metadata(args.output_dir, total, args.chunk_size, t2c, st, len(t2c), qparams, logger)
                logger.info(f"Successfully quantized {len(t2c)} tensors on {world} GPUs; {total} chunk files "
                            f"written by their ranks")
            except OSError as e:
                logger.error(f"Failed to save quantized model: {e}")
                rc = 1
    rc = _agree(rc, comm)
    if rc:      # nothing is published: every rank removes the chunk files it wrote
        tmp = _rank_stem(rank).split("{")[0]
        leftovers = renamed + [os.path.join(args.output_dir, f) for f in os.listdir(args.output_dir)
                               if f.startswith(tmp)]
        for f in leftovers:
            try:
                os.remove(f)
            except OSError:
                pass
    return rc


def _commit_rank_autoawq(args, loader, ordered: List[TensorInfo], mine: List[TensorInfo],
                         results: Dict[str, Dict[str, torch.Tensor]], passthrough: List[TensorInfo], rank: int,
                         world: int, failed: int, comm: torch.device, logger) -> int:
    """AutoAWQ checkpoint written by its ranks: rank r writes its quantized linears (and its
    linears that failed, unquantized) as one safetensors shard, rank 0 adds the passthrough
    tensors, and rank 0 writes model.safetensors.index.json (the transformers sharded-
    checkpoint index) plus the configs.  One rank with tensors writes model.safetensors."""
    import torch.distributed as dist
    from safetensors.torch import save_file
    not_quant = [i for i in mine if i.name not in results]
    has = bool(results or not_quant or (rank == 0 and passthrough))
    flags = [None] * world
    dist.all_gather_object(flags, {"failed": failed, "has": has, "n_ok": len(results)})
    if any(f["failed"] for f in flags):
        if rank == 0:
            logger.error("A rank failed; no output was published")
        return 1
    if sum(f["n_ok"] for f in flags) == 0:
        if rank == 0:
            logger.error("No tensors were successfully quantized")
        return 1
    writers = [r for r in range(world) if flags[r]["has"]]
    fname = ("model.safetensors" if len(writers) == 1 else
             f"model-{writers.index(rank) + 1:05d}-of-{len(writers):05d}.safetensors") if has else None
    keys, size, bad = [], 0, 0
    if has:
        try:
            tensors = autoawq_tensors(results, loader, passthrough if rank == 0 else [], not_quant)
            save_file(tensors, os.path.join(args.output_dir, fname), metadata={"format": "pt"})
            keys = list(tensors)
            size = sum(t.numel() * t.element_size() for t in tensors.values())
        except Exception as e:  # noqa: BLE001
            logger.error(f"rank {rank}: writing {fname} failed: {e}")
            bad = 1
    shards = [None] * world
    dist.all_gather_object(shards, {"file": fname, "keys": keys, "size": size, "bad": bad,
                                    "not_converted": [i.name[: -len(".weight")] for i in not_quant]})

    def unpublish():   # nothing is published: every rank removes the shard it wrote
        if fname and os.path.exists(os.path.join(args.output_dir, fname)):
            try:
                os.remove(os.path.join(args.output_dir, fname))
            except OSError:
                pass
    if any(s["bad"] for s in shards):
        unpublish()
        return 1
    rc = 0
    if rank == 0:
        try:
            if len(writers) > 1:
                wmap = {k: s["file"] for s in shards for k in s["keys"]}
                index = {"metadata": {"total_size": sum(s["size"] for s in shards)},
                         "weight_map": {k: wmap[k] for k in sorted(wmap)}}
                with open(os.path.join(args.output_dir, "model.safetensors.index.json"), "w") as f:
                    json.dump(index, f, indent=2)
            order = {i.name[: -len(".weight")]: k for k, i in enumerate(ordered)}
            nc = sorted((m for s in shards for m in s["not_converted"]), key=lambda m: order.get(m, 0))
            write_autoawq_configs(args.output_dir, args, loader, nc, logger)
            logger.info(f"Saved AutoAWQ checkpoint from {world} ranks: {sum(f['n_ok'] for f in flags)} quantized "
                        f"linear weights in {len(writers)} shard file(s)")
        except Exception as e:  # noqa: BLE001
            logger.error(f"Failed to save quantized model: {e}")
            rc = 1
    rc = _agree(rc, comm)
    if rc:
        unpublish()
    return rc


def _gather_and_write(args, loader, ordered: List[TensorInfo], results: Dict[str, Dict[str, torch.Tensor]],
                      passthrough: List[TensorInfo], rank: int, world: int, failed: int, comm: torch.device,
                      logger) -> int:
    """--dist_output gather: the packed results of every rank go to rank 0 in one batched
    point-to-point round (distributed.gather_to_rank0), rank 0 writes the single-process
    layout."""
    import torch.distributed as dist
    from . import distributed as D
    autoawq = args.output_format == "autoawq"
    # which tensors succeeded, and the shapes rank 0 must receive (tiny metadata)
    meta = {n: {f: (tuple(t.shape), str(t.dtype)) for f, t in r.items() if f not in _SCALARS}
            for n, r in results.items()}
    all_meta = [None] * world
    dist.all_gather_object(all_meta, {"failed": failed, "meta": meta})
    if any(m["failed"] for m in all_meta):
        if rank == 0:
            logger.error("A rank failed; no output was published")
        return 1
    ok_owner, shapes = {}, {}
    for r, m in enumerate(all_meta):
        for n, fields in m["meta"].items():
            ok_owner[n] = r
            shapes[n] = {f: (shp, getattr(torch, dt.split(".")[-1])) for f, (shp, dt) in fields.items()}
    payload = {n: {f: t.to(comm) for f, t in r.items() if f not in _SCALARS} for n, r in results.items()}
    merged = D.gather_to_rank0(payload, ok_owner, shapes, comm)
    rc = 0
    if rank == 0:
        scal = {"bits": torch.tensor(args.bits, dtype=torch.int32),
                "group_size": torch.tensor(args.group_size, dtype=torch.int32),
                "symmetric": torch.tensor(args.symmetric, dtype=torch.bool)}
        quantized = {}
        for info in ordered:
            if info.name in merged:
                d = _to_cpu(merged[info.name])
                if not autoawq:
                    d.update(scal)
                if args.output_format == "packed":
                    d["shape"] = torch.tensor(list(info.shape), dtype=torch.int64)
                quantized[info.name] = d
        if not quantized:
            logger.error("No tensors were successfully quantized")
            rc = 1
        else:
            logger.info(f"Successfully quantized {len(quantized)} tensors on {world} GPUs")
            try:
                if autoawq:
                    save_autoawq(quantized, loader, passthrough, args.output_dir, args, logger,
                                 failed=[i for i in ordered if i.name not in quantized])
                else:
                    save_model_in_chunks(quantized, args.output_dir, chunk_size=args.chunk_size,
                                         use_safetensors=args.save_safetensors, logger=logger)
            except Exception as e:  # noqa: BLE001
                logger.error(f"Failed to save quantized model: {e}")
                rc = 1
    return _agree(rc, comm)


if __name__ == "__main__":
    sys.exit(main())
