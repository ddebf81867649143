"""Safetensors loading for the quantizer's CLI — streaming, header-first.

Reference: src/awq_quantizer/model_loading/safetensors_loader.py:17-224, whose
load_tensors() reads every file whole into host RAM (safetensors load_file, :145-173)
before anything is quantized.  This loader keeps the same constructor, file discovery
and load_tensors() contract, and adds what the MI355X path needs:

  * tensor_index(): names / dtypes / shapes / sizes from the file headers only;
  * read(name): one tensor at a time (memory-mapped slice of its file), so the CLI can
    stream weights host -> HBM while the previous tensor is being quantized;
  * read_pinned(name): the same bytes read straight from the file into page-locked host
    memory (one pread per tensor at the offset the file header gives; the GIL is released
    during the read, so reader threads run in parallel), ready for an async H2D copy.
"""
import json
import os
import struct
import threading
from typing import Dict, Iterator, List, Optional, Tuple

import torch
from safetensors import safe_open

from ..utils.logger import get_logger
from ..utils.tensor_utils import convert_bf16_to_fp16, filter_consolidated_files, get_model_files, get_tensor_type

_DT = {"BF16": torch.bfloat16, "F16": torch.float16, "F32": torch.float32, "F64": torch.float64,
       "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
       "BOOL": torch.bool, "F8_E4M3": getattr(torch, "float8_e4m3fn", None),
       "F8_E5M2": getattr(torch, "float8_e5m2", None)}


class TensorInfo:
    __slots__ = ("name", "file", "dtype", "shape", "numel", "nbytes")

    def __init__(self, name, file, dtype, shape):
        self.name, self.file, self.dtype, self.shape = name, file, dtype, tuple(shape)
        n = 1
        for s in self.shape:
            n *= s
        self.numel = n
        self.nbytes = n * (torch.empty((), dtype=dtype).element_size() if dtype is not None else 1)


class SafetensorsLoader:
    def __init__(self, model_path: str, from_hub: bool = False, revision: str = "main",
                 token: Optional[str] = None, logger_name: str = "safetensors_loader",
                 logger_level: str = "INFO", logger_to_file: bool = False,
                 logger_file_path: Optional[str] = None, resume_download: bool = True,
                 force_download: bool = False):
        self.model_path = model_path
        self.from_hub = from_hub
        self.revision = revision
        self.token = token
        self.resume_download = resume_download
        self.force_download = force_download
        self.logger = get_logger(name=logger_name, level=logger_level, to_file=logger_to_file,
                                 file_path=logger_file_path)
        files = get_model_files(model_path)
        if not files:
            raise ValueError(f"No safetensor files found in {model_path}")
        self.model_files = filter_consolidated_files(files)
        self.logger.info(f"Loading {len(self.model_files)} safetensors files:")
        for f in self.model_files:
            self.logger.info(f"  - {os.path.basename(f)}")
        self.tensors: Dict[str, torch.Tensor] = {}
        self._index: Optional[List[TensorInfo]] = None
        self._handles = {}
        self._layouts: Dict[str, Tuple[int, Dict[str, Tuple[int, int]]]] = {}
        self._fds: Dict[str, int] = {}
        self._lock = threading.Lock()

    # ---- header-only index (file order, key order of safe_open) ----
    def tensor_index(self) -> List[TensorInfo]:
        if self._index is None:
            idx, seen = [], {}
            for path in self.model_files:
                with safe_open(path, framework="pt") as f:
                    for name in f.keys():
                        sl = f.get_slice(name)
                        info = TensorInfo(name, path, _DT.get(sl.get_dtype()), sl.get_shape())
                        if name in seen:
                            self.logger.warning(f"Duplicate tensor name: {name}")
                            idx[seen[name]] = info          # later file wins, position kept
                        else:
                            seen[name] = len(idx)
                            idx.append(info)
            self._index = idx
        return self._index

    def read(self, info: TensorInfo) -> torch.Tensor:
        """Read one tensor from its file (CPU tensor)."""
        key = (threading.get_ident(), info.file)      # one handle per reader thread and file
        h = self._handles.get(key)
        if h is None:
            h = safe_open(info.file, framework="pt")
            self._handles[key] = h
        return h.get_tensor(info.name)

    def _layout(self, path: str) -> Tuple[int, Dict[str, Tuple[int, int]]]:
        """(data start, name -> (begin, end) byte offsets) from a safetensors header:
        8-byte little-endian header length, JSON header, then the data block."""
        with self._lock:
            lay = self._layouts.get(path)
            if lay is None:
                with open(path, "rb") as f:
                    n = struct.unpack("<Q", f.read(8))[0]
                    hdr = json.loads(f.read(n))
                lay = (8 + n, {k: tuple(v["data_offsets"]) for k, v in hdr.items() if k != "__metadata__"})
                self._layouts[path] = lay
                self._fds[path] = os.open(path, os.O_RDONLY)
            return lay

    def data_location(self, info: TensorInfo) -> Tuple[int, int]:
        """(open file descriptor, absolute byte offset) of a tensor's data, for native
        readers (include/awq_hip.h awq_stream_*); the descriptor lives until close()."""
        start, offs = self._layout(info.file)
        return self._fds[info.file], start + offs[info.name][0]

    def read_pinned(self, info: TensorInfo) -> torch.Tensor:
        """Read one tensor into page-locked host memory."""
        if info.dtype is None:
            raise ValueError(f"{info.name}: unsupported dtype")
        return self.read_into(info, torch.empty(info.shape, dtype=info.dtype, pin_memory=True))

    def read_into(self, info: TensorInfo, out: torch.Tensor) -> torch.Tensor:
        """Read one tensor's bytes from its file into `out` (contiguous CPU tensor of the
        tensor's dtype and shape) with pread at the header's offsets."""
        start, offs = self._layout(info.file)
        begin, end = offs[info.name]
        nbytes = end - begin
        if not out.is_contiguous() or nbytes != out.numel() * out.element_size():
            raise ValueError(f"{info.name}: header size {nbytes} B does not match the destination "
                             f"{tuple(out.shape)} {out.dtype}")
        if nbytes:
            view = memoryview(out.view(-1).view(torch.uint8).numpy())
            fd, pos, done = self._fds[info.file], start + begin, 0
            while done < nbytes:
                got = os.preadv(fd, [view[done:]], pos + done)
                if got <= 0:
                    raise IOError(f"{info.name}: short read at byte {done} of {nbytes}")
                done += got
        return out

    def close(self) -> None:
        with self._lock:
            for fd in self._fds.values():
                os.close(fd)
            self._fds.clear()
            self._layouts.clear()

    def iter_tensors(self) -> Iterator[Tuple[str, torch.Tensor]]:
        for info in self.tensor_index():
            yield info.name, self.read(info)

    def verify_file(self, file_path: str) -> bool:
        try:
            with safe_open(file_path, framework="pt") as f:
                f.metadata()
                keys = list(f.keys())
                if keys:
                    f.get_slice(keys[0])
            return True
        except Exception as e:  # noqa: BLE001
            self.logger.warning(f"File verification failed for {file_path}: {e}")
            return False

    def load_tensors(self) -> Dict[str, torch.Tensor]:
        """Whole-model load (reference API, safetensors_loader.py:145-173)."""
        self.tensors = {}
        for name, t in self.iter_tensors():
            self.tensors[name] = t
        self.logger.info(f"Loaded {len(self.tensors)} total tensors")
        return self.tensors

    def save_tensors(self, tensors: Dict[str, torch.Tensor], output_dir: str,
                     filename: str = "model.safetensors") -> None:
        from safetensors.torch import save_file
        os.makedirs(output_dir, exist_ok=True)
        path = os.path.join(output_dir, filename)
        save_file(tensors, path)
        self.logger.info(f"Saved {len(tensors)} tensors to {path}")

    def convert_tensors_bf16_to_fp16(self, tensors: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """bf16 tensors of the dict as fp16 (RNE; out-of-range values become inf), others
        unchanged (reference safetensors_loader.py:205-225)."""
        out = {}
        for name, t in tensors.items():
            out[name] = convert_bf16_to_fp16(t)
            if out[name].dtype != t.dtype:
                self.logger.debug(f"Converted tensor {name} from {get_tensor_type(t)} to {get_tensor_type(out[name])}")
        return out
