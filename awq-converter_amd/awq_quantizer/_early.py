"""HIP's first-use work started before `import torch` (no torch import here).

`python -m awq_quantizer.main` spends ~1.5 s importing torch before main() runs, and the
first GPU work of a process then pays ~0.1 s more for the device's first hardware queue,
first large copy and the quantize kernels' code object (scripts/init_probe.py,
profiles/round4/r4e/, r4f/).  main.py calls start(argv) at the top of the module when it
is the program, so awq_runtime_warmup (include/awq_hip.h) runs on a native thread while
the interpreter imports torch.

The HIP runtime it initialises is torch's own: torch ships libamdhip64.so (soname
libamdhip64.so.7) and loads it when imported; loading that same file first by path makes
every later NEEDED libamdhip64.so.7 — torch's and libawq_hip.so's — resolve to it, as it
would have without this module.  Anything unusual (no torch HIP runtime, a multi-device
or torchrun run, an unparsable --device, an ABI mismatch) and start() does nothing: the
pipeline then warms the device itself when it starts.
"""
import atexit
import ctypes
import importlib.util
import os
from typing import List, Optional

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libawq_hip.so")
ABI_VERSION = 17          # include/awq_hip.h AWQ_HIP_ABI_VERSION

_started: Optional[int] = None


def device_index(argv: List[str]) -> Optional[int]:
    """The one GPU the CLI will use, from its arguments alone (None: not exactly one known
    device — CPU, --multi_gpu / all, torchrun, or an option this parser does not read)."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return None
    dev = "cuda"
    it = iter(argv)
    for tok in it:
        if tok == "--multi_gpu":
            return None
        if tok == "--device":
            dev = next(it, "")
        elif tok.startswith("--device="):
            dev = tok.split("=", 1)[1]
        elif tok.startswith("--dev") or tok.startswith("--multi"):
            return None           # an abbreviation argparse would accept: do not guess
    dev = dev.lower()
    if dev == "cuda":
        return 0                  # the current device of a fresh process
    if dev.startswith("cuda:") and dev[5:].isdigit():
        return int(dev[5:])
    return None


def start(argv: List[str]) -> Optional[int]:
    """Start the warm-up for the CLI's device; returns its index, or None if not started."""
    global _started
    idx = device_index(argv)
    if idx is None or _started is not None:
        return None
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return None
    hip = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if not (os.path.exists(hip) and os.path.exists(LIB_PATH)):
        return None
    try:
        ctypes.CDLL(hip)                     # torch's HIP runtime, the one torch will use
        lib = ctypes.CDLL(LIB_PATH)
        lib.awq_abi_version.restype = ctypes.c_int
        if lib.awq_abi_version() != ABI_VERSION:
            return None
        lib.awq_runtime_warmup.argtypes = [ctypes.c_int]
        lib.awq_runtime_warmup_wait.argtypes = [ctypes.c_int, ctypes.c_void_p]
        if lib.awq_runtime_warmup(idx) != 0:
            return None
    except (OSError, AttributeError):
        return None
    atexit.register(lib.awq_runtime_warmup_wait, idx, None)
    _started = idx
    return idx
