"""
AWQ Quantizer package — MI355X (gfx950) build.

Drop-in for shanefitch/AWQ-Converter's `awq_quantizer` (same import paths, CLI and
AWQQuantizer API); the quantization arithmetic runs in hand-written HIP kernels
(awq-converter_amd/csrc, C ABI in include/awq_hip.h).
"""

__version__ = "0.1.0"
