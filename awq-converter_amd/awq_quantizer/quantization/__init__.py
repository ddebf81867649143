"""
Quantization package.
"""

from .awq import AWQQuantizer

__all__ = ["AWQQuantizer"]
