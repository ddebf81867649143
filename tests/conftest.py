"""pytest setup: the `gpu` marker and import paths.

Layout: the drop-in package lives in awq-converter_amd/awq_quantizer (mirroring
the reference's src/awq_quantizer), the CPU oracle in oracle/ (test infra).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(ROOT, "awq-converter_amd")
for p in (ROOT, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # A/B of in-tree builds (scripts/cmd/*.sh): AWQ_TEST_LIB names another build of the
    # library for the whole session (test-only; the product never reads the environment)
    lib = os.environ.get("AWQ_TEST_LIB")
    if lib:
        from awq_quantizer import _hip
        _hip.load_library(os.path.join(ROOT, lib) if not os.path.isabs(lib) else lib)
