"""Console entry point `awq_quantizer` (pyproject [project.scripts]; the reference's points at
awq_quantizer.main:main, which this calls): the device warm-up starts before the CLI module
imports torch, as it does for `python -m awq_quantizer.main` (see _early.py)."""
import sys


def run() -> None:
    from . import _early
    _early.start(sys.argv[1:])
    from .main import main
    sys.exit(main())
