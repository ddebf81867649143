"""Logging helpers with the reference's interface and line format
(reference src/awq_quantizer/utils/logger.py:11-104: stdout handler, optional file
handler, "%(asctime)s - %(name)s - %(levelname)s - %(message)s")."""
import logging
import os
import sys
from typing import Optional

FORMAT = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"


class Logger:
    """Thin wrapper over a stdlib logger (handlers are reset on construction)."""

    def __init__(self, name: str = "awq_quantizer", level: str = "INFO", to_file: bool = False,
                 file_path: Optional[str] = None):
        lvl = getattr(logging, level.upper())
        self.logger = logging.getLogger(name)
        self.logger.setLevel(lvl)
        self.logger.propagate = False
        for h in list(self.logger.handlers):
            self.logger.removeHandler(h)
        handlers = [logging.StreamHandler(sys.stdout)]
        if to_file:
            path = file_path or "quantization.log"
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            handlers.append(logging.FileHandler(path))
        for h in handlers:
            h.setLevel(lvl)
            h.setFormatter(logging.Formatter(FORMAT))
            self.logger.addHandler(h)

    @property
    def level(self) -> int:
        return self.logger.level

    def debug(self, msg: str):
        self.logger.debug(msg)

    def info(self, msg: str):
        self.logger.info(msg)

    def warning(self, msg: str):
        self.logger.warning(msg)

    def error(self, msg: str):
        self.logger.error(msg)

    def critical(self, msg: str):
        self.logger.critical(msg)


def get_logger(name: str = "awq_quantizer", level: str = "INFO", to_file: bool = False,
               file_path: Optional[str] = None) -> Logger:
    return Logger(name=name, level=level, to_file=to_file, file_path=file_path)
