"""Logging with the reference's log4j line format.

``log4j.properties:2-8``: root logger INFO -> stdout console appender with pattern
``%d{yyyy-MM-dd HH:mm:ss} %-5p %c{1} - %m%n``.  Same format here (``%c{1}`` = last
component of the logger name, WARNING printed as ``WARN``).  Under data
parallelism the logger name carries the rank (``Main[r3]``) and ranks other than
0 only emit WARN and above.
"""
from __future__ import annotations

import json
import logging
import os
import sys

FORMAT = "%(asctime)s %(levelname)-5s %(shortname)s - %(message)s"
DATEFMT = "%Y-%m-%d %H:%M:%S"
_LEVEL_NAMES = {"WARNING": "WARN", "CRITICAL": "FATAL"}
_configured = False


class Log4jFormatter(logging.Formatter):
    def format(self, record):
        record.levelname = _LEVEL_NAMES.get(record.levelname, record.levelname)
        record.shortname = record.name.rsplit(".", 1)[-1]
        return super().format(record)


def setup(level: str = "INFO", rank: int | None = None, stream=None) -> None:
    global _configured
    root = logging.getLogger("euromillioner")
    for h in list(root.handlers):
        root.removeHandler(h)
    h = logging.StreamHandler(stream or sys.stdout)
    h.setFormatter(Log4jFormatter(FORMAT, DATEFMT))
    root.addHandler(h)
    lvl = getattr(logging, level.upper(), logging.INFO)
    if rank not in (None, 0) and lvl < logging.WARNING:
        lvl = logging.WARNING
    root.setLevel(lvl)
    root.propagate = False
    _configured = True


def get(name: str = "Main") -> logging.Logger:
    if not _configured:
        setup(os.environ.get("EUROM_LOG__LEVEL", "INFO"))
    rank = os.environ.get("RANK")
    multi = int(os.environ.get("WORLD_SIZE", "1")) > 1
    suffix = f"[r{rank}]" if multi and rank is not None else ""
    return logging.getLogger(f"euromillioner.{name}{suffix}")


def metrics_line(payload: dict, stream=None) -> None:
    """One machine-readable JSON line (the reference only prints a boolean, Main.java:143)."""
    out = stream or sys.stdout
    out.write(json.dumps(payload, default=float) + "\n")
    out.flush()
