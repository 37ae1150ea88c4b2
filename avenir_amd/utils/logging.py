"""Structured, per-rank logging.

* ``get_logger(name)`` — stdlib logger; with ``AVENIR_LOG_JSON=1`` records are emitted as JSON
  lines tagged with the rank, otherwise ``asctime - name - levelname - message`` like the
  reference's ``createLogger`` (``python/lib/util.py:978-1003``).
* ``create_logger(name, log_file, level)`` — the reference helper: a RotatingFileHandler of
  1 MB x 4 backups.
* ``debug.on`` in a job config raises the job logger to DEBUG (the Java jobs' idiom, e.g.
  ``J/tree/DecisionTreeBuilder.java:139-142``).
"""
from __future__ import annotations

import json
import logging
import logging.handlers
import os
import sys
import time

_FMT = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"


class _JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": round(time.time(), 3), "rank": int(os.environ.get("RANK", "0")),
             "name": record.name, "level": record.levelname, "msg": record.getMessage()}
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d)


_configured: set[str] = set()


def get_logger(name: str, level: int | str | None = None) -> logging.Logger:
    lg = logging.getLogger(f"avenir_amd.{name}")
    if name not in _configured:
        h = logging.StreamHandler(sys.stderr)
        if os.environ.get("AVENIR_LOG_JSON", "0") == "1":
            h.setFormatter(_JsonFormatter())
        else:
            h.setFormatter(logging.Formatter(_FMT))
        lg.addHandler(h)
        lg.propagate = False
        env_level = os.environ.get("AVENIR_LOG_LEVEL", "WARNING")
        lg.setLevel(level or env_level)
        _configured.add(name)
    elif level is not None:
        lg.setLevel(level)
    return lg


def create_logger(name: str, log_file: str | None = None, level: int | str = logging.INFO,
                  max_bytes: int = 1_000_000, backups: int = 4) -> logging.Logger:
    lg = logging.getLogger(name)
    lg.setLevel(level)
    if log_file:
        fh = logging.handlers.RotatingFileHandler(log_file, maxBytes=max_bytes, backupCount=backups)
        fh.setFormatter(logging.Formatter(_FMT))
        lg.addHandler(fh)
    return lg


createLogger = create_logger
