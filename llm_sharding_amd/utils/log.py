"""Structured logging with the reference's message prefixes (the reference
prints ``[INFO]`` / ``[CONFIG]`` / ``[WARNING]`` / ``[ERROR]`` lines, e.g.
``/root/reference/utils/node_worker.py:115-185``).

``get_logger(name).info("...")`` prints ``[INFO] ...`` (unbuffered, like the reference's
``PYTHONUNBUFFERED=1`` runs). ``LSA_LOG_LEVEL`` filters (DEBUG/INFO/WARNING/ERROR);
``LSA_LOG_JSON=1`` switches to one JSON object per line with timestamp, rank and logger name,
for log collection across the per-GPU processes.
"""
from __future__ import annotations

import json
import os
import sys
import time

LEVELS = {"DEBUG": 10, "CONFIG": 20, "INFO": 20, "WARNING": 30, "ERROR": 40}


class Logger:
    def __init__(self, name: str = "lsa"):
        self.name = name

    @staticmethod
    def _threshold() -> int:
        return LEVELS.get(os.environ.get("LSA_LOG_LEVEL", "INFO").upper(), 20)

    def log(self, level: str, msg: str, **fields) -> None:
        if LEVELS.get(level, 20) < self._threshold():
            return
        if os.environ.get("LSA_LOG_JSON") == "1":
            rec = {"ts": time.time(), "level": level, "rank": int(os.environ.get("RANK", "0")), "logger": self.name,
                   "msg": msg, **fields}
            line = json.dumps(rec, default=str)
        else:
            extra = (" " + " ".join(f"{k}={v}" for k, v in fields.items())) if fields else ""
            line = f"[{level}] {msg}{extra}"
        stream = sys.stderr if level == "ERROR" else sys.stdout
        print(line, file=stream, flush=True)

    def debug(self, msg, **kw):
        self.log("DEBUG", msg, **kw)

    def info(self, msg, **kw):
        self.log("INFO", msg, **kw)

    def config(self, msg, **kw):
        self.log("CONFIG", msg, **kw)

    def warning(self, msg, **kw):
        self.log("WARNING", msg, **kw)

    def error(self, msg, **kw):
        self.log("ERROR", msg, **kw)


_LOGGERS: dict = {}


def get_logger(name: str = "lsa") -> Logger:
    if name not in _LOGGERS:
        _LOGGERS[name] = Logger(name)
    return _LOGGERS[name]


__all__ = ["get_logger", "Logger"]
