"""Structured logging: stdlib ``logging`` with an optional JSON-lines formatter.

``FDX_LOG_JSON=1`` switches every framework logger to one JSON object per record (ts, level,
logger, msg, rank + any ``extra`` fields), suitable for log shipping; otherwise a compact human
format. ``FDX_LOG_LEVEL`` sets the level (default INFO).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time

_configured = False


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {"ts": time.time(), "level": record.levelname, "logger": record.name, "msg": record.getMessage(),
             "rank": int(os.environ.get("RANK", "0"))}
        for k, v in record.__dict__.items():
            if k.startswith("fdx_"):
                d[k[4:]] = v
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d, default=str)


def _configure() -> None:
    global _configured
    if _configured:
        return
    _configured = True
    root = logging.getLogger("fdx")
    root.setLevel(os.environ.get("FDX_LOG_LEVEL", "INFO").upper())
    h = logging.StreamHandler(sys.stderr)
    if os.environ.get("FDX_LOG_JSON") == "1":
        h.setFormatter(JsonFormatter())
    else:
        h.setFormatter(logging.Formatter("[%(asctime)s %(levelname)s %(name)s] %(message)s", "%H:%M:%S"))
    root.addHandler(h)
    root.propagate = False


def get_logger(name: str) -> logging.Logger:
    _configure()
    return logging.getLogger(f"fdx.{name}")
