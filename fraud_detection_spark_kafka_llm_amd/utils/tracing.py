"""Tracing spans.

``span(name)`` marks a region with a ROCm ``roctx`` range when the roctx library is loadable (so
rocprofv3 ``--marker-trace`` shows the framework phases next to the kernels) and, when
``FDX_TRACE=<path>`` is set, appends one JSON line per span with wall-clock start/duration.
Spans nest. When neither sink is active ``span`` returns a shared no-op context manager: the
trainers open several spans per tree level, and a generator-based context manager cost ~5 us
each on the host thread that drives the RF lanes.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time

_roctx = None
_trace_path = os.environ.get("FDX_TRACE")
_sync = os.environ.get("FDX_TRACE_SYNC") == "1"   # synchronise the device at span exit (attribution)
_lock = threading.Lock()
_depth = threading.local()


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx
    _roctx = False
    if os.environ.get("FDX_ROCTX", "1") == "0":
        return _roctx
    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so", "librocprofiler-sdk-roctx.so",
                 "/opt/rocm/lib/librocprofiler-sdk-roctx.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


def enable(path: str) -> None:
    global _trace_path
    _trace_path = path


class _NullSpan:
    __slots__ = ()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NULL = _NullSpan()
_ROCTX_ON = os.environ.get("FDX_ROCTX") == "1"


def refresh() -> None:
    """Re-read FDX_ROCTX / FDX_TRACE (tests toggle them at run time)."""
    global _ROCTX_ON, _trace_path
    _ROCTX_ON = os.environ.get("FDX_ROCTX") == "1"
    _trace_path = os.environ.get("FDX_TRACE", _trace_path)


def span(name: str, **attrs):
    if not (_trace_path or _ROCTX_ON):
        return _NULL
    return _span(name, **attrs)


@contextlib.contextmanager
def _span(name: str, **attrs):
    rt = _load_roctx() if _ROCTX_ON else None
    if rt:
        rt.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    d = getattr(_depth, "v", 0)
    _depth.v = d + 1
    try:
        yield
    finally:
        if _sync and _trace_path:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()
        _depth.v = d
        dt = time.perf_counter() - t0
        if rt:
            rt.roctxRangePop()
        if _trace_path:
            rec = {"name": name, "t": t0, "dur_ms": dt * 1e3, "depth": d, "pid": os.getpid(), **attrs}
            with _lock, open(_trace_path, "a") as fh:
                fh.write(json.dumps(rec) + "\n")
