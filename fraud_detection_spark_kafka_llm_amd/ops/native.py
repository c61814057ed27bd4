"""Loader for the in-tree native core ``_C.so`` (gfx950 kernels + host C++).

The extension is required: every hot op dispatches into it, on the GPU (HIP kernels) and on the
CPU (host C++). If the shared object is missing it is built in place with ``hipcc`` (the build is
incremental and takes ~20 s from scratch). There is deliberately no silent PyTorch fallback: a
GPU process that cannot load the native core raises.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch  # noqa: F401  (loads the HIP runtime the extension links against)

_lock = threading.Lock()
_mod = None


def lib():
    """Return the loaded ``_C`` module, building it first if needed."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            _mod = importlib.import_module("fraud_detection_spark_kafka_llm_amd._C")
        except ImportError as first:
            if os.environ.get("FDX_NO_AUTOBUILD"):
                raise ImportError(f"native core _C.so not built ({first}); run "
                                  "`python -m fraud_detection_spark_kafka_llm_amd._build`") from first
            from .. import _build

            _build.build()
            _mod = importlib.import_module("fraud_detection_spark_kafka_llm_amd._C")
    return _mod


def so_path() -> str:
    return lib().__file__


def default_device() -> torch.device:
    """``cuda:<LOCAL_RANK>`` when a GPU is visible, else CPU."""
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    return torch.device("cpu")
