"""Cheap HIP stream switching for the host threads that drive many streams.

``torch.cuda.stream(s)`` (StreamContext) looks the device up, builds Stream objects for the current
streams and goes through ``torch.cuda.set_stream`` on enter and exit: ~15-20 us of host time per
switch. The forest driver (models/forest_batch.py) switches streams at every step of every tree in
flight, and at a 1.25M-row data-parallel shard the host thread, not the GPU, is the critical path
(``bench/probes/rf_host_probe.py --forced``: ~5 % of the wall blocked on the device). A
:class:`StreamSwitch` is built once per stream and switches with torch's two low-level calls.
"""
from __future__ import annotations

import torch


class StreamSwitch:
    """Reusable context manager: make ``stream`` current (no-op for None), restore on exit."""

    __slots__ = ("sid", "didx", "dtype", "prev", "prev_dev")

    def __init__(self, stream):
        if stream is None:
            self.sid = None
        else:
            self.sid, self.didx, self.dtype = stream.stream_id, stream.device_index, stream.device_type

    def __enter__(self):
        if self.sid is not None:
            # (_cuda_setStream also makes the stream's device current: restored on exit)
            self.prev_dev = torch._C._cuda_getDevice()
            self.prev = torch._C._cuda_getCurrentStream(self.didx)
            torch._C._cuda_setStream(stream_id=self.sid, device_index=self.didx, device_type=self.dtype)
        return self

    def __exit__(self, *exc):
        if self.sid is not None:
            p = self.prev
            torch._C._cuda_setStream(stream_id=p[0], device_index=p[1], device_type=p[2])
            if self.prev_dev != self.didx:
                torch._C._cuda_setDevice(self.prev_dev)
        return False


NULL_SWITCH = StreamSwitch(None)
