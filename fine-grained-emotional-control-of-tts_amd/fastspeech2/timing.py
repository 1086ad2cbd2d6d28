"""HIP-event timing of tagged kernel launches on the launching (current) stream.

The events are created with ``hipEventDisableSystemFence``: a default (torch) timing event
records with a system-scope release, i.e. an L2 write-back and invalidate between the two
kernels it separates, which measured ~6 us of idle GPU on each side of every bracketed launch
(24 brackets per bench step ~ 0.3 ms).  Timing-only events need no such fence
(hip_runtime_api.h: "can be used for events that are only being used to measure timing").
FS2_TIMER_EVENTS=torch restores torch.cuda.Event for A/B runs."""

import ctypes
import os

import torch

_HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000
_hip = None


def _lib():
    global _hip
    if _hip is None:
        lib = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
        lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                            ctypes.c_void_p]
        lib.hipEventDestroy.argtypes = [ctypes.c_void_p]
        _hip = lib
    return _hip


class _NoFenceEvent:
    """A timing-only HIP event recorded without the system-scope release."""

    __slots__ = ("h",)

    def __init__(self):
        h = ctypes.c_void_p()
        if _lib().hipEventCreateWithFlags(ctypes.byref(h), _HIP_EVENT_DISABLE_SYSTEM_FENCE):
            raise RuntimeError("hipEventCreateWithFlags failed")
        self.h = h

    def record(self, stream):
        if _lib().hipEventRecord(self.h, ctypes.c_void_p(stream.cuda_stream)):
            raise RuntimeError("hipEventRecord failed")

    def elapsed_time(self, end):
        ms = ctypes.c_float()
        if _lib().hipEventElapsedTime(ctypes.byref(ms), self.h, end.h):
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    def __del__(self):
        if _hip is not None and self.h:
            _hip.hipEventDestroy(self.h)


class KernelTimer:
    def __init__(self):
        self.pending = {}
        self.pairs = {}
        self.torch_events = os.environ.get("FS2_TIMER_EVENTS", "nofence") == "torch"

    def _event(self):
        if self.torch_events:
            return torch.cuda.Event(enable_timing=True)
        return _NoFenceEvent()

    def start(self, tag):
        e = self._event()
        e.record(torch.cuda.current_stream())
        self.pending[tag] = e

    def stop(self, tag):
        e = self._event()
        e.record(torch.cuda.current_stream())
        self.pairs.setdefault(tag, []).append((self.pending.pop(tag), e))

    def reset(self):
        self.pending, self.pairs = {}, {}

    def summary(self):
        """tag -> (launches, mean ms); call after a synchronize."""
        out = {}
        for tag, prs in self.pairs.items():
            ts = [a.elapsed_time(b) for a, b in prs]
            out[tag] = (len(ts), sum(ts) / len(ts))
        return out
