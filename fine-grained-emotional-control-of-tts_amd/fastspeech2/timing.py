"""HIP-event timing of tagged kernel launches on the launching (current) stream.

The events are created with ``hipEventDisableSystemFence``: a default (torch) timing event
records with a system-scope release, i.e. an L2 write-back and invalidate between the two
kernels it separates, which measured ~6 us of idle GPU on each side of every bracketed launch
(24 brackets per bench step ~ 0.3 ms).  Timing-only events need no such fence
(hip_runtime_api.h: "can be used for events that are only being used to measure timing").
FS2_TIMER_EVENTS=torch restores torch.cuda.Event for A/B runs.

Events are pooled: creating a HIP event costs far more host time than recording one (the
bench's 40 brackets a step added ~4.6 ms of host enqueue time when each record created its
event), so ``reserve(n)`` creates them before a timed region and ``reset()`` returns recorded
events to the pool once their times have been read."""

import ctypes
import os

import torch

from . import _native as N

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

    def record(self, stream_ptr):
        if _lib().hipEventRecord(self.h, ctypes.c_void_p(stream_ptr)):
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
        self.free = []
        self.torch_events = os.environ.get("FS2_TIMER_EVENTS", "nofence") == "torch"

    def _event(self):
        return self.free.pop() if self.free else self._event_new()

    def _record(self, e):
        if self.torch_events:
            e.record(torch.cuda.current_stream())
        else:
            e.record(N.stream_ptr())

    def start(self, tag):
        e = self._event()
        self._record(e)
        self.pending[tag] = e

    def stop(self, tag):
        e = self._event()
        self._record(e)
        self.pairs.setdefault(tag, []).append((self.pending.pop(tag), e))

    def n_events(self):
        return 2 * sum(len(p) for p in self.pairs.values()) + len(self.pending)

    def reserve(self, n):
        """create events until n are pooled (outside a timed region)"""
        while len(self.free) < n:
            self.free.append(self._event_new())

    def _event_new(self):
        return torch.cuda.Event(enable_timing=True) if self.torch_events else _NoFenceEvent()

    def reset(self):
        """drop the recorded pairs (after their times were read); their events are reused"""
        for prs in self.pairs.values():
            for a, b in prs:
                self.free += (a, b)
        self.free += list(self.pending.values())
        self.pending, self.pairs = {}, {}

    def summary(self):
        """tag -> (launches, mean ms); call after a synchronize."""
        out = {}
        for tag, prs in self.pairs.items():
            ts = [a.elapsed_time(b) for a, b in prs]
            out[tag] = (len(ts), sum(ts) / len(ts))
        return out
