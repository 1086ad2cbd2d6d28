"""Cross-stream ordering for the train step's three streams without a system-scope fence.

``torch.cuda.Stream.wait_stream`` records a freshly created event on the producer stream.  A
default HIP event records with a system-scope release (a full L2 write-back so that the HOST
could observe the memory), and the producer's queue idles behind it: measured ~6-8 us of idle
main-stream GPU per fork, ~75 forks a step (the weight-gradient side stream forks off the main
stream before each weight gradient).  The streams here are all on one device, where the
agent-scope release every kernel already ends with makes its writes visible to the consumer
stream's kernels; so the links use pooled events created with hipEventDisableTiming |
hipEventDisableSystemFence.  ``hipStreamWaitEvent`` binds the consumer to the record made just
before it, so an event can be recorded again later without affecting earlier waits; the pool is
a ring anyway.  While a stream is being captured into a HIP graph the torch path is used (its
events become graph dependencies)."""

import ctypes

import torch

_HIP_EVENT_DISABLE_TIMING = 0x2
_HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000
_RING = 64

_hip = None
_ring = []
_pos = 0


def _lib():
    global _hip
    if _hip is None:
        lib = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
        lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        _hip = lib
    return _hip


def _event():
    global _pos
    if not _ring:
        lib = _lib()
        for _ in range(_RING):
            h = ctypes.c_void_p()
            if lib.hipEventCreateWithFlags(ctypes.byref(h), _HIP_EVENT_DISABLE_TIMING |
                                           _HIP_EVENT_DISABLE_SYSTEM_FENCE):
                raise RuntimeError("hipEventCreateWithFlags failed")
            _ring.append(h)
    e = _ring[_pos]
    _pos = (_pos + 1) % _RING
    return e


def wait(consumer, producer):
    """``consumer`` (a torch.cuda.Stream) runs its later work after everything queued so far on
    ``producer`` -- torch's ``consumer.wait_stream(producer)`` without the system fence."""
    if torch.cuda.is_current_stream_capturing():
        consumer.wait_stream(producer)
        return
    lib = _lib()
    e = _event()
    if lib.hipEventRecord(e, ctypes.c_void_p(producer.cuda_stream)):
        raise RuntimeError("hipEventRecord failed")
    if lib.hipStreamWaitEvent(ctypes.c_void_p(consumer.cuda_stream), e, 0):
        raise RuntimeError("hipStreamWaitEvent failed")


class Mark:
    """A fence-free event of its own (not from the ring): recorded on one stream now, waited
    on by another later in the step."""

    def __init__(self):
        h = ctypes.c_void_p()
        if _lib().hipEventCreateWithFlags(ctypes.byref(h), _HIP_EVENT_DISABLE_TIMING |
                                          _HIP_EVENT_DISABLE_SYSTEM_FENCE):
            raise RuntimeError("hipEventCreateWithFlags failed")
        self.h = h

    def record(self, stream):
        if _lib().hipEventRecord(self.h, ctypes.c_void_p(stream.cuda_stream)):
            raise RuntimeError("hipEventRecord failed")

    def wait(self, stream):
        if _lib().hipStreamWaitEvent(ctypes.c_void_p(stream.cuda_stream), self.h, 0):
            raise RuntimeError("hipStreamWaitEvent failed")
