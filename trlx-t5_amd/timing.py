"""Launch timers for the device-resident hot paths: HIP events created with
`hipEventDisableSystemFence` (hip_runtime_api.h).

A default event (torch.cuda.Event) performs a system-scope release when it is recorded —
an L2 write-back + invalidate on MI355X — so an event placed between two launches slows
the launch after it and charges that to the measurement (measured on the C2 step: the
experience launch reads 5-10 % slower right after an event than inside an uninstrumented
step).  Timing-only events skip that fence; they are recorded on the stream the kernels
are launched on, like torch's, and read back after the timed region has been synchronised.
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime this module binds)

_HIP_EVENT_DISABLE_TIMING = 0x2
_HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000
_hip = None


def _runtime():
    global _hip
    if _hip is None:
        lib = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)  # the runtime torch already loaded
        lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        lib.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        lib.hipEventDestroy.argtypes = [ctypes.c_void_p]
        lib.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        for f in ("hipEventCreateWithFlags", "hipEventRecord", "hipEventElapsedTime", "hipEventSynchronize",
                  "hipEventDestroy", "hipStreamWaitEvent"):
            getattr(lib, f).restype = ctypes.c_int
        _hip = lib
    return _hip


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def make_event():
    """A timing event: fence-free HIP event by default; TRLX_TIMING_EVENTS=torch selects
    torch.cuda.Event (default HIP event flags) for A/B comparisons."""
    if os.environ.get("TRLX_TIMING_EVENTS") == "torch":
        return torch.cuda.Event(enable_timing=True)
    return LaunchEvent()


class LaunchEvent:
    """A timing-only HIP event (no system-scope fence on record)."""

    __slots__ = ("_ev",)

    def __init__(self, timing: bool = True):
        """timing=False: an ordering-only event (hipEventDisableTiming; no timestamp write)."""
        ev = ctypes.c_void_p()
        flags = _HIP_EVENT_DISABLE_SYSTEM_FENCE | (0 if timing else _HIP_EVENT_DISABLE_TIMING)
        _check(_runtime().hipEventCreateWithFlags(ctypes.byref(ev), flags), "hipEventCreateWithFlags")
        self._ev = ev

    @property
    def handle(self):
        """The raw hipEvent_t (for C-ABI entry points that record it with a launch)."""
        return self._ev.value

    def record(self, stream):
        """stream: a torch.cuda.Stream (its raw hipStream_t is used)."""
        _check(_runtime().hipEventRecord(self._ev, ctypes.c_void_p(stream.cuda_stream)), "hipEventRecord")

    def wait(self, stream):
        """Make `stream` wait for this event (cross-stream ordering on one device; the kernels'
        own dispatch acquire / end-of-kernel release make the data visible)."""
        _check(_runtime().hipStreamWaitEvent(ctypes.c_void_p(stream.cuda_stream), self._ev, 0), "hipStreamWaitEvent")

    def synchronize(self):
        """Block the host until the work recorded before this event has finished."""
        _check(_runtime().hipEventSynchronize(self._ev), "hipEventSynchronize")

    def elapsed_time(self, end: "LaunchEvent") -> float:
        """Milliseconds between this event and `end` (waits for `end`)."""
        rt = _runtime()
        _check(rt.hipEventSynchronize(end._ev), "hipEventSynchronize")
        ms = ctypes.c_float()
        _check(rt.hipEventElapsedTime(ctypes.byref(ms), self._ev, end._ev), "hipEventElapsedTime")
        return float(ms.value)

    def __del__(self):
        if _hip is not None and self._ev:
            _hip.hipEventDestroy(self._ev)
