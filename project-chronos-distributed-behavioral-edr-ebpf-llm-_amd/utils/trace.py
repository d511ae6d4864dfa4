"""roctx ranges around scheduler phases.

``with trace.range("prefill"):`` pushes/pops a roctx range (``libroctx64.so`` through ctypes, no torch dependency),
so ``rocprofv3 --marker-trace --kernel-trace`` shows the engine's admit / prefill / decode-burst / harvest phases on
the same timeline as the HIP kernels they launch.  Off by default (one env lookup at import); enable with
``CHRONOS_ROCTX=1``.  A missing library leaves every range a no-op.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
ENABLED = os.environ.get("CHRONOS_ROCTX", "0") not in ("", "0")


def _load():
    global _lib, ENABLED
    if _lib is not None or not ENABLED:
        return _lib
    # rocprofv3 intercepts the rocprofiler-sdk roctx; the legacy roctracer library is the fallback
    for name in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "libroctx64.so",
                 "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            return lib
        except (OSError, AttributeError):
            continue
    ENABLED = False
    return None


def enable(on: bool = True) -> bool:
    """Turn ranges on/off at runtime; returns whether a roctx library is available."""
    global ENABLED
    ENABLED = on
    return _load() is not None if on else False


def push(name: str) -> None:
    if ENABLED and _load() is not None:
        _lib.roctxRangePushA(name.encode())


def pop() -> None:
    if ENABLED and _lib is not None:
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if ENABLED and _load() is not None:
        _lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001  (mirrors the roctx/nvtx API name)
    if not ENABLED:
        yield
        return
    push(name)
    try:
        yield
    finally:
        pop()
