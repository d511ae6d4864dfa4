"""Sensor filter policies.

Kernel side (reference chronos_sensor.py:74-92) lives in ``bpf/chronos_filters.h``; :func:`open_is_noise` here is a
pure-Python mirror used as the test oracle for the C++/BPF build of that header.  User-space lists are the
reference's ``ignore`` (comm substring, :134) and trigger keywords (event-string substring, :141).
"""
from __future__ import annotations

NOISE_PREFIXES = ("/lib", "/usr/lib", "/usr/share", "/etc/ssl", "/etc/fonts", "/etc/host", "/dev/", "/proc/")
NOISE_SUFFIXES = (".so", ".cache", ".mo", ".conf", ".crt", ".curlrc")
STRICT_PREFIXES = ("/etc/localtime",)
STRICT_SUFFIXES = ("curlrc",)

COMM_IGNORE = ("node", "code", "ollama", "python", "chrome", "vmtools", "git")
TRIGGERS = ("curl", "chmod", "bash", "nc", "cat")
MIN_CHAIN = 2

_PREFIX_SCAN = 20
_SUFFIX_SCAN = 10


def _c_prefix(path: bytes, prefix: bytes) -> bool:
    s = path + b"\0" * (_PREFIX_SCAN + 1)
    p = prefix[:_PREFIX_SCAN] + b"\0"
    for i in range(_PREFIX_SCAN):
        if p[i] == 0:
            return True
        if s[i] != p[i]:
            return False
    return True


def _c_suffix(path: bytes, suffix: bytes) -> bool:
    suf = suffix[:_SUFFIX_SCAN]
    return len(suf) <= len(path) and path.endswith(suf)


def open_is_noise(path: str | bytes, strict: bool = False) -> bool:
    """True when the kernel program would drop an OPEN of ``path`` (NUL-terminated semantics, 255-byte cap)."""
    b = path.encode() if isinstance(path, str) else path
    b = b[:255].split(b"\0", 1)[0]
    pre = NOISE_PREFIXES + (STRICT_PREFIXES if strict else ())
    suf = NOISE_SUFFIXES + (STRICT_SUFFIXES if strict else ())
    return any(_c_prefix(b, p.encode()) for p in pre) or any(_c_suffix(b, s.encode()) for s in suf)
