"""Importable alias for the framework package.

The framework lives in ``project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/`` at the repo root.  That
directory name is not a valid Python identifier, so this shim makes it importable as ``chronos``: every
``chronos.<sub>`` import is resolved inside that directory, and the real ``__init__.py`` runs in this namespace.
"""
import os as _os

PKG_DIR = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "project-chronos-distributed-behavioral-edr-ebpf-llm-_amd",
)
__path__ = [PKG_DIR]

_init = _os.path.join(PKG_DIR, "__init__.py")
with open(_init, "r", encoding="utf-8") as _f:
    exec(compile(_f.read(), _init, "exec"))
