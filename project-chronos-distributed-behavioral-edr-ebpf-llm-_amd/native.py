"""In-tree native build + loader for the framework's C++ / HIP libraries.

Three shared objects are built next to this file (never into site-packages, so they travel with the repo snapshot
to the GPU box and show up as in-tree loads):

  _sensor_native   g++      csrc/sensor_host/*.cpp      shared eBPF filter policy, data_t codec, chain tracker
  _constrain_native g++     csrc/constrain/*.cpp        JSON / verdict-schema token automaton compiler, tokenizer trie
  _C               hipcc    csrc/kernels/*.hip          gfx950 HIP kernels (MFMA/LDS) as torch ops

The HIP library is compiled with hipcc directly (``--offload-arch=gfx950``), not through torch's cpp_extension, so no
hipify pass ever touches the sources.  Rebuilds are keyed on a hash of sources + flags.
"""
from __future__ import annotations

import concurrent.futures as _cf
import glob
import hashlib
import importlib
import importlib.util
import os
import shutil
import subprocess
import sys
import sysconfig
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO_DIR, "csrc")
BUILD_DIR = os.path.join(REPO_DIR, "build", "native")
ARCH = os.environ.get("CHRONOS_GPU_ARCH", "gfx950")

_lock = threading.Lock()
_loaded: dict[str, object] = {}


def _py_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    return root, inc, os.path.join(root, "lib")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _hash(files: list[str], flags: list[str]) -> str:
    """Build key: repo-relative source paths + contents + flags with the repo location masked, so a snapshot of the
    tree at another path (the GPU box runs it from a scratch directory) keeps its prebuilt libraries instead of
    recompiling them on first import."""
    h = hashlib.sha256()
    for f in sorted(files, key=lambda x: os.path.relpath(x, REPO_DIR)):
        h.update(os.path.relpath(f, REPO_DIR).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(flags).replace(REPO_DIR, "<repo>").encode())
    return h.hexdigest()[:16]


class _BuildLock:
    """Inter-process lock around the stamp check + build: ranks of one job import the package at the same moment,
    and two of them rebuilding one library would load each other's half-written files."""

    def __init__(self, name: str):
        self.path = os.path.join(PKG_DIR, f".{name}.build.lock")
        self.fh = None

    def __enter__(self):
        import fcntl

        try:
            self.fh = open(self.path, "a")
        except OSError:  # read-only tree: nothing can be rebuilt here anyway
            return self
        fcntl.flock(self.fh, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        if self.fh is not None:
            import fcntl

            fcntl.flock(self.fh, fcntl.LOCK_UN)
            self.fh.close()


def _deps(pattern_dirs: list[str]) -> list[str]:
    out = []
    for d in pattern_dirs:
        for ext in ("*.h", "*.hpp", "*.cuh", "*.inc"):
            out += glob.glob(os.path.join(d, "**", ext), recursive=True)
    return out


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{r.stdout[-8000:]}")


def _build(name: str, sources: list[str], compiler: list[str], cflags: list[str], ldflags: list[str],
           deps: list[str], force: bool = False, jobs: int = 8) -> str:
    """Compile `sources` in parallel into PKG_DIR/<name><EXT_SUFFIX> unless the stamp matches."""
    with _BuildLock(name):
        return _build_locked(name, sources, compiler, cflags, ldflags, deps, force, jobs)


def _build_locked(name, sources, compiler, cflags, ldflags, deps, force, jobs) -> str:
    out = os.path.join(PKG_DIR, name + _ext_suffix())
    stamp = out + ".stamp"
    key = _hash(sources + deps, compiler + cflags + ldflags)
    if not force and os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == key:
                return out
    bdir = os.path.join(BUILD_DIR, name)
    os.makedirs(bdir, exist_ok=True)
    objs = [os.path.join(bdir, os.path.basename(s) + ".o") for s in sources]
    with _cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(sources)))) as ex:
        futs = [ex.submit(_run, compiler + cflags + ["-c", s, "-o", o]) for s, o in zip(sources, objs)]
        for f in futs:
            f.result()
    tmp = f"{out}.{os.getpid()}.tmp"
    _run(compiler + ["-shared", "-o", tmp] + objs + ldflags)
    os.replace(tmp, out)
    with open(stamp, "w") as fh:
        fh.write(key)
    return out


def build_sensor(force: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "sensor_host", "*.cpp")))
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall"] + _py_includes()
    deps = _deps([os.path.join(CSRC, "sensor_host"), os.path.join(PKG_DIR, "sensor", "bpf")])
    return _build("_sensor_native", srcs, ["g++"], flags, [], deps, force)


def build_constrain(force: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "constrain", "*.cpp")))
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall"] + _py_includes()
    deps = _deps([os.path.join(CSRC, "constrain")])
    return _build("_constrain_native", srcs, ["g++"], flags, [], deps, force)


def build_sanitize_harness(force: bool = False) -> str:
    """The host C++ cores (sensor_core.h, token_dfa_core.h) linked into one test executable under AddressSanitizer +
    UndefinedBehaviorSanitizer (GPU sanitizers are not available on the MI355X pool, so the
    sanitizers cover the host code).  Returns the executable's path; run it to exercise both cores."""
    src = os.path.join(CSRC, "tests", "host_sanitize.cpp")
    deps = _deps([os.path.join(CSRC, "tests"), os.path.join(CSRC, "sensor_host"), os.path.join(CSRC, "constrain"),
                  os.path.join(PKG_DIR, "sensor", "bpf")])
    flags = ["-O1", "-g", "-std=c++17", "-Wall", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=all"]
    out = os.path.join(BUILD_DIR, "host_sanitize")
    key = _hash([src] + deps, flags)
    stamp = out + ".stamp"
    if not force and os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return out
    os.makedirs(BUILD_DIR, exist_ok=True)
    _run(["g++"] + flags + [src, "-o", out])
    with open(stamp, "w") as fh:
        fh.write(key)
    return out


def hip_flags() -> tuple[list[str], list[str]]:
    import torch

    root, incs, libdir = _torch_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [
        f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fno-gpu-rdc", "-munsafe-fp-atomics",
        "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1", "-Wno-unused-result", "-Wno-deprecated-declarations",
        "-Wno-unused-command-line-argument",
        f"-I{os.path.join(CSRC, 'include')}",
    ] + [f"-I{i}" for i in incs] + [f"-I{sysconfig.get_paths()['include']}"]
    if os.environ.get("CHRONOS_GEMM_ABLATIONS") == "1":  # diagnostics build: gemm_lg's timing-only ablation ids
        cflags.append("-DCHRONOS_GEMM_ABLATIONS")
    ldflags = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
               "-ltorch_hip", "-ltorch_python", "-lamdhip64"]
    return cflags, ldflags


def build_kernels(force: bool = False, jobs: int = 8) -> str:
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) + glob.glob(os.path.join(CSRC, "kernels", "*.cpp")))
    cflags, ldflags = hip_flags()
    deps = _deps([os.path.join(CSRC, "kernels"), os.path.join(CSRC, "include")])
    return _build("_C", srcs, [hipcc], cflags, ldflags, deps, force, jobs)


def build_all(force: bool = False) -> None:
    build_sensor(force)
    build_constrain(force)
    build_kernels(force)


def _import_built(name: str, builder) -> object:
    with _lock:
        if name in _loaded:
            return _loaded[name]
        path = builder()
        spec = importlib.util.spec_from_file_location(f"chronos.{name}", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules[f"chronos.{name}"] = mod
        _loaded[name] = mod
        return mod


def sensor_lib():
    return _import_built("_sensor_native", build_sensor)


def constrain_lib():
    return _import_built("_constrain_native", build_constrain)


def kernels_lib():
    """Load the HIP kernel library (registers torch.ops.chronos.*).  Builds it in-tree if stale/missing."""
    with _lock:
        if "_C" in _loaded:
            return _loaded["_C"]
    import torch  # noqa: F401  (libtorch must be loaded before the extension)

    path = build_kernels()
    with _lock:
        torch.ops.load_library(path)
        _loaded["_C"] = path
    return path
