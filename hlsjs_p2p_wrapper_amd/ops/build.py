"""In-tree native build: ``_runtime`` (host C++) and ``_C`` (HIP kernels for gfx950).

Explicit ``g++`` / ``hipcc`` command lines (no hipify, no CUDA extension machinery):

* ``_runtime.<ext>`` — pybind11 module from ``csrc/runtime/*.cpp`` compiled with ``g++``.
  Needs no GPU and no torch; the CPU test tier builds it on demand.  ``sanitize=True``
  builds it with ASan/UBSan (host code only) for the race/memory test tier.
* ``_C.<ext>`` — CDNA4 kernels ``csrc/kernels/*.hip`` compiled by ``hipcc
  --offload-arch=gfx950`` into objects (fast: they include only ``hip_runtime.h``), plus the
  torch binding ``csrc/kernels/bindings.cpp``; linked by ``hipcc`` against libtorch.

Objects are cached under ``build/`` keyed by source mtime so rebuilds are incremental.
Run ``python -m hlsjs_p2p_wrapper_amd.ops.build`` to build everything.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import List, Optional

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
RUNTIME_SRC = CSRC / "runtime"
KERNEL_SRC = CSRC / "kernels"
REPO = HERE.parent.parent
BUILD = REPO / "build" / "native"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("HLSP2P_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _run(cmd: List[str], cwd: Optional[Path] = None) -> None:
    proc = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"command failed ({proc.returncode}): {' '.join(cmd)}\n{proc.stdout[-8000:]}")


def _stale(target: Path, deps: List[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _pybind_includes() -> List[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _jobs() -> int:
    try:
        return max(1, min(16, int(os.environ.get("MAX_JOBS", "0")) or (os.cpu_count() or 4)))
    except ValueError:
        return 4


def runtime_path() -> Path:
    return HERE / f"_runtime{EXT_SUFFIX}"


def asan_runtime_path() -> Path:
    return BUILD / "asan" / f"_runtime{EXT_SUFFIX}"


def device_path() -> Path:
    return HERE / f"_C{EXT_SUFFIX}"


def build_runtime(force: bool = False, sanitize: bool = False, verbose: bool = False) -> Path:
    srcs = sorted(RUNTIME_SRC.glob("*.cpp"))
    hdrs = sorted(RUNTIME_SRC.glob("*.hpp"))
    # the sanitizer build keeps the module name (_runtime) in its own directory; load it
    # with asan_runtime_path() under LD_PRELOAD=libasan (tests/test_asan_runtime.py)
    out = runtime_path() if not sanitize else asan_runtime_path()
    out.parent.mkdir(parents=True, exist_ok=True)
    if not force and not _stale(out, srcs + hdrs):
        return out
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]
    if sanitize:
        flags = ["-O1", "-g", "-std=c++17", "-fPIC", "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    objdir = BUILD / ("runtime_asan" if sanitize else "runtime")
    objdir.mkdir(parents=True, exist_ok=True)
    incs = _pybind_includes() + [f"-I{RUNTIME_SRC}"]

    def compile_one(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        if force or _stale(obj, [src] + hdrs):
            _run([cxx, *flags, *incs, "-c", str(src), "-o", str(obj)])
        return obj

    with cf.ThreadPoolExecutor(max_workers=_jobs()) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = out.with_suffix(out.suffix + ".tmp")
    link = [cxx, "-shared", *flags, *map(str, objs), "-o", str(tmp), "-lpthread"]
    _run(link)
    os.replace(tmp, out)
    if verbose:
        print(f"built {out}")
    return out


def _torch_paths():
    import torch.utils.cpp_extension as ce

    incs = [f"-I{p}" for p in ce.include_paths()]
    libdirs = ce.library_paths()
    return incs, libdirs


def build_device(force: bool = False, verbose: bool = False) -> Path:
    """Compile the HIP kernels for gfx950 and link the torch binding module ``_C``."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    kern = sorted(KERNEL_SRC.glob("*.hip"))
    hdrs = sorted(KERNEL_SRC.glob("*.h")) + sorted(KERNEL_SRC.glob("*.hpp"))
    # host-only translation units: bindings.cpp (torch ops) and rccl_comm.cpp (RCCL data plane)
    host_srcs = sorted(KERNEL_SRC.glob("*.cpp"))
    out = device_path()
    if not force and not _stale(out, kern + hdrs + host_srcs):
        return out
    objdir = BUILD / "device"
    objdir.mkdir(parents=True, exist_ok=True)
    kflags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
              "-D__HIP_PLATFORM_AMD__", f"-I{KERNEL_SRC}"]
    torch_incs, libdirs = _torch_paths()
    bflags = ["-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM", f"-I{ROCM}/include",
              "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", f"-I{KERNEL_SRC}",
              *torch_incs, *_pybind_includes()]

    def compile_kernel(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        if force or _stale(obj, [src] + hdrs):
            _run([hipcc, *kflags, "-c", str(src), "-o", str(obj)])
        return obj

    def compile_host(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        if force or _stale(obj, [src] + hdrs):
            # host-only translation unit: plain clang++ from the ROCm toolchain via hipcc
            _run([hipcc, *bflags, "-x", "c++", "-c", str(src), "-o", str(obj)])
        return obj

    with cf.ThreadPoolExecutor(max_workers=_jobs()) as ex:
        futs = [ex.submit(compile_kernel, s) for s in kern] + [ex.submit(compile_host, s) for s in host_srcs]
        objs = [f.result() for f in futs]
    tmp = out.with_suffix(out.suffix + ".tmp")
    link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp)]
    for d in libdirs:
        link += [f"-L{d}", f"-Wl,-rpath,{d}"]
    # -lrccl resolves to the librccl PyTorch ships (torch/lib comes first on the search path
    # and in the rpath): one RCCL runtime per process
    link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64", "-lrccl"]
    _run(link)
    os.replace(tmp, out)
    if verbose:
        print(f"built {out}")
    return out


# Host hot path compiled with Cython (pure-Python mode: the .py files stay the source of
# truth).  These modules run per fragment / per round (event dispatch, loaders, stream
# controller, swarm node, transmux bookkeeping); compiling them removes ~30 % of the
# interpreter overhead of the host path, which bounds segments/s per GPU once peers
# share the CDN work (N > 1).
ACCEL_MODULES = [
    "utils/events.py", "utils/xhr.py", "net/event_loop.py", "net/http.py", "net/origin.py",
    "player/controllers.py", "player/abr.py", "player/media.py", "player/transmux.py", "player/level.py",
    "player/playlist.py",
    "integration/p2p_loader.py", "agent/node.py", "agent/peer_agent.py",
    "models/segment_view.py", "models/track_view.py",
    "player/hls.py", "player/config.py", "utils/trace.py", "integration/player_interface.py",
    "models/media_map.py", "parallel/comm.py", "parallel/fleet.py", "ops/desc.py", "ops/aes.py", "ops/tsdemux.py",
    "ops/crc.py", "ops/segment.py",
]
ACCEL_MANIFEST = "_accel.json"


def _sha1(path: Path) -> str:
    import hashlib

    return hashlib.sha1(path.read_bytes()).hexdigest()


def build_accel(force: bool = False, verbose: bool = False) -> List[Path]:
    """Cython-compile ``ACCEL_MODULES`` in place (``<module>.cpython-*.so`` next to the
    ``.py``) and record each source's SHA-1 in ``_accel.json``: the package's import hook
    falls back to the ``.py`` for any module whose source changed since (never stale code),
    and ``HLSJS_P2P_PURE=1`` disables the compiled modules altogether."""
    import json

    try:
        from Cython.Build import cythonize
    except ImportError:  # optional: the pure-Python modules are the reference implementation
        if verbose:
            print("Cython not available: host hot path stays pure Python")
        return []
    pkg = HERE.parent
    objdir = BUILD / "accel"
    objdir.mkdir(parents=True, exist_ok=True)
    manifest_path = pkg / ACCEL_MANIFEST
    manifest = json.loads(manifest_path.read_text()) if manifest_path.exists() else {}
    todo = []
    for rel in ACCEL_MODULES:
        src = pkg / rel
        so = src.with_name(src.stem + EXT_SUFFIX)
        digest = _sha1(src)
        if force or not so.exists() or manifest.get(rel) != digest:
            todo.append((rel, src, so, digest))
    if not todo:
        return []
    cc = os.environ.get("CC", "gcc")
    incs = [f"-I{sysconfig.get_paths()['include']}"]
    # one cythonize call (the Cython compiler is not thread-safe), C files next to the
    # sources, moved into build/ right after
    cythonize([str(src) for _, src, _, _ in todo], language_level=3, quiet=True, force=True,
              compiler_directives={"binding": True,
                                   # HLSP2P_CYTHON_PROFILE=1: cProfile sees the compiled functions
                                   # (diagnostic builds only: the hooks cost ~2x per call)
                                   "profile": os.environ.get("HLSP2P_CYTHON_PROFILE") == "1"})
    c_files = {}
    for rel, src, _, _ in todo:
        c_file = objdir / (rel[:-3].replace("/", "__") + ".c")
        os.replace(src.with_suffix(".c"), c_file)
        c_files[rel] = c_file

    def one(item):
        rel, src, so, digest = item
        tmp = so.with_suffix(so.suffix + ".tmp")
        _run([cc, "-O2", "-fPIC", "-shared", "-fno-strict-aliasing", "-fwrapv", *incs, str(c_files[rel]), "-o",
              str(tmp)])
        os.replace(tmp, so)
        return rel, digest, None

    with cf.ThreadPoolExecutor(max_workers=_jobs()) as ex:
        done = list(ex.map(one, todo))
    for rel, digest, _ in done:
        manifest[rel] = digest
    manifest_path.write_text(json.dumps(manifest, indent=1, sort_keys=True))
    if verbose:
        print(f"cython-compiled {len(done)} host modules")
    return [pkg / rel for rel, _, _ in done]


def build_all(force: bool = False, verbose: bool = True) -> None:
    build_runtime(force=force, verbose=verbose)
    build_device(force=force, verbose=verbose)
    build_accel(force=force, verbose=verbose)


if __name__ == "__main__":
    force = "--force" in sys.argv
    if "--runtime" in sys.argv:
        build_runtime(force=force, verbose=True)
    elif "--device" in sys.argv:
        build_device(force=force, verbose=True)
    elif "--asan" in sys.argv:
        build_runtime(force=force, sanitize=True, verbose=True)
    elif "--accel" in sys.argv:
        build_accel(force=force, verbose=True)
    else:
        build_all(force=force)
