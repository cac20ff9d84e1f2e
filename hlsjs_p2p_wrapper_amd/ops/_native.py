"""Loading of the in-tree native modules.

* :func:`runtime` — ``_runtime`` (host C++).  Built on demand with ``g++`` if missing
  (a few seconds; the CPU test tier relies on this).
* :func:`device`  — ``_C`` (gfx950 kernels).  Built on demand with ``hipcc`` if missing.
  There is deliberately **no** PyTorch/eager fallback for device tensors: if the kernels
  cannot be loaded on a GPU box the op raises, so a run can never silently measure a
  non-native path.
"""
from __future__ import annotations

import importlib
import threading
from typing import Any

_lock = threading.Lock()
_rt: Any = None
_dev: Any = None


def runtime() -> Any:
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            from . import build

            try:
                mod = importlib.import_module("hlsjs_p2p_wrapper_amd.ops._runtime")
                if build._stale(build.runtime_path(), sorted(build.RUNTIME_SRC.glob("*.[ch]pp"))):
                    raise ImportError("stale")
            except ImportError:
                build.build_runtime()
                importlib.invalidate_caches()
                mod = importlib.import_module("hlsjs_p2p_wrapper_amd.ops._runtime")
            _rt = mod
    return _rt


def device() -> Any:
    global _dev
    if _dev is not None:
        return _dev
    with _lock:
        if _dev is None:
            import torch  # noqa: F401  (libtorch symbols must be loaded first)
            from . import build

            try:
                mod = importlib.import_module("hlsjs_p2p_wrapper_amd.ops._C")
            except ImportError:
                try:
                    build.build_device()
                except Exception as e:  # pragma: no cover - GPU box without toolchain
                    raise RuntimeError(
                        "hlsjs_p2p_wrapper_amd: the gfx950 kernel module _C is missing and could not be "
                        f"built ({e}); refusing to run device ops without native kernels") from e
                importlib.invalidate_caches()
                mod = importlib.import_module("hlsjs_p2p_wrapper_amd.ops._C")
            _dev = mod
    return _dev


def device_available() -> bool:
    try:
        device()
        return True
    except Exception:
        return False
