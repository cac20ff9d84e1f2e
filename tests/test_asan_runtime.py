"""the native host runtime (ring store, directory/planner, AES, CRC, TS
mux/demux oracle) built with -fsanitize=address,undefined and driven through every entry
point — including a TS demux fuzz over random / bit-flipped / truncated packets — in a
child process with libasan preloaded.  (GPU sanitizers are not available on the pool;
the device kernels are checked by numerics tests against these host oracles instead.)"""
import os
import subprocess
import sys
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent


def _libasan():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


@pytest.mark.slow
def test_runtime_under_asan_ubsan():
    lib = _libasan()
    if lib is None:
        pytest.skip("libasan not available")
    from hlsjs_p2p_wrapper_amd.ops.build import build_runtime

    so = build_runtime(sanitize=True)
    env = dict(os.environ)
    env["LD_PRELOAD"] = lib
    # CPython itself "leaks" at exit; halt on any real error (UBSan included)
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    p = subprocess.run([sys.executable, str(HERE / "asan_workload.py"), str(so)], env=env, capture_output=True,
                       text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "ASAN-WORKLOAD-OK" in p.stdout
    assert "runtime error" not in p.stderr  # UBSan reports
