"""tools/update_demo.py (reference ``update_demo.rb``): the P2P demo is
derived from the engine's stock demo and actually plays."""
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))

import update_demo  # noqa: E402


def test_patch_rewrites_constructor_and_import():
    src = (REPO / "examples/demo/engine_demo.py").read_text()
    out = update_demo.patch(src)
    assert "Hls(hlsjsConfig, p2pConfig)" in out and "Hls(hlsjsConfig)" not in out
    assert "from hlsjs_p2p_wrapper_amd import Hls" in out
    assert "from hlsjs_p2p_wrapper_amd.player.hls import Hls" not in out
    assert out.startswith('"""GENERATED')
    compile(out, "p2p_demo.py", "exec")


def test_committed_demo_is_fresh():
    src = (REPO / "examples/demo/engine_demo.py").read_text()
    assert (REPO / "examples/demo/p2p_demo.py").read_text() == update_demo.patch(src)


def test_patch_fails_loudly_on_unknown_demo():
    with pytest.raises(update_demo.PatchError):
        update_demo.patch("print('not the engine demo')\n")


def test_patched_demo_plays():
    # the committed demo is the patcher's output (test_committed_demo_is_fresh)
    p = subprocess.run([sys.executable, str(REPO / "examples/demo/p2p_demo.py"), "--seconds", "3"], cwd=REPO,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "DEMO-OK" in p.stdout and "cdn=" in p.stdout
