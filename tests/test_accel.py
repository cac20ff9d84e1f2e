"""Cython-compiled host modules (ops/build.py: build_accel) never shadow newer sources:
a module whose source SHA-1 differs from the build manifest, or every module under
HLSJS_P2P_PURE=1, is loaded from its .py."""
import importlib.machinery

from hlsjs_p2p_wrapper_amd import _accel


def test_stale_module_falls_back_to_source():
    f = _accel._SourceFallbackFinder(False, {"player/abr.py": "0" * 40, "utils/events.py": None})
    assert "hlsjs_p2p_wrapper_amd.player.abr" in f.fallback
    spec = f.find_spec("hlsjs_p2p_wrapper_amd.player.abr")
    assert spec is not None and isinstance(spec.loader, importlib.machinery.SourceFileLoader)
    assert spec.origin.endswith("player/abr.py")
    assert f.find_spec("hlsjs_p2p_wrapper_amd.player.media") is None  # not in the manifest: default import


def test_fresh_module_keeps_compiled_and_pure_mode_disables_all():
    import hashlib

    src = _accel._PKG_DIR / "player" / "abr.py"
    digest = hashlib.sha1(src.read_bytes()).hexdigest()
    assert not _accel._SourceFallbackFinder(False, {"player/abr.py": digest}).fallback
    pure = _accel._SourceFallbackFinder(True, {"player/abr.py": digest})
    assert pure.fallback == {"hlsjs_p2p_wrapper_amd.player.abr"}


def test_compiled_modules_report_is_consistent():
    for name in _accel.compiled_modules():
        assert name.startswith("hlsjs_p2p_wrapper_amd.") and name not in _accel.FINDER.fallback
