"""Developer tooling parity: ``npm run docs`` (jsdoc) -> ``tools/gen_api_docs.py`` and
``npm run lint`` (eslint) -> ``tools/lint.py`` (reference ``package.json:21-22``)."""
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))

import lint  # noqa: E402


def test_api_docs_are_current():
    """docs/API.md is what the generator produces from today's docstrings."""
    p = subprocess.run([sys.executable, str(REPO / "tools" / "gen_api_docs.py"), "--check"], cwd=REPO,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr


def test_api_docs_cover_the_public_surface():
    text = (REPO / "docs" / "API.md").read_text()
    for name in ("HlsjsP2PWrapper", "HlsjsP2PWrapperPrivate", "p2p_loader_generator", "PlayerInterface",
                 "SegmentView", "TrackView", "MediaMap", "PeerAgent", "SwarmNode", "getSegment",
                 "isSupported", "MANIFEST_LOADING"):
        assert name in text, name
    # every member row carries a description
    rows = [ln for ln in text.splitlines() if ln.startswith("| `")]
    assert rows and all(not ln.rstrip().endswith("|  |") for ln in rows)


def test_lint_is_clean_on_the_tree():
    findings = lint.lint(lint._py_files(lint.DEFAULT_TARGETS))
    assert findings == [], "\n".join(f"{p}:{n}: {c} {m}" for p, n, c, m in findings)


def test_lint_reports_each_check(tmp_path):
    bad = tmp_path / "bad.py"
    bad.write_text(
        "import os\n"
        "import json  # noqa\n"
        "from typing import Optional\n"
        "def f(x=[], *, y={}):\n"
        "    try:\n"
        "        pass\n"
        "    except:\n"
        "        pass\n"
        "    if x is 'a':\n"
        "        return f'plain'\n"
        "    assert (x, 'msg')\n"
        "    return f'{x:>4}'\n"
        "def f():\n"
        "    pass\n"
        "def g(a: 'Optional[int]') -> None:\t\n"
        "    return None  \n"
        "z = '" + "x" * 130 + "'\n")
    codes = sorted((n, c) for _, n, c, _ in lint.lint([bad]))
    assert codes == [(1, "L001"), (4, "L003"), (4, "L003"), (7, "L002"), (9, "L004"), (10, "L005"),
                     (11, "L009"), (13, "L006"), (15, "L007"), (16, "L007"), (17, "L008")]


def test_lint_cli_exit_status(tmp_path):
    good = tmp_path / "good.py"
    good.write_text("def f(x=None):\n    return x\n")
    bad = tmp_path / "bad2.py"
    bad.write_text("import os\n")
    run = lambda f: subprocess.run([sys.executable, str(REPO / "tools" / "lint.py"), str(f)],  # noqa: E731
                                   capture_output=True, text=True, timeout=60)
    assert run(good).returncode == 0
    r = run(bad)
    assert r.returncode == 1 and "L001" in r.stdout


def test_wheel_ships_every_compiled_module(tmp_path):
    """``pip wheel .`` (the reference's ``grunt`` dist build, C13): a platform-tagged wheel with
    the gfx950 kernels, the host runtime, every Cython-compiled module and the manifest
    that keeps stale compiled modules out of use."""
    import zipfile

    p = subprocess.run([sys.executable, "-m", "pip", "wheel", str(REPO), "--no-deps", "--no-build-isolation",
                        "--no-index", "-w", str(tmp_path)], capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    wheels = list(tmp_path.glob("*.whl"))
    assert len(wheels) == 1 and "-cp3" in wheels[0].name and "linux_x86_64" in wheels[0].name, wheels
    names = zipfile.ZipFile(wheels[0]).namelist()
    shipped = {n.split("hlsjs_p2p_wrapper_amd/", 1)[1] for n in names if "hlsjs_p2p_wrapper_amd/" in n}
    pkg = REPO / "hlsjs_p2p_wrapper_amd"
    built = {str(so.relative_to(pkg)) for so in pkg.rglob("*.so")}
    assert built and built <= shipped, sorted(built - shipped)
    assert "_accel.json" in shipped and "ops/csrc/kernels/aes_cbc.hip" in shipped


def test_scale_report_runs_each_n_and_tabulates(tmp_path):
    """SURVEY §5.5's bench reporter (``tools/scale_report.py``): one self-launched bench per N,
    a row each with segments/s, offload and weak-scaling efficiency against N x the 1-rank
    rate (CPU rehearsal here; on a node of MI355X the same command runs RCCL ranks)."""
    out = tmp_path / "scale.md"
    p = subprocess.run([sys.executable, str(REPO / "tools" / "scale_report.py"), "--gpus", "1", "2", "--cpu", "--out",
                        str(out), "--", "--players", "0", "--config", "hostcost-micro", "--steps", "4", "--warmup", "1",
                        "--inflight", "8", "--pool", "8", "--cache-gb", "0.5"], cwd=REPO, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    rows = [ln for ln in p.stdout.splitlines() if ln.startswith("| 1 |") or ln.startswith("| 2 |")]
    assert len(rows) == 2 and "| 1.00 |" in rows[0] and "| 0.500 |" in rows[1]
    text = out.read_text()
    assert text.count('"n_gpus": ') == 2


def test_scale_report_table_marks_failures():
    import scale_report

    rec = {"value": 100.0, "offload_ratio": 0.0, "goodput_GBps": 1.0, "ms_per_step": 2.0, "per_rank": [],
           "data_plane": {"data": "local"}}
    rec2 = dict(rec, value=350.0, offload_ratio=0.5, per_rank=[{"bound": "pcie"}, {"bound": "xgmi"}],
                data_plane={"data": "rccl-native"})
    t = scale_report.table([{"n": 1, "ok": True, "record": rec}, {"n": 2, "ok": True, "record": rec2},
                            {"n": 4, "ok": False, "error": "exit 1: boom"}])
    lines = t.splitlines()
    assert "| 1.75 |" in lines[3] and "pcie,xgmi" in lines[3] and "rccl-native" in lines[3]
    assert lines[4].startswith("| 4 | failed |") and "boom" in lines[4]
