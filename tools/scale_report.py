"""Scaling report: the headline bench at 1, 2, 4, 8 GPUs of one node, one row
per N -- segments/s, offload ratio, goodput, ms per step, weak-scaling efficiency against N x
the one-GPU rate, and each run's per-rank bound -- as a Markdown table plus the raw JSON lines.

Each N runs ``bench.py --gpus N`` as its own process (bench.py starts its N ranks itself, one
per GPU over the native RCCL plane), so a failing N is reported and the next one still runs.

    python tools/scale_report.py [--gpus 1 2 4 8] [--out scale.md] [-- bench.py args ...]
    python tools/scale_report.py --gpus 1 2 --cpu -- --players 0 --config hostcost-micro   # rehearsal

``--cpu`` passes ``--cpu`` through (gloo ranks on the host); ``HLSP2P_RCCL_REHEARSAL=socket``
in the environment rehearses the RCCL plane with ranks sharing one GPU.

``--project`` (one GPU): every N > 1 row is the single-GPU projection of one rank of an N-rank
swarm (``tools/project_swarm.py --peers N``: bench.py with N-1 synthetic peers and RCCL moving
the received bytes), scaled to the job as N x the rank's rate at max(measured step, the xGMI
receive roofline) -- a PROJECTION, labelled as such in the table, never a measurement.

    python tools/scale_report.py --project --out profiles/r6_scale_projection/scale.md
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _projected(n: int, proj: dict) -> dict:
    """A projection's output as a scaling row's record (job value = N x the rank's rate)."""
    rec = dict(proj["bench_record"])
    rec.update(value=proj["projected_job_value"], ms_per_step=proj["projected_ms_per_step"],
               goodput_GBps=rec.get("goodput_GBps", 0.0) * n, n_gpus=n, projection=proj["projection"])
    rec["data_plane"] = {"data": f"projection ({proj.get('plane', 'copy')})"}
    return rec


def run(n: int, extra: list, cpu: bool, timeout: float, project: bool = False) -> dict:
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = str(REPO) + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, str(REPO / "bench.py"), "--gpus", str(n), *(["--cpu"] if cpu else []), *extra]
    if project and n > 1:
        cmd = [sys.executable, str(REPO / "tools" / "project_swarm.py"), "--peers", str(n), *extra]
    t0 = time.monotonic()
    try:
        p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"n": n, "ok": False, "error": f"timed out after {timeout:.0f} s", "wall_s": timeout}
    wall = time.monotonic() - t0
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"n": n, "ok": False, "error": f"exit {p.returncode}: {p.stderr.strip().splitlines()[-1:] or ''}",
                "wall_s": wall}
    rec = json.loads(lines[-1])
    if project and n > 1:
        rec = _projected(n, rec)
    return {"n": n, "ok": True, "record": rec, "wall_s": wall}


def table(rows: list) -> str:
    base = next((r["record"]["value"] for r in rows if r["ok"] and r["n"] == 1), None)
    out = ["| GPUs | segments/s | offload | goodput GB/s | ms/step | weak-scaling efficiency | bound per rank "
           "| data plane | wire | CU reserve |", "|---:|---:|---:|---:|---:|---:|---|---|---|---|"]
    for r in rows:
        if not r["ok"]:
            out.append(f"| {r['n']} | failed | | | | | {r['error']} | | | |")
            continue
        rec = r["record"]
        eff = f"{rec['value'] / (r['n'] * base):.2f}" if base else "n/a"
        bounds = ",".join(sorted({p.get("bound", "?") for p in rec.get("per_rank", [])})) or "-"
        dp = rec.get("data_plane", {})
        plane = dp.get("data", "local")
        # the transport RCCL chose per pair (its connection log) and the HIP link types;
        # "-degraded" when one-GPU-per-rank pairs fell back to a network / shared-memory path
        wire = "/".join(dp.get("wire") or []) or "-"
        if dp.get("hip_links"):
            wire += f" ({'/'.join(dp['hip_links'])})"
        if dp.get("transport_degraded"):
            wire += " DEGRADED"
        cal = rec.get("calibration") or {}
        cu = str(cal.get("chosen", "-")) + (" (calibrated)" if cal.get("source") == "calibrated" else "")
        n_label = f"{r['n']} (projected)" if rec.get("projection") else str(r["n"])
        out.append(f"| {n_label} | {rec['value']:,.0f} | {rec['offload_ratio']:.3f} | {rec['goodput_GBps']:.1f} | "
                   f"{rec['ms_per_step']:.2f} | {eff} | {bounds} | {plane} | {wire} | {cu} |")
    return "\n".join(out)


def main() -> int:
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--timeout", type=float, default=1800.0, help="per N, seconds")
    ap.add_argument("--out", default=None, help="also write the report (Markdown + JSON lines) here")
    ap.add_argument("--project", action="store_true",
                    help="N > 1 rows from the single-GPU projection (tools/project_swarm.py), labelled as such")
    args = ap.parse_args(argv)
    rows = []
    for n in args.gpus:
        r = run(n, extra, args.cpu, args.timeout, args.project)
        rows.append(r)
        status = f"{r['record']['value']:,.0f} seg/s" if r["ok"] else r["error"]
        print(f"# N={n}: {status} ({r['wall_s']:.0f} s)", file=sys.stderr, flush=True)
    report = table(rows)
    print(report)
    if args.out:
        raw = "\n".join(json.dumps(r["record"]) for r in rows if r["ok"])
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(report + "\n\n```\n" + raw + "\n```\n")
    return 0 if all(r["ok"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
