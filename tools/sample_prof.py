"""Statistical host profiler for the bench's timed steps (pure-Python mode only: Cython
frames are invisible).  Usage:
    HLSJS_P2P_PURE=1 python tools/sample_prof.py [bench args...]
Prints self time by source line and inclusive time by function over the whole run."""
import collections
import os
import runpy
import signal
import sys

INTERVAL = float(os.environ.get("SAMPLE_INTERVAL_S", "0.0002"))
self_lines = collections.Counter()
incl_funcs = collections.Counter()
total = [0]


def _handler(sig, frame):
    f0 = frame
    while f0 is not None and f0.f_code.co_name != "step":
        f0 = f0.f_back
    if f0 is None:  # outside bench.step(): start-up, imports, reporting
        return
    total[0] += 1
    f = frame
    self_lines[(f.f_code.co_filename, f.f_lineno, f.f_code.co_name)] += 1
    seen = set()
    while f is not None:
        key = (f.f_code.co_filename, f.f_code.co_firstlineno, f.f_code.co_name)
        if key not in seen:
            incl_funcs[key] += 1
            seen.add(key)
        f = f.f_back


def main():
    sys.argv = ["bench.py"] + sys.argv[1:]
    # SIGALRM must reach only the main thread: runtime threads (HIP) created while it is
    # blocked inherit the mask and never see EINTR from the sampler
    signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGALRM})
    import torch

    if torch.cuda.is_available():
        torch.cuda.init()
        torch.empty(1, device="cuda")
    signal.pthread_sigmask(signal.SIG_UNBLOCK, {signal.SIGALRM})
    signal.signal(signal.SIGALRM, _handler)
    signal.setitimer(signal.ITIMER_REAL, INTERVAL, INTERVAL)
    try:
        runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bench.py"), run_name="__main__")
    except SystemExit:
        pass
    finally:
        signal.setitimer(signal.ITIMER_REAL, 0, 0)
    n = max(1, total[0])
    short = lambda p: p.split("hlsjs_p2p_wrapper_amd/")[-1].split("site-packages/")[-1]
    print(f"# {n} samples", file=sys.stderr)
    print("# self time by line", file=sys.stderr)
    for (fn, ln, name), c in self_lines.most_common(int(os.environ.get("SAMPLE_TOP", "60"))):
        print(f"{100.0 * c / n:6.2f}%  {short(fn)}:{ln} {name}", file=sys.stderr)
    print("# inclusive time by function", file=sys.stderr)
    for (fn, ln, name), c in incl_funcs.most_common(70):
        print(f"{100.0 * c / n:6.2f}%  {short(fn)}:{ln} {name}", file=sys.stderr)


if __name__ == "__main__":
    main()
