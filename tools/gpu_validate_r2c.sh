# Validation after the slotted per-fragment classes: GPU tests, smoke, headline bench,
# host-cost probe (3 runs each, for the A/B against profiles/r2_configs), hipGraph launch probe.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --verbose > $O/bench_1080p.log 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config hostcost --steps 40 --warmup 6 --verbose > $O/hostcost_$i.log 2>&1
done
timeout -k 10 120 python tools/graph_probe.py > $O/graph_probe.json 2> $O/graph_probe.err
