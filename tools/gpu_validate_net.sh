# Validation after the real-CDN origin + event-loop changes: GPU tests (incl. the HTTP-CDN
# swarm on the GPU), smoke, headline bench, host-cost probe x3 (A/B vs profiles/r2_slots).
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/net
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --verbose > $O/bench_1080p.log 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config hostcost --steps 40 --warmup 6 --verbose > $O/hostcost_$i.log 2>&1
done
