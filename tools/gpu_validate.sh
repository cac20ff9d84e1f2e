# Round validation on one MI355X: GPU tests, smoke, kernel bench, headline bench, host-cost probe.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/val
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/val/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val/smoke.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python tools/kernel_bench.py > gpurun_out/val/kb_$i.json 2> gpurun_out/val/kb_$i.err
done
timeout -k 10 300 python bench.py --verbose > gpurun_out/val/bench_1080p.log 2>&1
timeout -k 10 300 python bench.py --config hostcost --steps 30 --warmup 6 --verbose > gpurun_out/val/hostcost.log 2>&1
