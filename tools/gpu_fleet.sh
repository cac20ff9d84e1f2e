# Fleet mode (player processes per GPU, parallel/fleet.py): the fleet GPU tests, then the
# host-cost probe across player counts.   bash tools/gpu_fleet.sh [P ...]  (default 2 4 6)
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/fleet
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fleet.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/fleet_gpu_test.log 2>&1
for P in ${@:-2 4 6}; do
  timeout -k 10 200 python bench.py --config hostcost --steps 60 --warmup 6 --players $P --verbose > $O/hostcost_p$P.log 2>&1
  grep '^{' $O/hostcost_p$P.log
done
