# Round validation on one MI355X (what the driver runs, plus the two probes):
#   GPU tests, smoke(), the headline bench, the host-cost probe and the HBM-origin probe.
#   bash tools/gpu_validate.sh            -> gpurun_out/validate/*.log (VAL_OUT=<dir> to keep runs apart)
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${VAL_OUT:-validate}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --verbose > $O/headline.log 2>&1
timeout -k 10 300 python bench.py --config hostcost --steps 60 --warmup 6 --verbose > $O/hostcost.log 2>&1
timeout -k 10 300 python bench.py --ingest hbm --steps 60 --warmup 6 --verbose > $O/hbm.log 2>&1
grep -h '^{' $O/headline.log $O/hostcost.log $O/hbm.log
