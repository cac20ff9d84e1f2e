# Round-5 soak: the HBM-origin probe (device-bound) over 3,000 steps and the headline over
# 2,000 -- with the periodic GC thaw (utils/runtime.py) the long runs must stay flat.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r5_soak
mkdir -p $O
timeout -k 10 400 python -u bench.py --ingest hbm --steps 3000 --warmup 6 --verbose > $O/hbm3000.log 2>&1
timeout -k 10 400 python -u bench.py --steps 2000 --warmup 5 --verbose > $O/head2000.log 2>&1
grep -h '^{' $O/hbm3000.log $O/head2000.log | cut -c1-200
grep -h "step ms by tenth" $O/hbm3000.log $O/head2000.log
