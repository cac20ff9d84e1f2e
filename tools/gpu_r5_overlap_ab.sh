# Steady lag-2 pipeline A/B of the RCCL CU reserve, interleaved repeats (tools/overlap_n8.py).
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 500 python -u tools/overlap_n8.py --only-steady --steady 12 --iters 3 --repeat 4 --options base,r32,r64 > $O/overlap_ab.log 2>&1
grep -h '^{"option' $O/overlap_ab.log | cut -c1-200
