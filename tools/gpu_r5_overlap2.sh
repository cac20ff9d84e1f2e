# Round-5 overlap rehearsal, second pass: larger CU reserves and reserve + split combined.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 400 python -u tools/overlap_n8.py --iters 5 --options base,r32,r48,r64,r96,r32+split,r64+split > $O/overlap_n8_2.log 2>&1
grep -h '^{"option' $O/overlap_n8_2.log | cut -c1-300
