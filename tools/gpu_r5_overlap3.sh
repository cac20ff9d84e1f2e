# Round-5 overlap rehearsal, third pass: the bench's steady lag-2 pipeline per option.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 500 python -u tools/overlap_n8.py --iters 3 --steady 10 --options base,r32,r48,r64,r96,split,r64+split > $O/overlap_n8_3.log 2>&1
grep -h '^{"option' $O/overlap_n8_3.log | cut -c1-400
