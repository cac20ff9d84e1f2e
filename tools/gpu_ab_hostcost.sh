# Same-box A/B of the host-bound probe (hostcost): ab_head vs this tree, interleaved x4.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abhc
mkdir -p $O
for i in 1 2 3 4; do
  for v in base new; do
    if [ $v = base ]; then cd $R/ab_head; else cd $R; fi
    PYTHONPATH=$PWD timeout -k 10 200 python bench.py --config hostcost --steps 40 --warmup 6 --verbose > $O/${v}_$i.log 2>&1
  done
done
