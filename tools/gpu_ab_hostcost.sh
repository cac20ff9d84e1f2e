# Same-box A/B of the host-bound probe (hostcost): ab_head vs this tree, x6, alternating
# which variant runs first in each pair (order effects).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abhc
mkdir -p $O
for i in 1 2 3 4 5 6; do
  if [ $((i % 2)) = 1 ]; then order="base new"; else order="new base"; fi
  for v in $order; do
    if [ $v = base ]; then cd $R/ab_head; else cd $R; fi
    PYTHONPATH=$PWD timeout -k 10 200 python bench.py --config hostcost --steps 40 --warmup 6 --verbose > $O/${v}_$i.log 2>&1
  done
done
