# Fleet mode (player processes per GPU) vs the single-process bench, one box.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/fleet
mkdir -p $O
timeout -k 10 200 python bench.py --config hostcost --steps 40 --warmup 6 --verbose > $O/hc_p0.log 2>&1
for P in 1 2 3; do
  timeout -k 10 300 python bench.py --config hostcost --players $P --steps 40 --warmup 6 --verbose > $O/hc_p$P.log 2>&1
done
timeout -k 10 300 python bench.py --players 2 --verbose > $O/b1080_p2.log 2>&1
