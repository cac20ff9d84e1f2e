# Fleet variance check: single-process vs 1 / 2 / 3 player processes, interleaved x3.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/fleet3
mkdir -p $O
for i in 1 2 3; do
  for P in 0 1 2 3; do
    timeout -k 10 200 python bench.py --config hostcost --steps 60 --warmup 6 --players $P --verbose > $O/hc_p${P}_$i.log 2>&1
  done
done
