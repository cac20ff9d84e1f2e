# Where does the rank saturate? host-bound probe with 3..6 player processes, x2.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/fleet4
mkdir -p $O
for i in 1 2; do
  for P in 3 4 5 6; do
    timeout -k 10 200 python bench.py --config hostcost --steps 60 --warmup 6 --players $P --verbose > $O/hc_p${P}_$i.log 2>&1
  done
done
