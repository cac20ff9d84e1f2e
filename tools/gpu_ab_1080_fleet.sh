# Headline (1080p, PCIe-bound) with the fleet default vs one in-process player, interleaved x3.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/ab1080f
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --verbose > $O/p3_$i.log 2>&1
  timeout -k 10 200 python bench.py --players 0 --verbose > $O/p0_$i.log 2>&1
done
