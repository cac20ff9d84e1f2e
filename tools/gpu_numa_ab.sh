# NUMA placement A/B on one box: the host process (and its pinned CDN buffers) on the
# GPU's socket (auto), on the other socket (remote), or unbound (off); headline + hostcost.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/numa
mkdir -p $O
for i in 1 2; do
  for m in auto remote off; do
    timeout -k 10 200 python bench.py --numa $m --verbose > $O/b1080_${m}_$i.log 2>&1
    timeout -k 10 200 python bench.py --numa $m --config hostcost --steps 40 --warmup 6 > $O/hc_${m}_$i.log 2>&1
  done
done
