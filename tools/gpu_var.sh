# host-cost variance probe: unpinned vs pinned runs of the hostcost config
set -o pipefail
mkdir -p gpurun_out/var
cat /proc/loadavg > gpurun_out/var/env.txt; nproc >> gpurun_out/var/env.txt
python -c "import os; print(sorted(os.sched_getaffinity(0))[:8], len(os.sched_getaffinity(0)))" >> gpurun_out/var/env.txt
lscpu | grep -E "Model name|MHz|NUMA node|Socket" >> gpurun_out/var/env.txt
C=$(python -c "import os; a=sorted(os.sched_getaffinity(0)); print(a[len(a)//2])")
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --config hostcost --steps 60 --warmup 10 --verbose > gpurun_out/var/free_$i.log 2>&1 || exit 1
  timeout -k 10 120 taskset -c $C python bench.py --config hostcost --steps 60 --warmup 10 --verbose > gpurun_out/var/pin_$i.log 2>&1 || exit 1
done
cat /proc/loadavg >> gpurun_out/var/env.txt
