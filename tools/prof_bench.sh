set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench2.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/prof1.log 2>&1
ls -R $R/gpurun_out/prof1 | head -30
