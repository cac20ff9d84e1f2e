# rocprofv3 kernel + memory-copy trace of the headline bench at the current head.
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/profhead
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/profhead/trace -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/profhead/bench.log 2>&1
find $R/gpurun_out/profhead/trace -name "*stats.csv" -exec cp {} $R/gpurun_out/profhead/ \;
