# One bench.py run on one MI355X: bash tools/gpu_bench.sh NAME [bench.py args ...]
#   e.g. bash tools/gpu_bench.sh live --config 1080p6m-live --steps 40
#        bash tools/gpu_bench.sh hbm --ingest hbm --steps 3000      (soak)
#   -> gpurun_out/bench/NAME.log (the JSON line is the last line)
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
NAME=${1:?name}
shift
mkdir -p gpurun_out/bench
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --verbose "$@" > gpurun_out/bench/$NAME.log 2>&1
grep '^{' gpurun_out/bench/$NAME.log
