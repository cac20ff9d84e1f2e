# BASELINE configs at the round-4 head, one MI355X: the HBM-origin probe over 3,000 steps
# (flatness), 4K 25 Mb/s, the 5-rendition ABR ladder, the live edge and the clear 1080p stream.
#   bash tools/gpu_r4_configs.sh -> gpurun_out/r4_configs/*.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_configs
mkdir -p $O
timeout -k 10 400 python bench.py --ingest hbm --steps 3000 --warmup 10 > $O/hbm_3000.log 2>&1
timeout -k 10 300 python bench.py --config 4k25m --steps 40 --warmup 5 > $O/4k25m.log 2>&1
timeout -k 10 300 python bench.py --config abr5 --steps 40 --warmup 5 > $O/abr5.log 2>&1
timeout -k 10 300 python bench.py --config 1080p6m-clear --steps 40 --warmup 5 > $O/clear.log 2>&1
timeout -k 10 300 python bench.py --config 1080p6m-live --steps 40 --warmup 5 > $O/live.log 2>&1
for f in $O/*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; j=json.loads(sys.stdin.readline()); print(j["value"], j["ms_per_step"], j.get("goodput_GBps"), j["errors"], j["per_rank"][0]["bound"])')"; done
