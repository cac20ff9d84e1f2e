# Summarise the last tools/gpu_iter.sh run (local).
tail -1 gpurun_out/kern/tests.log
cat gpurun_out/kern/bench.json
for f in bench_1080p bench_hostcost; do grep "step ms" gpurun_out/host/$f.log; grep -o '"value": [0-9.]*' gpurun_out/host/$f.log; done
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/kern/prof/run_kernel_stats.csv')):
    print(r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs'])/1e3,1), round(float(r['MinNs'])/1e3,1))
PY
