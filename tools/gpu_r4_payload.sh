# Fleet payloads (gpuSwarm.fleetPayload: every player's onSuccess carries the fragment's bytes)
# after the round-4 rework (one async D2H per batch into the HIP-registered shared ring,
# zero-copy views on the players):  bash tools/gpu_r4_payload.sh -> gpurun_out/r4_payload/*
#   * the fleet GPU tests (payload bytes checked against the origin's CRC)
#   * headline with and without payloads, interleaved, 2 runs each; HBM-origin probe with payloads
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_payload
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fleet.py -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --verbose > $O/head_$i.log 2>&1
  timeout -k 10 300 python bench.py --fleet-payload --verbose > $O/head_payload_$i.log 2>&1
done
timeout -k 10 300 python bench.py --fleet-payload --ingest hbm --steps 100 --warmup 6 --verbose > $O/hbm_payload.log 2>&1
grep -h '^{' $O/*.log | cut -c1-300
