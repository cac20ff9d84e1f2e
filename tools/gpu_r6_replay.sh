#!/bin/bash
# One rank's host path per round at N = 1, 2, 4, 8 (fake peers, device work real), uncontended.
set -e
mkdir -p gpurun_out/r6_replay
for n in 1 2 4 8; do
  PYTHONPATH=. timeout -k 10 150 python -u tools/round_replay.py --device cuda --world $n --rounds 400 --warmup 40 \
    > gpurun_out/r6_replay/world$n.json 2> gpurun_out/r6_replay/world$n.err
  cat gpurun_out/r6_replay/world$n.json
done
