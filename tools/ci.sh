#!/usr/bin/env bash
# Local CI (same steps as .github/workflows/ci.yml, CPU job).
set -euo pipefail
cd "$(dirname "$0")/.."
python -c "import __graft_entry__ as g; g.build()"
python -m compileall -q hlsjs_p2p_wrapper_amd tests examples tools bench.py
python tools/lint.py
python tools/gen_api_docs.py --check
python -m pytest tests -x -q -m "not gpu"
