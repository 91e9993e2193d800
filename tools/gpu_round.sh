#!/bin/bash
# One GPU call: gpu tests, smoke, default bench line.  Each step under its own time limit; stops at the first failure.
#   tools/gpu_round.sh <outdir>
set -e
out=${1:-gpurun_out/round}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
timeout -k 10 180 python -u __graft_entry__.py smoke > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
cat "$out/bench.json"
