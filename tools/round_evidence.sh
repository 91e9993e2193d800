#!/bin/bash
# One call's round evidence: default bench line, rocprof kernel stats + PMC traffic of the bench workload,
# per-layer h2 conv timing, every BASELINE config.  Stops at the first failing step.
#   tools/round_evidence.sh <outdir>
set -e
out=${1:-gpurun_out/ev}
mkdir -p "$out"
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
bash tools/profile_round.sh "$out/prof"
python tools/pmc_traffic.py "$out/prof" --steps 4 --summaries "$out/r" > "$out/pmc_traffic.json"
timeout -k 10 300 python -u tools/perf_conv.py --math h2 > "$out/perf_conv.txt" 2> "$out/perf_conv.err"
bash tools/measure_configs.sh "$out/configs.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/bnprof" -o run -- python3 tools/perf_bn.py > "$out/perf_bn.txt" 2> "$out/perf_bn.err"
