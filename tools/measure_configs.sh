#!/bin/bash
# Every BASELINE config's bench line (h2 / x3 / x5 / bf16, bs 32 / 64, dual-stream, DT-Siamese, MMCR), one JSON line each.
#   tools/measure_configs.sh <out.jsonl>
set -e
out=${1:-gpurun_out/configs.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
run() { timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" >> "$out" 2>> "$out.err"; }
run --config baseline_siamese
run --config baseline_siamese --batch 64
run --config baseline_siamese --math x3
run --config baseline_siamese --math x5
run --config baseline_siamese --math bf16
run --config baseline_siamese --math bf16 --batch 64
run --config baseline_dualstream
run --config baseline_dualstream --batch 64
run --config dtsiamese
run --config siamese_mmcr_alpha0500 --batch 16
