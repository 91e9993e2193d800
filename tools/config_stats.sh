#!/bin/bash
# rocprof kernel statistics per step for every BASELINE config (tools/step_stats.py), one short bench run each.
#   tools/config_stats.sh <outdir>
set -e
out=${1:-gpurun_out/cfgstats}
export TMPDIR=/tmp
mkdir -p "$out"
one() {  # name per-step-kernel bench-args...
  local name=$1 psk=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name" -o run -- \
    python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing "$@" > "$out/$name.json" 2> "$out/$name.err"
  python3 tools/step_stats.py "$(find "$out/$name" -name 'run_kernel_trace.csv' | head -1)" --per-step-kernel "$psk" \
    --csv "$out/kernel_stats_$name.csv" > "$out/kernel_stats_$name.txt"
}
one baseline_siamese pjaccard_partial --config baseline_siamese
one baseline_siamese_bs64 pjaccard_partial --config baseline_siamese --batch 64
one baseline_dualstream pjaccard_partial --config baseline_dualstream
one dtsiamese jaccard_multi_partial --config dtsiamese
one siamese_mmcr_alpha0500 jaccard_multi_partial --config siamese_mmcr_alpha0500 --batch 16
