#!/bin/bash
# Round profile of the bench workload: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate passes.
#   tools/profile_round.sh <outdir>
set -e
out=$1
export TMPDIR=/tmp
mkdir -p "$out"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > "$out/trace.json" 2> "$out/trace.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing > "$out/fetch.json" 2> "$out/fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing > "$out/write.json" 2> "$out/write.err"
