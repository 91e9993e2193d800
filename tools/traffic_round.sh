#!/bin/bash
# Per-launch conv traffic of one config (tools/traffic_table.py): a FETCH_SIZE and a WRITE_SIZE pass, then the table.
#   tools/traffic_round.sh <outdir> [log args: --config X --batch B]
set -e
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 tools/traffic_table.py log --out "$out/fetch/launches.json" "$@" > "$out/fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 tools/traffic_table.py log --out "$out/write/launches.json" "$@" > "$out/write.log" 2>&1
python3 tools/traffic_table.py table "$out" --csv "$out/traffic_table.csv" > "$out/traffic_table.txt"
