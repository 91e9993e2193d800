#!/bin/bash
# Run a command with a heartbeat line appended to <file> every 60 s (a long single test, e.g. the bs=64 fp64 oracle,
# prints nothing for minutes); the command keeps its own time limit.
#   tools/gpu_heartbeat.sh <heartbeat file> <command...>
hb=$1; shift
( while true; do date +%T >> "$hb"; sleep 60; done ) &
pid=$!
"$@"
rc=$?
kill $pid 2>/dev/null
exit $rc
