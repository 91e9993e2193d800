#!/bin/bash
# Run GPU steps in order, each under its own time limit; continue past ordinary test failures (rc 1) but stop at
# the first crash, abort, fault or time-out.   tools/gpu_steps.sh <outdir> '<limit_s> <cmd...>' ...
out=$1; shift
mkdir -p "$out"
i=0
for step in "$@"; do
    i=$((i + 1))
    lim=${step%% *}
    cmd=${step#* }
    echo "[step $i] $cmd" | tee -a "$out/steps.log"
    timeout -k 10 "$lim" bash -c "$cmd" > "$out/step$i.log" 2>&1
    rc=$?
    echo "[step $i] rc=$rc" | tee -a "$out/steps.log"
    tail -3 "$out/step$i.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after rc=$rc" | tee -a "$out/steps.log"
        exit $rc
    fi
done
