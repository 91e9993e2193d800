#!/bin/bash
# A/B of two environment settings on the bench step, alternating processes on one box.
#   tools/ab_env.sh '<VAR=a ...>' '<VAR=b ...>' [rounds] [extra bench args...]
a=$1; b=$2; rounds=${3:-3}; shift 3
for r in $(seq "$rounds"); do
    for e in "$a" "$b"; do
        v=$(env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-kernel-timing --steps 12 --warmup 3 "$@" \
            | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit $?
        echo "round $r [$e]: $v"
    done
done
