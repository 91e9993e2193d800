#!/bin/bash
# Whole-step A/B of source trees in alternating processes on one box (same-box comparison across revisions):
#   tools/ab_revs.sh <rounds> <dir> [<dir> ...]    each dir holds bench.py + the package with its built library
n=$1; shift
for i in $(seq "$n"); do
  for d in "$@"; do
    (cd "$d" && timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$d', d['ms_per_step'], d['value'])") || exit 1
  done
done
