#!/bin/bash
# Whole-step A/B of two library builds in alternating processes on one box:
#   tools/ab_libs.sh <lib_a.so> <lib_b.so> [rounds] [extra bench args...]
a=$1; b=$2; n=${3:-3}; shift 3
for i in $(seq "$n"); do
  for lib in "$a" "$b"; do
    SCD_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing "$@" \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['ms_per_step'], d['value'])"
  done
done
