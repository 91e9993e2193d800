#!/bin/bash
# Ablation sweep of the x3 weight-grad kernel (perf experiment): 1 = no rows loads, 2 = no src loads,
# 8 = no MFMA, 16 = no split, combinations.
mkdir -p gpurun_out/ablw
for v in 0 1 2 3 8 16 11 27; do
  SCD_WGRAD_DBG=$v timeout -k 10 60 python tools/perf_conv.py --math x3 --only wgrad --reps 10 > gpurun_out/ablw/d$v.txt 2>&1 || exit 1
done
