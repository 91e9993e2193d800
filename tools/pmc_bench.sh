#!/bin/bash
# SQ / GRBM counter passes over the bench workload (2 steps), one rocprofv3 --pmc pass per counter group, then the
# per-kernel summary (tools/pmc_kernels.py).
#   tools/pmc_bench.sh <outdir> [bench.py args...]
set -e
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing "$@" > "$out/p$i.json" 2> "$out/p$i.err"
done
python3 tools/pmc_kernels.py "$out/p1" "$out/p2" "$out/p3" "$out/p4" --top 16 --csv "$out/pmc_kernels.csv" > "$out/pmc_kernels.txt"
