#!/bin/bash
# Counter passes over one conv layer (tools/perf_conv.py), one rocprofv3 --pmc pass per counter group.
#   tools/pmc_conv.sh <outdir> <perf_conv args...>
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
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 tools/perf_conv.py "$@" > "$out/p$i.log" 2>&1
done
