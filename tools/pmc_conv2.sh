#!/bin/bash
# Memory-side counter passes over one conv layer (tools/perf_conv.py), one rocprofv3 --pmc pass per group.
#   tools/pmc_conv2.sh <outdir> <perf_conv args...>
set -e
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for grp in "TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d "$out/q$i" -o run -- python3 tools/perf_conv.py "$@" > "$out/q$i.log" 2>&1
done
