mkdir -p gpurun_out/abl
for d in 0 1 2 3 4 8 16 3_4 11; do
  v=${d/_4/}; [ "$d" = "3_4" ] && v=7
  SCD_IGEMM_DBG=$v timeout -k 10 60 python tools/perf_conv.py --math x3 --only fwd --reps 10 > gpurun_out/abl/d$v.txt 2>&1 || exit 1
done
