set -e
out=gpurun_out/s3
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 200 python -u tools/perf_bn.py > $out/perf_bn.txt 2>&1
tail -8 $out/perf_bn.txt
timeout -k 10 300 python -u tools/perf_conv.py --math h2 --variants "tune=0,tune=0x10000000" > $out/perf_conv_t256.txt 2>&1
timeout -k 10 300 python -u tools/ab_step.py --variants "tune=0" "tune=0x10000000" --rounds 5 --steps 8 > $out/ab_t256.txt 2>&1
tail -3 $out/ab_t256.txt
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $out/trace.json 2> $out/trace.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err
cat $out/bench.json
