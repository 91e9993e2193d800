set -e
out=gpurun_out/s4
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 180 python -u __graft_entry__.py smoke > $out/smoke.log 2>&1
tail -1 $out/smoke.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $out/trace.json 2> $out/trace.err
timeout -k 10 300 python -u tools/ab_step.py --variants "tune=0" "tune=0x10000000" --rounds 5 --steps 8 > $out/ab_t256.txt 2>&1
tail -2 $out/ab_t256.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err
cat $out/bench.json
