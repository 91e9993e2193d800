set -e
out=gpurun_out/pack
mkdir -p $out
timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "batched_weight_pack or h2_weight_split" > $out/pytest_pack.log 2>&1 || { tail -30 $out/pytest_pack.log; exit 1; }
tail -1 $out/pytest_pack.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $out/trace.json 2> $out/trace.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err
cat $out/bench.json
