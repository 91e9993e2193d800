set -e
out=gpurun_out/c16h2
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_bf16_gpu.py tests/test_h2_gpu.py tests/test_model_gpu.py tests/test_workloads_gpu.py tests/test_blocks_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -2 $out/pytest.log
timeout -k 10 300 python -u tools/perf_conv.py --math bf16 --variants "tune=0,tune=0x10000000" > $out/perf_conv_bf16.txt 2>&1
timeout -k 10 300 python -u tools/ab_step.py --variants "math=bf16" "math=bf16,tune=0x10000000" --rounds 4 --steps 8 > $out/ab_bf16.txt 2>&1
cat $out/ab_bf16.txt | tail -4
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > $out/trace.json 2> $out/trace.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err
cat $out/bench.json
