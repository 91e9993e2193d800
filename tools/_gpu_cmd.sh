set -e
out=gpurun_out/fin
mkdir -p $out
bash tools/pmc_bench.sh $out/pmc
cat $out/pmc/pmc_kernels.txt | head -20
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 180 python -u __graft_entry__.py smoke > $out/smoke.log 2>&1
tail -1 $out/smoke.log
