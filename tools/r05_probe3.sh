set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_decoder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05d_pytest.log 2>&1 || { tail -30 gpurun_out/r05d_pytest.log; exit 1; }
tail -2 gpurun_out/r05d_pytest.log
timeout -k 10 120 ./tools/valu_cost > gpurun_out/r05d_valu_cost.log 2>&1 || { tail gpurun_out/r05d_valu_cost.log; exit 1; }
head -50 gpurun_out/r05d_valu_cost.log
timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 5 > gpurun_out/r05d_bench_c5.json 2> gpurun_out/r05d_bench_c5.err || { tail -20 gpurun_out/r05d_bench_c5.err; exit 1; }
echo done
