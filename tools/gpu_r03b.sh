# Round 3: full GPU suite + magnitude sweep with the hot-granule fallback (kHotS = 8).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1 || { tail -40 gpurun_out/r03b_pytest.log; exit 1; }
tail -2 gpurun_out/r03b_pytest.log
timeout -k 10 300 python -u tools/fast_tolerance.py --out gpurun_out/tol_r03b.json > gpurun_out/tol_r03b.log 2>&1 || { tail -5 gpurun_out/tol_r03b.log; exit 1; }
echo sweep done
