# queue-build variant A/B (QB0 = per-word while loops; prod = first bit straight-line) + score parity
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_mf.py tests/test_gpu_score_edge.py tests/test_gpu_large_n.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/g9_pytest.log 2>&1 || { tail -30 gpurun_out/g9_pytest.log; exit 1; }
tail -1 gpurun_out/g9_pytest.log
LIBS="QB0 prod" ROUNDS=3 bash scripts/gpu_ab_libs.sh > gpurun_out/g9_ab.log 2>&1 || { tail -20 gpurun_out/g9_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g9_ab.log
