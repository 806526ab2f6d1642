set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_sweep_flat.py tests/test_gpu_sweep.py tests/test_gpu_pipeline.py tests/test_gpu_regularize.py > gpurun_out/w_tests.log 2>&1; rc=$?; tail -3 gpurun_out/w_tests.log; [ $rc -ne 0 ] && exit $rc
SETS="--config c3|--config c3 --tune sweep_store_px=0" ROUNDS=2 bash scripts/bench_ab.sh
