set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_sweep_flat.py -k wide > gpurun_out/w_tests.log 2>&1; rc=$?; tail -3 gpurun_out/w_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/sweep_ab.py dtype=bf16 B=4 "" "sweep_store_px=4" "sweep_store_px=8" "sweep_store_px=8,sweep_store_nt=0" "sweep_store_px=4,sweep_store_nt=0" 2>&1 | grep median
timeout -k 10 300 python -u scripts/sweep_ab.py dtype=bf16 B=4 "" "sweep_store_px=4" "sweep_store_px=8" 2>&1 | grep median
