set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u scripts/diag_psnet64.py || exit 1
TESTS="tests/test_gpu_roots_split.py tests/test_gpu_precision.py tests/test_gpu_score_mf.py tests/test_gpu_ransac.py" PYTEST_ARGS="-s" LIBS="prod L0" ROUNDS=3 bash scripts/gpu_session.sh || exit $?
grep -E "C5 thr" gpurun_out/s_tests.log | head -60
for r in 1 2; do for sp in "" "--sparse"; do for k in 1 2; do
  timeout -k 10 120 python -u scripts/solve_time.py $sp roots_split=$k || exit 1
done; done; done
