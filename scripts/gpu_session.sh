set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_score_mf.py tests/test_gpu_score_edge.py tests/test_gpu_large_n.py tests/test_gpu_ransac.py tests/test_gpu_prune.py > gpurun_out/g1_tests.log 2>&1
rc=$?; tail -5 gpurun_out/g1_tests.log
[ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/ab_ref.pt
AB_REF=gpurun_out/ab_ref.pt LIBS="R3 prod T2 T0" STATS="T1S" ROUNDS=2 bash scripts/gpu_ab_libs.sh > gpurun_out/g1_ab.log 2>&1
rc=$?; grep -E "==|median|undecided|equal|Error|error" gpurun_out/g1_ab.log; exit $rc
