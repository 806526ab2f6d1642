# k_score_mf2 guided per-XCD range claiming: parity, A/B against static ranges, block balance
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_mf.py tests/test_gpu_score_edge.py tests/test_gpu_large_n.py tests/test_gpu_ransac.py tests/test_gpu_configs.py tests/test_gpu_prune.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/g12_pytest.log 2>&1 || { tail -30 gpurun_out/g12_pytest.log; exit 1; }
tail -1 gpurun_out/g12_pytest.log
SFM_HIP_LIB=scripts/exp/libsfm_hip_BLOCKTD.so timeout -k 10 200 python -u scripts/mf2_blockt.py > gpurun_out/g12_blockt.log 2>&1 || { tail -20 gpurun_out/g12_blockt.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g12_blockt.log
LIBS="DYN0 prod MC32 MC128" ROUNDS=3 bash scripts/gpu_ab_libs.sh > gpurun_out/g12_ab.log 2>&1 || { tail -20 gpurun_out/g12_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g12_ab.log | grep -v inliers
