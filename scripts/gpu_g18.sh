# span-aligned claims (CAS): parity, block balance, A/B against unaligned claims; sparse + c2 lines
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_mf.py tests/test_gpu_score_edge.py tests/test_gpu_large_n.py tests/test_gpu_ransac.py tests/test_gpu_configs.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/g18_pytest.log 2>&1 || { tail -30 gpurun_out/g18_pytest.log; exit 1; }
tail -1 gpurun_out/g18_pytest.log
SFM_HIP_LIB=scripts/exp/libsfm_hip_BLOCKTA.so timeout -k 10 200 python -u scripts/mf2_blockt.py > gpurun_out/g18_blockt.log 2>&1 || { tail -20 gpurun_out/g18_blockt.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g18_blockt.log | tail -2
LIBS="ALIGN0 prod" ROUNDS=3 bash scripts/gpu_ab_libs.sh > gpurun_out/g18_ab.log 2>&1 || { tail -20 gpurun_out/g18_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g18_ab.log | grep -v inliers
for cfg in sparse c2; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-regularize > gpurun_out/g18_bench_$cfg.log 2>&1 || { tail -20 gpurun_out/g18_bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/g18_bench_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
