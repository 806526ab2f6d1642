# k_solve_front on DPP quads: bit-identity, the RANSAC parity tests, stamps, bench lines
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_solve_coop.py tests/test_gpu_ransac.py tests/test_gpu_prune.py tests/test_gpu_configs.py tests/test_gpu_roots_split.py tests/test_gpu_corr.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/g3_pytest.log 2>&1 || { tail -30 gpurun_out/g3_pytest.log; exit 1; }
tail -2 gpurun_out/g3_pytest.log
SFM_HIP_LIB=scripts/exp/libsfm_hip_FRONTSTATS.so timeout -k 10 200 python -u scripts/front_stats.py 16 > gpurun_out/g3_front_stats.log 2>&1 || { tail -20 gpurun_out/g3_front_stats.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g3_front_stats.log
for cfg in sparse c2; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-regularize > gpurun_out/g3_bench_$cfg.log 2>&1 || { tail -20 gpurun_out/g3_bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/g3_bench_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['avg_launch_ms'], d['roofline_sweep']['avg_launch_ms'])"
done
