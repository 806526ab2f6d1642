# round-3 session 3: k_solve_front static elimination (bit-exactness + stamps), bench lines with roofline-only events
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
true
true
SFM_HIP_LIB=scripts/exp/libsfm_hip_FRONTSTATS.so timeout -k 10 200 python -u scripts/front_stats.py 16 8 > gpurun_out/g2_front_stats.log 2>&1 || { tail -20 gpurun_out/g2_front_stats.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g2_front_stats.log
for cfg in sparse c2; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-regularize > gpurun_out/g2_bench_$cfg.log 2>&1 || { tail -20 gpurun_out/g2_bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/g2_bench_$cfg.log | cut -c1-250
  grep '^{' gpurun_out/g2_bench_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['kernel_ms'], d['roofline']['avg_launch_ms'], d['roofline_sweep']['avg_launch_ms'])"
done
