# quad k_solve_back: bit-identity, RANSAC parity, sweep relative bars, sparse/c2 lines
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_solve_coop.py tests/test_gpu_ransac.py tests/test_gpu_roots_split.py tests/test_gpu_sweep.py tests/test_gpu_configs.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/g8_pytest.log 2>&1 || { tail -30 gpurun_out/g8_pytest.log; exit 1; }
tail -2 gpurun_out/g8_pytest.log
for cfg in sparse c2; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-regularize > gpurun_out/g8_bench_$cfg.log 2>&1 || { tail -20 gpurun_out/g8_bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/g8_bench_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['kernel_ms'])"
done
