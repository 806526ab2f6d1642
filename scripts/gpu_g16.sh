# adaptive chunk floor: parity (score/RANSAC), sparse + c2 lines
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_mf.py tests/test_gpu_score_edge.py tests/test_gpu_ransac.py tests/test_gpu_configs.py tests/test_gpu_sfmnet.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/g16_pytest.log 2>&1 || { tail -30 gpurun_out/g16_pytest.log; exit 1; }
tail -1 gpurun_out/g16_pytest.log
for cfg in sparse c2 sparse c2; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-regularize > gpurun_out/g16_bench_$cfg.log 2>&1 || { tail -20 gpurun_out/g16_bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/g16_bench_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms'])"
done
