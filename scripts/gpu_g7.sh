# --pipeline with the 8-wave scorer (room for sweep waves beside it) vs the 12-wave default
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for r in 1 2; do
  for L in prod W8; do
    if [ $L = prod ]; then LIB=deep-sfm-revisited_amd/sfm_amd/libsfm_hip.so; else LIB=scripts/exp/libsfm_hip_$L.so; fi
    for P in "" "--pipeline"; do
      SFM_HIP_LIB=$LIB timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-regularize $P > gpurun_out/g7.log 2>&1 || { tail -20 gpurun_out/g7.log; exit 1; }
      echo "round $r lib $L $P: $(grep '^{' gpurun_out/g7.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_sweep']['avg_launch_ms'])")"
    done
  done
done
