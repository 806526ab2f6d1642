set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 240 python -u scripts/event_ab.py sparse 20 3 > gpurun_out/g1_event_sparse.log 2>&1 || { tail -20 gpurun_out/g1_event_sparse.log; exit 1; }
timeout -k 10 240 python -u scripts/event_ab.py c2 10 2 > gpurun_out/g1_event_c2.log 2>&1 || { tail -20 gpurun_out/g1_event_c2.log; exit 1; }
for spec in "dtype=bf16 B=4" "dtype=bf16 B=8" "dtype=bf16 B=16" "dtype=fp32 B=4" "dtype=fp32 B=8"; do
  echo "== $spec" >> gpurun_out/g1_sweep_size.log
  timeout -k 10 200 python -u scripts/sweep_ab.py $spec >> gpurun_out/g1_sweep_size.log 2>&1 || { tail -20 gpurun_out/g1_sweep_size.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/g1_event_sparse.log gpurun_out/g1_event_c2.log gpurun_out/g1_sweep_size.log
SFM_HIP_LIB=scripts/exp/libsfm_hip_FRONTSTATS.so timeout -k 10 200 python -u scripts/front_stats.py 16 8 > gpurun_out/g1_front_stats.log 2>&1 || { tail -20 gpurun_out/g1_front_stats.log; exit 1; }
SFM_HIP_LIB=scripts/exp/libsfm_hip_FRONTSTATS.so timeout -k 10 200 python -u scripts/front_stats.py --sparse 16 >> gpurun_out/g1_front_stats.log 2>&1 || { tail -20 gpurun_out/g1_front_stats.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g1_front_stats.log
