set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for L in prod DYN0 prod; do
  if [ $L = prod ]; then LIB=deep-sfm-revisited_amd/sfm_amd/libsfm_hip.so; else LIB=scripts/exp/libsfm_hip_$L.so; fi
  echo "== $L"
  SFM_HIP_LIB=$LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_ransac.py -q -p no:cacheprovider --timeout 120 --timeout-method thread 2>&1 | tail -3
done
