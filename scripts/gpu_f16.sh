set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_regularize.py tests/test_gpu_sfmnet.py > gpurun_out/f16_tests.log 2>&1; rc=$?; grep -E "r16|fp16|passed|failed|Error" gpurun_out/f16_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/f16_bench.log 2>&1 || exit 1
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/f16_bench.log") if l.startswith("{")][-1])
for k in ("roofline_regularize", "roofline_regularize_fp16", "roofline_regularize_fp32"):
    v = d.get(k, {})
    print(k, v.get("ms_per_stack"), v.get("achieved"), v.get("frac"), v.get("error"))
PY
