mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_depth.py tests/test_gpu_regularize.py -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
tail -15 gpurun_out/t.log
[ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_reg -o run --output-format csv -- python3 scripts/bench_regularize.py > gpurun_out/prof_reg.log 2>&1 || exit $?
tail -1 gpurun_out/prof_reg.log
