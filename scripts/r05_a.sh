set -u
OUT=gpurun_out/r05/${RUN:-a1}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=15 > $OUT/gpu_tests.log 2>&1
rc=$?; tail -25 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_bench.py --variant base: --ids range,grouped,declared --workloads cfg2,cfg3,4096x256,8192x1024 --rounds 9 --launches 20 --segment > $OUT/ab_modes.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_modes.log | tail -8; exit $rc
