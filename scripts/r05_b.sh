#!/bin/bash
# GPU suite, then a same-process A/B of two library builds over ids modes.
set -u
OUT=gpurun_out/r05/${RUN:-b}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=10 > $OUT/gpu_tests.log 2>&1
rc=$?; tail -14 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_bench.py ${AB_VARIANTS:---variant old@feb9330: --variant new:} --ids ${AB_IDS:-range,grouped,declared} --workloads ${AB_WL:-cfg2,4096x256,8192x1024} --rounds 11 --launches 20 --segment > $OUT/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab.log | tail -5 | cut -c1-900; exit $rc
