#!/bin/bash
# Grouped persistent prologue (ZRC4_GR_FASTPRO): GPU suite on the new
# library, then a same-process A/B against HEAD and FASTPRO=0.
set -u
OUT=gpurun_out/r05/${RUN:-fp}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 600 python tools/ab_bench.py ${AB_VARIANTS} --ids ${AB_IDS:-grouped} --workloads ${AB_WL:-cfg5,262144x1024,131072x1024} --rounds ${AB_ROUNDS:-11} --launches 20 --segment > $OUT/ab.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; grep -v amdgpu.ids $OUT/ab.log | tail -4 | cut -c1-1500; exit $rc
