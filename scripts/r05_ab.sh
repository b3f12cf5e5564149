#!/bin/bash
# One same-process A/B (tools/ab_bench.py) without the test suite.
set -u
OUT=gpurun_out/r05/${RUN:-ab}; mkdir -p $OUT
timeout -k 10 ${AB_TIMEOUT:-500} python tools/ab_bench.py ${AB_VARIANTS} --ids ${AB_IDS:-range} --workloads ${AB_WL} --rounds ${AB_ROUNDS:-11} --launches ${AB_LAUNCHES:-20} --segment ${AB_EXTRA:-} > $OUT/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab.log | tail -6 | cut -c1-1500; exit $rc
