#!/bin/bash
# Window-kernel placement timelines (tools/kernel_timeline.py --placement),
# product loop and the SDWA-mask variant, at 2 048 / 3 072 / 4 096 streams.
set -u
OUT=gpurun_out/r05/${RUN:-tlw}; mkdir -p $OUT
timeout -k 10 300 python tools/kernel_timeline.py --placement --workloads 2048x1024,3072x1024,cfg2 > $OUT/tl_v17.log 2>&1 &&
timeout -k 10 300 python tools/kernel_timeline.py --placement --define ZRC4_WIN_SDWA=1 --workloads 2048x1024,3072x1024,cfg2 > $OUT/tl_sdwa.log 2>&1
rc=$?; tail -c 600 $OUT/tl_v17.log; exit $rc
