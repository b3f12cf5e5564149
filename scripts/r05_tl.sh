#!/bin/bash
# cfg2 per-workgroup timelines (ZRC4_TIMING build) for range / grouped /
# declared ids, and the window ubench with 2 streams per wave (mode 15).
set -u
OUT=gpurun_out/r05/${RUN:-tl}; mkdir -p $OUT
for ids in range grouped declared; do
  timeout -k 10 120 python tools/kernel_timeline.py --workloads cfg2 --ids $ids --launches 30 > $OUT/tl_cfg2_$ids.log 2>&1 || exit $?
  tail -1 $OUT/tl_cfg2_$ids.log | cut -c1-600
done
for m in 6 15 6 15; do
  timeout -k 10 60 tools/ubench/win_ubench 4096 1024 16 1 $m >> $OUT/win_ubench.jsonl 2>&1 || exit $?
done
cat $OUT/win_ubench.jsonl
