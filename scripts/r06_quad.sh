#!/bin/bash
# Consecutive-index S-box layout in the pipe ubench:
# classic product step vs the exact quad step and its patch-free skeleton,
# at 1, 4 and 8 waves per CU, bit-exact checks against the classic step and
# the CPU PRGA.  Two runs (same box) for the spread.
set -u
OUT=gpurun_out/r06/${RUN:-quad}; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 120 tools/ubench/pipe_ubench 86 >> $OUT/pipe_ubench.jsonl 2>&1 || exit $?
done
cat $OUT/pipe_ubench.jsonl
