#!/bin/bash
# Window-loop microbenchmarks (tools/ubench/win_ubench.hip): product asm (6),
# product rules in compiled HIP (1), repaired windows in compiled HIP (13).
set -u
OUT=gpurun_out/r05/${RUN:-win}; mkdir -p $OUT
for m in 6 1 13 6 13; do
  for ns in 4096 4; do
    timeout -k 10 60 tools/ubench/win_ubench $ns 1024 16 1 $m >> $OUT/win_ubench.jsonl 2>&1 || exit $?
  done
done
cat $OUT/win_ubench.jsonl
