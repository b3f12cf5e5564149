#!/bin/bash
# Window loop variant R (tools/ubench/win_var2.hpp, mode 16: the duplicate
# rule from ds_max_rtn) or S (win_var3.hpp, mode 17: SDWA byte masks)
# against the product loop (mode 6), interleaved (MODES="6 17").
set -u
OUT=gpurun_out/r05/${RUN:-win2}; mkdir -p $OUT
for r in 1 2 3; do
  for m in ${MODES:-6 16}; do
    for ns in ${NSS:-4096 1024 4}; do
      timeout -k 10 60 tools/ubench/win_ubench $ns 1024 16 1 $m >> $OUT/win_ubench.jsonl 2>&1 || exit $?
    done
  done
done
cat $OUT/win_ubench.jsonl
