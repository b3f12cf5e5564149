#!/bin/bash
# zrc4_crypt_host (pageable caller memory, host ids in random order) after
# the r06 pipelining: bench.py --host-inclusive --ids declared, cfg2/cfg3/cfg5.
set -u
OUT=gpurun_out/r06/${RUN:-hostinc3}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for wl in cfg2 cfg3 cfg5; do
  S=200; W=20; [ $wl = cfg5 ] && { S=20; W=3; }
  timeout -k 10 240 python bench.py --host-inclusive --workload $wl --steps $S --warmup $W --ids declared \
      > $OUT/hostinc_${wl}_declared.json 2> $OUT/hostinc_${wl}_declared.err
  rc=$?; echo "[$wl declared] rc=$rc $(tail -c 300 $OUT/hostinc_${wl}_declared.json)"
  [ $rc -eq 0 ] || exit $rc
done
