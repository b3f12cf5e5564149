#!/bin/bash
# Host-inclusive rates on the round-6 tree: pinned
# H2D -> kernel -> D2H (bench.py --host-inclusive, chunking by size), the
# kernels on pinned host memory in place (--zero-copy), and the engine's
# shape through zrc4_crypt_host (host ids in random slot order, bucketed and
# declared by the library: --ids declared), and the session engine's own
# path (zrc4_crypt_grouped_declared on pinned host blocks in place:
# --zero-copy --ids declared), for cfg2, cfg3 and cfg5.
set -u
OUT=gpurun_out/r06/${RUN:-hostinc}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for wl in cfg2 cfg3 cfg5; do
  S=200; W=20; [ $wl = cfg5 ] && { S=20; W=3; }
  for mode in copies zero_copy declared engine; do
    extra=""; [ $mode = zero_copy ] && extra="--zero-copy"; [ $mode = declared ] && extra="--ids declared"; [ $mode = engine ] && extra="--zero-copy --ids declared"
    timeout -k 10 240 python bench.py --host-inclusive --workload $wl --steps $S --warmup $W $extra \
        > $OUT/hostinc_${wl}_${mode}.json 2> $OUT/hostinc_${wl}_${mode}.err
    rc=$?; echo "[$wl $mode] rc=$rc $(tail -c 400 $OUT/hostinc_${wl}_${mode}.json)"
    [ $rc -eq 0 ] || exit $rc
  done
done
