#!/bin/bash
# §8f rows 3-4 on the final tree: batched KSA (connection storm) rates by key
# length, and the device framing scan / fused decrypt+frame, next to the
# CPU oracle on one thread.
set -u
OUT=gpurun_out/r06/${RUN:-aux}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for kl in 16 24 64; do
  timeout -k 10 200 python bench.py --ksa --workload cfg5 --key-len $kl --steps 50 --warmup 5 --cpu-seconds 3 \
      > $OUT/ksa_cfg5_k$kl.json 2> $OUT/ksa_cfg5_k$kl.err || exit $?
  echo "[ksa $kl] $(cut -c1-300 $OUT/ksa_cfg5_k$kl.json)"
done
for wl in cfg2 cfg3 cfg5; do
  for ids in range grouped; do
    timeout -k 10 300 python bench.py --frame --workload $wl --ids $ids --steps 50 --warmup 5 --cpu-seconds 3 \
        > $OUT/frame_${wl}_$ids.json 2> $OUT/frame_${wl}_$ids.err || exit $?
    echo "[frame $wl $ids] $(cut -c1-400 $OUT/frame_${wl}_$ids.json)"
  done
done
