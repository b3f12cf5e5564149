#!/bin/bash
# Round 4: framing fused into the persistent kernel's tail -- parity, then
# bench.py --frame (fused vs crypt + scan launches) at cfg5 / cfg3 / cfg2,
# range and grouped ids; the grouped window kernel's prefetch-before-claim A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04/${R04_TAG:-frame}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=10 step tests 900 python -u -m pytest tests/test_frame_scan.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider
for wl in cfg5 cfg3 cfg2; do
  for ids in range grouped; do
    step frame_${wl}_$ids 300 python bench.py --frame --workload $wl --ids $ids --steps 64 --warmup 16 --cpu-seconds 0
  done
done
step ab_win_grouped 600 python tools/ab_bench.py --variant new: --variant prev@628c07f: --ids grouped \
    --workloads cfg2,16384x1024,cfg3 --rounds 7 --launches 20
echo r04 frame done
