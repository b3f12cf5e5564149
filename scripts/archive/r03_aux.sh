#!/bin/bash
# Round-3 refresh of the auxiliary measurements (never the headline): the
# host-inclusive rate (pinned H2D -> kernel -> D2H, and zero-copy), the
# connection-storm KSA rate, the device framing scan.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03/aux
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name, seconds, args...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
    local rc=$?; echo "[$name] rc=$rc $(tail -c 400 $OUT/$name.json)"
    [ $rc -eq 0 ] || exit $rc
}
for wl in cfg2 cfg3 cfg5; do
  run hostinc_$wl 200 --host-inclusive --workload $wl --steps 10 --warmup 3
  run hostinc_zc_$wl 200 --host-inclusive --zero-copy --workload $wl --steps 10 --warmup 3
  run ksa_$wl 200 --ksa --workload $wl --steps 64 --warmup 8 --cpu-seconds 3
done
for wl in cfg2 cfg3 cfg4; do
  run frame_$wl 300 --frame --workload $wl --steps 64 --warmup 8 --cpu-seconds 3
done
echo aux done
