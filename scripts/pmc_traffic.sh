#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate, kernel-trace only) for the
# calibration kernels and the bench workloads.  usage: scripts/pmc_traffic.sh cfg2 cfg5 cfg3-grouped
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$ROOT/gpurun_out/traffic
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/calib_$C" -o run -- "$ROOT/tools/ubench/traffic_calib" > "$OUT/calib_$C.log" 2>&1
  rc=$?; echo "[calib $C] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for WL in "$@"; do
    # WL = cfgN or cfgN-<ids mode> (bench.py --ids grouped|scattered)
    W=${WL%%-*}; IDS=range; [ "$W" != "$WL" ] && IDS=${WL#*-}
    timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/${WL}_$C" -o run -- \
        python3 "$ROOT/bench.py" --workload "$W" --ids "$IDS" --steps 20 --warmup 2 --cpu-seconds 0 --companion-workload none > "$OUT/${WL}_$C.log" 2>&1
    rc=$?; echo "[$WL $C] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
echo traffic done
