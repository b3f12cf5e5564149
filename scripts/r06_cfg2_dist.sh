#!/bin/bash
# Round-6: per-launch kernel durations of cfg2 (rocprofv3 --kernel-trace) for
# the product window loop and the r05 SDWA-mask loop (ZSX_ZRC4_VARIANT=sdwa,
# built beforehand), 400 timed launches each, to see whether the SDWA loop's
# slower cfg2 median is a shifted or a bimodal distribution.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=${DIST_OUT:-gpurun_out/r06/cfg2dist}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for v in product sdwa product2 sdwa2; do
  if [ "${v%2}" = sdwa ]; then export ZSX_ZRC4_VARIANT=sdwa; else unset ZSX_ZRC4_VARIANT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/$OUT/$v -o run --output-format csv \
      -- python3 $ROOT/bench.py --steps 400 --warmup 20 --cpu-seconds 0 --companion-workload none \
      > $ROOT/$OUT/$v.log 2>&1
  rc=$?; echo "[$v] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo dist done
