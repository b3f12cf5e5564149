#!/bin/bash
# Round-6 A/B: the window loop head aligned (ZRC4_WIN_ALIGN=6/7, s_nop padding
# before it) and the r05 SDWA-mask loop (ZRC4_WIN_SDWA=1) with and without
# alignment, against the product build, same process (tools/ab_bench.py;
# libraries prebuilt with --build-only on the CPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${AB_OUT:-gpurun_out/r06/abalign}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python tools/ab_bench.py --variant base: --variant al6:ZRC4_WIN_ALIGN=6 \
    --variant al7:ZRC4_WIN_ALIGN=7 --variant sdwa:ZRC4_WIN_SDWA=1 \
    --variant sdwaal6:ZRC4_WIN_SDWA=1,ZRC4_WIN_ALIGN=6 \
    --workloads ${AB_WL:-cfg2,2048x1024,8192x1024,cfg4} --ids ${AB_IDS:-range,declared} \
    --rounds ${AB_ROUNDS:-11} --launches 20 > $OUT/ab.log 2>&1
rc=$?; echo "[ab] rc=$rc"; grep -v amdgpu.ids $OUT/ab.log | tail -40 | cut -c1-300
exit $rc
