#!/bin/bash
# Round-6 A/B: the lane kernels' block loop with each block's payload wait
# after its keystream (ZRC4_BLK_DEFER=1) against the product build.  First
# the parity tests of every kernel on the variant library (bit-exact), then
# same-process timing (tools/ab_bench.py; libraries prebuilt on the CPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${AB_OUT:-gpurun_out/r06/abdefer}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
ZSX_ZRC4_VARIANT=defer timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py \
    tests/test_gpu_declared.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    > $OUT/tests_defer.log 2>&1
rc=$?; echo "[tests defer] rc=$rc"; tail -2 $OUT/tests_defer.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_bench.py --variant base: --variant defer:ZRC4_BLK_DEFER=1 \
    --workloads ${AB_WL:-cfg3,65536x1024,16384x1024,32768x256,4096x256,65536x128} --ids ${AB_IDS:-range,declared} \
    --rounds ${AB_ROUNDS:-11} --launches 20 > $OUT/ab.log 2>&1
rc=$?; echo "[ab] rc=$rc"; grep -v amdgpu.ids $OUT/ab.log | grep -v "^{" | tail -10 | cut -c1-300
exit $rc
