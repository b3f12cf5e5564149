#!/bin/bash
# Round-3 A/B: crypt_stream2_kernel with progress-balanced priority (s2b)
# against s2 (static alternation) and the product kernel; timeline of s2b;
# staged-path parity on the s2b build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u tools/ab_bench.py --variant base: --variant s2:ZRC4_STREAM2=1,ZRC4_XADD16=0,ZRC4_BAL=0 \
    --variant s2b:ZRC4_STREAM2=1,ZRC4_XADD16=0,ZRC4_BAL=1 \
    --workloads cfg5,262144x1024,1048576x256 --rounds 7 --launches 40 > gpurun_out/r03/ab_bal.log 2>&1
rc=$?; echo "[ab] rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/ab_bal.log | tail -4 | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/stream_timeline.py --s2 --define ZRC4_BAL=1 --workloads cfg5 > gpurun_out/r03/tl_s2b.log 2>&1
rc=$?; echo "[tl s2b] rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/tl_s2b.log | tail -1 | cut -c1-2500; [ $rc -eq 0 ] || exit $rc
ZSX_ZRC4_VARIANT=s2b timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "staged or baseline or stream or frame" > gpurun_out/r03/s2b_parity.log 2>&1
rc=$?; echo "[s2b parity] rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/s2b_parity.log | tail -3; exit $rc
