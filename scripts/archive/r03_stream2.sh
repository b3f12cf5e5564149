#!/bin/bash
# Round-3 A/B: crypt_stream2_kernel (one 512-thread workgroup per CU, two
# images in lockstep) against the product stream kernel, plus the XADD16=0
# control; then the staged-path parity tests on the s2 build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u tools/ab_bench.py --variant base: --variant x0:ZRC4_XADD16=0 \
    --variant s2:ZRC4_STREAM2=1,ZRC4_XADD16=0 \
    --workloads cfg5,262144x1024,131072x1024,1048576x256 --rounds 7 --launches 40 > gpurun_out/r03/ab_stream2.log 2>&1
rc=$?; echo "[ab] rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/ab_stream2.log | tail -6; [ $rc -eq 0 ] || exit $rc
ZSX_ZRC4_VARIANT=s2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r03/s2_parity.log 2>&1
rc=$?; echo "[s2 parity] rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/s2_parity.log | tail -3; exit $rc
