#!/bin/bash
# Round-2 probe 28: x-index update as a 16-bit VOP2 add (ZRC4_XADD16) --
# parity of the product build, then a same-process A/B against the SDWA add.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_xadd.log 2>&1
rc=$?; echo "[gpu_parity] rc=$rc"; grep -v amdgpu.ids gpurun_out/gpu_xadd.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_bench.py --variant sdwa:ZRC4_XADD16=0 --variant u16:ZRC4_XADD16=1 \
    --workloads cfg2,cfg3,cfg5 --rounds 7 --launches 20 > gpurun_out/ab_xadd16.log 2>&1
rc=$?; echo "[ab] rc=$rc"; tail -12 gpurun_out/ab_xadd16.log; exit $rc
