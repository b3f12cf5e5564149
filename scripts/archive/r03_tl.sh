#!/bin/bash
# Round-3 timelines: the product stream kernel (wave-0 stamps per workgroup)
# and crypt_stream2_kernel (per-wave stamps), cfg5 steady state.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/stream_timeline.py --s2 --workloads cfg5 ${TL_EXTRA:-} > gpurun_out/r03/tl_s2.log 2>&1
rc=$?; echo "[tl s2] rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/tl_s2.log | tail -2 | cut -c1-3000; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/stream_timeline.py --workloads cfg5 > gpurun_out/r03/tl_base.log 2>&1
rc=$?; echo "[tl base] rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/tl_base.log | tail -1 | cut -c1-1500; exit $rc
