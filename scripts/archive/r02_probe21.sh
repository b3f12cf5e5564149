#!/bin/bash
# Round-2 probe 21: host-pointer batches bucketed into grouped launches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_capi.py tests/test_frame.py tests/test_hooks.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_host_grouped.log 2>&1
rc=$?; echo "[gpu_host_grouped] rc=$rc"; grep -v amdgpu.ids gpurun_out/gpu_host_grouped.log | tail -4 | cut -c1-400
exit $rc
