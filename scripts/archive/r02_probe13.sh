#!/bin/bash
# Round-2 probe 13: throughput-kernel workgroup timing by placement.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
timeout -k 10 300 python tools/stream_timeline.py --workloads cfg5,131072x1024 > $OUT/stream_tl3.log 2>&1
rc=$?; echo "[stream_tl3] rc=$rc"; grep -v amdgpu.ids $OUT/stream_tl3.log | grep -v '^{' | cut -c1-3000
exit $rc
