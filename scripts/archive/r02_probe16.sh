#!/bin/bash
# Round-2 probe 16: steady-state (150 launches in) throughput-kernel timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/stream_timeline.py --workloads cfg5,262144x1024,131072x1024 --footprint-mib 640 > gpurun_out/stl_ss.log 2>&1
rc=$?; echo "[stl_ss] rc=$rc"; grep -v amdgpu.ids gpurun_out/stl_ss.log | grep -v '^{' | cut -c1-1800
exit $rc
