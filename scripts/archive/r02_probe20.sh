#!/bin/bash
# Round-2 probe 20: alternating wave priority between a CU's two workgroups.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python tools/ab_bench.py --variant p1:ZRC4_PRIO=1 --variant p3:ZRC4_PRIO=3 --workloads cfg5,262144x1024,131072x1024,1048576x256 --rounds 7 --launches 20 --segment > gpurun_out/ab_prio3.log 2>&1
rc=$?; echo "[ab_prio] rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_prio3.log | grep -v '^{' | tail -4 | cut -c1-400
exit $rc
