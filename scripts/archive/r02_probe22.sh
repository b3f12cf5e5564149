#!/bin/bash
# Round-2 probe 22: workgroup -> group permutation for whole-group launches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python tools/ab_bench.py --variant wp0:ZRC4_WPERM=0 --variant wp97:ZRC4_WPERM=97 --workloads cfg3,65536x1024,32768x512 --rounds 9 --launches 20 --segment > gpurun_out/ab_wperm.log 2>&1
rc=$?; echo "[ab_wperm] rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_wperm.log | grep -v '^{' | tail -3 | cut -c1-400
exit $rc
