#!/bin/bash
# Round-2 probe 17: wave roles picked by SIMD (ZRC4_ROLE A/B) on the 4-wave kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | grep -v '^{' | tail -${TAILN:-2} | cut -c1-900
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=5 step ab_role 700 python tools/ab_bench.py --variant r0:ZRC4_ROLE=0 --variant r1:ZRC4_ROLE=1 --variant r2:ZRC4_ROLE=2 --variant r3:ZRC4_ROLE=3 --workloads cfg3,65536x1024,131072x1024,cfg5 --rounds 7 --launches 10 --segment --ksa
echo probe17 done
