#!/bin/bash
# Round-2 probe 10: throughput loop without its payload stores (and loads).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-600
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=4 step ab_io2 500 python tools/ab_bench.py --variant base: --variant nost:ZRC4_LL_AB=5 --variant noio:ZRC4_LL_AB=6 --variant ldsink:ZRC4_LL_AB=2 --workloads cfg5,131072x1024 --rounds 5 --launches 10 --segment --no-check
bash scripts/pmc_sq.sh cfg5 nost:ZRC4_LL_AB=5 noio:ZRC4_LL_AB=6 || exit $?
echo probe10 done
