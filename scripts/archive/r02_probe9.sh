#!/bin/bash
# Round-2 probe 9: what the throughput loop's I/O costs (timing-only ablations:
# stores to the sink, loads from the sink, no transpose) + SQ stall buckets.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-500
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=4 step ab_io 500 python tools/ab_bench.py --variant base: --variant stsink:ZRC4_LL_AB=1 --variant ldsink:ZRC4_LL_AB=2 --variant notp:ZRC4_LL_AB=3 --variant sinks:ZRC4_LL_AB=4 --workloads cfg5,131072x1024 --rounds 5 --launches 10 --segment --no-check
bash scripts/pmc_sq.sh cfg5 base: sinks:ZRC4_LL_AB=4 || exit $?
echo probe9 done
