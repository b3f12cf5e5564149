#!/bin/bash
# Round-2 probe 14: is the timing build slower, or the timeline harness?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | grep -v '^{' | tail -${TAILN:-2} | cut -c1-700
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=2 step ab_tim 300 python tools/ab_bench.py --variant base: --variant tim:ZRC4_TIMING=1 --workloads cfg5 --rounds 5 --launches 10 --segment
TAILN=2 step stl_640 300 python tools/stream_timeline.py --workloads cfg5 --footprint-mib 640
TAILN=2 step stl_1200 300 python tools/stream_timeline.py --workloads cfg5 --footprint-mib 1200
echo probe14 done
