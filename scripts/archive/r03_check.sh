#!/bin/bash
# Round-3 health check: default bench line (self-contained N=1 incl. the
# configs[4] companion), then the full GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r03
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
step bench_default 300 python bench.py --steps 20 --warmup 5
TAILN=4 step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
echo check done
