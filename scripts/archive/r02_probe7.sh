#!/bin/bash
# Round-2 probe 7: where the slow waves of a chain-bound launch ran (HW_ID /
# XCC_ID per wave, timing build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-300
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
step place_cfg2 200 python tools/kernel_timeline.py --workloads cfg2 --placement
step place_w1 200 python tools/kernel_timeline.py --workloads 16384x1024 --active-waves 1 --placement
step place_w4 200 python tools/kernel_timeline.py --workloads 4096x1024 --placement
echo probe7 done
