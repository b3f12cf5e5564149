#!/bin/bash
# Round-2 probe 23: permuted workgroup -> group mapping (default now): parity,
# cfg3 bench line and PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-700
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=3 step gpu_wperm 600 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_cfg3_wperm 200 python bench.py --workload cfg3 --steps 200 --warmup 20 --cpu-seconds 0
bash scripts/pmc_traffic.sh cfg3 || exit $?
echo probe23 done
