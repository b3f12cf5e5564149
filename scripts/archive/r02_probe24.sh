#!/bin/bash
# Round-2 probe 24: half image issued before the SIMD exchange.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | grep -v '^{' | tail -${TAILN:-2} | cut -c1-600
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=3 step gpu_early 400 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not staged and not cfg5"
TAILN=4 step ab_early 300 python tools/ab_bench.py --variant old@HEAD: --variant new: --workloads cfg2,4096x256,16384x1024 --rounds 9 --launches 20 --segment
TAILN=3 step tl_early 200 python tools/kernel_timeline.py --workloads cfg2
echo probe24 done
