#!/bin/bash
# Round-2 probe 6: half-group workgroups padded to 256 threads (working waves
# on two SIMDs) vs 128 threads; parity of the half paths; timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
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
TAILN=3 step gpu_half 300 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "grouped or fused or ragged or edge or cfg2 or cfg4"
TAILN=6 step tl_pad 200 python tools/kernel_timeline.py --workloads cfg2,16384x1024
TAILN=8 step ab_pad 400 python tools/ab_bench.py --variant pad:ZRC4_HALF_PAD=1 --variant nopad:ZRC4_HALF_PAD=0 --workloads cfg2,4096x256,16384x1024,32768x256 --rounds 7 --launches 20 --segment
echo probe6 done
