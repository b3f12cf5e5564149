#!/bin/bash
# Round-2 probe 18: next group's line 0 loaded behind the final half.
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
TAILN=3 step gpu_stream2 500 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
TAILN=4 step ab_next0 500 python tools/ab_bench.py --variant old@HEAD: --variant new: --workloads cfg5,262144x1024,1048576x256 --rounds 7 --launches 20 --segment
TAILN=3 step stl_next0 300 python tools/stream_timeline.py --workloads cfg5 --footprint-mib 640
echo probe18 done
