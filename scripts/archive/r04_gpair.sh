#!/bin/bash
# Round 4: wave-pair grouped buckets -- grouped parity, A/B against the
# committed tree (c1 = dde45ad), boundary-0 stamps (range vs grouped).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04/${R04_TAG:-gpair2}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-700
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=4 step tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "${R04_K:-grouped or fused or reservoir}"
step ab_grouped 600 python tools/ab_bench.py --variant new: --variant c1@dde45ad: --ids grouped \
    --workloads cfg5,262144x1024 --rounds 5 --launches 30
step stl_grouped 300 python tools/stream_timeline.py --workloads cfg5 --ids grouped --dump $OUT/grp
step stl_range 300 python tools/stream_timeline.py --workloads cfg5 --dump $OUT/rng
echo r04 gpair done
