#!/bin/bash
# Round 4: what the grouped claims cost -- grouped parity (window kernel's
# deferred claim check), the window-kernel A/B against c4aa2a0, and claim
# placement / timing-only claim forms in the grouped persistent kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04/${R04_TAG:-claim}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-700
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=3 step tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "grouped or window or fused"
step ab_claim 1200 python tools/ab_bench.py --variant new: --variant pc0:ZRC4_GR_PRECLAIM=0 \
    --ids grouped --workloads cfg5,262144x1024,131072x1024 --rounds 7 --launches 30
echo r04 claim done
