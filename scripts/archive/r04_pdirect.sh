#!/bin/bash
# Round 4: wave pairs in whole-group range launches (crypt_kernel<kRange>) --
# parity of the direct paths, then A/B against workgroup barriers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04/${R04_TAG:-pdirect}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-700
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=3 step tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "dispatch or baseline or staged or range or fused or state"
step ab_direct 900 python tools/ab_bench.py --variant new: --variant pd0:ZRC4_PAIR_DIRECT=0 \
    --workloads cfg3,65536x1024,65536x512,65536x128 --rounds 9 --launches 20
echo r04 pdirect done
