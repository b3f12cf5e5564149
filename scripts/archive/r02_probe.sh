#!/bin/bash
# Round-2 probe: GPU parity suite, per-wave kernel timeline (diagnostic build),
# A/B of the refactored kernels against round 1 (849e847) in one process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-8}
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
fi
step timeline 300 python tools/kernel_timeline.py --workloads ${TL_WLS:-cfg2,cfg3,65536x1024,16384x1024,4096x256}
step ab 400 python tools/ab_bench.py ${AB_VARIANTS:---variant r01@849e847: --variant base:} --workloads ${AB_WLS:-cfg2,cfg3,65536x1024,cfg5} --rounds 7 --launches 20 --segment
echo probe done
