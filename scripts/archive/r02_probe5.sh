#!/bin/bash
# Round-2 probe 5: grouped batches on half-group workgroups (tests, timeline
# range vs grouped, ids bench).
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
TAILN=3 step gpu_grouped 400 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py tests/test_hooks.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "grouped or fused or hooks"
TAILN=6 step tl_range 200 python tools/kernel_timeline.py --workloads cfg2,cfg3,16384x1024
TAILN=6 step tl_grouped 200 python tools/kernel_timeline.py --workloads cfg2,cfg3,16384x1024 --ids grouped
for ids in range grouped; do
  step ids_cfg3_$ids 200 python bench.py --workload cfg3 --ids $ids --steps 100 --warmup 10 --cpu-seconds 0
  step ids_cfg2_$ids 200 python bench.py --workload cfg2 --ids $ids --steps 100 --warmup 10 --cpu-seconds 0
done
echo probe5 done
