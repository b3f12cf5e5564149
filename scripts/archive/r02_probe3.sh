#!/bin/bash
# Round-2 probe 3: GPU suite (half-group + permuting grouped kernels), A/B
# half vs whole-group workgroups, timeline, slot-id modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-600
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=4 step gpu_tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py tests/test_capi.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
TAILN=8 step ab_half 400 python tools/ab_bench.py --variant half: --variant full:ZRC4_HALF=0 --workloads cfg2,4096x256,16384x1024,32768x256 --rounds 7 --launches 20 --segment
TAILN=2 step tl_cfg2 200 python tools/kernel_timeline.py --workloads cfg2,cfg3
for ids in range grouped scattered; do
  step ids_cfg3_$ids 200 python bench.py --workload cfg3 --ids $ids --steps 100 --warmup 10 --cpu-seconds 0
done
step ids_cfg2_grouped 200 python bench.py --workload cfg2 --ids grouped --steps 100 --warmup 10 --cpu-seconds 0
step bench_cfg2_k20 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 4
echo probe3 done
