#!/bin/bash
# Round-2 probe 2: chain rate per waves/CU (timeline), bench lines (driver
# shape K=20 W=5, and K=200), slot-id modes at cfg3/cfg2, fused decrypt+frame.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-400
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=2 step tl_w4 200 python tools/kernel_timeline.py --workloads 4096x1024 --active-waves 4
TAILN=2 step tl_w2 200 python tools/kernel_timeline.py --workloads 8192x1024 --active-waves 2
TAILN=2 step tl_w1 200 python tools/kernel_timeline.py --workloads 16384x1024 --active-waves 1
step bench_cfg2_k20 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 4
step bench_cfg2_k200 200 python bench.py --steps 200 --warmup 20 --cpu-seconds 0
for ids in range grouped scattered; do
  step ids_cfg3_$ids 200 python bench.py --workload cfg3 --ids $ids --steps 100 --warmup 10 --cpu-seconds 0
done
step ids_cfg2_grouped 200 python bench.py --workload cfg2 --ids grouped --steps 100 --warmup 10 --cpu-seconds 0
for wl in cfg2 cfg3; do
  step frame_$wl 300 python bench.py --frame --workload $wl --steps 64 --warmup 8 --cpu-seconds 2
done
echo probe2 done
