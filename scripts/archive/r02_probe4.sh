#!/bin/bash
# Round-2 probe 4: grouped kernel with speculative image issue (tests + ids
# bench), rocprofv3 kernel stats of the bench workloads, PMC traffic passes.
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
for ids in range grouped; do
  step ids_cfg3_$ids 200 python bench.py --workload cfg3 --ids $ids --steps 100 --warmup 10 --cpu-seconds 0
  step ids_cfg2_$ids 200 python bench.py --workload cfg2 --ids $ids --steps 100 --warmup 10 --cpu-seconds 0
done
cd /tmp && export TMPDIR=/tmp
for wl in cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_$wl -o run --output-format csv \
      -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 200 --warmup 20 --cpu-seconds 0 \
      > $GRAFT_REPO_ROOT/$OUT/prof_$wl.log 2>&1
  rc=$?; echo "[rocprof $wl] rc=$rc"; tail -1 $GRAFT_REPO_ROOT/$OUT/prof_$wl.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
bash $GRAFT_REPO_ROOT/scripts/pmc_traffic.sh cfg2 cfg3 cfg3-grouped cfg5 || exit $?
echo probe4 done
