#!/bin/bash
# Round-2 validation: full GPU suite, smoke, default bench line, steady-state
# cfg5 line, rocprofv3 kernel stats, PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out/val
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/val
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-900
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=4 step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_default 300 python bench.py
step bench_cfg5 300 python bench.py --workload cfg5 --steps 200 --warmup 120 --cpu-seconds 0
step bench_cfg3 200 python bench.py --workload cfg3 --steps 200 --warmup 20 --cpu-seconds 0
cd /tmp && export TMPDIR=/tmp
for wl in cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_$wl -o run --output-format csv \
      -- python3 $ROOT/bench.py --workload $wl --steps 200 --warmup 20 --cpu-seconds 0 \
      > $ROOT/$OUT/prof_$wl.log 2>&1
  rc=$?; echo "[rocprof $wl] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd $ROOT
bash scripts/pmc_traffic.sh cfg2 cfg5 || exit $?
echo validate done
