#!/bin/bash
# Round-6 validation: full GPU suite, smoke, the default bench line (with its
# configs[4] companion), steady-state cfg5 (range and grouped ids) and cfg3
# lines, rocprofv3 kernel stats per config, PMC traffic (range and grouped).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=${VAL_OUT:-gpurun_out/r06/val}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-600
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
# VAL_PHASE=bench: tests, smoke and bench lines; VAL_PHASE=prof: rocprofv3
# kernel stats and PMC traffic only (two calls: each fits gpurun's limit)
PHASE=${VAL_PHASE:-all}
if [ "$PHASE" != prof ]; then
if [ -z "${VAL_SKIP_TESTS:-}" ]; then
  TAILN=4 step gpu_tests 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_default 300 python bench.py --steps 20 --warmup 5
[ -n "${VAL_QUICK:-}" ] && { echo "quick validation done"; exit 0; }
step bench_default_200 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0
step bench_cfg2_grouped 300 python bench.py --ids grouped --steps 200 --warmup 20 --cpu-seconds 0 --companion-workload none
step bench_cfg2_declared 300 python bench.py --ids declared --steps 200 --warmup 20 --cpu-seconds 0 --companion-workload none
step bench_cfg5 300 python bench.py --workload cfg5 --steps 200 --warmup 120 --cpu-seconds 0
step bench_cfg5_grouped 300 python bench.py --workload cfg5 --ids grouped --steps 200 --warmup 120 --cpu-seconds 0
step bench_cfg3 200 python bench.py --workload cfg3 --steps 200 --warmup 20 --cpu-seconds 0
step bench_cfg3_declared 200 python bench.py --workload cfg3 --ids declared --steps 200 --warmup 20 --cpu-seconds 0
step bench_cfg4 200 python bench.py --workload cfg4 --steps 50 --warmup 5 --cpu-seconds 0
[ "$PHASE" = bench ] && { echo "bench phase done"; exit 0; }
fi
cd /tmp && export TMPDIR=/tmp
for wl in cfg2 cfg3 cfg4 cfg5 cfg5-grouped cfg2-grouped cfg2-declared cfg3-declared; do
  W=20; [ ${wl%%-*} = cfg5 ] && W=120
  IDS=range; [ "${wl#*-}" != "$wl" ] && IDS=${wl#*-}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_$wl -o run --output-format csv \
      -- python3 $ROOT/bench.py --workload ${wl%%-*} --ids $IDS --steps 200 --warmup $W --cpu-seconds 0 \
      --companion-workload none > $ROOT/$OUT/prof_$wl.log 2>&1
  rc=$?; echo "[rocprof $wl] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd $ROOT
bash scripts/pmc_traffic.sh ${VAL_PMC:-cfg2 cfg5 cfg5-grouped cfg2-grouped cfg2-declared cfg3 cfg3-declared cfg4} || exit $?
echo validate done
