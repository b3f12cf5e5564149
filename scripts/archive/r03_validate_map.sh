#!/bin/bash
# After the xcd_run_map change: full GPU suite, smoke, default + cfg3 bench
# lines, rocprof stats for cfg3, PMC traffic for cfg3 and cfg2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/r03/final3
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-400
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=3 step gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py --steps 20 --warmup 5
step bench_cfg3 200 python bench.py --workload cfg3 --steps 200 --warmup 20 --cpu-seconds 0
step ab_shard 300 python -u tools/ab_bench.py --variant base: --workloads 65536x1024,cfg3,131072x1024 --rounds 7 --launches 20 --segment
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_cfg3 -o run --output-format csv \
    -- python3 $ROOT/bench.py --workload cfg3 --steps 200 --warmup 20 --cpu-seconds 0 --companion-workload none \
    > $ROOT/$OUT/prof_cfg3.log 2>&1 || exit 7
echo "[rocprof cfg3] ok"
cd $ROOT
bash scripts/pmc_traffic.sh cfg3 cfg2 || exit $?
echo validate done
