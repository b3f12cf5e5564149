#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout stops the script
# (no further GPU work in the call).  Outputs land in gpurun_out/.
#   usage: scripts/gpu_session.sh [workload ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
WLS="${*:-cfg2}"

stop_on_fault() {  # $1 = rc, $2 = step name
    local rc=$1
    echo "[$2] rc=$rc"
    if [ "$rc" -ge 124 ] || [ "$rc" -lt 0 ]; then
        echo "[$2] fault/timeout (rc=$rc): stopping GPU work in this call"
        exit "$rc"
    fi
}

timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -5 $OUT/gpu_tests.log; stop_on_fault $rc pytest-gpu
[ $rc -eq 0 ] || { echo "gpu tests failed; skipping bench"; exit 1; }

timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; cat $OUT/smoke.log | tail -2; stop_on_fault $rc smoke

for wl in $WLS; do
  timeout -k 10 300 python bench.py --workload $wl --steps 200 --warmup 20 --cpu-seconds 6 \
      > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err
  rc=$?; cat $OUT/bench_$wl.json; stop_on_fault $rc bench-$wl
done

for wl in $WLS; do
  timeout -k 10 200 python bench.py --workload $wl --host-inclusive --steps 20 --warmup 3 \
      > $OUT/hostinc_$wl.json 2> $OUT/hostinc_$wl.err
  rc=$?; cat $OUT/hostinc_$wl.json; stop_on_fault $rc hostinc-$wl
done

cd /tmp && export TMPDIR=/tmp
for wl in $WLS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_$wl -o run \
      --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 200 --warmup 20 --cpu-seconds 0 \
      > $GRAFT_REPO_ROOT/$OUT/prof_$wl.log 2>&1
  rc=$?; stop_on_fault $rc rocprof-$wl
done
echo done
