#!/bin/bash
# The driver's exact N=1 command under rocprofv3 --kernel-trace --stats, so the
# headline line's HIP-event kernel average can be checked against the
# profiler's average for the same launches (bench.py's roofline contract).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=${PROF_OUT:-gpurun_out/r06/driver_prof}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv \
    -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $ROOT/$OUT/bench.log 2>&1
rc=$?; echo "[driver cmd under rocprofv3] rc=$rc"; tail -1 $ROOT/$OUT/bench.log | cut -c1-200
exit $rc
