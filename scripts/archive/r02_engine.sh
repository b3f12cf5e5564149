#!/bin/bash
# Round-2 GPU call: full GPU suite, engine loopback sweep + rocprof trace,
# frame-scan bench (separate vs fused decrypt+frame).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests.log 2>&1
rc=$?; tail -4 $OUT/gpu_tests.log; echo "[gpu-tests] rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/frame_session.sh 2 skip-tests || exit $?
for wl in cfg2 cfg3; do
  timeout -k 10 300 python bench.py --frame --workload $wl --steps 64 --warmup 8 --cpu-seconds 3 \
      > $OUT/frame_$wl.json 2> $OUT/frame_$wl.err
  rc=$?; cat $OUT/frame_$wl.json; [ $rc -eq 0 ] || exit $rc
done
echo engine done
