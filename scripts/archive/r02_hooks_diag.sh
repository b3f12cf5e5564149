#!/bin/bash
# Reservoir hooks at 2 048 sessions on coherent pinned memory: byte-checked
# random spans (3 seeds), then the loopback sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/hooks_diag2.jsonl
: > $OUT
for seed in 3 4 5; do
  timeout -k 10 120 tools/bin/hooks_check device 2048 60 $seed >> $OUT 2>&1
  rc=$?; echo "[check seed=$seed rc=$rc]" | tee -a $OUT; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 tools/bin/hooks_check direct 1024 30 4 >> $OUT 2>&1; rc=$?; echo "[direct rc=$rc]"; [ $rc -eq 0 ] || exit $rc
cut -c1-200 $OUT
bash scripts/frame_session.sh 2 skip-tests
