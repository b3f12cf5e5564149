#!/bin/bash
# Round-2 probe 25: reservoir hooks with the parallel host XOR: GPU hooks tests,
# then the loopback sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_hooks.py tests/test_frame.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_hooks_par.log 2>&1
rc=$?; echo "[gpu_hooks_par] rc=$rc"; tail -2 gpurun_out/gpu_hooks_par.log; [ $rc -eq 0 ] || exit $rc
bash scripts/frame_session.sh 2 skip-tests
