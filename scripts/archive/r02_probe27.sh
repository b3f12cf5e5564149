#!/bin/bash
# Round-2 probe 27: the drop-in mirror over the keystream reservoir: C-ABI and
# mirror tests on the GPU, then the per-call cost with and without a ring.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_capi.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "mirror or capi or edge or kat" > gpurun_out/gpu_ks.log 2>&1
rc=$?; echo "[gpu_ks] rc=$rc"; grep -v amdgpu.ids gpurun_out/gpu_ks.log | tail -3; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/mirror_bench.jsonl
for ring in 8192 16384 65536; do
  for cfg in "2 1024" "64 1024" "2 256"; do
    set -- $cfg
    ZSX_RC4_RING=$ring timeout -k 10 60 tools/bin/mirror_bench $1 $2 2 >> gpurun_out/mirror_bench.jsonl
    rc=$?; [ $rc -eq 0 ] || { echo "[mirror_bench $ring $cfg] rc=$rc"; exit $rc; }
  done
done
cat gpurun_out/mirror_bench.jsonl
