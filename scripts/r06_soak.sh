#!/bin/bash
# Round-6 randomised soak on the validated library (test-side only): the
# 84-call C-ABI sweep (tests/test_gpu_fuzz.py) and the fused decrypt+frame
# case (tests/test_frame_scan.py) from many seeds, one pytest process each;
# KSA_SEEDS adds the batched KSA (tests/test_gpu_fuzz.py::test_ksa_soak) and
# ENGINE_SEEDS the engine's echo parity (tests/test_frame.py) on the device hooks.
# ZRC4_SOAK_SEEDS='a-b' or 'a,b,c' (default 1-30); FUSED_SEEDS / FUZZ_SEEDS
# override it per sweep ('none' skips one), SOAK_SECS bounds each step (default 540).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${SOAK_OUT:-gpurun_out/r06/soak}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
export ZRC4_SOAK_SEEDS=${ZRC4_SOAK_SEEDS:-1-30}
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -3 | cut -c1-600
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
S=${SOAK_SECS:-540}
[ "${FUSED_SEEDS:-}" != none ] && ZRC4_SOAK_SEEDS=${FUSED_SEEDS:-$ZRC4_SOAK_SEEDS} step fused_soak $S python -u -m pytest tests/test_frame_scan.py -m gpu -k soak -x -v --durations=0 \
    --timeout 240 --timeout-method thread -p no:cacheprovider
[ "${FUZZ_SEEDS:-}" != none ] && ZRC4_SOAK_SEEDS=${FUZZ_SEEDS:-$ZRC4_SOAK_SEEDS} step fuzz_soak $S python -u -m pytest tests/test_gpu_fuzz.py -m gpu -k random_call_sequence_soak -x -v --durations=0 \
    --timeout 240 --timeout-method thread -p no:cacheprovider
if [ -n "${KSA_SEEDS:-}" ]; then
ZRC4_SOAK_SEEDS=$KSA_SEEDS step ksa_soak $S python -u -m pytest tests/test_gpu_fuzz.py -m gpu -k ksa_soak -x -v \
    --durations=0 --timeout 240 --timeout-method thread -p no:cacheprovider
fi
if [ -n "${ENGINE_SEEDS:-}" ]; then
ZRC4_SOAK_SEEDS=$ENGINE_SEEDS step engine_soak $S python -u -m pytest tests/test_frame.py -m gpu -k soak -x -v \
    --durations=0 --timeout 240 --timeout-method thread -p no:cacheprovider
fi
echo soak done
