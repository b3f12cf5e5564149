#!/bin/bash
# Round 4: KSA window path (off-pattern key lengths) -- parity, then the
# same-process A/B against the round-3 tree by key length.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04/${R04_TAG:-ksa}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=6 step tests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "ksa"
for kl in ${R04_KL:-16 17 20 24 40 48}; do
  step ab_ksa_kl$kl 300 python tools/ab_bench.py --variant new: --variant old@4754ac6: --ksa --key-len $kl \
      --workloads cfg2,cfg5 --rounds 3 --launches 10
done
echo r04 ksa done
