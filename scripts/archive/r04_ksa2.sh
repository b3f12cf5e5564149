#!/bin/bash
# Round 4: KSA window path with E built from dword reads + byte aligns and
# 32-step chunks -- parity, then A/B against 628c07f by key length.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04/${R04_TAG:-ksa2}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=4 step tests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "ksa"
for kl in ${R04_KL:-16 17 20 24 40 48 13}; do
  step ab_ksa_kl$kl 300 python tools/ab_bench.py --variant new: --variant prev@628c07f: --ksa --key-len $kl \
      --workloads cfg5,cfg2 --rounds 5 --launches 10
done
echo r04 ksa2 done
