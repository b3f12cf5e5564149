#!/bin/bash
# Round 4: KSA fetch path for keys over 48 bytes as dwords -- parity, then
# A/B against 74a1ddf (17 byte loads per chunk) by key length.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r04/${R04_TAG:-ksa4}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-700
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=3 step tests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "ksa"
for kl in 16 49 65 100 128 256; do
  step ab_ksa_kl$kl 300 python tools/ab_bench.py --variant new: --variant c3@74a1ddf: --ksa --key-len $kl \
      --workloads cfg5,cfg2 --rounds 5 --launches 10
done
echo r04 ksa4 done
