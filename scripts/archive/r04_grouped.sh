#!/bin/bash
# Round 4: grouped buckets on the persistent kernel, the KSA window path and
# the asm line-0 -- parity, then same-process A/B: new (this tree), l0c (next
# line 0 as compiler loads, ZRC4_LINE0_ASM=0) and old (the round-3 tree,
# 4754ac6), for grouped and range batches, and KSA by key length.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04/${R04_TAG:-grp}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=6 step tests 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "${R04_K:-grouped or staged or dispatch or window or baseline or ksa or reservoir}"
V="--variant new: --variant l0c:ZRC4_LINE0_ASM=0 --variant old@4754ac6:"
step ab_grouped 600 python tools/ab_bench.py $V --ids grouped --workloads cfg5,262144x1024,cfg2,cfg3 --rounds 5 --launches 20
step ab_range 600 python tools/ab_bench.py $V --workloads cfg5,262144x1024,131072x1024,cfg2 --rounds 5 --launches 20
for kl in 16 17 20 24 40; do
  step ab_ksa_kl$kl 300 python tools/ab_bench.py --variant new: --variant old@4754ac6: --ksa --key-len $kl \
      --workloads cfg2,cfg5 --rounds 3 --launches 10
done
echo r04 grouped done
