#!/bin/bash
# Round 4: parity subset + same-process A/Bs (new = this tree, prev = the
# round-4 KSA-window commit 628c07f, old = the round-3 tree 4754ac6).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04/${R04_TAG:-ab}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=4 step tests 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "${R04_K:-grouped or window or dispatch or ksa}"
V="--variant new: --variant prev@628c07f: --variant old@4754ac6:"
step ab_range 600 python tools/ab_bench.py $V --workloads cfg2,cfg3 --rounds 9 --launches 20
step ab_grouped 600 python tools/ab_bench.py $V --ids grouped --workloads cfg2,cfg3 --rounds 9 --launches 20
for kl in ${R04_KL:-16 17 20 24}; do
  step ab_ksa_kl$kl 300 python tools/ab_bench.py --variant new: --variant prev@628c07f: --ksa --key-len $kl \
      --workloads cfg5 --rounds 5 --launches 10
done
step ab_pair 600 python tools/ab_bench.py --variant new: --variant pair:ZRC4_PAIR_AB=1 --no-check \
    --workloads cfg5,262144x1024 --rounds 5 --launches 30
step ab_shards 600 python tools/ab_bench.py --variant new: \
    --workloads cfg5,262144x1024,131072x1024,65536x1024 --rounds 7 --launches 30
echo r04 ab done
