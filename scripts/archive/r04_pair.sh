#!/bin/bash
# Round 4: wave-pair half-groups in the range persistent kernel -- parity of
# every stream-kernel path, then same-process A/B: new (pair meets), pair0
# (the same tree with workgroup barriers, ZRC4_PAIR=0), prev (628c07f).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04/${R04_TAG:-pair}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
TAILN=4 step tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_scan.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "${R04_K:-staged or baseline or grouped or fused or dispatch or stream}"
V="${R04_V:---variant new: --variant pair0:ZRC4_PAIR=0 --variant prev@628c07f:}"
step ab_range 900 python tools/ab_bench.py $V --workloads ${R04_RANGE_WL:-cfg5,262144x1024,131072x1024,cfg2} --rounds 7 --launches 30
step ab_grouped 600 python tools/ab_bench.py $V --ids grouped --workloads ${R04_GROUPED_WL:-cfg5,cfg2} --rounds 5 --launches 30
for kl in ${R04_KSA_KL:-}; do
  step ab_ksa_kl$kl 300 python tools/ab_bench.py --variant new: --variant w16:ZRC4_KSA_WIN32=0 --variant eab:ZRC4_KSA_EAB=1 \
      --no-check --ksa --key-len $kl --workloads cfg5 --rounds 5 --launches 10
done
echo r04 pair done
