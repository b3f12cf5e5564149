#!/bin/bash
# Round-3: (1) the reference's own frame code on the GPU mirror (tests);
# (2) cfg3 range-launch write excess: WRITE_SIZE and the TCC write-request
# split per variant (base, start stagger) and per shape; grouped for contrast;
# (3) SQ stall buckets of the cfg5 stream kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out/r03/pmc
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_reference_frame.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r03/ref_frame_gpu.log 2>&1
rc=$?; echo "[ref frame gpu] rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/ref_frame_gpu.log | tail -4; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $ROOT/gpurun_out/r03/pmc/counters.txt 2>&1
grep -o "TCC_EA0_WR[A-Z0-9_]*\|TCC_EA_WR[A-Z0-9_]*" $ROOT/gpurun_out/r03/pmc/counters.txt | sort -u | head -20
OUT=$ROOT/gpurun_out/r03/pmc
for VA in base: stg16:ZRC4_STAGGER=16 stg64:ZRC4_STAGGER=64; do
  V=${VA%%:*}
  for WL in 65536x256 65536x128 65536x512; do
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/${V}_${WL}_W" -o run -- \
        python3 "$ROOT/tools/ab_bench.py" --variant "$VA" --workloads "$WL" --rounds 1 --launches 10 --no-check \
        > "$OUT/${V}_${WL}_W.log" 2>&1
    rc=$?; echo "[$V $WL WRITE_SIZE] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
for WL in cfg3-range cfg3-grouped; do
  W=${WL%%-*}; IDS=${WL#*-}
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/${WL}_REQ" -o run -- \
      python3 "$ROOT/bench.py" --workload "$W" --ids "$IDS" --steps 20 --warmup 2 --cpu-seconds 0 --companion-workload none \
      > "$OUT/${WL}_REQ.log" 2>&1
  rc=$?; echo "[$WL REQ] rc=$rc (counter names: see counters.txt)"; [ $rc -eq 124 ] && exit $rc; [ $rc -eq 137 ] && exit $rc
done
bash $ROOT/scripts/pmc_sq.sh cfg5 base: || exit $?
echo cfg3 done
