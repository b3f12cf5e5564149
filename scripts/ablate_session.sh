#!/bin/bash
# Timing-only ablations of the crypt kernel (tools/ab_bench.py, one process)
# plus FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs) on a few of
# them.  Variant libraries are built beforehand on the CPU side:
#   python tools/ab_bench.py $(scripts/ablate_session.sh --variants) --build-only
# usage: scripts/ablate_session.sh [workloads]   (default cfg3,cfg5,131072x1024)
set -u
VARIANTS="--variant base: --variant st:ZRC4_STAGED_STORE=1 --variant st_nostore:ZRC4_STAGED_STORE=1,ZRC4_ABLATE=1 \
--variant st_nostage:ZRC4_STAGED_STORE=1,ZRC4_ABLATE=4 --variant st_noload:ZRC4_STAGED_STORE=1,ZRC4_ABLATE=2 \
--variant st_noimg:ZRC4_STAGED_STORE=1,ZRC4_ABLATE=24 --variant st_nomem:ZRC4_STAGED_STORE=1,ZRC4_ABLATE=30"
if [ "${1:-}" = "--variants" ]; then echo "$VARIANTS"; exit 0; fi
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$ROOT/gpurun_out/ablate
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
WLS="${1:-cfg3,cfg5,131072x1024}"
timeout -k 10 400 python "$ROOT/tools/ab_bench.py" $VARIANTS --workloads "$WLS" --rounds 5 --launches 10 --no-check \
    > "$OUT/ab.log" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/ab.log" | tail -4; echo "[ab] rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for V in base st_nostore st_nostage; do
  VA=$(echo "$VARIANTS" | tr ' ' '\n' | grep "^$V:")
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/${V}_$C" -o run -- \
        python3 "$ROOT/tools/ab_bench.py" --variant "$VA" --workloads cfg5 --rounds 1 --launches 10 --no-check \
        > "$OUT/${V}_$C.log" 2>&1
    rc=$?; echo "[$V $C] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
echo ablate done
