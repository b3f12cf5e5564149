#!/bin/bash
# SQ stall buckets + GRBM clock counters (one rocprofv3 pass per variant) on a
# workload, for libzrc4 variants prebuilt by tools/ab_bench.py --build-only.
# usage: scripts/pmc_sq.sh <workload> <variant-spec> [<variant-spec> ...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$ROOT/gpurun_out/pmc_sq
mkdir -p "$OUT"
WL=$1; shift
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
CTRS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
for VA in "$@"; do
  V=${VA%%:*}
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/${V}_$WL" -o run -- \
      python3 "$ROOT/tools/ab_bench.py" --variant "$VA" --workloads "$WL" --rounds 1 --launches 10 --no-check \
      > "$OUT/${V}_$WL.log" 2>&1
  rc=$?; echo "[$V $WL] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo pmc_sq done
