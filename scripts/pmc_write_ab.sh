#!/bin/bash
# WRITE_SIZE (one rocprofv3 pass per variant) on a workload, for libzrc4
# variants prebuilt by tools/ab_bench.py --build-only.
# usage: scripts/pmc_write_ab.sh <counter> <workload> <variant-spec> [...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$ROOT/gpurun_out/pmc_ab
mkdir -p "$OUT"
CTR=$1; WL=$2; shift 2
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for VA in "$@"; do
  V=${VA%%:*}
  timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d "$OUT/${V}_${WL}_$CTR" -o run -- \
      python3 "$ROOT/tools/ab_bench.py" --variant "$VA" --workloads "$WL" --rounds 1 --launches 10 --no-check \
      > "$OUT/${V}_${WL}_$CTR.log" 2>&1
  rc=$?; echo "[$V $WL $CTR] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo pmc_ab done
