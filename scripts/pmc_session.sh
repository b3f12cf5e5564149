#!/bin/bash
# PMC passes (one rocprofv3 --pmc pass per counter group, kernel-trace only;
# never combined with sys/runtime traces) over bench.py for one workload.
#   usage: scripts/pmc_session.sh <workload> [steps]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
WL=${1:-cfg5}
STEPS=${2:-20}
OUT=$ROOT/gpurun_out/pmc_$WL
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
PASSES=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VALU SQ_ACTIVE_INST_LDS"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TA_BUSY_avr TCP_UTCL1_TRANSLATION_MISS_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_WAVES"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/bench.py" --workload "$WL" --steps "$STEPS" --warmup 2 --cpu-seconds 0 \
      > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "[pmc pass $i] rc=$rc ($P)"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
done
echo pmc done
