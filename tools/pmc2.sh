#!/bin/bash
# Instruction-mix / stall PMC passes (one rocprofv3 --pmc run per group, --kernel-trace only).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pmc2}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-parity --no-profile --no-e2e}
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
      python3 bench.py $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pass $i failed"; tail -5 "$OUT/p$i.err"; exit 1; }
done <<GROUPS
${PMC_GROUPS:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum
TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum
FETCH_SIZE
WRITE_SIZE}
GROUPS
echo "== done"
