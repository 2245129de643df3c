#!/bin/bash
# Detailed PMC passes (TA/TD/LDS/issue/I-cache) over one bench configuration.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pmcd}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-parity --no-profile --no-e2e}
i=0
for grp in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVE_CYCLES" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_VALU" \
           ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
      python3 bench.py $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pass $i failed"; tail -5 "$OUT/p$i.err"; exit 1; }
done
echo "== done"
