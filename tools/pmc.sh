#!/bin/bash
# PMC passes over one bench configuration (each counter group in its own
# rocprofv3 run with --kernel-trace only, as MI355X_MICROARCH.md prescribes).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-parity --no-profile --no-e2e --no-latency}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
      python3 bench.py $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pass $i failed"; tail -5 "$OUT/p$i.err"; exit 1; }
done
echo "== done"
