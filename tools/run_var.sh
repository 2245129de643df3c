#!/bin/bash
# GPU suite on variant V (var/exp_V), A/B against the in-tree lib, STAMPS clocks of
# VST (optional).  usage: V=va2 VST=va2st bash tools/run_var.sh
set -euo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/$V
mkdir -p $O
JB_LIB=$PWD/var/exp_$V/libjiebahip.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
TAG=$V REPS=${REPS:-2} bash tools/abtest.sh lib $V
if [ -n "${VST:-}" ]; then
  for v in st0 $VST; do
    JB_LIB=$PWD/var/exp_$v/libjiebahip.so JB_STAMPS=1 timeout -k 10 200 python -u bench.py --no-parity --no-e2e --no-latency --steps 2 --warmup 1 > $O/$v.json 2> $O/$v.err
    grep "k_zh clocks" $O/$v.err | tail -1
  done
fi
