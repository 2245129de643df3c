#!/bin/bash
# GPU suite on the in-tree lib, 1 GiB A/B against var/exp_$B, and the STAMPS per-wave
# clocks of var/exp_$BST and var/exp_$LST.  usage: B=head BST=hst LST=st1 bash tools/run_ab_st.sh
set -euo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-abst}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
TAG=${TAG:-abst}/big REPS=${REPS:-2} bash tools/abtest.sh lib $B
for v in $BST $LST; do
  JB_LIB=$PWD/var/exp_$v/libjiebahip.so JB_STAMPS=1 timeout -k 10 200 python -u bench.py --no-parity --no-e2e --no-latency --steps 2 --warmup 1 > $O/$v.json 2> $O/$v.err
  grep "k_zh clocks" $O/$v.err | tail -1
done
