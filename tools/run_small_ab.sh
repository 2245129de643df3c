#!/bin/bash
# GPU suite on the in-tree lib, then S10k (HMM off/on) and the 1 GiB headline, A/B
# against var/exp_$B, REPS rounds.  usage: B=head bash tools/run_small_ab.sh
set -euo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-sab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for r in $(seq 1 ${REPS:-2}); do
  for v in lib $B; do
    if [ "$v" = lib ]; then L=$PWD/jieba-go_amd/lib/libjiebahip.so; else L=$PWD/var/exp_$v/libjiebahip.so; fi
    for h in 0 1; do
      JB_LIB=$L timeout -k 10 200 python bench.py --workload s10k --hmm $h --no-e2e --steps 200 --warmup 20 > $O/$v.s$h.$r.json 2> $O/$v.s$h.$r.err
      python -c "import json; d=json.load(open('$O/$v.s$h.$r.json')); print('$v s10k hmm$h', d['ms_per_step'], 'parity', (d['parity'] or {}).get('bit_exact'))"
    done
  done
done
TAG=${TAG:-sab}/big REPS=${REPS:-2} bash tools/abtest.sh lib $B
