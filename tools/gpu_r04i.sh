#!/bin/bash
# Round-4 evidence on the current build: concurrent Cut rates, smoke, PMC + rocprofv3 stats +
# the full bench line (tools/final_profile.sh), the other configs, sentence kernel stats.
set -o pipefail
T=${TAG:-r04i}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k concurrent -s --timeout 250 --timeout-method thread > gpurun_out/$T/concurrent.log 2>&1 || { echo CONC_FAILED; tail -20 gpurun_out/$T/concurrent.log; exit 1; }
grep -E "serial|concurrent threads" gpurun_out/$T/concurrent.log
TAG=$T bash tools/round_end.sh || { echo ROUND_END_FAILED; exit 1; }
tail -c 1500 gpurun_out/$T/bench.json
for f in gpurun_out/$T/cfg/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['ms_per_step'], round(d['value']/1e9,3), (d.get('parity') or {}).get('bit_exact'))"; done
