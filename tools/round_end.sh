#!/bin/bash
# One GPU call of round-end evidence: smoke, the headline profile (tools/final_profile.sh),
# the other configs (tools/configs.sh) and rocprofv3 kernel stats of the sentence
# workload (k_small).  usage: TAG=r02f tools/round_end.sh
set -euo pipefail
cd "$(dirname "$0")/.."
T=${TAG:-final}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
TAG=$T tools/final_profile.sh
TAG=$T/cfg tools/configs.sh
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/sent_stats -o run --output-format csv -- \
    python3 bench.py --workload sentence --sentence-iters 2000 > gpurun_out/$T/sent_stats.json 2>&1
echo "round_end done"
