#!/bin/bash
# k_small DP without branches: k_small parity, sentence latency (phase clocks), concurrent calls
set -o pipefail
OUT=gpurun_out/${RUN:-r04t}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "small or sentence or concurrent or edge or golden or c_abi" \
  -s --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -E "serial threads|concurrent threads" $OUT/pytest.log | tail -2
timeout -k 10 200 python -u bench.py --workload sentence --sentence-iters 3000 > $OUT/sentence.json 2> $OUT/sentence.err || exit 1
python -c "import json; d=json.loads(open('$OUT/sentence.json').read().strip().splitlines()[-1]); print('sentence ms', d['ms_per_step'])"
JB_DEBUG=1 timeout -k 10 120 python -u bench.py --workload sentence --sentence-iters 300 --no-parity > /dev/null 2> $OUT/sentence_dbg.err || exit 1
python - <<'PY'
import re, numpy as np
rows=[]
for ln in open('gpurun_out/r04t/sentence_dbg.err'):
    m=re.search(r"phases \(us\): ([\d. ]+);", ln)
    if m and len(m.group(1).split())==15: rows.append([float(x) for x in m.group(1).split()])
a=np.array(rows); c=np.zeros((len(a),16)); c[:,1:]=a
print(len(a), "calls; median us: load", np.median(c[:,1]), "codes", np.median(c[:,6]), "dag", np.median(c[:,7]), "DP end", np.median(c[:,12]), "fwd+vit end", np.median(c[:,13]), "end", np.median(c[:,11]))
PY
