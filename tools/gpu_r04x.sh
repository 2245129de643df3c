#!/bin/bash
# long blocks: speculative choices + decided chain (JB_LONG_SPEC=1) — parity, then 5b timing against the exact chain
set -o pipefail
OUT=gpurun_out/${RUN:-r04x}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
  -k "long or edge or golden or overflow or degenerate or split or config4" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
  || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 1 0 1; do
  JB_LONG_SPEC=$v timeout -k 10 300 python bench.py --workload long-oov --steps 3 --warmup 1 --no-e2e > $OUT/long_spec$v.json 2> $OUT/long_spec$v.err || { tail -5 $OUT/long_spec$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/long_spec$v.json').read().strip().splitlines()[-1]); k=d['kernels_ms']; print('JB_LONG_SPEC=$v', d['ms_per_step'], {a: round(b,3) for a,b in k.items() if b > 0.05}, 'parity', (d.get('parity') or {}).get('bit_exact'))"
done
