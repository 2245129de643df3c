# k_zh group size at 1 GiB with the wide form (JB_ZH_GROUP, runtime: at most the compiled 6 KiB), A/B x2
set -o pipefail
O=gpurun_out/r06ap; mkdir -p $O
for r in 1 2; do for g in 6144 5632 5120; do
  JB_ZH_WIDE=1 JB_ZH_GROUP=$g timeout -k 10 300 python -u bench.py --no-e2e --no-parity --steps 20 --warmup 3 > $O/g${g}_$r.json 2> $O/g${g}_$r.err || exit 1
done; done
