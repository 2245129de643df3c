# per-GPU rate of one rank's shard (2/4/8 GPUs) and the full GiB on one box, after the k_nonzh change
set -o pipefail
O=gpurun_out/r06ba; mkdir -p $O
for n in 1 2 4 8; do
  a="--shard-of $n"; [ $n = 1 ] && a=""
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 $a --no-e2e --no-latency > $O/shard$n.json 2> $O/shard$n.err || exit 1
done
