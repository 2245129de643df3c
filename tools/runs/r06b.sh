# k_zh tail / group sweep at one GPU's shard of an 8-GPU job (128 MiB), A/B x2
set -o pipefail
mkdir -p gpurun_out/r06b
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --shard-of 8 --no-parity --no-e2e --no-latency \
     > gpurun_out/r06b/$name.json 2> gpurun_out/r06b/$name.err || exit 1
}
for rep in 1 2; do
  run base$rep JB_X=0
  run t16k2k$rep JB_ZH_TAIL_KIB=16384 JB_ZH_TAIL_GROUP=2048
  run t32k2k$rep JB_ZH_TAIL_KIB=32768 JB_ZH_TAIL_GROUP=2048
  run t16k3k$rep JB_ZH_TAIL_KIB=16384 JB_ZH_TAIL_GROUP=3072
  run t8k1k$rep JB_ZH_TAIL_KIB=8192 JB_ZH_TAIL_GROUP=1024
  run g3k$rep JB_ZH_GROUP=3072 JB_ZH_WIDE=1
  run g4k$rep JB_ZH_GROUP=4096 JB_ZH_WIDE=1
done
JB_DEBUG=2 timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06b/host_probe.txt 2>&1
python - <<'PY' > gpurun_out/r06b/cpu.txt 2>&1
import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))
print(open('/proc/cpuinfo').read().split('\n\n')[0])
PY
