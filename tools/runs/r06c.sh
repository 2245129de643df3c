# balanced k_zh groups + k_nonzh word sharing: parity, then A/B by shard size
set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "edge_cases or nonzh or zh_groups or docs_corpus or zh_blocks_from_lane or config4 or s10k or long_document or one_large or packed_spans or long_wait" \
  > gpurun_out/r06c/pytest.log 2>&1 || exit 1
run() {  # name, bench args..., then env after --
  local name=$1; shift
  timeout -k 10 300 "$@" > gpurun_out/r06c/$name.json 2> gpurun_out/r06c/$name.err || exit 1
}
B="python -u bench.py --steps 30 --warmup 3 --no-e2e --no-latency"
for rep in 1 2; do
  for n in 8 4 2; do
    run s${n}_off$rep env JB_ZH_BALANCE=0 $B --shard-of $n --no-parity
    run s${n}_on$rep env JB_ZH_BALANCE=1 $B --shard-of $n $( [ $rep = 2 ] && echo --no-parity )
  done
  run g1_off$rep env JB_ZH_BALANCE=0 $B --no-parity
  run g1_on$rep env JB_ZH_BALANCE=1 $B $( [ $rep = 2 ] && echo --no-parity )
done
for sp in 0 1; do
  JB_SPAN_PACK=$sp JB_DEBUG=1 timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06c/host_probe_pack$sp.txt 2>&1 || exit 1
done
