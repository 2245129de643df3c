# host path: AVX-512 span decoder with streaming stores (lib) against the packed-spans commit (exp_pack); parity on the host paths first
set -o pipefail
mkdir -p gpurun_out/r06o
P=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "packed_spans or cut_batch_into or multi_device or one_large or c_abi or cpp_tok or config4" > gpurun_out/r06o/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  JB_LIB=$P/var/exp_pack/libjiebahip.so timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06o/pack_$rep.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06o/avx_$rep.txt 2>&1 || exit 1
  JB_DECODE_AVX512=0 timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06o/ntscalar_$rep.txt 2>&1 || exit 1
done
