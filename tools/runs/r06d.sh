# packed spans (2 B per token): parity on the host paths, then the host probe
set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "packed_spans or cut_batch_into or multi_device or one_large or c_abi or cpp_tok or golden or mini_dict or random_mixed or long_document" \
  > gpurun_out/r06d/pytest.log 2>&1 || exit 1
for sp in 1 0; do
  JB_SPAN_PACK=$sp JB_DEBUG=2 timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06d/host_probe_pack$sp.txt 2>&1 || exit 1
done
