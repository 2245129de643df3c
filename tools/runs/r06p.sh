# u32 spans (jb_cut_batch_into32) and the AVX-512 decoder: parity on the host paths, then the host probe x2
set -o pipefail
mkdir -p gpurun_out/r06p
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "into32 or packed_spans or cut_batch_into or multi_device or one_large or c_abi or cpp_tok or config4 or small_batches or concurrent" > gpurun_out/r06p/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06p/probe_$rep.txt 2>&1 || exit 1
done
