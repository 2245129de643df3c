# host path timelines (per piece: H2D done, kernels done, results back) for spans, u32 spans and masks
set -o pipefail
mkdir -p gpurun_out/r06q
JB_DEBUG=2 timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06q/probe.txt 2>&1 || exit 1
