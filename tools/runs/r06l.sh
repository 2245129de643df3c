# the whole GPU suite on the current build
set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06l/pytest_gpu.log 2>&1 || exit 1
