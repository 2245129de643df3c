# full GPU suite on the current build
set -o pipefail
mkdir -p gpurun_out/r06ae
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r06ae/pytest_gpu.log 2>&1
