set -o pipefail
R=${R:-hp3}
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pieces or masks or multi_device or concurrent or split" > gpurun_out/$R/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/$R/pytest.log; exit 1; }
tail -3 gpurun_out/$R/pytest.log
timeout -k 10 240 python -u tools/host_probe.py > gpurun_out/$R/probe.log 2>&1; grep -v "nbytes=" gpurun_out/$R/probe.log | tail -30
