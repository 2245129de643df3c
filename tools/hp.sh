set -o pipefail
mkdir -p gpurun_out/hp2
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pieces or masks or multi_device or concurrent or split" > gpurun_out/hp2/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/hp2/pytest.log; exit 1; }
tail -3 gpurun_out/hp2/pytest.log
timeout -k 10 240 python -u tools/host_probe.py > gpurun_out/hp2/probe.log 2>&1; tail -25 gpurun_out/hp2/probe.log
