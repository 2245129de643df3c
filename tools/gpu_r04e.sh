set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r04e/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04e/pytest.log; exit 1; }
tail -2 gpurun_out/r04e/pytest.log
TAG=r04e/ab REPS=2 bash tools/envab.sh JB_ZH_WIDE=0 -
