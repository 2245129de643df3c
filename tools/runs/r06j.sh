# list the PMC counters of this gfx950 (names for the LDS passes)
set -o pipefail
mkdir -p gpurun_out/r06j
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r06j/counters.txt 2>&1 || exit 1
