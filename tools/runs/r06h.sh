# S10k under rocprofv3: real kernel durations and the gaps between them in the graph replay
set -o pipefail
mkdir -p gpurun_out/r06h
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06h/s10k_h0 -o s10k -- python3 $GRAFT_REPO_ROOT/bench.py --workload s10k --hmm 0 --steps 200 --warmup 20 --no-e2e --no-parity --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r06h/s10k_h0.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06h/s10k_h0.err || exit 1
