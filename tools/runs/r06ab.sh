# S10k kernel trace of graph-replayed steps (per-kernel durations and the gaps between them), HMM off and on
set -o pipefail
mkdir -p gpurun_out/${TAG:-r06ab}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for h in 0 1; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG:-r06ab}/kt$h -o s10k -- python3 -u bench.py --workload s10k --hmm $h --steps 100 --warmup 5 --no-e2e --no-parity --no-profile > gpurun_out/${TAG:-r06ab}/kt$h.log 2>&1 || exit 1
done
