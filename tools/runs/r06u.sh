# S10k: kernel trace of graph-replayed steps; A/B of k_zh's claim skip (lib) against HEAD (var/exp_base)
set -o pipefail
mkdir -p gpurun_out/r06u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06u/kt -o s10k -- python3 -u bench.py --workload s10k --hmm 0 --steps 50 --warmup 5 --no-e2e --no-parity --no-profile > gpurun_out/r06u/kt.log 2>&1 || exit 1
for r in 1 2 3; do for h in 0 1; do for v in base lib; do
  if [ $v = lib ]; then L=$PWD/jieba-go_amd/lib/libjiebahip.so; else L=$PWD/var/exp_$v/libjiebahip.so; fi
  JB_LIB=$L timeout -k 10 300 python -u bench.py --workload s10k --hmm $h --steps 300 --warmup 20 --no-e2e $( [ $r = 1 ] && [ $v = lib ] || echo --no-parity ) \
     > gpurun_out/r06u/t_h${h}_${v}_$r.json 2> gpurun_out/r06u/t_h${h}_${v}_$r.err || exit 1
done; done; done
