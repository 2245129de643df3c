# LDS counters of the headline kernels (one rocprofv3 --pmc pass, kernel trace only)
set -o pipefail
mkdir -p gpurun_out/r06k
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL \
  -d gpurun_out/r06k/p1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-parity --no-profile --no-e2e --no-latency \
  > gpurun_out/r06k/p1.json 2> gpurun_out/r06k/p1.err || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_ATOMIC SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES \
  -d gpurun_out/r06k/p2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-parity --no-profile --no-e2e --no-latency \
  > gpurun_out/r06k/p2.json 2> gpurun_out/r06k/p2.err || exit 1
