# host path: non-temporal staging and decode stores, decode threads; A/B on one box
set -o pipefail
mkdir -p gpurun_out/r06n
P=$PWD
for rep in 1 2; do
  JB_LIB=$P/var/exp_pack/libjiebahip.so timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06n/pack_$rep.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06n/nt_$rep.txt 2>&1 || exit 1
  JB_NT_STAGE=0 timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06n/ntdec_$rep.txt 2>&1 || exit 1
  JB_DECODE_THREADS=12 timeout -k 10 300 python -u tools/host_probe.py > gpurun_out/r06n/nt12_$rep.txt 2>&1 || exit 1
done
