set -o pipefail
mkdir -p gpurun_out/hp10
JB_PIECE_KIB=65536 JB_DEBUG=2 timeout -k 10 200 python -u tools/host_probe.py > gpurun_out/hp10/p.log 2>&1 || exit 1
grep -v "nbytes=" gpurun_out/hp10/p.log | grep -E "rep "
grep -v "nbytes=" gpurun_out/hp10/p.log | grep -B 19 -E "pinned rep 2" | head -19
HIP_FORCE_DEV_KERNARG=0 JB_PIECE_KIB=65536 JB_DEBUG=1 timeout -k 10 200 python -u tools/host_probe.py > gpurun_out/hp10/k0.log 2>&1 || exit 1
echo "== HIP_FORCE_DEV_KERNARG=0"; grep -v "nbytes=" gpurun_out/hp10/k0.log | grep -E "rep "
