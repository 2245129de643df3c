# host path at several piece sizes (diagnostic): usage bash tools/hp_piece.sh
set -o pipefail
mkdir -p gpurun_out/hpp
for kib in 1048576 262144 65536; do
  JB_PIECE_KIB=$kib JB_DEBUG=2 timeout -k 10 200 python -u tools/host_probe.py > gpurun_out/hpp/p$kib.log 2>&1 || exit 1
  echo "== piece $kib KiB"; grep -v "nbytes=" gpurun_out/hpp/p$kib.log | grep -E "rep 3|pinned rep 2|host range" | tail -4
  grep -B 30 "pinned rep 2" gpurun_out/hpp/p$kib.log | grep "^\[jb\]   " | tail -8
done
