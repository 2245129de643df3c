set -e
for cap in 2304 3584 4608; do
  make -s -C jieba-go_amd clean && make -s -C jieba-go_amd STAMPS=1 ZH_CAP=$cap -j8 > /dev/null 2>&1
  echo "== cap $cap"
  SPECS="JB_ABLATE=256" PAR_MIB=1 STEPS=2 TAG=r2f_$cap bash tools/envsweep.sh
done
