#!/bin/bash
# Build experiment variants of libjiebahip.so under exp/<name>/ (EXTRA switches).
# usage: tools/variants.sh name1 "-DFOO=1" name2 "-DBAR=2" ...
set -euo pipefail
cd "$(dirname "$0")/../jieba-go_amd"
while [ $# -ge 2 ]; do
  n=$1; x=$2; shift 2
  make -s OUT=../exp/$n OBJ=../exp/obj_$n EXTRA="$x" ../exp/$n/libjiebahip.so &
done
wait
