#!/bin/bash
# Build experiment variants of libjiebahip.so under var/<name>/ (EXTRA switches).
# usage: tools/variants.sh name1 "-DFOO=1" name2 "-DBAR=2" ...
set -euo pipefail
cd "$(dirname "$0")/../jieba-go_amd"
while [ $# -ge 2 ]; do
  n=$1; x=$2; shift 2
  make -s OUT=../var/$n OBJ=../var/${n}_obj EXTRA="$x" ../var/$n/libjiebahip.so &
done
wait
