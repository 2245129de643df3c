#!/bin/bash
# Build experiment variants of libjiebahip.so under var/exp_<name>/ (EXTRA switches); var/
# travels to the GPU box, exp/ does not.  usage: tools/variants.sh name1 "-DFOO=1" name2 "-DBAR=2" ...
set -euo pipefail
cd "$(dirname "$0")/../jieba-go_amd"
while [ $# -ge 2 ]; do
  n=$1; x=$2; shift 2
  make -s OUT=../var/exp_$n OBJ=../var/obj_$n EXTRA="$x" ../var/exp_$n/libjiebahip.so &
done
wait
