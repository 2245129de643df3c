#!/bin/bash
# Build the committed sources of a git revision (default HEAD) into var/exp_<name> for A/B runs
# (tools/abtest.sh), without touching the working tree.  usage: tools/build_base.sh [rev] [name]
set -euo pipefail
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
NAME=${2:-base}
T=$(mktemp -d /tmp/jbbase.XXXX)
mkdir -p "$T/jieba-go_amd/csrc" "$T/include"
for f in $(git ls-tree --name-only "$REV" jieba-go_amd/csrc/); do git show "$REV:$f" > "$T/$f"; done
git show "$REV:include/jiebahip.h" > "$T/include/jiebahip.h"
rm -rf "var/exp_$NAME" "jieba-go_amd/_obj_$NAME"
make -s -C jieba-go_amd -j8 SRC="$T/jieba-go_amd/csrc" OUT="../var/exp_$NAME" OBJ="_obj_$NAME"
rm -rf "$T"
ls -la "var/exp_$NAME/libjiebahip.so"
