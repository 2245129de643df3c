#!/bin/bash
# One GPU call, made of the steps named by the arguments, in order.  Each step has its own
# time limit, and the call stops at the first step that fails (no retries).  Output goes to
# gpurun_out/$RUN/.
#   test              the whole -m gpu suite on the in-tree library
#   test:EXPR         the -m gpu tests matching -k EXPR
#   testv:V           the whole -m gpu suite on variant V (var/exp_V)
#   ab:V1,V2,...      A/B of the headline bench: lib against each var/exp_V, REPS rounds (tools/abtest.sh)
#   abw:W:V1,...      the same on workload W (sentence, s10k, long-oov, ...)
#   req:V             one PMC pass of L1->L2 read requests and L1 accesses per kernel (V = lib or a variant)
#   pmc               every PMC pass of the headline (tools/final_profile.sh: summary, stats, bench line)
#   bench             the default bench line
#   cfg               the other BASELINE configs (tools/configs.sh)
#   smoke             __graft_entry__.smoke()
#   roundend          tools/round_end.sh (smoke, final profile, configs, sentence stats)
#   long5b            config 5b: one SQ PMC pass and rocprofv3 kernel stats
#   conc              the concurrent-Cut test (16 threads x 1,000 jb_cut calls), its rates printed
#   hostprobe         the host-batch tests and tools/host_probe.py (host-memory pipeline clocks)
#   stamps:V          per-wave phase clocks of the headline from STAMPS build V (lib_st or a variant)
#   envab:W:K=V       workload W with the in-tree library, default env against K=V, REPS rounds
#   sclk:V            k_small phase clocks (JB_DEBUG) on the benchmark sentence and a 4 KiB batch, library V
# usage: RUN=r05a bash tools/gpu.sh test ab:nosort req:lib req:nosort
set -o pipefail
cd "$(dirname "$0")/.."
RUN=${RUN:-g}
OUT=gpurun_out/$RUN
mkdir -p "$OUT"
export TMPDIR=/tmp
libof() { if [ "$1" = lib ]; then echo "$PWD/jieba-go_amd/lib/libjiebahip.so"; else echo "$PWD/var/exp_$1/libjiebahip.so"; fi; }
fail() { echo "FAILED: $1"; tail -30 "$2"; exit 1; }
for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    test)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
        > "$OUT/pytest.log" 2>&1 || fail "$step" "$OUT/pytest.log"
      tail -1 "$OUT/pytest.log" ;;
    test:*)
      k=${step#test:}
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -k "$k" --timeout 150 --timeout-method thread \
        > "$OUT/pytest_k.log" 2>&1 || fail "$step" "$OUT/pytest_k.log"
      tail -1 "$OUT/pytest_k.log" ;;
    testv:*)
      v=${step#testv:}
      JB_LIB=$(libof "$v") timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
        > "$OUT/pytest_$v.log" 2>&1 || fail "$step" "$OUT/pytest_$v.log"
      tail -1 "$OUT/pytest_$v.log" ;;
    ab:*)
      IFS=, read -ra vs <<< "${step#ab:}"
      TAG=$RUN/ab REPS=${REPS:-2} bash tools/abtest.sh lib "${vs[@]}" || fail "$step" /dev/null ;;
    abw:*)
      rest=${step#abw:}; w=${rest%%:*}
      IFS=, read -ra vs <<< "${rest#*:}"
      for r in $(seq 1 ${REPS:-2}); do
        for v in lib "${vs[@]}"; do
          JB_LIB=$(libof "$v") timeout -k 10 300 python bench.py --workload "$w" --no-e2e --no-parity ${BENCH_ARGS:-} \
            > "$OUT/abw_${w}_$v.$r.json" 2> "$OUT/abw_${w}_$v.$r.err" || fail "$step" "$OUT/abw_${w}_$v.$r.err"
          python -c "import json; d=json.load(open('$OUT/abw_${w}_$v.$r.json')); print('$w', '$v', d['ms_per_step'], {k: round(x, 4) for k, x in (d.get('kernels_ms') or {}).items()})"
        done
      done ;;
    req:*)
      v=${step#req:}
      JB_LIB=$(libof "$v") timeout -s KILL 180 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
        -d "$OUT/req_$v" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-parity --no-profile --no-e2e --no-latency \
        > "$OUT/req_$v.log" 2>&1 || fail "$step" "$OUT/req_$v.log"
      python3 - "$OUT/req_$v" <<'EOF'
import csv, glob, re, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[a-z_0-9]+)", r["Kernel_Name"])
        acc[m.group(1) if m else r["Kernel_Name"][:30]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in ("k_mark_walk", "k_zh"):
    print(k, {c: "%.1fM" % (sum(v) / len(v) / 1e6) for c, v in acc[k].items()})
EOF
      ;;
    pmc)
      TAG=$RUN/fp bash tools/final_profile.sh || fail "$step" /dev/null ;;
    bench)
      timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || fail "$step" "$OUT/bench.err"
      head -c 1500 "$OUT/bench.json"; echo ;;
    cfg)
      TAG=$RUN/cfg bash tools/configs.sh || fail "$step" /dev/null ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail "$step" "$OUT/smoke.log"
      tail -1 "$OUT/smoke.log" ;;
    roundend)
      TAG=$RUN/re bash tools/round_end.sh || fail "$step" /dev/null ;;
    long5b)
      timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/l5b_pmc" -o run --output-format csv -- \
        python3 bench.py --workload long-oov --steps 1 --warmup 1 --no-parity --no-e2e --no-profile \
        > "$OUT/l5b_pmc.log" 2>&1 || fail "$step" "$OUT/l5b_pmc.log"
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/l5b_stats" -o run --output-format csv -- \
        python3 bench.py --workload long-oov --steps 3 --warmup 1 --no-parity --no-e2e --no-profile \
        > "$OUT/l5b_stats.log" 2>&1 || fail "$step" "$OUT/l5b_stats.log"
      find "$OUT/l5b_stats" -name "*kernel_stats.csv" | head -1 ;;
    conc)
      timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k concurrent -s \
        --timeout 150 --timeout-method thread > "$OUT/conc.log" 2>&1 || fail "$step" "$OUT/conc.log"
      grep -E "JB_SMALL_SLOTS|serial threads|concurrent threads" "$OUT/conc.log" ;;
    hostprobe)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
        -k "pieces or masks or multi_device or split" > "$OUT/hp_pytest.log" 2>&1 || fail "$step" "$OUT/hp_pytest.log"
      timeout -k 10 240 python -u tools/host_probe.py > "$OUT/hp_probe.log" 2>&1 || fail "$step" "$OUT/hp_probe.log"
      grep -v "nbytes=" "$OUT/hp_probe.log" | tail -30 ;;
    stamps:*)
      v=${step#stamps:}
      if [ "$v" = lib_st ]; then L=$PWD/jieba-go_amd/lib_st/libjiebahip.so; else L=$(libof "$v"); fi
      JB_LIB=$L JB_STAMPS=1 timeout -k 10 200 python -u bench.py --no-parity --no-e2e --no-profile --no-latency \
        --steps 2 --warmup 1 ${BENCH_ARGS:-} > "$OUT/stamps_$v.json" 2> "$OUT/stamps_$v.err" || fail "$step" "$OUT/stamps_$v.err"
      grep "\[jb\]" "$OUT/stamps_$v.err" | tail -3 ;;
    envab:*)
      rest=${step#envab:}; w=${rest%%:*}; kv=${rest#*:}
      for r in $(seq 1 ${REPS:-2}); do
        for e in "" "$kv"; do
          tag=$( [ -z "$e" ] && echo default || echo "${e//=/_}" )
          env $e timeout -k 10 300 python bench.py --workload "$w" --no-e2e --no-parity ${BENCH_ARGS:-} \
            > "$OUT/envab_${w}_$tag.$r.json" 2> "$OUT/envab_${w}_$tag.$r.err" || fail "$step" "$OUT/envab_${w}_$tag.$r.err"
          python -c "import json; d=json.load(open('$OUT/envab_${w}_$tag.$r.json')); print('$w', '$tag', d['ms_per_step'], {k: round(x, 4) for k, x in (d.get('kernels_ms') or {}).items()})"
        done
      done ;;
    sclk:*)
      v=${step#sclk:}
      JB_LIB=$(libof "$v") JB_DEBUG=1 timeout -k 10 200 python -u tools/small_clocks.py > "$OUT/sclk_$v.log" 2> "$OUT/sclk_$v.err" \
        || fail "$step" "$OUT/sclk_$v.err"
      cat "$OUT/sclk_$v.log"; grep "k_small" "$OUT/sclk_$v.err" | tail -1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all done $(date +%T)"
