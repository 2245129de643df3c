# nonzh_block mask fast path: parity subset (non-Han heavy) + headline/S10k A/B vs HEAD
export PYK="random_mixed or edge_cases or invalid_utf8 or synthetic_golden or reference_kats or nonzh_blocks or docs_corpus or real_data or caller_arrays or s10k"
export HLREPS=3 SREPS=2
bash tools/runs/abrun.sh r06at
