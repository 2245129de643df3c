# k_nonzh: chunk neighbourhoods prefetched (walk-back step, block end, block bytes) vs HEAD
export PYK="random_mixed or edge_cases or invalid_utf8 or synthetic_golden or reference_kats or nonzh_blocks or docs_corpus or caller_arrays or s10k or small_batches or long_document or empty_batch or repeat_runs"
export HLREPS=3 SREPS=2
bash tools/runs/abrun.sh r06aw
