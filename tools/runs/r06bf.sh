# k_nonzh: a block inside its alnum chunk tokenized from the chunk's own 16 bytes (no loads) vs HEAD
export PYK="nonzh or random_mixed or edge_cases or invalid_utf8 or synthetic_golden or reference_kats or docs_corpus or caller_arrays or s10k or small_batches"
export HLREPS=3 SREPS=1
bash tools/runs/abrun.sh r06bf
