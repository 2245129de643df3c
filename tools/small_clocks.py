"""k_small phase clocks on the benchmark sentence and on a 4 KiB batch (JB_DEBUG=1
prints them per call; the last of 200 calls is kept)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jieba-go_amd", "python"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gen"))
import jiebahip as J  # noqa: E402
import synth  # noqa: E402

dp, ep = synth.Synth(nwords=350_000).write_files(os.environ.get("TMPDIR", "/tmp"))
tk = J.Tokenizer(J.make_config(dict_path=dp, emit_path=ep))
for text in ("我昨天去上海交通大學與老師討論量子力學", "我昨天去上海交通大學與老師討論量子力學，" * 68):
    for _ in range(200):
        tk.cut_spans(text, True)
    t0 = time.perf_counter_ns()
    for _ in range(200):
        tk.cut_spans(text, True)
    print(len(text.encode()), "bytes:", (time.perf_counter_ns() - t0) / 200 / 1000, "us per call", flush=True)
