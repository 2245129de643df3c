"""Print ms/step, the two big kernels and parity of bench JSON lines (A/B summaries)."""
import glob
import json
import sys

for f in sorted(sum((glob.glob(p) for p in sys.argv[1:]), [])):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            k = d.get("kernels_ms") or {}
            print(f.split("/")[-1], d["ms_per_step"], "mw", k.get("k_mark_walk"), "zh", k.get("k_zh"),
                  "bit_exact", (d.get("parity") or {}).get("bit_exact"))
