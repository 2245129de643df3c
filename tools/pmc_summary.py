#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per kernel.

Writes a JSON with, per kernel: dispatches, mean duration, mean value of each
counter per dispatch, and HBM traffic per launch computed as the guide
prescribes (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) counts 64-B requests
and reads 1/2 of a wide coalesced stream's bytes on gfx950 -> x2; WRITE_SIZE
(KiB) is exact for 16-B/lane stores.  Both raw and corrected values are kept.

usage: pmc_summary.py <pmc dir with p*/run_counter_collection.csv> <out.json> [note ...]
The workload key (bench.py's docs:<bytes>:hmm:prefix form, which bench.py matches
before it uses the traffic) is taken from the passes' bench lines (p1.json).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[a-z_0-9]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][:40]


def main():
    d, out = sys.argv[1], sys.argv[2]
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    res = {}
    for k, cs in vals.items():
        e = {"dispatches": max(len(v) for v in cs.values()),
             "mean_ms_profiled": sum(dur[k].values()) / max(1, len(dur[k]))}
        for c, v in cs.items():
            e[c] = sum(v) / len(v)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["fetch_bytes_raw"] = e["FETCH_SIZE"] * 1024
            e["fetch_bytes_x2"] = e["FETCH_SIZE"] * 1024 * 2
            e["write_bytes"] = e["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = e["fetch_bytes_x2"] + e["write_bytes"]
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e:
            t = e["TCC_HIT_sum"] + e["TCC_MISS_sum"]
            e["l2_hit_rate"] = e["TCC_HIT_sum"] / t if t else None
        res[k] = e
    meta = {"source": d, "note": " ".join(sys.argv[3:]),
            "method": "rocprofv3 --kernel-trace --pmc, one counter group per run; FETCH_SIZE x2 (gfx950)"}
    wkey = None
    try:
        with open(os.path.join(d, "p1.json")) as f:
            wkey = json.loads(f.read().strip().splitlines()[-1]).get("workload_key")
    except (OSError, ValueError, IndexError):
        pass
    with open(out, "w") as f:
        json.dump({"meta": meta, "workload_key": wkey, "kernels": res}, f, indent=1)
    for k, e in sorted(res.items(), key=lambda x: -x[1]["mean_ms_profiled"]):
        print(f"{k:22s} ms={e['mean_ms_profiled']:.3f} " + " ".join(
            f"{c}={e[c]:.4g}" for c in ("hbm_bytes_per_launch", "l2_hit_rate", "TCC_EA0_RDREQ_sum", "TCC_HIT_sum",
                                        "TCC_MISS_sum", "SQ_INSTS_VMEM_RD", "SQ_WAVES", "SQ_INSTS_VALU",
                                        "TCP_TCC_READ_REQ_sum", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
                                        "SQ_WAVE_CYCLES") if e.get(c) is not None))


if __name__ == "__main__":
    main()
