#!/usr/bin/env python3
"""Summarise tools/tlb_counters.sh: every counter per reduction call (the 5 calls of
bench.py's PMC child, each call = its 64 MiB window dispatches summed), per GiB of
algorithmic traffic ((8 + 1) x bucket bytes per call), and the kernel trace's per-call and
per-window durations.  FETCH_SIZE is doubled (gfx950 counts half a wide streaming read,
MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import json
import os
import statistics
import sys

CALLS = 5
TREE = "k_tree_sum_buf"


def rows(d, name):
    out = []
    for f in glob.glob(os.path.join(d, "**", name), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main(o):
    res = {}
    for mib in (256, 1024):
        algo = 9 * mib * (1 << 20)
        ent = {"algo_bytes_per_call": algo, "counters_per_call": {}, "per_GiB": {}}
        for p in (1, 2, 3, 4, 5, 7, 8):
            d = os.path.join(o, f"{mib}MiB_p{p}")
            acc = {}
            for r in rows(d, "*counter_collection.csv"):
                if TREE in r.get("Kernel_Name", ""):
                    acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            for k, v in acc.items():
                per = v / CALLS
                if k == "FETCH_SIZE":
                    per = 2 * per * 1024   # KiB, halved on gfx950 -> bytes
                elif k == "WRITE_SIZE":
                    per = per * 1024
                ent["counters_per_call"][k] = per
                ent["per_GiB"][k] = per / (algo / (1 << 30))
        kt = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in
                    rows(os.path.join(o, f"{mib}MiB_p6"), "*kernel_trace.csv") if TREE in r.get("Kernel_Name", ""))
        if kt:
            w = len(kt) // CALLS
            durs = [(e - s) / 1e3 for s, e in kt]
            calls = [sum(durs[i * w:(i + 1) * w]) for i in range(CALLS)]
            ent["windows_per_call"] = w
            ent["call_us"] = [round(c, 1) for c in calls]
            ent["frac_of_8TBs_median_call"] = round(algo / (statistics.median(calls) * 1e-6) / 8e12, 4)
            # window position within a call: median over calls
            ent["window_us_by_position"] = [round(statistics.median(durs[i * w + j] for i in range(CALLS)), 1)
                                            for j in range(w)]
        c = ent["counters_per_call"]
        for kind in ("RD", "WR"):   # average requests in flight / latency proxy per request
            lv, rq = c.get(f"TCC_EA0_{kind}REQ_LEVEL_sum"), c.get(f"TCC_EA0_{kind}REQ_sum")
            if lv and rq:
                ent[f"ea_{kind.lower()}_level_per_request"] = round(lv / rq, 1)
        res[f"{mib}MiB"] = ent
    miss = {k: res[k]["per_GiB"].get("TCP_UTCL1_TRANSLATION_MISS_sum") for k in res}
    res["utcl1_miss_per_GiB_ratio_1024_over_256"] = (miss["1024MiB"] / miss["256MiB"]
                                                     if miss.get("256MiB") and miss.get("1024MiB") else None)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
