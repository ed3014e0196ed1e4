"""Split a rocprofv3 kernel trace of `bench.py` by launch shape: the C2 (8 x 64 MiB) and
gate (8 x 256 MiB) launches of the production tree kernel run the same code object, so
rocprof's per-kernel statistics mix them; durations separate them cleanly (~92 vs ~380
us).  usage: split_trace.py RUN_kernel_trace.csv TAG > kernel_trace_split.json"""
import csv
import json
import statistics
import sys


def main():
    path, tag = sys.argv[1], sys.argv[2]
    durs = []
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if "k_tree_sum_buf<esgd::F32, 8, 4, 2, 16, false" in name:
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    c2 = [d for d in durs if d < 200]
    gate = [d for d in durs if d >= 200]
    out = {"source": "rocprofv3 --kernel-trace --stats of `bench.py --no-pmc --no-cpu-baseline "
                     "--steps 100` (%s)" % tag,
           "k_tree_sum_buf<F32,8,4,nt,sc1>": {}}
    for key, xs, b in (("C2_8x64MiB", c2, 9 * 64 << 20), ("gate_8x256MiB", gate, 9 * 256 << 20)):
        if not xs:
            continue
        avg = statistics.fmean(xs)
        out["k_tree_sum_buf<F32,8,4,nt,sc1>"][key] = {
            "dispatches": len(xs), "avg_us": round(avg, 2), "median_us": round(statistics.median(xs), 2),
            "algo_bytes": b, "frac_of_8TBs": round(b / (avg * 1e-6) / 8e12, 4)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
