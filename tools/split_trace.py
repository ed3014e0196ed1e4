"""Split a rocprofv3 kernel trace of `bench.py` into its two shapes: the gate calls
(8 x 256 MiB, run as 64 MiB windows: four dispatches per call), which the bench runs
first, right after the last fill kernel, and the C2 launches (8 x 64 MiB, one dispatch
each) that follow them.
usage: split_trace.py RUN_kernel_trace.csv TAG > kernel_trace_split.json"""
import csv
import json
import statistics
import sys

WINDOWS_PER_GATE_CALL = 4   # 256 MiB / kWindowBytes (reduce_kernels.hip)
GATE_CALLS = 130            # bench.gate_256: 10 warm-up + 20 + 100 calls


def main():
    path, tag = sys.argv[1], sys.argv[2]
    rows = []
    with open(path) as f:
        for row in csv.DictReader(f):
            rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row["Kernel_Name"]))
    rows.sort()
    last_fill = max(i for i, r in enumerate(rows) if "k_fill_uniform" in r[2])
    tree = [r for i, r in enumerate(rows) if "k_tree_sum_buf<esgd::F32, 8, 4, 2, 16, false" in r[2] and i > last_fill]
    # bench.py runs the gate leg first (10 warm-up + 20 timed-singly + 100 back-to-back
    # calls of four 64 MiB windows), then the C2 warm-up and timed launches, then host_e2e
    # (whose launches follow PCIe copies, ms apart)
    gw = tree[:GATE_CALLS * WINDOWS_PER_GATE_CALL]
    calls = [gw[j:j + WINDOWS_PER_GATE_CALL] for j in range(0, len(gw), WINDOWS_PER_GATE_CALL)]
    rest = tree[GATE_CALLS * WINDOWS_PER_GATE_CALL:]
    c2r = rest[:1]
    for r in rest[1:]:
        if r[0] - c2r[-1][1] > 1_000_000:   # the host_e2e leg
            break
        c2r.append(r)
    c2 = [(r[1] - r[0]) / 1e3 for r in c2r]
    # a call's kernel time: its windows' durations summed (the gaps between them are
    # dispatch gaps, a few us; the span also swallows host syncs between timed loops)
    gate = [sum(r[1] - r[0] for r in c) / 1e3 for c in calls]
    span = [(c[-1][1] - c[0][0]) / 1e3 for c in calls]
    out = {"source": "rocprofv3 --kernel-trace --stats of `bench.py --no-pmc --no-cpu-baseline "
                     "--steps 100` (%s)" % tag,
           "k_tree_sum_buf<F32,8,4,nt,sc1>": {}}
    for key, xs, b, unit in (("C2_8x64MiB", c2, 9 * 64 << 20, "dispatches"),
                             ("gate_8x256MiB", gate, 9 * 256 << 20, "calls (4 windows each)")):
        if not xs:
            continue
        avg = statistics.fmean(xs)
        out["k_tree_sum_buf<F32,8,4,nt,sc1>"][key] = {
            unit: len(xs), "avg_us": round(avg, 2), "median_us": round(statistics.median(xs), 2),
            "algo_bytes": b, "frac_of_8TBs": round(b / (avg * 1e-6) / 8e12, 4)}
    if span:
        out["k_tree_sum_buf<F32,8,4,nt,sc1>"]["gate_8x256MiB"]["median_span_us"] = round(statistics.median(span), 2)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
