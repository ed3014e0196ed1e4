"""Split a rocprofv3 kernel trace of `bench.py` into its two shapes: the C2 launches
(8 x 64 MiB, one dispatch each) and the gate calls (8 x 256 MiB, run as 64 MiB windows:
four dispatches per call).  The bench fills the gate buckets after the C2 loop, so the
tree-kernel dispatches after the last fill kernel are the gate's; a call's time is the
span from its first window's start to its last window's end.
usage: split_trace.py RUN_kernel_trace.csv TAG > kernel_trace_split.json"""
import csv
import json
import statistics
import sys

WINDOWS_PER_GATE_CALL = 4   # 256 MiB / kWindowBytes (reduce_kernels.hip)


def main():
    path, tag = sys.argv[1], sys.argv[2]
    rows = []
    with open(path) as f:
        for row in csv.DictReader(f):
            rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row["Kernel_Name"]))
    rows.sort()
    last_fill = max(i for i, r in enumerate(rows) if "k_fill_uniform" in r[2])
    tree = [(i, r) for i, r in enumerate(rows) if "k_tree_sum_buf<esgd::F32, 8, 4, 2, 16, false" in r[2]]
    c2 = [(r[1] - r[0]) / 1e3 for i, r in tree if i < last_fill]
    # after the gate's fills the bench also runs host_e2e, whose tree launches are single
    # (serial leg) or read host memory for ms (esgd_reduce_host): a gate call is a run of
    # exactly four back-to-back HBM windows (gaps of a few us)
    gw = [r for i, r in tree if i > last_fill and r[1] - r[0] < 1_000_000]
    runs, cur = [], []
    for r in gw:
        if cur and r[0] - cur[-1][1] > 50_000:
            runs.append(cur)
            cur = []
        cur.append(r)
    if cur:
        runs.append(cur)
    calls = [run[j:j + WINDOWS_PER_GATE_CALL] for run in runs if len(run) % WINDOWS_PER_GATE_CALL == 0
             for j in range(0, len(run), WINDOWS_PER_GATE_CALL)]
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
