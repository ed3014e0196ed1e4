#!/usr/bin/env python3
"""Summarise an ESGD_IPC_TRACE_FILE log of a test session (does the
refused export follow the forkserver's inherited address layout?): how many processes
exported arena chunks, how many distinct virtual addresses their first exports used, how
often two processes exported the same VA (over the session, and within one job: pids
that opened each other's handles), and every refused export with its VA and pid (refusals simulated by ESGD_FAIL_EXPORTS for
the fallback tests are counted apart; a log from before that tag existed lists them as
refused).

  python tools/ipc_export_stats.py <trace.log> [--csv exports.csv]
"""
import argparse
import collections
import json

ap = argparse.ArgumentParser()
ap.add_argument("log")
ap.add_argument("--csv", default=None, help="write pid,what,va,bytes of every export / refusal")
a = ap.parse_args()

ex = collections.defaultdict(list)      # pid -> [va of each export, in order]
refused = []
simulated = 0                           # ESGD_FAIL_EXPORTS refusals (the fallback tests)
opened = collections.defaultdict(set)   # pid -> handles it opened (bytes 0-11 = exporter VA + pid)
handle_owner = {}                       # handle -> exporting pid
rows = []
for line in open(a.log):
    f = line.split()
    if len(f) < 12 or f[0] != "esgd-ipc":
        continue
    pid, what, va, nbytes, h = int(f[2]), f[3], f[7], int(f[9]), f[11]
    if what == "export":
        ex[pid].append(va)
        handle_owner[h] = pid
        rows.append((pid, what, va, nbytes))
    elif what == "export-refused-simulated":
        simulated += 1
    elif what == "export-refused":
        refused.append({"pid": pid, "va": va, "bytes": nbytes})
        rows.append((pid, what, va, nbytes))
    elif what == "open":
        opened[pid].add(h)

pids = sorted(ex)
first = collections.Counter(ex[p][0] for p in pids)
any_va = collections.Counter(v for p in pids for v in set(ex[p]))
# jobs: connected components of "pid opened a handle exported by pid"
parent = {p: p for p in pids}


def find(p):
    while parent[p] != p:
        parent[p] = parent[parent[p]]
        p = parent[p]
    return p


for p, hs in opened.items():
    for h in hs:
        q = handle_owner.get(h)
        if q is not None and p in parent and q in parent:
            parent[find(p)] = find(q)
jobs = collections.defaultdict(list)
for p in pids:
    jobs[find(p)].append(p)
same_va_jobs = 0
for members in jobs.values():
    if len(members) < 2:
        continue
    c = collections.Counter(v for p in members for v in set(ex[p]))
    if any(n > 1 for n in c.values()):
        same_va_jobs += 1
out = {
    "exporting_processes": len(pids),
    "exports": sum(len(v) for v in ex.values()),
    "distinct_first_export_vas": len(first),
    "most_common_first_vas": first.most_common(5),
    "vas_exported_by_more_than_one_process": sum(1 for n in any_va.values() if n > 1),
    "distinct_vas": len(any_va),
    "multi_rank_jobs": sum(1 for m in jobs.values() if len(m) > 1),
    "jobs_where_two_ranks_exported_the_same_va": same_va_jobs,
    "refused": refused,
    "simulated_refusals": simulated,
}
print(json.dumps(out, indent=1))
if a.csv:
    with open(a.csv, "w") as fh:
        fh.write("pid,what,va,bytes\n")
        for r in rows:
            fh.write("%d,%s,%s,%d\n" % r)
