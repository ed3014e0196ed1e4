#!/usr/bin/env python3
"""Does a refused (or mis-mapped) IPC export follow VA reuse across processes?
(DESIGN.md §5 "Refused exports").

Rank processes forked from one forkserver inherit its address layout, so a fresh job's
first arena chunk lands at the same VA as the previous job's.  This probe runs job A
(2 ranks: allocate, export, allreduce), keeps A's processes alive with their exports and
mappings open, and meanwhile runs job B (2 ranks, same allocation sequence, so the same
VAs under forkserver) -- then the same with A finished before B, and with B's ranks
spawned (fresh interpreters: ASLR, different VAs).  Per case: both jobs' VAs, every
export / refusal (ESGD_IPC_TRACE_FILE), and B's wrong elements.

  python tools/va_reuse_probe.py [--out gpurun_out/va_reuse] [--repeat 3]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eager-sgd_amd"), os.path.join(ROOT, "tests")]

import mp_workers  # noqa: E402


def start(ctx, world, kw, env):
    q = ctx.Queue()
    port = mp_workers.free_port()
    procs = [ctx.Process(target=mp_workers._entry, args=("gpu_va_reuse", r, world, port, kw, q, env))
             for r in range(world)]
    for p in procs:
        p.start()
    return procs, q


def finish(procs, q, timeout=180):
    status, payload = q.get(timeout=timeout)
    for p in procs:
        p.join(30)
    return status, payload


def trace_lines(path):
    if not os.path.exists(path):
        return []
    out = []
    for line in open(path):
        f = line.split()
        if len(f) >= 8 and f[3] in ("export", "export-refused"):
            out.append({"pid": int(f[2]), "what": f[3], "va": f[7]})
    return out


def case(name, ctx_a, ctx_b, overlap, tmp, env, world=2):
    trace = os.path.join(tmp, f"trace_{name}.log")
    env = dict(env, ESGD_IPC_TRACE_FILE=trace)
    ready, hold = os.path.join(tmp, f"ready_{name}"), os.path.join(tmp, f"hold_{name}")
    pa, qa = start(ctx_a, world, dict(value=1000, ready_file=ready, hold_file=hold if overlap else None), env)
    res = {"case": name}
    if overlap:
        t0 = time.time()
        while not all(os.path.exists(f"{ready}.{r}") for r in range(world)) and time.time() - t0 < 120:
            time.sleep(0.05)
        pb, qb = start(ctx_b, world, dict(value=2000), env)
        sb, outb = finish(pb, qb)
        open(hold, "w").close()
        sa, outa = finish(pa, qa)
    else:
        sa, outa = finish(pa, qa)
        pb, qb = start(ctx_b, world, dict(value=2000), env)
        sb, outb = finish(pb, qb)
    res["job_a"] = outa if sa == "ok" else {"error": str(outa)[-400:]}
    res["job_b"] = outb if sb == "ok" else {"error": str(outb)[-400:]}
    ex = trace_lines(trace)
    res["exports"] = ex
    res["refused"] = [e for e in ex if e["what"] == "export-refused"]
    if sa == "ok" and sb == "ok":
        res["same_vas_across_jobs"] = sorted({o["va"] for o in outa} & {o["va"] for o in outb})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "va_reuse"))
    ap.add_argument("--repeat", type=int, default=3)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    fs = mp.get_context("forkserver")
    fs.set_forkserver_preload(["numpy", "torch", "torch.distributed"])
    sp = mp.get_context("spawn")
    env = dict(os.environ)
    with tempfile.TemporaryDirectory() as tmp:
        for i in range(a.repeat):
            for name, cb, ov in (("forkserver_overlap", fs, True), ("forkserver_sequential", fs, False),
                                 ("spawn_b_overlap", sp, True)):
                r = case(f"{name}_{i}", fs, cb, ov, tmp, env)
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
