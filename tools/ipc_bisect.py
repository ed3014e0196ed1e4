"""Bisect the IPC re-export fault ("IPC arena").

Round 2 found that once a bucket that peers had mapped is freed and its memory re-used by
a bigger bucket that is exported again, peers read wrong data through their fresh
mappings -- in esgd (8 ranks, a 16 MiB bucket, then a 256 MiB one), but not in a plain
HIP reproducer.  This script starts from that reproducer and adds esgd's steps one at a
time, cumulatively, in ONE GPU session:

  plain        export, peers map, read the whole buffer through the mapping with the tree
               kernel, close, free; then the same with a bigger buffer
  +hostreg     a host page registered with hipHostRegisterMapped (the node segment)
  +nbstream    the reads on a non-blocking stream (the round stream)
  +suballoc    the bucket at a 2 MiB offset inside a bigger allocation (arena carving)
  +keepmaps    mappings kept open and cached per handle, never closed before the free
               (the (peer, chunk) mapping cache)
  +engine      the esgd communicator up (progress thread, registered segment, a schedule)

and finally esgd itself with the arena bypassed (ESGD_ARENA_BYPASS=1: every bucket its
own hipMalloc, freed exported or not) on the C5 churn pattern -- the original trigger.
Round 3's first session: every step above correct, and the bypassed esgd correct too
(its peers now keep their mappings until shutdown).  What the cumulative steps never did
is round 2's ORDER: deletion was local, so an owner freed its bucket while peers still
mapped it, and the peers closed their old mapping only later, around opening the next
bucket.  The `late-close` lines do exactly that (on top of `plain` and of `+engine`):
the owner frees right after the reads, the peers close the old mapping only after opening
the next buffer's handle.
Every line prints the mismatches per size and rank.

  python tools/ipc_bisect.py [--world 8] [--only plain,+hostreg,...]
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import mp_workers  # noqa: E402

MiB = 1 << 20
STEPS = ["plain", "+hostreg", "+nbstream", "+suballoc", "+keepmaps", "+engine"]


class Handle(C.Structure):
    _fields_ = [("reserved", C.c_char * 64)]


def worker(rank, world, sizes, steps, late_close=False):
    import torch.distributed as dist

    import esgd
    from esgd import device as dev
    hip = C.CDLL("libamdhip64.so.7")   # the runtime torch (and libesgd) already loaded
    vp = C.c_void_p
    hip.hipIpcOpenMemHandle.argtypes = [C.POINTER(vp), Handle, C.c_uint]
    on = set(steps)
    if "+engine" in on:
        from esgd import comm
        comm.init()
        eb = dev.DeviceBuffer(4096)
        s0 = comm.Schedule(0, None, eb, 4096, buf=comm.BUF_DEVICE)
        s0.post(); s0.wait()
    if "+hostreg" in on:
        hb = (C.c_char * (1 << 20))()
        assert hip.hipHostRegister(hb, C.c_size_t(1 << 20), 2) == 0
    stream = dev.Stream() if "+nbstream" in on else None
    loc = dev.DeviceBuffer(max(sizes) // 4)
    pad = 2 * MiB if "+suballoc" in on else 0
    cache = {}
    pending = []
    out = []
    for si, size in enumerate(sizes):
        p = vp()
        assert hip.hipMalloc(C.byref(p), C.c_size_t(size + 2 * pad)) == 0
        buf = p.value + pad
        val = (rank * 16 + si + 1) & 0xFF
        assert hip.hipMemset(vp(buf), val, C.c_size_t(size)) == 0
        assert hip.hipDeviceSynchronize() == 0
        h = Handle()
        assert hip.hipIpcGetMemHandle(C.byref(h), p) == 0
        hs = [None] * world
        dist.all_gather_object(hs, bytes(h))
        opened, bad = [], []
        for q in range(world):
            if q == rank:
                continue
            key = (q, hs[q])
            if "+keepmaps" in on and key in cache:
                m = cache[key]
            else:
                mm = vp()
                rc = hip.hipIpcOpenMemHandle(C.byref(mm), Handle.from_buffer_copy(hs[q]), 1)
                assert rc == 0, rc
                m = mm.value
                cache[key] = m
                opened.append(m)
            want = (q * 16 + si + 1) & 0xFF
            dev.reduce(esgd.FLOAT, [m + pad], loc, size // 4, stream=stream)   # the whole buffer
            dev.synchronize(stream)
            for off in (0, size // 2, size - 4096):
                b = (C.c_uint8 * 4096)()
                assert hip.hipMemcpy(b, vp(loc.ptr + off), C.c_size_t(4096), 2) == 0
                got = set(b)
                if got != {want}:
                    bad.append((q, off, sorted(got)[:4], want))
        dist.barrier()
        if late_close:
            # round 2's order: the owner frees at once; peers close the old mappings only
            # after they opened the next buffer's (below, at the next size)
            hip.hipFree(p)
            for m in pending:
                hip.hipIpcCloseMemHandle(vp(m))
            pending = opened
            cache.clear()
            dist.barrier()
            out.append((size, len(bad), bad[:2]))
            continue
        if "+keepmaps" not in on:
            for m in opened:
                hip.hipIpcCloseMemHandle(vp(m))
            cache.clear()
        dist.barrier()
        hip.hipFree(p)
        dist.barrier()
        out.append((size, len(bad), bad[:2]))
    if "+engine" in on:
        s0.delete()
        comm.finalize()
    return out


mp_workers.ipc_bisect_worker = worker

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--only", default=None)
    ap.add_argument("--no-esgd", action="store_true")
    ap.add_argument("--repeat", type=int, default=1, help="runs of each esgd bypass mode")
    a = ap.parse_args()
    sizes = [16 * MiB, 256 * MiB]
    names = a.only.split(",") if a.only else STEPS + ["late-close", "late-close+engine", "late-close-3"]
    if a.only == "none":
        names = []
    for name in names:
        late = name.startswith("late-close")
        steps = (["plain", "+engine"] if name.endswith("+engine") else ["plain"]) if late \
            else STEPS[: STEPS.index(name) + 1]
        sz = [16 * MiB, 256 * MiB, 64 * MiB] if name == "late-close-3" else sizes
        res = mp_workers.run("ipc_bisect_worker", a.world, sizes=sz, steps=steps, late_close=late, timeout=300)
        nbad = [[n for _, n, _ in per] for per in res]
        print(f"world {a.world} {name:10s} mismatches per rank x size {nbad}", flush=True)
        for r, per in enumerate(res):
            for size, n, ex in per:
                if n:
                    print(f"  rank {r} size {size}: {ex}", flush=True)
                    break
    if not a.no_esgd:
        # esgd itself, arena bypassed: 16 MiB schedule used, deleted, bucket freed, then
        # 256 MiB (mp_workers.gpu_config: head / middle / tail of every rank vs the oracle);
        # mode 2 also closes the peers' mappings at each deletion (round 2's lifetime: an
        # owner may free before a slower peer closed); "2 close-first" puts a barrier
        # between every rank's deletion and any free (the IPC contract: no free under a
        # peer's mapping)
        for mode, cbf in (("1", False), ("2", False), ("2", True)):
            os.environ["ESGD_ARENA_BYPASS"] = mode
            for rep in range(a.repeat):
                try:
                    outs = mp_workers.run("gpu_config", a.world, kind=2,
                                          counts=[(16 * MiB) // 4, (256 * MiB) // 4], rounds=2,
                                          close_before_free=cbf, timeout=300)
                    res = f"ok per rank x size {[[v[3] for v in per] for per in outs]}"
                except AssertionError as e:
                    lines = [ln for ln in str(e).splitlines() if "esgd_schedule_create" in ln]
                    res = "ERROR " + " | ".join(ln.split("esgd_schedule_create: ")[-1] for ln in lines)
                print(f"world {a.world} esgd-arena-bypass={mode}{' close-first' if cbf else ''} "
                      f"#{rep}: {res}", flush=True)
