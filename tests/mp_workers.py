"""Multi-process harness: one process per rank, torch.distributed (gloo) for rendezvous
and result collection, the esgd engine for everything under test.

Worker functions live here (importable by spawned children).  `run(fn, world, **kw)`
starts `world` ranks on 127.0.0.1 and returns rank 0's result.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import queue
import socket
import sys
import time
import zlib
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "eager-sgd_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(fn_name, rank, world, port, kw, q, env=None):
    try:
        if env is not None:   # the parent's environment at run() time (forkserver children
            os.environ.clear()   # are forked from a server started earlier)
            os.environ.update(env)
        os.environ.setdefault("ESGD_TIMEOUT_S", "60")
        if os.environ.get("ESGD_HANG_DUMP_DIR"):   # diagnostics: every rank's Python stacks
            import faulthandler   # after ESGD_HANG_DUMP_S seconds, and again every period
            d = os.environ["ESGD_HANG_DUMP_DIR"]
            os.makedirs(d, exist_ok=True)
            _entry.dump = open(os.path.join(d, f"stacks_rank{rank}.txt"), "w")
            faulthandler.dump_traceback_later(float(os.environ.get("ESGD_HANG_DUMP_S", "60")), repeat=True,
                                              file=_entry.dump)
        # one GPU per rank where the box has them (device = rank % device_count, set in
        # _comm()): on a full node the data plane then crosses xGMI; on a 1-GPU box every
        # rank shares device 0
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        out = globals()[fn_name](rank, world, **kw)
        outs = [None] * world
        dist.all_gather_object(outs, out)
        if rank == 0:
            q.put(("ok", outs))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put(("err", f"rank {rank}: " + traceback.format_exc()))


_CTX = None


def _context():
    """Rank processes start from a forkserver that has imported torch once (ESGD_TEST_START=
    spawn restores a fresh interpreter per rank): a spawned rank spent ~2-3 s importing
    torch, most of a multi-rank GPU test.  The server is a fresh interpreter that never
    touches HIP (torch's import does not initialise the device), so every forked rank
    initialises its own HIP runtime, as a spawned one does."""
    global _CTX
    if _CTX is None:
        method = os.environ.get("ESGD_TEST_START", "forkserver")
        ctx = mp.get_context(method)
        if method == "forkserver":
            ctx.set_forkserver_preload(["numpy", "torch", "torch.distributed"])
        _CTX = ctx
    return _CTX


def run(fn_name: str, world: int, timeout: float = 240.0, **kw):
    ctx = _context()
    q = ctx.Queue()
    port = free_port()
    env = dict(os.environ)
    procs = [ctx.Process(target=_entry, args=(fn_name, r, world, port, kw, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        status, payload = q.get(timeout=timeout)
    finally:
        deadline = time.time() + 30
        for p in procs:
            p.join(max(0.1, deadline - time.time()))
        for p in procs:
            if p.is_alive():
                p.kill()
    if status != "ok":
        # the first error usually names a peer's failure: add every other rank's last line
        more = []
        while True:
            try:
                st, pl = q.get(timeout=0.5)
            except queue.Empty:
                break
            if st == "err":
                more.append(pl.strip().splitlines()[0] + " ... " + pl.strip().splitlines()[-1])
        raise AssertionError(payload + "".join("\n" + m for m in more))
    return payload


# --------------------------------------------------------------------------- workers

def wait_until(deadline: float):
    """Until time.perf_counter() reaches `deadline`: asleep while more than 2 ms remain (a
    spinning thread starves the rank's own progress thread on a box's few cores: r06k), then
    a spin (time.sleep cannot do tens of microseconds)."""
    while True:
        left = deadline - time.perf_counter()
        if left <= 0:
            return
        if left > 2e-3:
            time.sleep(left - 2e-3)


def set_test_knobs(**knobs):
    """The library's test hooks (ESGD_TEST, runtime.cpp test_knob): most are read once per
    process, at the hook's first use, so set them before the first schedule (fail_connect is
    read at every creation); e.g. set_test_knobs(fail_exports=2, shadow=1); None values are
    left out."""
    have = dict(kv.split("=", 1) for kv in os.environ.get("ESGD_TEST", "").split(",") if "=" in kv)
    have.update({k: str(int(v)) for k, v in knobs.items() if v is not None})
    os.environ["ESGD_TEST"] = ",".join(f"{k}={v}" for k, v in have.items())


def local_device(rank=None):
    """rank % device_count (0 when there is no device)."""
    import esgd
    n = esgd.device_count()
    r = int(os.environ.get("LOCAL_RANK", "0")) if rank is None else rank
    return r % n if n > 0 else 0


def _comm():
    """Join the esgd communicator on device rank % device_count.  Where the box has a GPU
    per rank, the ranks MUST be on distinct devices (the multi-rank tests then cover the
    cross-GPU data plane: xGMI peer loads, two L2s); a silent fall-back to a shared
    device would pass as cross-GPU coverage, so it fails here instead."""
    import ctypes as C

    import esgd
    from esgd import comm
    n = esgd.device_count()
    if n > 0:
        esgd.check(esgd.lib().esgd_set_device(local_device()), "esgd_set_device")
    comm.init()
    world = comm.world()
    if n > 0 and world > 1:
        import torch.distributed as dist
        d = C.c_int()
        esgd.check(esgd.lib().esgd_get_device(C.byref(d)), "esgd_get_device")
        devs = [None] * world
        dist.all_gather_object(devs, d.value)
        if n >= world:
            assert len(set(devs)) == world, f"{n} GPUs but ranks share devices: {devs}"
        os.environ["ESGD_TEST_DEVICES"] = ",".join(map(str, devs))
    return comm


def cp_rounds(rank, world, kind, rounds, async_=0, seed=0, straggler=-1, delay=0.0,
              first_poster_rotates=False, barrier_each=False, use_test=False):
    """Control plane only (ESGD_BUF_NONE): drive `rounds` post/wait cycles and return
    this rank's per-round log, post roles and stats."""
    comm = _comm()
    s = comm.Schedule(kind, None, None, 0, async_=async_, seed=seed, buf=comm.BUF_NONE)
    roles = []
    for t in range(1, rounds + 1):
        if barrier_each:
            comm.barrier()
        if first_poster_rotates:
            if rank == t % world:
                roles.append(s.post())
                comm.barrier()
            else:
                comm.barrier()
                time.sleep(0.02)
                roles.append(s.post())
        else:
            if rank == straggler:
                time.sleep(delay)
            roles.append(s.post())
        if use_test:
            while not s.test():
                time.sleep(0.0005)
        else:
            s.wait()
    comm.barrier()
    out = {"log": s.log(), "roles": roles, "stats": s.stats()}
    s.delete()
    comm.finalize()
    return out


class Mismatch(dict):
    """A failed round's verdict: falsy (so `all(verdicts)` still fails), and it says where --
    the round, the first wrong element, got / want, how many elements are wrong, every
    rank's input at that element, and this rank's schedule stats (fresh / carried rounds,
    transport, whether its bucket was shadowed)."""

    def __bool__(self):
        return False


def mismatch(t, got, want, xs, sched=None):
    import numpy as np
    gb, wb = got.view(np.uint8), want.view(np.uint8)
    bad = np.nonzero(gb.reshape(len(got), -1) != wb.reshape(len(want), -1))[0]
    i = int(bad[0]) if len(bad) else -1
    m = Mismatch(round=t, index=i, bad_elements=int(len(np.unique(bad))), count=int(len(got)))
    if i >= 0:
        val = (lambda a: float(a[i]) if a.dtype.kind == "f" else int(a[i]))
        m.update(got=val(got), want=val(want), inputs=[val(x) for x in xs])
    if sched is not None:
        try:
            m["stats"] = sched.stats()
        except Exception as e:   # noqa: BLE001 -- diagnostics only
            m["stats"] = repr(e)
    m["env"] = {k: v for k, v in os.environ.items() if k in ("ESGD_TEST", "ESGD_SMALL_ROUND_BYTES")}
    return m


def gpu_allreduce(rank, world, dtype_name="fp32", count=100003, rounds=3, kind=0, buf="device",
                  in_place=False, transport="ipc", shadow_ranks=(), small_bytes=None,
                  piece_bytes=None, host_chunk=None, device_flags=None, wire=False,
                  fail_exports=None, batch=None, fail_maps=None):
    """Data plane on the GPU: every rank reduces its splitmix bucket; returns the
    result bytes' digest per round plus a bit-exactness verdict against the oracle.
    shadow_ranks: ranks whose device buckets go through the owned shadow bucket.
    small_bytes: ESGD_SMALL_ROUND_BYTES (buckets up to it run as one launch per round;
    "0" forces the five-launch path).
    wire: fp32 buckets with bf16 on the wire (ESGD_SCHED_WIRE_BF16): the expected result
    is the oracle's bf16 tree of the bf16-rounded inputs, widened to fp32."""
    import numpy as np

    set_test_knobs(shadow=1 if rank in shadow_ranks else None,
                   # this rank's first N chunk exports fail / N mappings "show other memory"
                   fail_exports=fail_exports[rank] if fail_exports is not None and fail_exports[rank] else None,
                   fail_maps=fail_maps[rank] if fail_maps is not None and fail_maps[rank] else None,
                   piece_bytes=piece_bytes, host_chunk_bytes=host_chunk)
    if small_bytes is not None:
        os.environ["ESGD_SMALL_ROUND_BYTES"] = str(small_bytes)
    if device_flags is not None:
        os.environ["ESGD_DEVICE_FLAGS"] = str(device_flags)

    from esgd import _lib
    from esgd import device as dev
    from oracle import ffref
    comm = _comm()
    comm.set_transport(transport)
    if batch is not None:
        comm.set_config("batch_rounds", batch)
    seed = 0x5EEDE56D
    dt = {"fp32": _lib.FLOAT, "int32": _lib.INT32, "fp64": _lib.DOUBLE, "int64": _lib.INT64,
          "bf16": _lib.BF16}[dtype_name]
    verdicts = []
    if buf == "device":
        rb = dev.DeviceBuffer(count, dt)
        sb = None if in_place else dev.DeviceBuffer(count, dt)
        s = comm.Schedule(kind, sb, rb, count, dtype=dt, buf=comm.BUF_DEVICE,
                          flags=comm.WIRE_BF16 if wire else 0)
    else:
        npdt = dev.NP_DTYPE[dt]
        sb_h = None if in_place else np.zeros(count, npdt)
        rb_h = np.zeros(count, npdt)
        s = comm.Schedule(kind, sb_h, rb_h, count, dtype=dt, buf=comm.BUF_HOST,
                          flags=comm.WIRE_BF16 if wire else 0)
    for t in range(rounds):
        xs = []
        for r in range(world):
            if dt == _lib.FLOAT:
                x = ffref.fill_uniform(seed + t, r, count)
            elif dt == _lib.BF16:
                x = ffref.f32_to_bf16(ffref.fill_uniform(seed + t, r, count))
            elif dt in (_lib.INT32, _lib.INT64):
                x = (np.arange(count) + t + 7 * r).astype(dev.NP_DTYPE[dt])   # allreduce.c:49
            else:
                x = ffref.fill_uniform(seed + t, r, count).astype(np.float64) * 1e-3
            xs.append(x)
        mine = xs[rank]
        if buf == "device":
            (rb if in_place else sb).upload(mine)
        else:
            (rb_h if in_place else sb_h)[:] = mine
        comm.barrier()
        s.post()
        s.wait()
        got = rb.download() if buf == "device" else rb_h.copy()
        # Every rank gets rank 0's recursive-doubling result.  For power-of-two P that is
        # what every reference rank holds; for other P the reference leaves some ranks
        # with partial sums (ffallreduce.c:140) and esgd deliberately completes them.
        if wire and world > 1:
            want = ffref.bf16_to_f32(ffref.tree_sum_bf16([ffref.f32_to_bf16(x) for x in xs]))
        elif dt == _lib.BF16:
            want = ffref.tree_sum_bf16(xs)
        elif dt in (_lib.INT32, _lib.INT64):
            want = ffref.allreduce_rd(xs)[0]
            exact = sum(x.astype(np.int64) for x in xs).astype(want.dtype)   # (i+j)*P form
            assert np.array_equal(want, exact)
        else:
            want = ffref.allreduce_rd(xs)[0]
        same = bool(np.array_equal(got.view(np.uint8), want.view(np.uint8)))
        if not same:   # self-describing: a falsy verdict that says what came out wrong
            verdicts.append(mismatch(t, got, want, xs, s))
        else:
            verdicts.append(same)
        comm.barrier()
    s.delete()
    comm.finalize()
    return verdicts


def gpu_churn(rank, world, plan=(("fp32", 1 << 22), ("fp32", 64), ("fp32", 1001), ("fp32", 64),
                                  ("bf16", 1 << 23), ("fp32", 1 << 22), ("bf16", 1 << 15)), rounds=2):
    """Schedules created, run, deleted and their buckets freed one after another (the
    bench's C5 / C4 sequence in small): later schedules reuse freed addresses and cached
    sub-allocation chunks, while peers keep their IPC mappings of earlier buckets open.
    Every round of every schedule must still be bit-exact."""
    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    from oracle import ffref
    comm = _comm()
    verdicts = []
    for i, (dname, count) in enumerate(plan):
        dt = _lib.FLOAT if dname == "fp32" else _lib.BF16
        rb = dev.DeviceBuffer(count, dt)
        s = comm.Schedule(2, None, rb, count, dtype=dt, seed=6545343, buf=comm.BUF_DEVICE)
        for t in range(rounds):
            xs = [ffref.fill_uniform(0x5EED + 17 * i + t, r, count) for r in range(world)]
            if dt == _lib.BF16:
                xs = [ffref.f32_to_bf16(x) for x in xs]
                want = ffref.tree_sum_bf16(xs)
            else:
                want = ffref.tree_sum(xs)
            rb.upload(xs[rank])
            comm.barrier()
            s.post()     # majority: every rank posts, the drawn activator starts the round
            s.wait()
            got = rb.download()
            bad = np.nonzero(got.view(np.uint8) != want.view(np.uint8))[0]
            verdicts.append((i, dname, count, t, int(bad.size),
                             int(bad[0]) if bad.size else -1, int(bad[-1]) if bad.size else -1))
            comm.barrier()
        s.delete()
        rb.close()
    comm.finalize()
    return verdicts


def gpu_partial_semantics(rank, world, kind, rounds, async_=3, seed=6545343, straggler=1,
                          delay=0.05, count=4096):
    """eager-SGD semantics with data: rank r writes tag_r(t) = t * 64**r into its send
    buffer before posting round t (exact in fp32 for P <= 4, t < 64).  The reduced
    value of a round decodes which posted round each rank's buffer held when that rank
    joined — checked against the round logs."""
    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    comm = _comm()
    sb = dev.DeviceBuffer(count, _lib.FLOAT)
    rb = dev.DeviceBuffer(count, _lib.FLOAT)
    sb.zero(); dev.synchronize()
    s = comm.Schedule(kind, sb, rb, count, dtype=_lib.FLOAT, async_=async_, seed=seed,
                      buf=comm.BUF_DEVICE)
    results = []
    for t in range(1, rounds + 1):
        if rank == straggler:
            time.sleep(delay)
        sb.upload(np.full(count, float(t * 64 ** rank), np.float32))
        s.post()
        s.wait()
        v = rb.download()
        assert np.all(v == v[0]), "non-uniform result"
        results.append(float(v[0]))
    comm.barrier()
    out = {"log": s.log(), "results": results, "stats": s.stats()}
    s.delete()
    comm.finalize()
    return out


LATE_S = 0.03   # how late a delayed rank calls the op (>> one round of these sizes)


def late_ranks(mode, world, step, seed=6545343):
    """Ranks that call the op LATE in `step` so that a partial round's contributor set is
    deterministic: majority -- the activator (ffrand_allreduce.c:88, rand_r sequence) posts
    after every other rank has posted, so its round takes every fresh gradient; solo --
    every rank but 0, so rank 0's post activates the (asynchronous) round and the late
    ranks are carried through it with a zeroed send bucket (ffactivation.c:11-106, the
    wrapper's zeroing opt_esgd_solo_imagenet_imbalance.py:311-314)."""
    from oracle import ffref
    if mode == "majority":
        return {ffref.activators(seed, world, step + 1)[step]}
    if mode == "solo":
        return set(range(1, world))
    return set()


def expected_inputs(mode, xs):
    """The per-rank inputs the round reduces under late_ranks' ordering."""
    import numpy as np
    if mode == "solo":
        return [xs[0]] + [np.zeros_like(x) for x in xs[1:]]
    return xs


def op_host(rank, world, mode="allreduce", steps=3, count=5000):
    """deep500 op, host path (the reference's CPU-registered TF kernel contract).  Step 0
    creates the schedule (collective, racing the first post); steps >= 1 run in
    late_ranks' order and are checked bit for bit against the oracle tree of
    expected_inputs."""
    import numpy as np

    from esgd import deep500
    from oracle import ffref
    comm = _comm()
    deep500.configure(mode, 32, 6545343)
    op = deep500.AllreduceOp((count // 100, 100) if count % 100 == 0 else (count,))
    ok = []
    for t in range(steps):
        xs = [ffref.fill_uniform(0xABC + t, r, count) for r in range(world)]
        comm.barrier()          # evaluation/solo_allreduce_correctness.c:84 pattern
        if t > 0 and rank in late_ranks(mode, world, t):
            time.sleep(LATE_S)
        out = op.forward(xs[rank])
        if t > 0:
            want = ffref.tree_sum(expected_inputs(mode, xs))
            ok.append(bool(np.array_equal(out.view(np.uint32), want.view(np.uint32))))
    rep = op.report()
    comm.barrier()
    comm.finalize()
    return {"ok": ok, "report": rep, "cuda": op.supports_cuda()}


def op_device_late(rank, world, async_=3, steps=9, count=100003, on_time=0):
    """deep500 op, device path, solo, every rank but `on_time` calling late every step.
    Asynchronous rounds: the on-time rank activates, the late ranks are carried through
    with a zeroed send bucket, and their late gradient is DROPPED (not carried into the
    next round): the result is x_on_time / P.  Synchronous rounds (every async+1-th,
    ffsolo_limiter.c:4-35): every rank's fresh gradient.  Both on every rank, bit for bit."""
    import numpy as np
    import torch

    from esgd import deep500
    from oracle import ffref
    comm = _comm()
    dev = torch.device("cuda", local_device())
    torch.cuda.set_device(dev)
    deep500.configure("solo", async_, 6545343)
    op = deep500.AllreduceOp((count,))
    stream = torch.cuda.current_stream().cuda_stream
    ok, fresh = [], []
    for t in range(steps):
        xs = [ffref.fill_uniform(0x1A7E + t, r, count) for r in range(world)]
        g = torch.from_numpy(xs[rank]).to(dev)
        comm.barrier()
        if t > 0 and rank != on_time:
            time.sleep(LATE_S)
        op.forward_cuda_div(g, g, world, stream)
        got = g.cpu().numpy()
        rnd = t + 1
        scaled = [x / np.float32(world) for x in xs]
        if t == 0:
            continue
        sync = rnd % (async_ + 1) == 0
        want = ffref.tree_sum(scaled if sync else
                              [x if r == on_time else np.zeros_like(x) for r, x in enumerate(scaled)])
        ok.append(bool(np.array_equal(got.view(np.uint32), want.view(np.uint32))))
        fresh.append(sync)
    comm.barrier()
    comm.finalize()
    return {"ok": ok, "sync_rounds": fresh}


def op_device_pattern(rank, world, count=25559081, steps=9, mode="solo", packed=False, delay=0.05,
                      barrier=False, host=False):
    """deep500 op, device path, NO barrier between steps (unless `barrier`): in step t the
    ranks drawn as in the reference's imbalance loop (resnet_run_loop_solo_imagenet_300.py:
    290-294, seeded by t) sleep `delay` before calling the op.  Every rank must receive
    the same bits every step, and each step's result must be the tree of SOME subset of
    the ranks' inputs (the contributors of that partial round) -- returned per step."""
    import itertools

    import numpy as np
    import torch

    from esgd import deep500
    from oracle import ffref
    comm = _comm()
    dev = torch.device("cuda", local_device())
    torch.cuda.set_device(dev)
    deep500.configure(mode, 32, 6545343)
    op = deep500.AllreduceOp((count,))
    stream = torch.cuda.current_stream().cuda_stream
    m = min(count, 1 << 16)   # checked slice (head)
    out = []
    comm.barrier()
    for t in range(steps):
        np.random.seed(t)
        late = rank == np.random.randint(world) or rank == np.random.randint(world)
        if barrier:
            comm.barrier()
        if late and t > 0:
            time.sleep(delay)
        x = ffref.fill_uniform(0x7A77 + t, rank, count)
        if host:   # the reference's contract: host buffers, the wrapper's steps in the op
            res = op.forward(x / np.float32(world))
            got = res[:m]
            xs = [ffref.fill_uniform(0x7A77 + t, r, m) / np.float32(world) for r in range(world)]
            who = None
            for k in range(world, 0, -1):
                for sub in itertools.combinations(range(world), k):
                    want = ffref.tree_sum([v if r in sub else np.zeros_like(v) for r, v in enumerate(xs)])
                    if np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                        who = list(sub)
                        break
                if who is not None:
                    break
            out.append({"t": t, "late": bool(late), "contributors": who, "digest": zlib.crc32(res.tobytes())})
            continue
        g = torch.from_numpy(x).to(dev)
        if packed:
            half = count // 3
            parts = [g[:half], g[half:]]
            op.forward_cuda_packed(parts, parts, world, stream)
        else:
            op.forward_cuda_div(g, g, world, stream)
        got = g[:m].cpu().numpy()
        xs = [ffref.fill_uniform(0x7A77 + t, r, m) / np.float32(world) for r in range(world)]
        who = None
        for k in range(world, 0, -1):
            for sub in itertools.combinations(range(world), k):
                want = ffref.tree_sum([x if r in sub else np.zeros_like(x) for r, x in enumerate(xs)])
                if np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                    who = list(sub)
                    break
            if who is not None:
                break
        out.append({"t": t, "late": bool(late), "contributors": who,
                    "digest": zlib.crc32(g.cpu().numpy().tobytes())})
    comm.barrier()
    comm.finalize()
    return out


def optimizer_step(rank, world, mode="allreduce", steps=2, fuse=False, wire="fp32", pipeline=True, bucket_mb=None,
                   **opt_kw):
    """EagerSGDOptimizer on PyTorch-ROCm: every rank's p.grad after apply_gradients must
    equal the oracle tree of (grad_r / P) over ranks, bit for bit (allreduce), or over
    expected_inputs' contributors when the ranks call every op in late_ranks' order
    (solo / majority; step 0, which creates the schedules collectively, is not checked).
    wire="bf16": the same contributors, the oracle's bf16 tree of the rounded inputs, widened."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from esgd import deep500
    from esgd.optim import EagerSGDOptimizer
    from oracle import ffref
    comm = _comm()
    torch.manual_seed(1234)
    dev = torch.device("cuda", local_device())
    torch.cuda.set_device(dev)
    model = torch.nn.Sequential(torch.nn.Linear(64, 48), torch.nn.ReLU(), torch.nn.Linear(48, 10)).to(dev)
    captured = {}
    if opt_kw.get("overlap"):   # the local gradients, taken before the optimizer's hooks post them
        for prm in model.parameters():
            prm.register_post_accumulate_grad_hook(lambda q: captured.__setitem__(id(q), q.grad.detach().clone()))
    cls = EagerSGDOptimizer
    if bucket_mb is not None:   # the fused buckets' size is a class attribute
        cls = type("SmallBuckets", (EagerSGDOptimizer,), {"bucket_mb": bucket_mb})
    opt = cls(torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9), world, mode=mode,
              fuse=fuse, wire=wire, pipeline=pipeline, **opt_kw)
    ok = []
    for t in range(steps):
        g = torch.Generator().manual_seed(100 * t + rank)
        x = torch.randn(32, 64, generator=g).to(dev)
        y = torch.randint(0, 10, (32,), generator=g).to(dev)
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x), y)
        gvs = opt.compute_gradients(loss)
        if captured:   # the rounds posted in backward may have written p.grad already
            local = [(captured[id(p)].float() / world).cpu().numpy().ravel() for _, p in gvs]
        else:
            local = [(gr.detach().float() / world).cpu().numpy().ravel() for gr, _ in gvs]
        allg = [None] * world
        dist.all_gather_object(allg, local)
        comm.barrier()
        late = t > 0 and rank in late_ranks(mode, world, t)
        names = ("forward_cuda_div", "forward_cuda_packed", "post_many_io")
        orig = {n: getattr(deep500.AllreduceOp, n) for n in names}
        if late:   # every op call (or post) of this step comes LATE_S after the peers'
            def delayed(fn):
                def f(self, *a, **k):
                    time.sleep(LATE_S)
                    return fn(self, *a, **k)
                return f
            for n in names:
                setattr(deep500.AllreduceOp, n, delayed(orig[n]))
        try:
            opt.apply_gradients(gvs)
        finally:
            for n in names:
                setattr(deep500.AllreduceOp, n, orig[n])
        torch.cuda.synchronize()
        if t == 0 and mode != "allreduce":
            continue
        for i, (_, p) in enumerate(gvs):
            xs = expected_inputs(mode, [allg[r][i] for r in range(world)])
            want = (ffref.bf16_to_f32(ffref.tree_sum_bf16([ffref.f32_to_bf16(x) for x in xs]))
                    if wire == "bf16" else ffref.tree_sum(xs))
            got = p.grad.detach().float().cpu().numpy().ravel()
            ok.append(bool(np.array_equal(got.view(np.uint32), want.view(np.uint32))))
    params = torch.cat([p.detach().float().cpu().ravel() for p in model.parameters()]).numpy()
    comm.barrier()
    nbytes = opt.bytes_reduced()
    comm.finalize()
    return {"ok": ok, "params_digest": params.tobytes().hex()[:64] + str(params.sum()), "bytes": nbytes}


def op_group(rank, world, steps=3, sizes=(1, 17, 1000, 4099, 262147, (2 << 20) + 5, 64, 300007)):
    """allreducef_forward_cuda_post_many_io / _wait_many against the single-op path: one set
    of ops posted as a group over 16-B aligned tensors (the rounds read and write them
    themselves), one over tensors 4 bytes off that alignment (the group goes the copy-in way
    and wait_many copies out), a third driven by forward_cuda_div one op at a time
    (allreduce mode: every rank posts every round, so all must give the same bits, the
    oracle tree of grad_r / P); plus the misuse rules: a group post over an op still posted
    fails with ESGD_INVALID_ARG and leaves it posted, wait_many skips ops not posted."""
    import numpy as np
    import torch

    from esgd import deep500
    from esgd._lib import EsgdError
    from oracle import ffref
    comm = _comm()
    dev = torch.device("cuda", local_device())
    torch.cuda.set_device(dev)
    deep500.configure("allreduce", 32, 6545343)
    fio = [deep500.AllreduceOp((n,)) for n in sizes]   # aligned: the rounds do the copies
    grp = [deep500.AllreduceOp((n,)) for n in sizes]   # unaligned: copy-in / copy-out
    one = [deep500.AllreduceOp((n,)) for n in sizes]
    ok, errs = [], {}

    def unaligned(x):   # a copy of x starting 4 bytes past a 16-B boundary
        buf = torch.empty(x.numel() + 4, dtype=torch.float32, device=dev)
        v = buf[1:1 + x.numel()]
        v.copy_(x)
        assert v.data_ptr() % 16 == 4
        return v

    for t in range(steps):
        xs = [[ffref.fill_uniform(0xA11 + 13 * t + i, r, n) for r in range(world)] for i, n in enumerate(sizes)]
        k = [torch.from_numpy(x[rank]).to(dev) for x in xs]
        g = [unaligned(ki) for ki in k]
        h = [ki.clone() for ki in k]
        comm.barrier()
        deep500.AllreduceOp.post_many_io(fio, k, k, float(world))
        deep500.AllreduceOp.wait_many(fio, k)
        deep500.AllreduceOp.post_many_io(grp, g, g, float(world))
        deep500.AllreduceOp.wait_many(grp, g)
        for op, hi in zip(one, h):
            op.forward_cuda_div(hi, hi, float(world))
        torch.cuda.synchronize()
        for i, x in enumerate(xs):
            want = ffref.tree_sum([np.float32(xr) / np.float32(world) for xr in x])
            a, b, c = g[i].cpu().numpy(), h[i].cpu().numpy(), k[i].cpu().numpy()
            ok.append(bool(np.array_equal(a.view(np.uint32), want.view(np.uint32)) and
                           np.array_equal(a.view(np.uint32), b.view(np.uint32)) and
                           np.array_equal(a.view(np.uint32), c.view(np.uint32))))
    # misuse: op 0 posted alone, then a group post naming it fails and leaves it posted
    x = [torch.ones(n, device=dev) for n in sizes]
    deep500.AllreduceOp.post_many_io(fio[:1], x[:1], x[:1], float(world))
    try:
        deep500.AllreduceOp.post_many_io(fio, x, x, float(world))
        errs["post_many_over_posted"] = None
    except EsgdError as e:
        errs["post_many_over_posted"] = e.rc
    deep500.AllreduceOp.wait_many(fio, x)   # waits op 0 only (the others are not posted)
    torch.cuda.synchronize()
    want0 = ffref.tree_sum([np.ones(sizes[0], np.float32) / np.float32(world)] * world)
    errs["drained_op0"] = bool(np.array_equal(x[0].cpu().numpy(), want0))
    comm.barrier()
    comm.finalize()
    return {"ok": ok, "errs": errs}


def op_torch_registered(rank, world, shapes=((1000,), (64, 33), (4099,))):
    """esgd::allreducef (the registered PyTorch operator) inside a torch.fx-traced module on
    the GPU, allreduce mode: every output is the oracle tree of x_r / P over ranks, bit for
    bit; the traced graph holds one op node per tensor; backward gives the reference op's zero
    input gradients (allreducef::backward writes nothing)."""
    import numpy as np
    import torch
    import torch.fx

    from esgd import deep500
    from oracle import ffref
    comm = _comm()
    dev = torch.device("cuda", local_device())
    torch.cuda.set_device(dev)
    deep500.configure("allreduce", 32, 6545343)
    mods = [deep500.AllreduceModule(sh, divisor=float(world)) for sh in shapes]

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.ars = torch.nn.ModuleList(mods)

        def forward(self, a, b, c):   # fixed arity: torch.fx traces no *args
            return self.ars[0](a), self.ars[1](b), self.ars[2](c)

    gm = torch.fx.symbolic_trace(Net())
    nodes = sum(1 for n in gm.graph.nodes if n.op == "call_function" and n.target is torch.ops.esgd.allreducef)
    ok = []
    for t in range(2):
        xs = [[ffref.fill_uniform(0x70C + 7 * t + i, r, int(np.prod(sh))).reshape(sh) for r in range(world)]
              for i, sh in enumerate(shapes)]
        ins = [torch.from_numpy(x[rank]).to(dev).requires_grad_(True) for x in xs]
        comm.barrier()
        outs = gm(*ins)
        sum(o.sum() for o in outs).backward()
        torch.cuda.synchronize()
        for x, o, i in zip(xs, outs, ins):
            want = ffref.tree_sum([np.float32(xr.ravel()) / np.float32(world) for xr in x])
            got = o.detach().cpu().numpy().ravel()
            ok.append(bool(np.array_equal(got.view(np.uint32), want.view(np.uint32))))
            ok.append(bool(torch.count_nonzero(i.grad).item() == 0))
    comm.barrier()
    for m in mods:   # every rank in the same order: the schedules' deletion is collective
        m.close()
    comm.finalize()
    return {"ok": ok, "nodes": nodes}


def cp_ordered(rank, world, nsched=3, rounds=6, seed=7):
    """Ordered (rccl-style) issue: several schedules posted with per-rank random jitter;
    every rank must issue the rounds in the same global order (ticket ring)."""
    import random

    from esgd import comm
    comm.init()
    comm.set_transport("rccl")
    scheds = [comm.Schedule(comm.SOLO if i % 2 else comm.ALLREDUCE, None, None, 0, async_=2,
                            buf=comm.BUF_NONE) for i in range(nsched)]
    rng = random.Random(seed * 100 + rank)
    for t in range(rounds):
        order = list(range(nsched))
        rng.shuffle(order)                 # ranks post the buckets in different orders
        for i in order:
            time.sleep(rng.random() * 0.003)
            scheds[i].post()
        for i in order:
            scheds[i].wait()
    comm.barrier()
    log = comm.issue_log()
    for s in scheds:
        s.delete()
    comm.set_transport("ipc")
    comm.finalize()
    return log


def cp_create_failure(rank, world, bad_rank=1):
    """A creation that fails on one rank fails on every rank (voted registration), and
    the communicator stays usable: the next creation and its rounds work."""
    from esgd import comm
    from esgd._lib import EsgdError
    comm.init()
    kind = comm.MAJORITY if rank == bad_rank else comm.SOLO   # creation order mismatch
    err = None
    try:
        comm.Schedule(kind, None, None, 0, async_=2, buf=comm.BUF_NONE)
    except EsgdError as e:
        err = str(e)
    t0 = time.time()
    s = comm.Schedule(comm.ALLREDUCE, None, None, 0, buf=comm.BUF_NONE)
    for _ in range(3):
        s.post()
        s.wait()
    s.delete()
    comm.finalize()
    return {"err": err, "recovered_s": time.time() - t0}


def cp_churn_inflight(rank, world, rounds=300, churn=40):
    """Schedules created and deleted while another schedule's rounds are in flight (a
    thread posts / waits it back to back): delete must not free a schedule the progress
    thread is still stepping (engine.cpp: sched_delete waits two progress epochs)."""
    import threading

    comm = _comm()
    a = comm.Schedule(comm.ALLREDUCE, None, None, 0, buf=comm.BUF_NONE)
    errs = []

    def pump():
        try:
            for _ in range(rounds):
                a.post()
                a.wait()
        except Exception as e:   # pragma: no cover - reported below
            errs.append(repr(e))

    th = threading.Thread(target=pump)
    th.start()
    for j in range(churn):
        b = comm.Schedule(comm.SOLO if j % 2 else comm.MAJORITY, None, None, 0, async_=2, seed=7,
                          buf=comm.BUF_NONE)
        b.post()
        b.wait()
        b.delete()
    th.join()
    st = a.stats()
    a.delete()
    comm.finalize()
    return {"errs": errs, "completed": st["completed"]}


SEED = 0x5EEDE56D


def _download_slice(buf, start, n):
    """Elements [start, start + n) of a DeviceBuffer, to the host."""
    import numpy as np

    from esgd import device as dev
    from esgd._lib import check, lib
    out = np.empty(n, dtype=dev.NP_DTYPE[buf.dtype])
    es = out.itemsize
    check(lib().esgd_memcpy_async(out.ctypes.data, buf.ptr + start * es, n * es, 1, None), "d2h")
    dev.synchronize()
    return out


def gpu_config(rank, world, kind, counts, dtype_name="fp32", rounds=2, async_=32, seed=6545343,
               check=65536, transport="ipc", keep=False, detail=False, free=True, env=None,
               alloc_ahead=False, close_before_free=False):
    """A BASELINE.json workload: one in-place bucket per rank per size in `counts`, every
    rank's bucket written BEFORE a barrier and then posted (the pattern of
    evaluation/{solo,rand}_allreduce_correctness.c:76-97: whichever rank activates, every
    rank's data is fresh, so solo / majority rounds equal the plain allreduce).  Inputs
    come from the device generator shared with the oracle; head, middle and tail slices of
    every rank's result are compared bit for bit with the oracle tree."""
    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    from oracle import ffref
    os.environ.update(env or {})
    comm = _comm()
    comm.set_transport(transport)
    dt = _lib.FLOAT if dtype_name == "fp32" else _lib.BF16
    out, kept = [], []
    nxt = None
    for i, count in enumerate(counts):
        rb = nxt if nxt is not None else dev.DeviceBuffer(count, dt)
        nxt = None
        s = comm.Schedule(kind, None, rb, count, dtype=dt, async_=async_, seed=seed, buf=comm.BUF_DEVICE)
        for t in range(rounds[i] if isinstance(rounds, (list, tuple)) else rounds):
            sd = SEED + 7919 * i + t
            dev.fill_uniform(rb, sd, rank)
            dev.synchronize()
            comm.barrier()
            s.post()
            s.wait()
            comm.barrier()
            m = min(count, check)
            ok = True
            for start in sorted({0, (count - m) // 2, count - m}):
                got = _download_slice(rb, start, m)
                xs = [ffref.fill_uniform(sd, r, m, start=start) for r in range(world)]
                if dt == _lib.BF16:
                    want = ffref.tree_sum_bf16([ffref.f32_to_bf16(x) for x in xs])
                else:
                    want = ffref.tree_sum(xs)
                good = bool(np.array_equal(got.view(np.uint8), want.view(np.uint8)))
                if not good and detail:
                    bad = np.nonzero(got.view(np.uint32 if dt == _lib.FLOAT else np.uint16) !=
                                     want.view(np.uint32 if dt == _lib.FLOAT else np.uint16))[0]
                    e = int(bad[0])
                    print(f"[r{rank}] count={count} t={t} slice@{start}: {bad.size} bad, first {e + start} "
                          f"got {got[e]} want {want[e]}; last {bad[-1] + start}; inputs there "
                          f"{[float(x[e]) for x in xs]}", flush=True)
                ok &= good
            out.append((count, dtype_name, t, ok))
        comm.barrier()
        if keep:
            kept.append((s, rb))
        else:
            s.delete()
            if close_before_free:
                # every rank's deletion (closing its peer mappings under ESGD_TEST arena_bypass=2)
                # happens before any rank frees a bucket a peer had mapped
                comm.barrier()
            if alloc_ahead and i + 1 < len(counts):
                nxt = dev.DeviceBuffer(counts[i + 1], dt)
            if free:
                rb.close()
            else:
                kept.append((None, rb))
    for sch, buf in kept:
        if sch is not None:
            sch.delete()
        buf.close()
    comm.set_transport("ipc")
    comm.finalize()
    return out


def gpu_straggler(rank, world, kind, count, rounds, async_=3, seed=6545343, delay=None, delay_frac=None):
    """eager-SGD's partial rounds with a straggler (the last rank), contributor-counted
    like evaluation/rsgd.c:87,100: every rank's gradient is 1.0, zeroed after use, so a
    round's result is the number of ranks whose fresh gradient it took.  On-time ranks
    write theirs before the round's barrier; the straggler writes and posts `delay` after
    it (default 4x the no-straggler round T, at least 20 ms; delay_frac: that fraction of
    T, e.g. BASELINE C4's 20 %).  Returns this rank's per-round (round, contributors,
    uniform result) and the round log."""
    import statistics

    import numpy as np
    import torch
    import torch.distributed as dist

    from esgd import _lib
    from esgd import device as dev
    from esgd._lib import check, lib
    comm = _comm()
    ones = dev.DeviceBuffer(count)
    ones.upload(np.ones(count, np.float32))
    sb, rb = dev.DeviceBuffer(count), dev.DeviceBuffer(count)
    sb.zero(); rb.zero()
    dev.synchronize()
    s = comm.Schedule(kind, sb, rb, count, dtype=_lib.FLOAT, async_=async_, seed=seed, buf=comm.BUF_DEVICE)
    late = world - 1

    def fill():
        check(lib().esgd_memcpy_async(sb.ptr, ones.ptr, count * 4, 2, None), "d2d")
        dev.synchronize()

    def one(d):
        if rank != late or d == 0:
            fill()
        comm.barrier()
        tb = time.perf_counter()
        tf = tb
        if rank == late and d > 0:   # wait to the deadline, then the late gradient is written
            wait_until(tb + d)
            tf = time.perf_counter()
            fill()
        t0 = time.perf_counter()
        achieved.append(t0 - tb)   # barrier -> post, as this rank saw it (the write included)
        fills.append(t0 - tf)
        s.post()
        s.wait()
        el = time.perf_counter() - t0
        sb.zero()
        dev.synchronize()
        m = min(count, 4096)
        head, tail = _download_slice(rb, 0, m), _download_slice(rb, count - m, m)
        comm.barrier()
        uniform = bool(np.all(head == head[0]) and np.all(tail == head[0]))
        both = np.concatenate([head, tail])
        slices.append((float(both.min()), float(both.max()), zlib.crc32(both.tobytes())))
        return el, float(head[0]), uniform

    slices = []                            # per round: (min, max, crc32) of head + tail
    achieved = []                          # per round: barrier -> post on this rank (s)
    fills = []                             # ... of which the late gradient's write
    warm = [one(0)[0] for _ in range(3)]   # rounds 1..3: everyone on time
    tt = torch.tensor([statistics.median(warm)], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    T = float(tt.item())
    d = delay if delay is not None else (delay_frac * T if delay_frac is not None else max(4 * T, 0.02))
    res = []
    for t in range(4, 4 + rounds):
        _, c, u = one(d)
        res.append((t, c, u))
    out = {"rounds": res, "log": s.log(), "T_s": T, "delay_requested_s": d,
           "delay_achieved_s": statistics.median(achieved[3:]), "fill_s": statistics.median(fills[3:]),
           "slices": slices[3:]}
    comm.barrier()
    s.delete()
    comm.finalize()
    return out


def cp_stale_segment(rank, world, job):
    """A segment file left behind under this job id by a crashed run (its creator is
    dead) must not be joined: ranks > 0 wait for rank 0's fresh one (shm.cpp)."""
    comm = _comm_job(job)
    s = comm.Schedule(comm.ALLREDUCE, None, None, 0, buf=comm.BUF_NONE)
    for _ in range(3):
        s.post()
        s.wait()
    s.delete()
    comm.finalize()
    return True


def _comm_job(job):
    from esgd import comm
    comm.init(job_id=job)
    return comm


def gpu_big(rank, world, count, rounds=1):
    """One bucket of `count` fp32 per rank (up to ff.h's 2^31 - 1): creation, a round and
    head / tail slices checked; returns the wall time of each step."""
    import numpy as np

    from esgd import device as dev
    from oracle import ffref
    comm = _comm()
    t = {}
    t0 = time.perf_counter()
    rb = dev.DeviceBuffer(count)
    dev.fill_uniform(rb, SEED, rank)
    dev.synchronize()
    t["alloc_fill_s"] = time.perf_counter() - t0
    comm.barrier()
    t0 = time.perf_counter()
    s = comm.Schedule(comm.ALLREDUCE, None, rb, count, buf=comm.BUF_DEVICE)
    t["create_s"] = time.perf_counter() - t0
    ok = True
    for i in range(rounds):
        if i:   # in place: fresh inputs every round
            dev.fill_uniform(rb, SEED + i, rank)
            dev.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        s.post()
        s.wait()
        t.setdefault("round_s", []).append(time.perf_counter() - t0)
        m = 1 << 16
        for start in (0, count // 2, count - m):
            got = _download_slice(rb, start, m)
            want = ffref.tree_sum([ffref.fill_uniform(SEED + i, r, m, start=start) for r in range(world)])
            ok &= bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
    t["ok"] = ok
    comm.barrier()
    t0 = time.perf_counter()
    s.delete()
    t["delete_s"] = time.perf_counter() - t0
    comm.finalize()
    return t


def cp_hold(rank, world, hold_s=0.3):
    """ESGD_SCHED_HOLD on the control plane: after wait() a rank joins no further round
    of the schedule until release(); waiting again before releasing is an error."""
    from esgd._lib import EsgdError
    comm = _comm()
    s = comm.Schedule(comm.SOLO, None, None, 0, async_=100, buf=comm.BUF_NONE, flags=comm.HOLD)
    out = {}
    s.post()
    s.wait()
    try:
        s.wait()
        out["double_wait"] = "no error"
    except EsgdError as e:
        out["double_wait"] = str(e)
    comm.barrier()
    if rank == 1:
        time.sleep(hold_s)       # rank 0's round 2 cannot complete before this release
        s.release()
        s.post()
        s.wait()
        s.release()
    else:
        s.release()
        t0 = time.time()
        s.post()                 # activates round 2 (solo, asynchronous)
        s.wait()
        out["round2_s"] = time.time() - t0
        s.release()
    comm.barrier()
    out["log"] = s.log()
    s.delete()
    comm.finalize()
    return out


def gpu_stress(rank, world, kind, count, rounds=600, async_=3, seed=34495645, jitter_us=300, buf="device",
               wire=False):
    """Activation stress on the GPU data plane (the reference loops its activation test
    300 times to catch nondeterministic failures, test_activation.sh:5-7): every rank
    runs `rounds` steps with a random per-step delay and NO barrier between steps, so
    rounds are activated by whichever rank gets there first (solo) or by the drawn rank
    (majority) and ranks are carried through rounds they have not posted yet.
    Schedules as the deep500 op uses them (ESGD_SCHED_HOLD | ZERO_SB): the gradient for
    step t+1 is written while round t is held, then released.  int32 round tags: rank r
    writes (t mod 2^b) << (b r), b = min(10, 31 // P), so every element of round t's
    result must decode to tag t for EVERY rank -- each round took exactly the right
    generation of every rank's bucket, whole (no stale, torn or doubly counted data).
    buf="host": the reference's
    host buckets (HOLD only; the host bucket keeps its tag after the snapshot, refilled
    each step the same way).  wire=True: fp32 buckets with bf16 on the wire
    (ESGD_SCHED_WIRE_BF16); the tags are then ((t mod 2) + 1) << (2 r) (P <= 4; a missing
    share decodes as 0, a stale one as the other parity) or (t mod 2) << r (P > 4), sums
    below 256 that bf16 carries exactly.
    Returns per-round verdicts, the round log and the stats."""
    import random

    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    comm = _comm()
    host = buf == "host"
    # tag bits per rank: int32 without overflow at any P; over the wire the sum must stay
    # below 256 (bf16's 8 significant bits): 2 bits up to P = 4, 1 bit (the parity) above
    bits = (2 if world <= 4 else 1) if wire else min(10, 31 // world)
    dt, npdt = (_lib.FLOAT, np.float32) if wire else (_lib.INT32, np.int32)

    def tag(t):
        if wire:
            return (t % 2) + 1 if bits == 2 else t % 2
        return t % (1 << bits)

    if host:
        sb, rb = np.zeros(count, npdt), np.zeros(count, npdt)
    else:
        sb, rb = dev.DeviceBuffer(count, dt), dev.DeviceBuffer(count, dt)
        rb.zero()
        dev.synchronize()

    def fill(t):
        v = tag(t) << (bits * rank)
        if host:
            sb[:] = v
        else:
            sb.upload(np.full(count, v, npdt))

    fill(1)
    s = comm.Schedule(kind, sb, rb, count, dtype=dt, async_=async_, seed=seed,
                      buf=comm.BUF_HOST if host else comm.BUF_DEVICE,
                      flags=comm.HOLD | (0 if host else comm.ZERO_SB) | (comm.WIRE_BF16 if wire else 0))
    rng = random.Random(1000 + rank)
    m = min(count, 2048)
    bad = []
    fresh = []
    comm.barrier()
    for t in range(1, rounds + 1):
        time.sleep(rng.random() * jitter_us * 1e-6)
        s.post()
        fresh.append(s.wait())
        if host:
            head, tail = rb[:m].copy(), rb[count - m:].copy()
        else:
            head, tail = _download_slice(rb, 0, m), _download_slice(rb, count - m, m)
        v = int(head[0])
        tags = [(v >> (bits * q)) & ((1 << bits) - 1) for q in range(world)]
        if not (np.all(head == head[0]) and np.all(tail == head[0]) and tags == [tag(t)] * world):
            bad.append((t, tags, bool(np.all(head == head[0])), bool(np.all(tail == head[0]))))
        fill(t + 1)
        s.release()
    comm.barrier()
    out = {"bad": bad[:10], "nbad": len(bad), "fresh": sum(fresh), "log": s.log(), "stats": s.stats()}
    s.delete()
    comm.finalize()
    return out


def gpu_stress_multi(rank, world, kind, counts=(4096, 65536, (1 << 20) + 3, 300007), rounds=200, async_=3,
                     seed=34495645, jitter_us=200):
    """gpu_stress over several schedules at once, the way the wrapper drives its 161
    per-tensor ops (opt_esgd_solo_imagenet_imbalance.py:301-316): every step runs the
    schedules one after the other (post, wait, read, refill, release), with random delays
    between them and no barrier, so rounds of different schedules -- one-launch and
    five-launch sizes mixed -- are activated, issued (the node's issue ring) and carried
    through in interleaved orders on different ranks.  Same int32 tag check per round."""
    import random

    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    comm = _comm()
    bits = min(10, 31 // world)
    scheds = []
    for i, n in enumerate(counts):
        sb, rb = dev.DeviceBuffer(n, _lib.INT32), dev.DeviceBuffer(n, _lib.INT32)
        rb.zero()
        sb.upload(np.full(n, 1 << (bits * rank), np.int32))
        s = comm.Schedule(kind, sb, rb, n, dtype=_lib.INT32, async_=async_, seed=seed + i,
                          buf=comm.BUF_DEVICE, flags=comm.HOLD | comm.ZERO_SB)
        scheds.append((s, sb, rb, n))
    rng = random.Random(2000 + rank)
    bad = []
    comm.barrier()
    for t in range(1, rounds + 1):
        for i, (s, sb, rb, n) in enumerate(scheds):
            time.sleep(rng.random() * jitter_us * 1e-6)
            s.post()
            s.wait()
            m = min(n, 1024)
            head, tail = _download_slice(rb, 0, m), _download_slice(rb, n - m, m)
            v = int(head[0])
            tags = [(v >> (bits * q)) & ((1 << bits) - 1) for q in range(world)]
            if not (np.all(head == v) and np.all(tail == v) and tags == [t % (1 << bits)] * world):
                bad.append((i, t, tags))
            sb.upload(np.full(n, ((t + 1) % (1 << bits)) << (bits * rank), np.int32))
            s.release()
    comm.barrier()
    logs = [s.log() for s, *_ in scheds]
    autos = sum(s.stats()["auto_rounds"] for s, *_ in scheds)
    for s, sb, rb, _ in scheds:
        s.delete()
    comm.finalize()
    return {"bad": bad[:10], "nbad": len(bad), "logs": logs, "auto_rounds": autos}


def gpu_stress_fresh(rank, world, kind, count, rounds=600, async_=3, seed=34495645, jitter_us=300,
                     buf="device"):
    """ESGD_SCHED_HOLD | FRESH_ONLY -- how the deep500 op drives its schedule -- under the
    same stress, in the wrapper's own (racy) order: the gradient for step t is written
    AFTER round t-1 was released, right before the post (opt_esgd_solo...py:301), so a
    peer's activation may carry this rank into round t while it is still writing.  int32
    tags as in gpu_stress; returns every round's decoded result and this rank's fresh
    flags: a rank's share of round t must be its tag t if it had posted the round before
    joining it, and 0 if it had not (never a torn or stale bucket)."""
    import random

    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    comm = _comm()
    host = buf == "host"
    bits = min(10, 31 // world)
    if host:
        sb, rb = np.zeros(count, np.int32), np.zeros(count, np.int32)
    else:
        sb, rb = dev.DeviceBuffer(count, _lib.INT32), dev.DeviceBuffer(count, _lib.INT32)
        rb.zero()
        dev.synchronize()
    s = comm.Schedule(kind, sb, rb, count, dtype=_lib.INT32, async_=async_, seed=seed,
                      buf=comm.BUF_HOST if host else comm.BUF_DEVICE, flags=comm.HOLD | comm.FRESH_ONLY)
    rng = random.Random(3000 + rank)
    m = min(count, 2048)
    vals, fresh, torn = [], [], []
    comm.barrier()
    for t in range(1, rounds + 1):
        time.sleep(rng.random() * jitter_us * 1e-6)
        v = (t % (1 << bits)) << (bits * rank)
        if host:
            sb[:] = v
        else:
            sb.upload(np.full(count, v, np.int32))
        s.post()
        fresh.append(s.wait())
        if host:
            head, tail = rb[:m].copy(), rb[count - m:].copy()
        else:
            head, tail = _download_slice(rb, 0, m), _download_slice(rb, count - m, m)
        vals.append(int(head[0]))
        if not (np.all(head == head[0]) and np.all(tail == head[0])):
            torn.append(t)
        s.release()
    comm.barrier()
    out = {"vals": vals, "fresh": fresh, "torn": torn[:10], "bits": bits, "stats": s.stats()}
    s.delete()
    comm.finalize()
    return out


def gpu_stress_pipelined(rank, world, kind, counts=(4096, 65536, 17, (1 << 20) + 3, 300007, 1025, 65536 * 3,
                                                  (5 << 20) + 1), rounds=150, async_=3, seed=34495645,
                         jitter_us=200, batch=None, fail_exports=None, env=None):
    """The optimizer's pipelined per-tensor order under the activation stress: HOLD |
    FRESH_ONLY schedules (how the deep500 op drives them), every step writes each
    schedule's send bucket in the wrapper's racy order (after the release, right before
    the post) and posts ALL of them, then waits for all, reads and releases -- so many
    rounds of different schedules come due together (shared k_round_batch launches, cut
    differently on every rank, one five-launch size among them) while peers' activations
    carry ranks through rounds they have not posted.  A rank's share of every round must
    be its tag iff it had posted the round before joining it, never torn.  batch: rounds
    per shared launch for this rank (a list: one value per rank).  fail_exports: per rank,
    how many of its first chunk exports fail (ESGD_TEST fail_exports, the runtime's refusals)."""
    import random

    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    if fail_exports is not None and fail_exports[rank]:
        set_test_knobs(fail_exports=fail_exports[rank])
    os.environ.update(env or {})   # data-plane switches, read at their first use
    comm = _comm()
    if batch is not None:
        comm.set_config("batch_rounds", batch[rank] if isinstance(batch, (list, tuple)) else batch)
    bits = min(10, 31 // world)
    scheds = []
    for i, n in enumerate(counts):
        sb, rb = dev.DeviceBuffer(n, _lib.INT32), dev.DeviceBuffer(n, _lib.INT32)
        rb.zero()
        s = comm.Schedule(kind, sb, rb, n, dtype=_lib.INT32, async_=async_, seed=seed + i,
                          buf=comm.BUF_DEVICE, flags=comm.HOLD | comm.FRESH_ONLY)
        scheds.append((s, sb, rb, n))
    dev.synchronize()
    rng = random.Random(4000 + rank)
    vals = [[] for _ in scheds]
    fresh = [[] for _ in scheds]
    torn = []
    progress = os.environ.get("ESGD_PROGRESS_FILE")   # diagnostics: rank, step every 50 steps
    comm.barrier()
    for t in range(1, rounds + 1):
        if progress and t % 50 == 0:
            with open(progress, "a") as f:
                f.write(f"{time.time():.3f} rank {rank} step {t}\n")
        v = (t % (1 << bits)) << (bits * rank)
        for s, sb, rb, n in scheds:
            if rng.random() < 0.3:
                time.sleep(rng.random() * jitter_us * 1e-6)
            sb.upload(np.full(n, v, np.int32))
            s.post()
        for i, (s, sb, rb, n) in enumerate(scheds):
            fresh[i].append(s.wait())
            m = min(n, 1024)
            head, tail = _download_slice(rb, 0, m), _download_slice(rb, n - m, m)
            vals[i].append(int(head[0]))
            if not (np.all(head == head[0]) and np.all(tail == head[0])):
                torn.append((i, t))
            s.release()
    comm.barrier()
    autos = sum(s.stats()["auto_rounds"] for s, *_ in scheds)
    launches = comm.get_config("launches")
    for s, *_ in scheds:
        s.delete()
    comm.set_config("batch_rounds", -1)
    comm.finalize()
    return {"vals": vals, "fresh": fresh, "torn": torn[:10], "bits": bits, "auto_rounds": autos,
            "launches": launches}


def cp_peer_lost(rank, world, stall_s=5.0):
    """Failure detection (the reference has none: a lost peer hangs its ranks, SURVEY.md
    §5): with ESGD_TIMEOUT_S=2 the last rank stops posting after two rounds; every other
    rank's wait for the synchronous round 3 must fail with a timeout error instead of
    hanging, and the job must still shut down once the stalled rank returns."""
    import torch.distributed as dist

    from esgd._lib import EsgdError
    os.environ["ESGD_TIMEOUT_S"] = "2"
    comm = _comm()
    s = comm.Schedule(comm.ALLREDUCE, None, None, 0, buf=comm.BUF_NONE)
    for _ in range(2):
        s.post()
        s.wait()
    out = {"error": None, "elapsed_s": None}
    if rank == world - 1:
        time.sleep(stall_s)
    else:
        s.post()
        t0 = time.perf_counter()
        try:
            s.wait()
        except EsgdError as e:
            out["error"] = str(e)
        out["elapsed_s"] = time.perf_counter() - t0
    dist.barrier()
    s.delete()
    comm.finalize()
    return out


def gpu_stress_churn(rank, world, kind, count=65536, rounds=240, every=20,
                     churn_counts=(16384, (8 << 20) // 4 + 5, 300007, (64 << 20) // 4), jitter_us=200):
    """Schedules created and deleted while another schedule's rounds run under the random
    activation stress (the arena recycles the deleted schedules' buckets; peers keep their
    mappings): every `every` steps all ranks create a temporary allreduce schedule of the
    next size in `churn_counts`, run two rounds of it (checked bitwise against the oracle
    tree) and delete it, between steps of the persistent HOLD | FRESH_ONLY schedule, whose
    rounds are checked as in gpu_stress_fresh."""
    import random

    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    from oracle import ffref
    comm = _comm()
    bits = min(10, 31 // world)
    sb, rb = dev.DeviceBuffer(count, _lib.INT32), dev.DeviceBuffer(count, _lib.INT32)
    rb.zero()
    dev.synchronize()
    s = comm.Schedule(kind, sb, rb, count, dtype=_lib.INT32, async_=3, seed=34495645, buf=comm.BUF_DEVICE,
                      flags=comm.HOLD | comm.FRESH_ONLY)
    rng = random.Random(4000 + rank)
    vals, fresh, torn, churn_ok = [], [], [], []
    comm.barrier()
    for t in range(1, rounds + 1):
        if t % every == 0:
            n = churn_counts[(t // every) % len(churn_counts)]
            tb = dev.DeviceBuffer(n)
            for rr in range(2):
                tb.upload(ffref.fill_uniform(SEED + t + rr, rank, n))
                ts = comm.Schedule(comm.ALLREDUCE, None, tb, n, buf=comm.BUF_DEVICE) if rr == 0 else ts
                ts.post()
                ts.wait()
                m = min(n, 4096)
                got = _download_slice(tb, n - m, m)
                want = ffref.tree_sum([ffref.fill_uniform(SEED + t + rr, q, m, start=n - m) for q in range(world)])
                churn_ok.append(bool(np.array_equal(got.view(np.uint32), want.view(np.uint32))))
            ts.delete()
            tb.close()
        time.sleep(rng.random() * jitter_us * 1e-6)
        sb.upload(np.full(count, (t % (1 << bits)) << (bits * rank), np.int32))
        s.post()
        fresh.append(s.wait())
        head, tail = _download_slice(rb, 0, 2048), _download_slice(rb, count - 2048, 2048)
        vals.append(int(head[0]))
        if not (np.all(head == head[0]) and np.all(tail == head[0])):
            torn.append(t)
        s.release()
    comm.barrier()
    out = {"vals": vals, "fresh": fresh, "torn": torn[:10], "bits": bits, "churn_ok": churn_ok}
    s.delete()
    comm.finalize()
    return out


def gpu_stress_threads(rank, world, kind, counts=(65536, (1 << 20) + 3, 4096), rounds=200, jitter_us=200):
    """The ABI's threading contract (post / wait may come from a thread other than the one
    that initialised, ff.h's callers run ops from framework threads): three
    schedules, each driven by its own thread through the FRESH_ONLY stress at once, so
    posts, waits and releases of different schedules interleave inside the library.
    Returns per schedule the decoded results and this rank's fresh flags."""
    import random
    import threading

    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    comm = _comm()
    bits = min(10, 31 // world)
    scheds = []
    for i, n in enumerate(counts):
        sb, rb = dev.DeviceBuffer(n, _lib.INT32), dev.DeviceBuffer(n, _lib.INT32)
        rb.zero()
        s = comm.Schedule(kind, sb, rb, n, dtype=_lib.INT32, async_=3, seed=34495645 + i, buf=comm.BUF_DEVICE,
                          flags=comm.HOLD | comm.FRESH_ONLY)
        scheds.append((s, sb, rb, n))
    dev.synchronize()
    res = [None] * len(scheds)
    errs = []

    def drive(i):
        try:
            s, sb, rb, n = scheds[i]
            rng = random.Random(5000 + 10 * rank + i)
            vals, fresh, torn = [], [], []
            m = min(n, 1024)
            for t in range(1, rounds + 1):
                time.sleep(rng.random() * jitter_us * 1e-6)
                sb.upload(np.full(n, (t % (1 << bits)) << (bits * rank), np.int32))
                s.post()
                fresh.append(s.wait())
                head, tail = _download_slice(rb, 0, m), _download_slice(rb, n - m, m)
                vals.append(int(head[0]))
                if not (np.all(head == head[0]) and np.all(tail == head[0])):
                    torn.append(t)
                s.release()
            res[i] = {"vals": vals, "fresh": fresh, "torn": torn[:10]}
        except Exception as e:   # reported, not swallowed
            errs.append(repr(e))

    comm.barrier()
    th = [threading.Thread(target=drive, args=(i,)) for i in range(len(scheds))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    comm.barrier()
    for s, *_ in scheds:
        s.delete()
    comm.finalize()
    return {"res": res, "errs": errs, "bits": bits}


def gpu_visibility(rank, world, rounds=6, count=(1 << 20) + 3, small_bytes=None, flag_mode=0, strict=0):
    """Writer-then-post, the hand-off fflib2 orders with a send after the comp and a comp
    after the recv (colls/ffallreduce.c:145-162): right before posting round t, every rank
    rewrites its bucket on a producer stream (no host sync in between) with round t's
    values, and passes that stream to post().  Every element of every round's result must
    be the oracle's tree of round t's buckets -- across GPUs that checks the producer
    ordering, the peers' reads of freshly written HBM over xGMI (the writer's release and
    the reader's acquire) and the pairing flags of the chosen kind (host memory, uncached
    or fine-grained HBM)."""
    import numpy as np

    from esgd import device as dev
    from oracle import ffref
    comm = _comm()
    if small_bytes is not None:
        comm.set_config("small_round_bytes", small_bytes)
    comm.set_config("device_flags", flag_mode)
    comm.set_config("strict_handoffs", strict)
    rb = dev.DeviceBuffer(count)
    s = comm.Schedule(comm.ALLREDUCE, None, rb, count, buf=comm.BUF_DEVICE)
    prod = dev.Stream()
    bad = []
    for t in range(rounds):
        seed = 0x715B + 97 * t
        comm.barrier()
        dev.fill_uniform(rb, seed, rank, stream=prod)   # queued, not waited for
        s.post(prod)
        s.wait()
        got = rb.download()
        want = ffref.tree_sum([ffref.fill_uniform(seed, r, count) for r in range(world)])
        nbad = int(np.count_nonzero(got.view(np.uint32) != want.view(np.uint32)))
        if nbad:
            bad.append((t, nbad))
        comm.barrier()
    s.delete()
    comm.finalize()
    return {"bad": bad, "devices": os.environ.get("ESGD_TEST_DEVICES")}


def gpu_canary(rank, world, count, transport="ipc", path="one_launch", strict=0, rounds=3):
    """The cross-GPU canary (tests/test_dataplane_gpu.py): the writer-then-post pattern of
    gpu_visibility on one transport / round path, and on a mismatch everything needed to
    tell the layers apart -- this rank's device and every rank's, the round, the number of
    bad elements, the first bad index with its value and the oracle's."""
    import numpy as np

    from esgd import device as dev
    from oracle import ffref
    comm = _comm()
    comm.set_transport(transport)
    comm.set_config("small_round_bytes", count * 4 if path == "one_launch" else 0)
    comm.set_config("strict_handoffs", strict)
    rb = dev.DeviceBuffer(count)
    s = comm.Schedule(comm.ALLREDUCE, None, rb, count, buf=comm.BUF_DEVICE)
    prod = dev.Stream()
    bad = []
    for t in range(rounds):
        seed = 0xCA7A + 131 * t
        comm.barrier()
        dev.fill_uniform(rb, seed, rank, stream=prod)   # queued, not waited for
        s.post(prod)
        s.wait()
        got = rb.download()
        want = ffref.tree_sum([ffref.fill_uniform(seed, r, count) for r in range(world)])
        diff = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
        if diff.size:
            i = int(diff[0])
            bad.append({"round": t + 1, "nbad": int(diff.size), "first": i, "got": float(got[i]),
                        "want": float(want[i])})
        comm.barrier()
    s.delete()
    for k in ("small_round_bytes", "strict_handoffs"):
        comm.set_config(k, -1)
    comm.finalize()
    return {"rank": rank, "device": local_device(), "devices": os.environ.get("ESGD_TEST_DEVICES", ""),
            "transport": transport, "path": path, "strict": strict, "count": count, "rounds": rounds,
            "bad": bad}


def _inputs(dname, seed, world, count):
    """Every rank's bucket of one round: splitmix fp32 (and its bf16 / fp64 forms), or the
    int patterns of evaluation/allreduce.c:49 -- with the oracle's result for them."""
    import numpy as np

    from oracle import ffref
    if dname == "fp32":
        xs = [ffref.fill_uniform(seed, r, count) for r in range(world)]
        return xs, ffref.tree_sum(xs)
    if dname == "bf16":
        xs = [ffref.f32_to_bf16(ffref.fill_uniform(seed, r, count)) for r in range(world)]
        return xs, ffref.tree_sum_bf16(xs)
    if dname == "fp64":
        xs = [ffref.fill_uniform(seed, r, count).astype(np.float64) * 1e-3 for r in range(world)]
        return xs, ffref.tree_sum(xs)
    npdt = {"int32": np.int32, "int64": np.int64}[dname]
    xs = [(np.arange(count) + seed % 1000 + 7 * r).astype(npdt) for r in range(world)]
    return xs, ffref.tree_sum(xs)


def gpu_many(rank, world, specs, rounds=3, batch=None, small_bytes=None, strict=0, pipelined=True,
             seed=0xBA7C, straggle_us=0):
    """One ALLREDUCE schedule per (dtype, count) in `specs` (device buckets, in place), every
    round: each rank writes all its buckets, a barrier, then posts every schedule and waits
    for every one (the optimizer's per-tensor pipelining; pipelined=False: post, wait, one
    schedule after the other).  batch: rounds per shared launch (esgd_set_config
    "batch_rounds"), one value for every rank or a list with one per rank -- ranks may cut
    the issue ring into launches differently.  straggle_us: each rank sleeps a random time
    (up to that) between its posts.  Returns every mismatch and this rank's launch count."""
    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    comm = _comm()
    if batch is not None:
        comm.set_config("batch_rounds", batch[rank] if isinstance(batch, (list, tuple)) else batch)
    if small_bytes is not None:
        comm.set_config("small_round_bytes", small_bytes)
    comm.set_config("strict_handoffs", strict)
    dts = {"fp32": _lib.FLOAT, "bf16": _lib.BF16, "fp64": _lib.DOUBLE, "int32": _lib.INT32, "int64": _lib.INT64}
    bufs = [dev.DeviceBuffer(c, dts[d]) for d, c in specs]
    scheds = [comm.Schedule(comm.ALLREDUCE, None, b, c, dtype=dts[d], buf=comm.BUF_DEVICE)
              for b, (d, c) in zip(bufs, specs)]
    rng = np.random.default_rng(1000 + rank)
    bad = []
    workers = []   # pipelined=False: the last shared launch's workers after each round
    l0 = comm.get_config("launches")
    for t in range(rounds):
        wants = []
        for i, ((d, c), b) in enumerate(zip(specs, bufs)):
            xs, want = _inputs(d, seed + 7919 * t + 31 * i, world, c)
            b.upload(xs[rank])
            wants.append(want)
        comm.barrier()
        if pipelined:
            for s in scheds:
                if straggle_us:
                    time.sleep(rng.uniform(0, straggle_us) * 1e-6)
                s.post()
            for s in scheds:
                s.wait()
        else:
            for s in scheds:
                s.post()
                s.wait()
                workers.append(comm.get_config("batch_workers"))
        for i, (b, want) in enumerate(zip(bufs, wants)):
            got = b.download()
            diff = np.nonzero(got.view(np.uint8) != want.view(np.uint8))[0]
            if diff.size:
                bad.append({"round": t + 1, "sched": i, "spec": specs[i], "nbad_bytes": int(diff.size),
                            "first_byte": int(diff[0])})
        comm.barrier()
    launches = comm.get_config("launches") - l0
    for s in scheds:
        s.delete()
    for k in ("batch_rounds", "small_round_bytes", "strict_handoffs"):
        comm.set_config(k, -1)
    comm.finalize()
    return {"bad": bad, "launches": launches, "rounds": rounds * len(specs), "workers": workers}


def gpu_va_reuse(rank, world, value, count=4099, ready_file=None, hold_file=None, rounds=2):
    """One job of tools/va_reuse_probe.py: every rank allocates its bucket (the first arena
    chunk of a fresh process), exports it through an allreduce schedule, checks the sum,
    and reports the bucket's VA.  ready_file: touched (".<rank>") once the rounds are done;
    hold_file: the job does not finalize (its exports and its peers' mappings stay alive)
    until that file exists -- so a second job can export the same VAs meanwhile."""
    import numpy as np

    from esgd import device as dev
    comm = _comm()
    rb = dev.DeviceBuffer(count)
    s = comm.Schedule(comm.ALLREDUCE, None, rb, count, buf=comm.BUF_DEVICE)
    ok = []
    for t in range(rounds):
        rb.upload(np.full(count, float(value + rank + t), np.float32))
        comm.barrier()
        s.post()
        s.wait()
        got = rb.download()
        want = np.float32(sum(float(value + q + t) for q in range(world)))
        ok.append(int(np.count_nonzero(got != want)))
        comm.barrier()
    if ready_file:
        open(f"{ready_file}.{rank}", "w").close()
    if hold_file:
        t0 = time.time()
        while not os.path.exists(hold_file) and time.time() - t0 < 120:
            time.sleep(0.05)
    s.delete()
    comm.finalize()
    return {"rank": rank, "pid": os.getpid(), "va": hex(rb.ptr), "bad_elements": ok}


def gpu_reinit(rank, world, count=4099):
    """A finalized job that mapped its peers' buckets must refuse a second multi-process
    job in the same process (re-opening closed IPC handles: DESIGN.md §5)."""
    import numpy as np

    from esgd import device as dev
    from esgd._lib import EsgdError
    comm = _comm()
    rb = dev.DeviceBuffer(count)
    rb.upload(np.ones(count, np.float32))
    s = comm.Schedule(comm.ALLREDUCE, None, rb, count, buf=comm.BUF_DEVICE)
    s.post(); s.wait()
    ok = bool(np.all(rb.download() == world))
    s.delete()
    comm.finalize()
    err = None
    try:
        comm.init()
        comm.finalize()
    except EsgdError as e:
        err = str(e)
    return {"ok": ok, "err": err}


def gpu_finalize_held(rank, world, n=4, count=1024, delete_first=False):
    """Finalize (or delete) while rounds wait in the pending shared launch: with batch_hold
    nothing but an explicit flush sends it, so after every rank has launched its rounds into
    it (posted, pumped, held), fffinalize -- or each schedule's deletion -- must send them
    while the schedules are alive (the launch used to be flushed after the
    teardown, on freed schedules).  The rounds then pair up across ranks and land: every
    bucket holds the int32 sum of allreduce.c's (i + 7 r) inputs."""
    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    comm = _comm()
    comm.set_config("batch_hold", 1)
    rbs = [dev.DeviceBuffer(count, _lib.INT32) for _ in range(n)]
    for k, rb in enumerate(rbs):
        rb.upload((np.arange(count) + 7 * rank + k).astype(np.int32))
    scheds = [comm.Schedule(comm.ALLREDUCE, None, rb, count, dtype=_lib.INT32, buf=comm.BUF_DEVICE)
              for rb in rbs]
    l0 = comm.get_config("launches")
    comm.barrier()
    for s in scheds:
        s.post()
    time.sleep(0.5)   # every rank's progress thread joins and launches them: held
    import torch.distributed as dist
    dist.barrier()
    launched_before = comm.get_config("launches") - l0
    if delete_first:
        for s in scheds:
            s.delete()
    comm.finalize()
    ok = []
    for k, rb in enumerate(rbs):
        want = sum((np.arange(count) + 7 * r + k) for r in range(world)).astype(np.int32)
        ok.append(bool(np.array_equal(rb.download(), want)))
    return {"ok": ok, "launched_before_finalize": launched_before}


def gpu_post_io(rank, world, count=4099, rounds=3, small_bytes=None, batch=None, shadow_ranks=(),
                plain_ranks=(), divisor=None, separate_dst=True, dtype_name="fp32"):
    """esgd_schedule_post_io on the data plane: every round of an allreduce schedule reads
    this rank's tensor src / divisor itself and writes the result into dst (a separate
    buffer, or src itself), never the send bucket -- checked bit for bit against the
    oracle tree of (x_r / divisor), with rb left to the round.  plain_ranks post their
    share through the send bucket instead (a mixed job); shadow_ranks' buckets are
    shadowed (one-launch rounds of their own beside peers' shared launches)."""
    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    from oracle import ffref
    if rank in shadow_ranks:
        set_test_knobs(shadow=1)
    if small_bytes is not None:
        os.environ["ESGD_SMALL_ROUND_BYTES"] = str(small_bytes)
    comm = _comm()
    if batch is not None:
        comm.set_config("batch_rounds", batch)
    dt = {"fp32": _lib.FLOAT, "int32": _lib.INT32}[dtype_name]
    div = float(world if divisor is None else divisor) if dt == _lib.FLOAT else 1.0
    sb, rb = dev.DeviceBuffer(count, dt), dev.DeviceBuffer(count, dt)
    src, dst = dev.DeviceBuffer(count, dt), dev.DeviceBuffer(count, dt)
    s = comm.Schedule(comm.ALLREDUCE, sb, rb, count, dtype=dt, buf=comm.BUF_DEVICE)
    verdicts, fresh = [], []
    for t in range(rounds):
        if dt == _lib.FLOAT:
            xs = [ffref.fill_uniform(0x10D + t, r, count) for r in range(world)]
        else:
            xs = [(np.arange(count) + t + 7 * r).astype(np.int32) for r in range(world)]
        if rank in plain_ranks:
            sb.upload(xs[rank] / np.float32(div) if dt == _lib.FLOAT else xs[rank])
        else:
            src.upload(xs[rank])
        dst.upload(np.full(count, 7, dtype=xs[0].dtype))
        comm.barrier()
        if rank in plain_ranks:
            s.post()
        else:
            s.post_io(src, dst if separate_dst else src, div)
        fresh.append(s.wait())
        out = rb if rank in plain_ranks else (dst if separate_dst else src)
        got = out.download()
        want = ffref.tree_sum([x / np.float32(div) for x in xs]) if dt == _lib.FLOAT else \
            sum(x.astype(np.int64) for x in xs).astype(np.int32)
        same = bool(np.array_equal(got.view(np.uint8), want.view(np.uint8)))
        verdicts.append(same if same else mismatch(t, got, want, xs, s))
        comm.barrier()
    s.delete()
    comm.finalize()
    return {"verdicts": verdicts, "fresh": fresh}


def gpu_post_io_late(rank, world, count=4099, steps=8, async_=3, late=1):
    """post_io under solo's asynchronous rounds: HOLD | FRESH_ONLY (how the deep500 op runs
    them), rank `late` posts LATE_S after its peers every step.  A round the early rank's
    activation carries the late rank through before its post does not take its data: wait
    says fresh = 0, its dst keeps what it held, and the round's result (its share zero) is
    in rb; a round it posted in time takes src and writes dst.  Every rank's result must be
    the oracle tree of (x_r / P if rank r's round was fresh else 0), the same bits on every
    rank."""
    import numpy as np
    import torch.distributed as dist

    from esgd import device as dev
    from oracle import ffref
    comm = _comm()
    rb = dev.DeviceBuffer(count)
    src, dst = dev.DeviceBuffer(count), dev.DeviceBuffer(count)
    s = comm.Schedule(comm.SOLO, None, rb, count, async_=async_, seed=6545343, buf=comm.BUF_DEVICE,
                      flags=comm.HOLD | comm.FRESH_ONLY)
    out = []
    for t in range(steps):
        xs = [ffref.fill_uniform(0x1A7E + t, r, count) for r in range(world)]
        src.upload(xs[rank])
        dst.upload(np.full(count, 3.0, np.float32))
        comm.barrier()
        if rank == late and t > 0:
            time.sleep(LATE_S)
        s.post_io(src, dst, float(world))
        f = s.wait()
        res = (dst if f else rb).download()
        untouched = f or bool(np.all(dst.download() == np.float32(3.0)))
        s.release()
        fr = [None] * world
        dist.all_gather_object(fr, bool(f))
        want = ffref.tree_sum([x / np.float32(world) if fr[r] else np.zeros_like(x) for r, x in enumerate(xs)])
        out.append({"t": t, "fresh": fr, "untouched": untouched, "ok": bool(np.array_equal(res.view(np.uint32),
                                                                                          want.view(np.uint32))),
                    "digest": zlib.crc32(res.tobytes())})
    comm.barrier()
    s.delete()
    comm.finalize()
    return out


def gpu_residency(rank, world, hog_ms=6000, free_cus=2, rounds=4, counts=(1 << 20, 65536, 17, 300007, 1025)):
    """Batched rounds while a concurrent kernel holds almost the whole GPU (verdict r04 item
    3): rank 0 starts k_occupy (tools/bin/libesgd_sweeps.so) on a side stream -- 2 x CUs -
    2 x free_cus workgroups of 16 waves, resident for hog_ms -- then every rank posts one
    round of five one-launch schedules (one shared k_round_batch launch per rank) and waits.
    Those rounds must complete on the few workgroup slots left, long before the hog ends:
    workers take tiles from the launch's counter, so the resident ones do every tile
    (first_round_s; the five are held -- batch_hold -- until all are in the pending launch,
    then sent together: 64 + 1 + ... tiles per phase, more workers than fit).  The
    launch's workgroups that did not fit are dispatched, find the list done and leave once
    the hog does -- only then can the stream's next launch start, so the later rounds
    (checked for their bits) wait for the hog.  int32 inputs of allreduce.c, (i + t + 7 r)."""
    import ctypes as C

    import numpy as np

    from esgd import _lib
    from esgd import device as dev
    comm = _comm()
    sw = C.CDLL(os.path.join(ROOT, "tools", "bin", "libesgd_sweeps.so"))
    sw.esgd_sweep_occupy.restype, sw.esgd_sweep_occupy.argtypes = C.c_int, [C.c_int, C.c_uint64, C.c_void_p]
    sw.esgd_sweep_cu_count.restype = C.c_int
    bufs = [(dev.DeviceBuffer(n, _lib.INT32), dev.DeviceBuffer(n, _lib.INT32)) for n in counts]
    scheds = [comm.Schedule(comm.ALLREDUCE, sb, rb, n, dtype=_lib.INT32, buf=comm.BUF_DEVICE)
              for n, (sb, rb) in zip(counts, bufs)]
    ok, times = [], []

    def one_round(t, held=False):
        for n, (sb, _) in zip(counts, bufs):
            sb.upload((np.arange(n) + t + 7 * rank).astype(np.int32))
        comm.barrier()
        if held:   # every round joined and launched into the pending shared launch first
            comm.set_config("batch_hold", 1)
        t0 = time.perf_counter()
        for s_ in scheds:
            s_.post()
        if held:
            time.sleep(0.3)
            t0 = time.perf_counter()
            comm.set_config("batch_hold", 0)   # the next progress pass sends all of them
        for s_ in scheds:
            s_.wait()
        times.append(time.perf_counter() - t0)
        for n, (_, rb) in zip(counts, bufs):
            want = sum((np.arange(n) + t + 7 * r) for r in range(world)).astype(np.int32)
            ok.append(bool(np.array_equal(rb.download(), want)))

    t_start = time.perf_counter()

    def note(what):   # progress on stderr (shown with the failure if the test times out)
        print(f"[gpu_residency r{rank} +{time.perf_counter() - t_start:.2f}s] {what}", file=sys.stderr, flush=True)

    for t in range(2):   # warm: the descriptors exist before the hog
        one_round(t)
    note("warm rounds done")
    side = dev.Stream()
    comm.barrier()
    t_hog = time.perf_counter()
    if rank == 0:
        blocks = 2 * sw.esgd_sweep_cu_count() - 2 * free_cus
        assert sw.esgd_sweep_occupy(blocks, int(hog_ms * 1000), side.handle) == 0
        time.sleep(0.2)   # resident before the round starts
    comm.barrier()
    note("hog launched" if rank == 0 else "past the hog barrier")
    for t in range(2, 2 + rounds):
        one_round(t, held=t == 2)
        note(f"round {t} done in {times[-1]:.3f}s")
    side.synchronize()
    hog_s = time.perf_counter() - t_hog
    note(f"hog stream synchronized after {hog_s:.2f}s")
    comm.barrier()
    workers = comm.get_config("batch_workers")
    for s_ in scheds:
        s_.delete()
    note("schedules deleted")
    comm.finalize()
    return {"first_round_s": times[2], "round_s": times, "hog_s": hog_s, "ok": ok, "workers": workers}


def gpu_late_peer_after_timeout(rank, world, cases, delay_s=4.0):
    """The failure contract: the last rank's GPU runs the
    round `delay_s` late -- its post names a producer stream on which a 1-workgroup k_occupy
    (tools/bin/libesgd_sweeps.so) holds it, as a backward pass still writing the gradient
    would -- so the other ranks' GPU flag waits time out (ESGD_TIMEOUT_S, set by the caller)
    first.  They must fail.  The late rank must fail too, or return the oracle's sum of the
    data that really arrived -- never success with a sum built from its peers' shards, which
    they folded from its STALE bucket (the previous round's result).  Each case (kind, path)
    runs one good round (data A), then the late round (data B).  int32 inputs, exact."""
    import ctypes as C

    import numpy as np
    import torch.distributed as dist

    from esgd import _lib
    from esgd import device as dev
    comm = _comm()
    sw = C.CDLL(os.path.join(ROOT, "tools", "bin", "libesgd_sweeps.so"))
    sw.esgd_sweep_occupy.restype, sw.esgd_sweep_occupy.argtypes = C.c_int, [C.c_int, C.c_uint64, C.c_void_p]
    late = world - 1
    side = dev.Stream()   # the late rank's "backward": the producer of its late round
    kinds = {"allreduce": comm.ALLREDUCE, "solo": comm.SOLO, "majority": comm.MAJORITY}
    out = []
    for kind, path in cases:
        count = (3 << 20) if path == "five" else 300007   # 12 MiB: above the one-launch threshold
        comm.set_config("batch_rounds", 0 if path == "one" else -1)
        sb, rb = dev.DeviceBuffer(count, _lib.INT32), dev.DeviceBuffer(count, _lib.INT32)
        # solo with async 1: round 2 is synchronous, joined at each rank's own post (an async
        # round would carry the late rank through on a peer's activation, without its producer)
        s_ = comm.Schedule(kinds[kind], sb, rb, count, dtype=_lib.INT32, buf=comm.BUF_DEVICE, async_=1, seed=7)
        a = [(np.arange(count) * 3 + 11 * r).astype(np.int32) for r in range(world)]
        b = [(np.arange(count) % 977 + 1000 * r + 5).astype(np.int32) for r in range(world)]
        sb.upload(a[rank])
        dist.barrier()   # gloo: esgd's own barrier times out with the 2 s limit
        s_.post()
        s_.wait()
        good = bool(np.array_equal(rb.download(), sum(a).astype(np.int32)))
        sb.upload(b[rank])
        dist.barrier()   # gloo: esgd's own barrier times out with the 2 s limit
        t0 = time.perf_counter()
        if rank == late:
            assert sw.esgd_sweep_occupy(1, int(delay_s * 1e6), side.handle) == 0
            s_.post(stream=side)
            # the host's own wait limit counts from wait(): wait only shortly before the GPU
            # runs the round, so the GPU's flag protocol decides rank 1's outcome
            time.sleep(delay_s - 0.5)
        else:
            s_.post()
        err, result = None, None
        try:
            s_.wait()
            got = rb.download()
            result = "oracle" if np.array_equal(got, sum(b).astype(np.int32)) else "WRONG"
        except Exception as e:   # esgd.EsgdError
            err = str(e).splitlines()[0][:300]
        side.synchronize()
        el = time.perf_counter() - t0
        dist.barrier()   # gloo: esgd's own barrier times out with the 2 s limit
        s_.delete()
        comm.set_config("batch_rounds", -1)
        out.append({"kind": kind, "path": path, "first_round_ok": good, "failed": err is not None,
                    "result": result, "err": err, "elapsed_s": round(el, 2),
                    # the round's failure words (this rank's GPU, or a peer's), not the host's
                    # own wait limit ("wait timed out [rank ...")
                    "gpu_failure": err is not None and ("failed round" in err or "GPU waited" in err)})
        print(f"[late_peer r{rank}] {kind}/{path}: {out[-1]}", file=sys.stderr, flush=True)
    comm.finalize()
    return out


def op_void_peer_lost(rank, world, count=5000):
    """The deep500-shaped void entry point under ESGD_OP_ON_ERROR_LOCAL: rank 1 runs one
    step and leaves; rank 0's next (synchronous) round times out, and instead of aborting
    the process the op writes rank 0's own gradient to the output and keeps the status."""
    import numpy as np

    from esgd import deep500
    os.environ["ESGD_TIMEOUT_S"] = "3"
    comm = _comm()
    deep500.configure("allreduce", 32, 6545343)
    deep500.on_error("local")
    op = deep500.AllreduceOp((count,))
    x = np.full(count, 0.5 + rank, np.float32)
    first = op.forward_void(x)          # step 1: both ranks
    out = {"first_ok": bool(np.all(first == sum(0.5 + r for r in range(world))))}
    if rank == 0:
        t0 = time.time()
        second = op.forward_void(x)     # rank 1 never posts this round
        out.update(elapsed=time.time() - t0, own=bool(np.array_equal(second, x)), status=op.status())
    return out


def cp_connect_failure(rank, world, bad_rank=1):
    """One rank's connect fails: every rank's creation fails at the connect vote (the
    second creation barrier), none waits for the timeout, and the communicator stays
    usable for the next schedule."""
    if rank == bad_rank:
        set_test_knobs(fail_connect=rank)
    from esgd import comm
    from esgd._lib import EsgdError
    comm.init()
    err, s = None, None
    t0 = time.time()
    try:
        s = comm.Schedule(comm.ALLREDUCE, None, None, 0, buf=comm.BUF_NONE)
    except EsgdError as e:
        err = str(e)
    t_fail = time.time() - t0
    if s is not None:
        s.delete()
    os.environ.pop("ESGD_TEST", None)
    comm.barrier()
    s2 = comm.Schedule(comm.ALLREDUCE, None, None, 0, buf=comm.BUF_NONE)
    for _ in range(2):
        s2.post()
        s2.wait()
    s2.delete()
    comm.finalize()
    return {"create_err": err, "t_fail": t_fail}


def cp_fresh_queue(rank, world, rounds=300):
    """wait()'s fresh bit survives any run-ahead: rank 0 posts round 1, then
    rank 1 activates rounds 1..`rounds` (solo, no synchronous round in between), so rank
    0's progress thread joins rounds 2..rounds on those activations before rank 0 waits
    for anything.  Rank 0's waits must then report round 1 fresh and every later one not
    (a 256-slot ring indexed by round reported round 1 as round 257's)."""
    comm = _comm()
    s = comm.Schedule(comm.SOLO, None, None, 0, async_=100000, buf=comm.BUF_NONE)
    if rank == 0:
        s.post()
    comm.barrier()
    if rank == 1:
        for _ in range(rounds):
            s.post()
    comm.barrier()
    t0 = time.time()
    while s.stats()["joined"] < rounds and time.time() - t0 < 30:
        time.sleep(0.001)
    fresh = [s.wait() for _ in range(rounds)] if rank == 0 else []
    if rank == 1:
        for _ in range(rounds):
            s.wait()
    joined = s.stats()["joined"]
    comm.barrier()
    s.delete()
    comm.finalize()
    return {"fresh": fresh, "joined": joined}


def cp_pipelined_steps(rank, world, steps=50, kind=2, n=161, idle=0):
    """The per-tensor call pattern on the control plane alone (ESGD_BUF_NONE: join, ticket,
    issue ring and completion with a transport that moves nothing): `n` schedules, every
    step posts all of them, then waits for all.  Median step and, on the last step, the
    host timeline relative to the first post (tools/host_engine_probe.py)."""
    import statistics

    import numpy as np
    comm = _comm()
    # `idle` more schedules, never posted (a process that keeps other jobs' schedules alive:
    # every progress pass still walks them)
    others = [comm.Schedule(kind, None, None, 0, seed=6545343, buf=comm.BUF_NONE) for _ in range(idle)]
    scheds = [comm.Schedule(kind, None, None, 0, seed=6545343, buf=comm.BUF_NONE) for _ in range(n)]
    ts = []
    for _ in range(steps):
        comm.barrier()
        t0 = time.perf_counter()
        for s in scheds:
            s.post()
        for s in scheds:
            s.wait()
        ts.append(time.perf_counter() - t0)
    rows = []
    for s in scheds:
        tl = s.timeline().astype(np.int64)
        tl = tl[(tl[:, 0] > 0) & (tl[:, 5] > 0)]
        if len(tl):
            rows.append(tl[-1])
    tl = np.array(rows)
    t0 = tl[:, 0].min()
    rel = {k: round(float(tl[:, i].max() - t0) / 1e3, 1) for k, i in
           (("last_post", 0), ("last_join", 1), ("last_launch_queued", 3), ("last_completion", 4),
            ("last_wait", 5))}
    # per schedule, in creation order: post, join, launch, completion relative to the first post
    per = [[round(float(r[i] - t0) / 1e3, 1) for i in (0, 1, 3, 4, 5)] for r in tl]
    comm.barrier()
    for s in scheds + others:
        s.delete()
    comm.finalize()
    return {"step_us_median": round(statistics.median(ts[2:]) * 1e6, 1), "last_step": rel, "per_sched": per}


def cp_post_group(rank, world, n=12, rounds=20, kind=2):
    """esgd_schedule_post_group on the control plane: `n` schedules, every round posted as
    one group on half the steps and one by one on the others; the roles, the round logs and
    the activators must be those of single posts (the same draws in the same order)."""
    comm = _comm()
    scheds = [comm.Schedule(kind, None, None, 0, seed=6545343 + i, async_=3, buf=comm.BUF_NONE)
              for i in range(n)]
    roles = []
    for t in range(rounds):
        comm.barrier()
        roles.append(comm.post_group(scheds) if t % 2 == 0 else [s.post() for s in scheds])
        for s in scheds:
            s.wait()
    comm.barrier()
    logs = [s.log() for s in scheds]
    for s in scheds:
        s.delete()
    comm.finalize()
    return {"roles": roles, "logs": logs}


def cp_profile(rank, world, n=5, rounds=10):
    """esgd_comm_profile counts what the progress thread did: every round joined once."""
    comm = _comm()
    p0 = comm.profile()
    scheds = [comm.Schedule(comm.ALLREDUCE, None, None, 0, buf=comm.BUF_NONE) for _ in range(n)]
    for _ in range(rounds):
        comm.post_group(scheds)
        for s in scheds:
            s.wait()
    p1 = comm.profile()
    comm.barrier()
    for s in scheds:
        s.delete()
    comm.finalize()
    return {k: p1[k] - p0[k] for k in p0}


def cp_create_many(rank, world, n=161, rounds=1):
    """`n` schedules created back to back (the per-tensor wrapper's 161 buckets,
    opt_esgd_solo_imagenet_imbalance.py:85-248), each run for `rounds` rounds, then deleted:
    the creation cost per schedule (two node barriers each) on the control plane."""
    from esgd import comm
    comm.init()
    comm.barrier()
    t0 = time.perf_counter()
    scheds = [comm.Schedule(comm.SOLO, None, None, 0, buf=comm.BUF_NONE) for _ in range(n)]
    t_create = time.perf_counter() - t0
    for _ in range(rounds):
        for s in scheds:
            s.post()
        for s in scheds:
            s.wait()
    for s in scheds:
        s.delete()
    comm.finalize()
    return {"create_ms_per_schedule": t_create * 1e3 / n}


def gpu_post_iov(rank, world, count=4099, rounds=3, in_place=False):
    """esgd_schedule_post_iov: the round's data in three fp32 pieces (sizes 1, 1000 and the
    rest; the middle one starting off any 16-B boundary), packed / divisor into the bucket
    and unpacked into the destinations by the round itself (one-launch rounds: a launch of
    their own; larger: the five launches) -- the oracle tree of (x_r / P), bit for bit, in
    every piece, every round."""
    import numpy as np

    from esgd import device as dev
    from oracle import ffref
    comm = _comm()
    sizes = [1, 1000, count - 1001]
    sb, rb = dev.DeviceBuffer(count), dev.DeviceBuffer(count)
    s = comm.Schedule(comm.ALLREDUCE, sb, rb, count, buf=comm.BUF_DEVICE)
    srcs = [dev.DeviceBuffer(n) for n in sizes]
    dsts = srcs if in_place else [dev.DeviceBuffer(n) for n in sizes]
    ok, fresh = [], []
    for t in range(rounds):
        xs = [ffref.fill_uniform(0x10F + t, r, count) for r in range(world)]
        o = 0
        for b, n in zip(srcs, sizes):
            b.upload(xs[rank][o:o + n])
            o += n
        comm.barrier()
        s.post_iov(srcs, dsts, float(world))
        fresh.append(s.wait())
        got = np.concatenate([b.download() for b in dsts])
        want = ffref.tree_sum([x / np.float32(world) for x in xs])
        same = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
        ok.append(same if same else mismatch(t, got, want, xs, s))
        comm.barrier()
    s.delete()
    comm.finalize()
    return {"ok": ok, "fresh": fresh}
