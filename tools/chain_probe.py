"""Where does a 161-bucket step go?  The reference's wrapper reduces one bucket per
ResNet-50 gradient tensor, one after another (opt_esgd_solo_imagenet_imbalance.py:24-44,
301-316).  Run under torch.distributed.run; prints, per rank, the step time, the sum of
the per-round timelines split into stages, and the host gap between one round's wait and
the next round's post.  Diagnostic tool only."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "eager-sgd_amd"))


def main():
    import torch  # noqa: F401  (one HIP runtime: torch first)
    import torch.distributed as dist

    import esgd
    from esgd import comm, device as dev

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    esgd.check(esgd.lib().esgd_set_device(int(os.environ.get("LOCAL_RANK", "0")) % esgd.device_count()),
               "set_device")
    dist.init_process_group("gloo")
    comm.init()
    kind = {"allreduce": comm.ALLREDUCE, "solo": comm.SOLO, "majority": comm.MAJORITY}[
        os.environ.get("LAT_KIND", "majority")]
    with open(os.path.join(ROOT, "tests", "golden", "resnet50_buckets.json")) as f:
        lengths = json.load(f)["lengths"]
    pre = []   # CHAIN_PRE=MiB,MiB,...: live schedules over big buckets first (bench's earlier legs)
    for mib in [float(x) for x in os.environ.get("CHAIN_PRE", "").split(",") if x]:
        b = dev.DeviceBuffer(int(mib * (1 << 20)) // 4)
        dev.fill_uniform(b, 2, rank)
        dev.synchronize()
        s = comm.Schedule(kind, None, b, b.count, seed=6545343, async_=32, buf=comm.BUF_DEVICE)
        for _ in range(3):
            s.post()
            s.wait()
        pre.append((s, b))
    if os.environ.get("CHAIN_EARLY") == "1":   # first round (and round stream) before the streams
        b = dev.DeviceBuffer(1024)
        s0 = comm.Schedule(kind, None, b, b.count, seed=6545343, async_=32, buf=comm.BUF_DEVICE)
        s0.post()
        s0.wait()
        pre.append((s0, b))
    extra = []  # CHAIN_STREAMS=n: n more streams with one memset each (HW queue count)
    for _ in range(int(os.environ.get("CHAIN_STREAMS", "0"))):
        st = dev.Stream()
        z = dev.DeviceBuffer(1024)
        z.zero(st)
        st.synchronize()
        extra.append((st, z))
    if os.environ.get("CHAIN_PAGEABLE") == "1":   # one 4-byte D2H into pageable memory
        from esgd._lib import check, lib
        z = dev.DeviceBuffer(1024)
        cell = np.zeros(1, np.float32)
        check(lib().esgd_memcpy_async(cell.ctypes.data, z.ptr, 4, 1, None))
        dev.synchronize()
        extra.append((None, z))
    bufs = [dev.DeviceBuffer(n) for n in lengths]
    for b in bufs:
        dev.fill_uniform(b, 1, rank)
    dev.synchronize()
    scheds = [comm.Schedule(kind, None, b, b.count, seed=6545343, async_=32, buf=comm.BUF_DEVICE)
              for b in bufs]
    steps = int(os.environ.get("CHAIN_STEPS", "6"))
    walls = []
    for _ in range(steps):
        comm.barrier()
        t0 = time.perf_counter()
        for s in scheds:
            s.post()
            s.wait()
        walls.append(time.perf_counter() - t0)
    names = ["post_join", "join_launch", "launch_host", "gpu_round", "wake"]
    tl = np.stack([s.timeline().astype(np.int64)[-1] for s in scheds])   # last step
    d = np.stack([tl[:, i + 1] - tl[:, i] for i in range(5)], 1) / 1e3
    gap = (tl[1:, 0] - tl[:-1, 5]) / 1e3          # wait returned -> next post
    small = np.array(lengths) * 4 <= (4 << 20)
    out = {"rank": rank, "step_ms_median": round(float(np.median(walls)) * 1e3, 3),
           "rounds_small": int(small.sum()), "rounds_large": int((~small).sum()),
           "sum_us_small": {n: round(float(d[small, i].sum()), 1) for i, n in enumerate(names)},
           "sum_us_large": {n: round(float(d[~small, i].sum()), 1) for i, n in enumerate(names)},
           "median_us_small": {n: round(float(np.median(d[small, i])), 1) for i, n in enumerate(names)},
           "host_gap_us_sum": round(float(gap.sum()), 1),
           "host_gap_us_median": round(float(np.median(gap)), 1)}
    if tl[:, 11].any():
        gn = ["g_wait_ready", "g_rs", "g_wait_reduced", "g_ag", "g_wait_done"]
        out["gpu_median_us_small"] = {n: round(float(np.median(tl[small, 6 + i])) / 1e3, 1)
                                      for i, n in enumerate(gn)}
    print("[chain] " + json.dumps(out), flush=True)
    comm.barrier()
    for s in scheds:
        s.delete()
    for b in bufs:
        b.close()
    for s, b in pre:
        s.delete()
        b.close()
    comm.finalize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
