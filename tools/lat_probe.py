"""Where does a small round's time go?  Run under torch.distributed.run (N ranks, any
GPUs); per bucket size prints the median of each stage of the per-round timeline
(esgd_schedule_timeline) on every rank, in microseconds.  Diagnostic tool only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "eager-sgd_amd"))


def main():
    import torch  # noqa: F401  (one HIP runtime: torch first)
    import torch.distributed as dist

    import esgd
    from esgd import comm, device as dev
    from esgd import _lib

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = esgd.device_count()
    esgd.check(esgd.lib().esgd_set_device(int(os.environ.get("LOCAL_RANK", "0")) % ndev), "set_device")
    dist.init_process_group("gloo")
    comm.init()
    kind = {"allreduce": comm.ALLREDUCE, "solo": comm.SOLO, "majority": comm.MAJORITY}[
        os.environ.get("LAT_KIND", "allreduce")]
    names = ["post->join", "join->launch", "launch(host)", "queued->done", "done->wait", "post->wait"]
    kept = []
    for nbytes in [int(x) for x in os.environ.get("LAT_SIZES", "65536,4194304,67108864").split(",")]:
        count = nbytes // 4
        buf = dev.DeviceBuffer(count, _lib.FLOAT)
        dev.fill_uniform(buf, 1, rank)
        dev.synchronize()
        s = comm.Schedule(kind, None, buf, count, buf=comm.BUF_DEVICE, async_=3, seed=6545343)
        iters = int(os.environ.get("LAT_ITERS", "60"))
        comm.barrier()
        for _ in range(iters):
            s.post()
            s.wait()
        tl = s.timeline().astype(np.int64)[10:]
        d = np.stack([tl[:, 1] - tl[:, 0], tl[:, 2] - tl[:, 1], tl[:, 3] - tl[:, 2],
                      tl[:, 4] - tl[:, 3], tl[:, 5] - tl[:, 4], tl[:, 5] - tl[:, 0]], 1) / 1e3
        ok = tl[:, 0] > 0
        med = np.median(d[ok], 0)
        # round period (post of t+1 - post of t)
        per = np.median(np.diff(tl[:, 0])) / 1e3
        line = " ".join(f"{n}={m:.1f}" for n, m in zip(names, med))
        g = np.median(tl[:, 6:12], 0) / 1e3
        if g.any():
            line += " | gpu " + " ".join(f"{n}={m:.1f}" for n, m in zip(
                ["w_ready", "rs", "w_reduced", "ag", "w_done", "total"], g))
        print(f"[lat] rank {rank} bytes {nbytes}: {line} period={per:.1f}us", flush=True)
        if os.environ.get("LAT_KEEP") == "1":
            kept.append((s, buf))
        elif os.environ.get("LAT_NOFREE") == "1":   # delete the schedule, keep the bucket
            s.delete()
            kept.append((None, buf))
        else:
            s.delete()
            buf.close()
    for s, buf in kept:
        if s is not None:
            s.delete()
        buf.close()
    comm.finalize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
