"""Which host-side HIP action puts a process's peer-reading kernels into the slow state?
Run under torch.distributed.run (2 ranks).  A 64 KiB allreduce schedule is timed (median
post->wait over 200 rounds), then one action is applied on every rank, then it is timed
again, for a list of actions in order.  Diagnostic tool only."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "eager-sgd_amd"))


def main():
    import torch  # noqa: F401  (one HIP runtime: torch first)
    import torch.distributed as dist

    import esgd
    from esgd import _lib, comm, device as dev

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    esgd.check(esgd.lib().esgd_set_device(0), "set_device")
    dist.init_process_group("gloo")
    comm.init()
    n = 16384
    buf = dev.DeviceBuffer(n)
    dev.fill_uniform(buf, 1, rank)
    dev.synchronize()
    s = comm.Schedule(comm.ALLREDUCE, None, buf, n, buf=comm.BUF_DEVICE)

    def measure(tag):
        comm.barrier()
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            s.post()
            s.wait()
            ts.append(time.perf_counter() - t0)
        med = statistics.median(ts[20:]) * 1e6
        if rank == 0:
            print(f"[slow] after {tag:38s} round {med:7.1f} us", flush=True)

    keep = []
    st = dev.Stream()

    def a_big_alloc_free():
        b = dev.DeviceBuffer(16 << 20)
        b.close()

    def a_small_alloc():
        keep.append(dev.DeviceBuffer(64))

    def a_small_free():
        keep.pop().close()

    def a_memset_async_big():
        b = dev.DeviceBuffer(16 << 20)
        b.zero(stream=st)
        st.synchronize()
        keep.append(b)

    def a_memset_sync_small():
        b = dev.DeviceBuffer(64)
        esgd.check(esgd.lib().esgd_memset_async(b.ptr, 0, 256, None), "memset")
        dev.synchronize()
        keep.append(b)

    def a_d2h():
        buf.download()

    def a_other_schedule():
        b = dev.DeviceBuffer(n)
        o = comm.Schedule(comm.ALLREDUCE, None, b, n, buf=comm.BUF_DEVICE)
        o.post(); o.wait()
        o.delete()
        keep.append(b)

    def a_free_kept():
        while keep:
            keep.pop().close()

    measure("start")
    for name, fn in (("16 MiB alloc+free", a_big_alloc_free), ("64-element alloc", a_small_alloc),
                     ("64-element free", a_small_free), ("memsetAsync 16 MiB (own stream)", a_memset_async_big),
                     ("memset 256 B (library stream)", a_memset_sync_small), ("D2H download", a_d2h),
                     ("free everything kept", a_free_kept),
                     ("another schedule created+deleted", a_other_schedule)):
        fn()
        dev.synchronize()
        measure(name)
    s.delete()
    buf.close()
    comm.finalize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
