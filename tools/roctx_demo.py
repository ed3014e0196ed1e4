"""A few rounds of one schedule in one process, for `rocprofv3 --marker-trace`
(ESGD_ROCTX=1): shows the round / launch / wait ranges next to the round's kernels."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "eager-sgd_amd"))


def main():
    import torch  # noqa: F401  (one HIP runtime in the process, as in the tests)
    from esgd import _lib, comm
    from esgd import device as dev
    comm.init(job_id="roctx-demo-%d" % os.getpid(), rank=0, world=1)
    for count in (1 << 14, 1 << 22):
        rb = dev.DeviceBuffer(count, _lib.FLOAT)
        sb = dev.DeviceBuffer(count, _lib.FLOAT)
        dev.fill_uniform(sb, 1, 0)
        s = comm.Schedule(comm.SOLO, sb, rb, count, async_=2, buf=comm.BUF_DEVICE)
        for _ in range(6):
            s.post()
            s.wait()
        s.delete()
        rb.close()
        sb.close()
    comm.finalize()
    print("roctx demo done")


if __name__ == "__main__":
    main()
