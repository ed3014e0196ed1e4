"""Scratch: pure HIP IPC reproducer (no esgd kernels).  P processes on one GPU export a
buffer, import every peer's, check a few bytes through the mapping, close, free; then
the same with a bigger buffer.  Prints mismatches per (size, peer)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import mp_workers  # noqa: E402


class Handle(C.Structure):
    _fields_ = [("reserved", C.c_char * 64)]


def worker(rank, world, sizes, free=True, kernel=False, read_first=True, hostreg=False, engine=False):
    import torch.distributed as dist
    import esgd
    from esgd import device as dev
    hip = C.CDLL("libamdhip64.so")
    hip.hipSetDevice(0)
    if engine:   # the esgd node communicator: registered segment + progress thread
        from esgd import comm
        comm.init()
        s0 = comm.Schedule(0, None, dev.DeviceBuffer(4096), 4096, buf=comm.BUF_DEVICE)
    if hostreg:
        hb = (C.c_char * (1 << 20))()
        assert hip.hipHostRegister(hb, C.c_size_t(1 << 20), 2) == 0
    loc = dev.DeviceBuffer(max(sizes) // 4)
    vp = C.c_void_p
    hip.hipSetDevice(0)
    out = []
    keep = []
    for si, size in enumerate(sizes):
        p = vp()
        assert hip.hipMalloc(C.byref(p), C.c_size_t(size)) == 0
        val = (rank * 16 + si + 1) & 0xFF
        assert hip.hipMemset(p, val, C.c_size_t(size)) == 0
        assert hip.hipDeviceSynchronize() == 0
        h = Handle()
        assert hip.hipIpcGetMemHandle(C.byref(h), p) == 0
        hs = [None] * world
        dist.all_gather_object(hs, bytes(h))
        maps = []
        bad = []
        for q in range(world):
            if q == rank:
                continue
            m = vp()
            hh = Handle.from_buffer_copy(hs[q])
            hip.hipIpcOpenMemHandle.argtypes = [C.POINTER(vp), Handle, C.c_uint]
            rc = hip.hipIpcOpenMemHandle(C.byref(m), hh, 1)
            assert rc == 0, rc
            maps.append(m)
            want = (q * 16 + si + 1) & 0xFF
            if si == 0 and not read_first:
                continue
            for off in (0, size // 2, size - 4096):
                buf = (C.c_uint8 * 4096)()
                if kernel:   # the whole peer buffer read through the mapping by the tree kernel
                    if off == 0:
                        dev.reduce(esgd.FLOAT, [m.value], loc, size // 4)
                        dev.synchronize()
                    assert hip.hipMemcpy(buf, C.c_void_p(loc.ptr + off), C.c_size_t(4096), 2) == 0
                else:
                    assert hip.hipMemcpy(buf, C.c_void_p(m.value + off), C.c_size_t(4096), 2) == 0
                got = set(buf)
                if got != {want}:
                    bad.append((q, off, sorted(got)[:4], want))
        dist.barrier()
        for m in maps:
            hip.hipIpcCloseMemHandle(m)
        dist.barrier()
        if free:
            hip.hipFree(p)
        else:
            keep.append(p)
        dist.barrier()
        out.append((size, bad))
    return out


mp_workers.ipc_worker = worker

if __name__ == "__main__":
    MiB = 1 << 20
    for name, kw in [("noread", dict(read_first=False)), ("hostreg", dict(read_first=False, hostreg=True)),
                     ("engine", dict(read_first=False, engine=True))]:
        if True:
            world = 8
            res = mp_workers.run("ipc_worker", world, sizes=[16 * MiB, 256 * MiB], free=True, kernel=True,
                                 timeout=300, **kw)
            nbad = [[len(b) for _, b in per] for per in res]
            print(f"world {world} {name}: mismatches per size {nbad}", flush=True)
            for r, per in enumerate(res):
                for size, b in per:
                    if b:
                        print(f"  rank {r} size {size}: {b[:3]}", flush=True)
                        break
