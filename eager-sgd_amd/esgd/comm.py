"""Node communicator and persistent partial-allreduce schedules (esgd.h C ABI).

Mirrors fflib2's collective surface (src/ff.h:161-165, src/ffschedule.c) one level
below the optimizer wrapper:

    comm.init()                                   # ffinit (rendezvous + progress thread)
    s = comm.Schedule(comm.SOLO, sb, rb, count, async_=32)   # ffsolo_allreduce
    s.post(); s.wait()                            # ffschedule_post / ffschedule_wait

Buffers are device pointers (ints, DeviceBuffer or torch tensors), host numpy arrays
(host staging mode, the reference's contract) or None with buf=NONE (control plane only).
"""
from __future__ import annotations

import ctypes as C
import os
import uuid

import numpy as np

from . import _lib
from ._lib import check, lib

ALLREDUCE, SOLO, MAJORITY = 0, 1, 2
BUF_DEVICE, BUF_HOST, BUF_NONE = 0, 1, 2
HOLD, ZERO_SB, WIRE_BF16, FRESH_ONLY = 0x1, 0x2, 0x4, 0x8   # esgd_schedule_create_ex flags (esgd.h)


class SchedStats(C.Structure):
    _fields_ = [("posted", C.c_uint32), ("joined", C.c_uint32), ("completed", C.c_uint32),
                ("waited", C.c_uint32), ("activated", C.c_uint32), ("last_activator", C.c_int32),
                ("fresh_rounds", C.c_uint64), ("auto_rounds", C.c_uint64),
                ("activations", C.c_uint64)]


def _bind(h):
    vp, i, u32, u64 = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64
    sigs = {
        "esgd_comm_init": (i, [C.c_char_p, i, i]),
        "esgd_comm_finalize": (i, []),
        "esgd_comm_rank": (i, [C.POINTER(i)]),
        "esgd_comm_size": (i, [C.POINTER(i)]),
        "esgd_barrier": (i, []),
        "esgd_schedule_create": (i, [i, i, vp, vp, u64, i, i, C.c_uint, C.POINTER(u64)]),
        "esgd_schedule_create_ex": (i, [i, i, vp, vp, u64, i, i, C.c_uint, C.c_uint, C.POINTER(u64)]),
        "esgd_schedule_wait_ex": (i, [u64, C.POINTER(i)]),
        "esgd_schedule_post_iov": (i, [u64, i, C.POINTER(vp), C.POINTER(vp), C.POINTER(u64), C.c_float, vp,
                                       C.POINTER(i)]),
        "esgd_schedule_release": (i, [u64, vp]),
        "esgd_schedule_post": (i, [u64, vp, C.POINTER(i)]),
        "esgd_schedule_wait": (i, [u64]),
        "esgd_schedule_test": (i, [u64, C.POINTER(i)]),
        "esgd_schedule_delete": (i, [u64]),
        "esgd_schedule_stats": (i, [u64, C.POINTER(SchedStats)]),
        "esgd_schedule_log": (i, [u64, C.POINTER(u32), C.POINTER(C.c_uint8), C.POINTER(C.c_uint8),
                                  C.POINTER(C.c_int16), u32, C.POINTER(u32)]),
        "esgd_schedule_stream": (i, [u64, C.POINTER(vp)]),
        "esgd_schedule_timeline": (i, [u64, C.POINTER(u64), u32, C.POINTER(u32)]),
        "esgd_set_transport": (i, [C.c_char_p]),
        "esgd_set_config": (i, [C.c_char_p, C.c_int64]),
        "esgd_get_config": (i, [C.c_char_p, C.POINTER(C.c_int64)]),
        "esgd_comm_issue_log": (i, [C.POINTER(u32), C.POINTER(u32), u32, C.POINTER(u32)]),
        "esgd_comm_profile": (i, [C.POINTER(u64), i]),
        "esgd_schedule_post_group": (i, [C.POINTER(u64), i, vp, C.POINTER(i)]),
        "esgd_schedule_release_group": (i, [C.POINTER(u64), i, vp]),
        "esgd_schedule_post_io": (i, [u64, vp, vp, C.c_float, vp, C.POINTER(i)]),
        "esgd_schedule_post_group_io": (i, [C.POINTER(u64), i, C.POINTER(vp), C.POINTER(vp), C.c_float, vp,
                                            C.POINTER(i)]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(h, name)
        fn.restype, fn.argtypes = res, args


_lib.register_signatures(_bind)

_state = {"init": False}


def _default_job_id(rank: int, world: int) -> str:
    """A job id every rank agrees on: broadcast over torch.distributed when it is up,
    else derived from the launcher's environment."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            obj = [uuid.uuid4().hex if dist.get_rank() == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            return obj[0]
    except Exception:
        pass
    if os.environ.get("ESGD_JOB_ID"):
        return os.environ["ESGD_JOB_ID"]
    if os.environ.get("TORCHELASTIC_RUN_ID"):
        return f"{os.environ['TORCHELASTIC_RUN_ID']}-{os.environ.get('MASTER_PORT', '0')}"
    if world == 1:
        return f"single-{os.getpid()}"
    raise RuntimeError("esgd.comm.init: no job id (pass job_id= or set ESGD_JOB_ID)")


def init(job_id: str | None = None, rank: int | None = None, world: int | None = None):
    """Join the node communicator (collective).  Uses the current HIP device."""
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    if world is None:
        world = int(os.environ.get("WORLD_SIZE", "1"))
    if job_id is None:
        job_id = _default_job_id(rank, world)
    check(lib().esgd_comm_init(job_id.encode(), rank, world), "esgd_comm_init")
    _state["init"] = True
    return rank, world


def finalize():
    if _state["init"]:
        check(lib().esgd_comm_finalize(), "esgd_comm_finalize")
        _state["init"] = False


def rank() -> int:
    v = C.c_int()
    check(lib().esgd_comm_rank(C.byref(v)))
    return v.value


def world() -> int:
    v = C.c_int()
    check(lib().esgd_comm_size(C.byref(v)))
    return v.value


def set_transport(name: str):
    """Data plane of schedules created afterwards: "ipc" (default) or "rccl"."""
    check(lib().esgd_set_transport(name.encode()), "esgd_set_transport")


def set_config(key: str, value: int):
    """Data-plane setting captured by schedules created afterwards (esgd_set_config):
    "small_round_bytes" (one-launch rounds up to this size), "device_flags" (0 host,
    1 uncached HBM, 2 fine-grained HBM pairing flags) or "strict_handoffs" (1: acq_rel
    counts, release gates and an L2 write-back in one-launch rounds); -1 restores the default.  Every
    rank must set the same value before the same creations."""
    check(lib().esgd_set_config(key.encode(), int(value)), "esgd_set_config")


def get_config(key: str) -> int:
    v = C.c_int64()
    check(lib().esgd_get_config(key.encode(), C.byref(v)), "esgd_get_config")
    return v.value


def issue_log():
    """(schedule id, round) in the order this rank issued ordered (rccl) rounds."""
    n = C.c_uint32()
    check(lib().esgd_comm_issue_log(None, None, 0, C.byref(n)))
    cap = n.value
    a = (C.c_uint32 * max(1, cap))(); b = (C.c_uint32 * max(1, cap))()
    check(lib().esgd_comm_issue_log(a, b, cap, C.byref(n)))
    return [(a[i], b[i]) for i in range(min(cap, n.value))]


PROFILE_KEYS = ("passes", "pass_ns", "launch_ns", "joins", "join_ns", "launches", "flush_ns")


def profile() -> dict:
    """The progress thread's host-side profile since init (esgd_comm_profile): monotonic
    counters -- subtract two readings."""
    v = (C.c_uint64 * len(PROFILE_KEYS))()
    check(lib().esgd_comm_profile(v, len(PROFILE_KEYS)), "esgd_comm_profile")
    return dict(zip(PROFILE_KEYS, (int(x) for x in v)))


def barrier():
    check(lib().esgd_barrier(), "esgd_barrier")


def _buf_arg(x, buf):
    if x is None:
        return None
    if buf == BUF_HOST:
        assert isinstance(x, np.ndarray) and x.flags.c_contiguous
        return x.ctypes.data
    from .device import as_ptr
    return as_ptr(x)


def _stream_arg(stream):
    s = None if stream is None else (stream.handle if hasattr(stream, "handle") else int(stream))
    return 1 if s == 0 else s   # 0: the legacy default stream (ESGD_STREAM_NULL)


def post_group(scheds, stream=None) -> list:
    """Post every schedule in this order with ONE producer event (esgd_schedule_post_group);
    returns the roles (1 activated, 0 passive, 2 synchronous)."""
    n = len(scheds)
    hs = (C.c_uint64 * n)(*[s.handle for s in scheds])
    roles = (C.c_int * n)(*([-1] * n))
    check(lib().esgd_schedule_post_group(hs, n, _stream_arg(stream), roles), "esgd_schedule_post_group")
    return list(roles)


def release_group(scheds, stream=None):
    """Release every HOLD schedule with ONE consumer event (esgd_schedule_release_group)."""
    n = len(scheds)
    hs = (C.c_uint64 * n)(*[s.handle for s in scheds])
    check(lib().esgd_schedule_release_group(hs, n, _stream_arg(stream)), "esgd_schedule_release_group")


class Schedule:
    """A persistent schedule (ffallreduce / ffsolo_allreduce / ffrand_allreduce)."""

    def __init__(self, kind: int, sb, rb, count: int, dtype: int = _lib.FLOAT,
                 async_: int = 0, seed: int = 0, buf: int | None = None, flags: int = 0):
        if buf is None:
            buf = BUF_HOST if isinstance(rb, np.ndarray) else BUF_NONE if rb is None else BUF_DEVICE
        self.kind, self.buf, self.count, self.dtype = kind, buf, int(count), dtype
        self._keep = (sb, rb)   # host arrays must outlive the schedule
        h = C.c_uint64()
        check(lib().esgd_schedule_create_ex(kind, buf, _buf_arg(sb, buf), _buf_arg(rb, buf),
                                            self.count, dtype, int(async_), int(seed) & 0xFFFFFFFF,
                                            int(flags), C.byref(h)), "esgd_schedule_create")
        self.handle = h.value

    def post(self, stream=None) -> int:
        """stream: producer of sb (None = no producer; 0 = the legacy default stream,
        e.g. torch's default stream, passed on as ESGD_STREAM_NULL)."""
        role = C.c_int()
        s = None if stream is None else (stream.handle if hasattr(stream, "handle") else int(stream))
        if s == 0:
            s = 1   # ESGD_STREAM_NULL
        check(lib().esgd_schedule_post(self.handle, s, C.byref(role)), "esgd_schedule_post")
        return role.value

    def post_io(self, src, dst, divisor: float = 1.0, stream=None) -> int:
        """esgd_schedule_post_io: the round reads src / divisor instead of the send bucket
        and writes its result into dst (device pointers, 16-B aligned) -- if this rank joins
        it at or after this post (wait() then returns True); otherwise dst is untouched and
        the result is in rb."""
        from .device import as_ptr
        role = C.c_int()
        s = None if stream is None else (stream.handle if hasattr(stream, "handle") else int(stream))
        if s == 0:
            s = 1   # ESGD_STREAM_NULL
        check(lib().esgd_schedule_post_io(self.handle, as_ptr(src), as_ptr(dst), float(divisor), s, C.byref(role)),
              "esgd_schedule_post_io")
        return role.value

    def post_iov(self, srcs, dsts, divisor: float = 1.0, stream=None) -> int:
        """esgd_schedule_post_iov: the round's data in fp32 pieces (tensors / buffers whose
        sizes sum to the schedule's count): packed (/ divisor) into the bucket and the result
        unpacked into dsts by the round itself, if this rank joins it at or after this post."""
        from .device import ptr_array_of
        n = len(srcs)
        counts = (C.c_uint64 * max(1, n))(*[int(x.numel()) if hasattr(x, "numel") else int(x.count)
                                            for x in srcs])
        role = C.c_int()
        s = None if stream is None else (stream.handle if hasattr(stream, "handle") else int(stream))
        if s == 0:
            s = 1   # ESGD_STREAM_NULL
        src = ptr_array_of(srcs)
        dst = src if dsts is srcs else ptr_array_of(dsts)
        check(lib().esgd_schedule_post_iov(self.handle, n, src, dst, counts, float(divisor), s,
                                           C.byref(role)), "esgd_schedule_post_iov")
        return role.value

    def wait(self) -> bool:
        """Returns whether this rank had posted the round before joining it (False: a
        peer's activation carried it through with what its send bucket held)."""
        f = C.c_int()
        check(lib().esgd_schedule_wait_ex(self.handle, C.byref(f)), "esgd_schedule_wait")
        return bool(f.value)

    def release(self, stream=None):
        """HOLD schedules: done with the last round's buckets (work queued on `stream`
        is waited for by the next round's snapshot; 0 = the legacy default stream)."""
        s = None if stream is None else (stream.handle if hasattr(stream, "handle") else int(stream))
        if s == 0:
            s = 1   # ESGD_STREAM_NULL
        check(lib().esgd_schedule_release(self.handle, s), "esgd_schedule_release")

    def test(self) -> bool:
        f = C.c_int()
        check(lib().esgd_schedule_test(self.handle, C.byref(f)), "esgd_schedule_test")
        return bool(f.value)

    def stats(self) -> dict:
        st = SchedStats()
        check(lib().esgd_schedule_stats(self.handle, C.byref(st)), "esgd_schedule_stats")
        return {k: getattr(st, k) for k, _ in SchedStats._fields_}

    def log(self):
        n = C.c_uint32()
        check(lib().esgd_schedule_log(self.handle, None, None, None, None, 0, C.byref(n)))
        cap = n.value
        r = (C.c_uint32 * cap)(); f = (C.c_uint8 * cap)(); s = (C.c_uint8 * cap)()
        a = (C.c_int16 * cap)()
        check(lib().esgd_schedule_log(self.handle, r, f, s, a, cap, C.byref(n)))
        return [{"round": r[i], "fresh": bool(f[i]), "sync": bool(s[i]), "activator": a[i]}
                for i in range(min(cap, n.value))]

    def timeline(self):
        """Per completed round (numpy uint64, rounds x 12): CLOCK_MONOTONIC ns of post,
        join, launch start, launch queued, completion seen, wait returned; then GPU spans
        in ns (ESGD_GPU_TRACE=1): ready wait, reduce-scatter, reduced wait, all-gather,
        done wait, total."""
        n = C.c_uint32()
        check(lib().esgd_schedule_timeline(self.handle, None, 0, C.byref(n)))
        out = np.zeros((max(1, n.value), 12), np.uint64)
        check(lib().esgd_schedule_timeline(self.handle, out.ctypes.data_as(C.POINTER(C.c_uint64)),
                                           n.value, C.byref(n)))
        return out[: n.value]

    def stream(self) -> int:
        v = C.c_void_p()
        check(lib().esgd_schedule_stream(self.handle, C.byref(v)))
        return v.value or 0

    def delete(self):
        if self.handle:
            check(lib().esgd_schedule_delete(self.handle), "esgd_schedule_delete")
            self.handle = 0
