"""Multi-rank data plane on the GPU: P processes (all on device 0 of the test box, one
per GPU on a full node) run persistent schedules over IPC-mapped peer buffers.

Bar: every rank's receive buffer is bit-identical to the oracle's restatement of
fflib2's recursive doubling (src/colls/ffallreduce.c:138-171) for the same inputs;
int32 also matches the known answer of evaluation/allreduce.c:59-63.  Partial
(solo / majority) rounds are checked through round tags: rank r contributes
t * 64**r in round t, so the reduced value names the round each rank's buffer held.
"""
import pytest

from mp_workers import run
from oracle import ffref

pytestmark = pytest.mark.gpu
ALLREDUCE, SOLO, MAJORITY = 0, 1, 2


SMALL = {"one_launch": None, "five_launch": 0}   # ESGD_SMALL_ROUND_BYTES per round path


@pytest.mark.parametrize("path", sorted(SMALL))
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("dtype", ["fp32", "int32", "bf16", "fp64", "int64"])
def test_allreduce_bitwise_device(world, dtype, path):
    verdicts = run("gpu_allreduce", world, dtype_name=dtype, count=100003, rounds=2,
                   small_bytes=SMALL[path])
    assert all(all(v) for v in verdicts), verdicts


@pytest.mark.parametrize("path", sorted(SMALL))
@pytest.mark.parametrize("world", [2, 3, 8])
def test_allreduce_ragged_and_tiny(world, path):
    for count in (1, 17, 1023, 4099):
        verdicts = run("gpu_allreduce", world, count=count, rounds=1, small_bytes=SMALL[path])
        assert all(all(v) for v in verdicts), (count, verdicts)


@pytest.mark.parametrize("world", [2, 5])
def test_one_launch_rounds_back_to_back(world):
    # many consecutive one-launch rounds of one schedule (flags, counters and fin reused
    # every round), at the size limit of the one-launch path and just above it
    for count, small in ((1 << 20, 4 << 20), ((1 << 20) + 3, 4 << 20)):
        verdicts = run("gpu_allreduce", world, count=count, rounds=6, small_bytes=small)
        assert all(all(v) for v in verdicts), (count, verdicts)


@pytest.mark.parametrize("in_place", [False, True])
def test_allreduce_host_buffers(in_place):
    # the reference's contract: host buckets in, host result out (staged through HBM)
    verdicts = run("gpu_allreduce", 2, count=262144, rounds=2, buf="host", in_place=in_place)
    assert all(all(v) for v in verdicts), verdicts


@pytest.mark.parametrize("in_place", [False, True])
@pytest.mark.parametrize("world", [1, 2, 3])
def test_allreduce_host_chunked(world, in_place):
    # host buckets of >= 2 chunks run chunk by chunk (H2D of one chunk beside the D2H of
    # the previous); 64 KiB chunks: 7 chunks, the last one ragged, 3 rounds back to back
    verdicts = run("gpu_allreduce", world, count=100003, rounds=3, buf="host", in_place=in_place,
                   host_chunk=65536)
    assert all(all(v) for v in verdicts), verdicts


@pytest.mark.parametrize("dtype", ["fp64", "bf16", "int32"])
def test_allreduce_host_chunked_dtypes(dtype):
    verdicts = run("gpu_allreduce", 2, dtype_name=dtype, count=70001, rounds=2, buf="host",
                   host_chunk=32768)
    assert all(all(v) for v in verdicts), verdicts


def test_allreduce_host_chunked_default_size():
    # 36 MB host bucket: three 16 MiB-class chunks at the default chunk size
    verdicts = run("gpu_allreduce", 2, count=9_000_003, rounds=2, buf="host")
    assert all(all(v) for v in verdicts), verdicts


def test_allreduce_in_place_device():
    verdicts = run("gpu_allreduce", 4, count=65536 * 4 + 5, rounds=2, in_place=True)
    assert all(all(v) for v in verdicts), verdicts


@pytest.mark.parametrize("world", [2, 3])
def test_allreduce_in_pieces(world):
    # shards are moved in pieces of at most 1 GiB (ff.h's 2^31 - 1 fp32 bucket has 4 GiB
    # shards at P = 2); 4 KiB pieces drive the same code with a small bucket, ragged last
    # pieces and more than 16 gather segments included
    for count in (100003, 65536 * 3 + 1):
        verdicts = run("gpu_allreduce", world, count=count, rounds=2, small_bytes=0, piece_bytes=4096)
        assert all(all(v) for v in verdicts), (count, verdicts)


def test_schedule_and_bucket_churn():
    # create / run / delete / free, again and again, mixing sizes, dtypes and tiny
    # sub-allocated buckets: mappings of freed buckets stay open on the peers
    verdicts = run("gpu_churn", 2)
    # (step, dtype, count, round, mismatched bytes, first, last) per rank and round
    bad = [v for per_rank in verdicts for v in per_rank if v[4]]
    assert not bad, bad


@pytest.mark.parametrize("kind", [SOLO, MAJORITY])
def test_solo_majority_round_tags(kind):
    world, rounds, async_ = 2, 9, 3
    outs = run("gpu_partial_semantics", world, kind=kind, rounds=rounds, async_=async_,
               straggler=1, delay=0.05)
    digits = lambda v, r: int(v // 64 ** r) % 64  # noqa: E731
    fast = outs[0]
    acts = ffref.activators(6545343, world, rounds)
    prev = [0] * world
    for t, v in enumerate(fast["results"], start=1):
        d = [digits(v, r) for r in range(world)]
        assert v == sum(d[r] * 64 ** r for r in range(world)), v
        for r in range(world):
            assert d[r] <= t and d[r] >= prev[r], (t, d)   # buffers only move forward
        prev = d
        if kind == SOLO:
            assert d[0] == t                                 # the fast rank is always fresh
            if t % (async_ + 1) == 0:
                assert d == [t] * world                      # synchronous round: everyone
        else:
            assert d[acts[t - 1]] == t                       # the activator is fresh
    # a rank that joined a round it had posted contributed that round's tag
    for r, o in enumerate(outs):
        for e in o["log"]:
            if e["fresh"] and r == 0:
                assert digits(fast["results"][e["round"] - 1], r) == e["round"]


@pytest.mark.parametrize("kind", [ALLREDUCE, SOLO])
def test_rccl_transport_single_rank(kind):
    # RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so on a 1-GPU box the
    # RCCL transport can only run at world size 1: communicator bring-up, ticket ring,
    # the full round protocol and the copy paths (host and device buckets).
    for buf in ("device", "host"):
        verdicts = run("gpu_allreduce", 1, count=300007, rounds=3, kind=kind, buf=buf,
                       transport="rccl")
        assert all(all(v) for v in verdicts), (buf, verdicts)


@pytest.mark.parametrize("in_place", [False, True])
def test_shadowed_device_buckets(in_place):
    # a rank whose device bucket cannot be exported reduces through an owned shadow
    # bucket (copy in at the snapshot, out at the finish); mixed with direct ranks
    verdicts = run("gpu_allreduce", 3, count=200003, rounds=2, in_place=in_place, shadow_ranks=(1,))
    assert all(all(v) for v in verdicts), verdicts
