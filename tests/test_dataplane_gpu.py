"""Multi-rank data plane on the GPU: P processes (device rank % device_count: all on
device 0 of a 1-GPU box, one per GPU on a full node, where the peer reads cross xGMI)
run persistent schedules over IPC-mapped peer buffers.

Bar: every rank's receive buffer is bit-identical to the oracle's restatement of
fflib2's recursive doubling (src/colls/ffallreduce.c:138-171) for the same inputs;
int32 also matches the known answer of evaluation/allreduce.c:59-63.  Partial
(solo / majority) rounds are checked through round tags: rank r contributes
t * 64**r in round t, so the reduced value names the round each rank's buffer held.
"""
import os

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


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("world", [2, 3])
def test_device_pairing_flags(world, mode):
    # ESGD_DEVICE_FLAGS (opt-in): pairing flags in uncached (1) / fine-grained (2) HBM pages,
    # every kind of round: one launch, five launches, chunked host buckets, majority
    for kw in (dict(count=4099, small_bytes=4 << 20), dict(count=300007, small_bytes=0),
               dict(count=(32 << 20) // 4 + 5, buf="host", host_chunk=16 << 20),
               dict(count=65536, kind=2)):
        verdicts = run("gpu_allreduce", world, rounds=3, device_flags=mode, **kw)
        assert all(all(v) for v in verdicts), (kw, verdicts)


@pytest.mark.parametrize("world", [2, 5])
def test_one_launch_rounds_back_to_back(world):
    # many consecutive one-launch rounds of one schedule (flags, counters and fin reused
    # every round), at the size limit of the one-launch path and just above it
    for count, small in ((1 << 20, 4 << 20), ((1 << 20) + 3, 4 << 20)):
        verdicts = run("gpu_allreduce", world, count=count, rounds=6, small_bytes=small)
        assert all(all(v) for v in verdicts), (count, verdicts)


# ---- batched one-launch rounds (k_round_batch) -----------------------------------------
# Rounds that come due together in issue order share one launch: a flag agent publishes
# every round's ready flag at once and turns peers' flags into gates, workers walk the
# rounds' tiles in ring order.  Every round must give the oracle's bits, however the
# ranks cut the ring into launches.

MIXED = [("fp32", 1), ("fp32", 17), ("fp32", 4099), ("fp32", 65536 + 3), ("fp32", 300007),
         ("fp32", (1 << 20) + 3), ("fp32", 1000), ("fp32", 64), ("fp32", 262144), ("fp32", 5)]


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_batched_rounds_bitwise(world):
    # ten schedules of ragged sizes posted back to back then waited (the optimizer's
    # pipelined per-tensor pattern): fewer launches than rounds, every round bit-exact
    outs = run("gpu_many", world, specs=MIXED, rounds=3)
    for o in outs:
        assert not o["bad"], o["bad"]
        assert o["launches"] < o["rounds"], o


def test_batched_rounds_mixed_dtypes_and_five_launch_rounds():
    # a dtype change cuts the launch; a bucket above the one-launch size goes out as a
    # five-launch round between batched ones (the pending launch is flushed first)
    specs = [("fp32", 4099), ("int32", 70001), ("bf16", 65539), ("fp64", 1025), ("fp32", (2 << 20) + 7),
             ("int64", 333), ("fp32", 100003), ("bf16", 9)]
    outs = run("gpu_many", 3, specs=specs, rounds=3, small_bytes=1 << 20)
    for o in outs:
        assert not o["bad"], o["bad"]


def test_batched_launch_grid_for_every_dtype():
    # every dtype's shared launch gets the workers its tiles ask for: bf16's dtype code (16)
    # once fell outside the residency cache, every bf16 launch ran ONE worker and bf16
    # rounds were 10-20x slower (bench sweep_c5_majority_bf16, round 4)
    specs = [(d, 1 << 18) for d in ("fp32", "bf16", "fp64", "int32", "int64")]
    outs = run("gpu_many", 2, specs=specs, rounds=1, pipelined=False)
    for o in outs:
        assert not o["bad"], o["bad"]
        assert len(o["workers"]) == len(specs)
        for (d, _), w in zip(specs, o["workers"]):
            assert w >= 8, (d, o["workers"])


def test_batched_rounds_cut_differently_per_rank():
    # rank 0 batches up to 64 rounds, rank 1 one round per launch (k_round_small), rank 2
    # three, rank 3 two; random delays between posts: no deadlock, every round bit-exact
    outs = run("gpu_many", 4, specs=MIXED * 3, rounds=3, batch=[64, 0, 3, 2], straggle_us=300)
    for o in outs:
        assert not o["bad"], o["bad"]


@pytest.mark.parametrize("strict", [0, 1])
def test_batched_rounds_resnet50_table(strict):
    # the reference's 161 per-tensor buckets (opt_esgd_solo_imagenet_imbalance.py:86-248):
    # at the default one-launch size 156 of them go out in shared launches, 5 as
    # five-launch rounds; relaxed and strict hand-offs
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "resnet50_buckets.json")) as f:
        lengths = json.load(f)["lengths"]
    outs = run("gpu_many", 2, specs=[("fp32", n) for n in lengths], rounds=2, strict=strict, timeout=400)
    for o in outs:
        assert not o["bad"], o["bad"][:5]
        assert o["launches"] < o["rounds"], o


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
    # the wire flag is accepted on this transport; a world of one returns the bucket
    verdicts = run("gpu_allreduce", 1, count=300007, rounds=2, kind=kind, wire=True, transport="rccl")
    assert all(all(v) for v in verdicts), verdicts


@pytest.mark.parametrize("in_place", [False, True])
def test_shadowed_device_buckets(in_place):
    # a rank whose device bucket cannot be exported reduces through an owned shadow
    # bucket (copy in at the snapshot, out at the finish); mixed with direct ranks
    verdicts = run("gpu_allreduce", 3, count=200003, rounds=2, in_place=in_place, shadow_ranks=(1,))
    assert all(all(v) for v in verdicts), verdicts


@pytest.mark.parametrize("count", [1, 17, 4099])
def test_shadowed_rank_beside_batched_ranks(count):
    # a shadowed rank's one-launch rounds go out one per launch (k_round_small + copy-out)
    # while its peers' go out in shared launches (k_round_batch): the same flags, the same
    # bits; tiny buckets leave a rank with an empty shard
    for world, shadow in ((2, (0,)), (2, (1,)), (3, (1,))):
        verdicts = run("gpu_allreduce", world, count=count, rounds=3, shadow_ranks=shadow)
        assert all(all(v) for v in verdicts), (world, shadow, verdicts)


@pytest.mark.parametrize("batch", [None, 0])
@pytest.mark.parametrize("count", [1, 17, 4099])
def test_refused_export_on_one_rank(count, batch):
    # the runtime refused a fresh process's first chunk export on ONE rank (round 4, r04d:
    # count 1 at P = 2 then came out wrong on both ranks); ESGD_TEST fail_exports on that rank
    # only: its published shard moves to a fresh chunk and its bucket is shadowed, while
    # the peer's rounds stay batched
    for fails in ((1, 0), (2, 0), (0, 2)):
        verdicts = run("gpu_allreduce", 2, count=count, rounds=3, fail_exports=fails, batch=batch)
        assert all(all(v) for v in verdicts), (fails, verdicts)


@pytest.mark.parametrize("count,small", [(17, None), (4099, None), (300007, 0)])
@pytest.mark.parametrize("fails", [(1, 0), (0, 2), (3, 0)])
def test_wrong_mapping_is_remapped(fails, count, small):
    # round 5 (r05b): a fresh mapping of a peer's chunk showed the importer's OWN exported
    # chunk (the seal caught it).  ESGD_TEST fail_maps makes a rank's first N sealed mappings
    # count as such: the exporter moves the publication to a new chunk (its own bucket is
    # shadowed), every rank maps again, up to kRemapTries (3) times -- then bit-exact rounds
    verdicts = run("gpu_allreduce", 2, count=count, rounds=2, fail_maps=fails, small_bytes=small)
    assert all(all(v) for v in verdicts), (fails, verdicts)


def test_wrong_mapping_retries_exhausted_fails_every_rank():
    # four wrong mappings in a row on rank 0 (initial connect + 3 retries): the creation
    # fails on every rank, naming the mapping, instead of hanging or summing other memory
    with pytest.raises(AssertionError, match="other memory|another rank failed"):
        run("gpu_allreduce", 2, count=4099, rounds=1, fail_maps=(4, 0), timeout=120)


# ---- BASELINE.json's workloads (C1, C3, C4, C5) at their full sizes -----------------
# Every rank writes its bucket before a barrier and posts (the pattern of
# evaluation/{solo,rand}_allreduce_correctness.c:76-97): solo / majority rounds then
# equal the plain allreduce, checked bit for bit on head, middle and tail slices of
# every rank's result (mp_workers.gpu_config).

def _all_ok(outs):
    bad = [(r, v) for r, per in enumerate(outs) for v in per if not v[3]]
    assert not bad, bad


def test_c1_majority_2_ranks_1mib():
    # C1: 2-rank majority-allreduce of one 1 MiB fp32 bucket, seed 6545343
    _all_ok(run("gpu_config", 2, kind=MAJORITY, counts=[262144], rounds=4, seed=6545343))


@pytest.mark.timeout(900)
def test_c3_solo_8_ranks_256mib():
    # C3: 8-rank solo-allreduce of one 256 MiB fp32 bucket per rank (LIMITER 32)
    _all_ok(run("gpu_config", 8, kind=SOLO, counts=[64 << 20], rounds=2, async_=32, timeout=420))


@pytest.mark.timeout(900)
def test_c4_majority_8_ranks_resnet50():
    # C4: 8-rank majority-allreduce of the ResNet-50 fused gradient, 25 559 081 fp32
    # (opt_esgd_solo_imagenet_imbalance.py:86-248 summed; ragged: not a multiple of 4)
    _all_ok(run("gpu_config", 8, kind=MAJORITY, counts=[25559081], rounds=3, timeout=420))


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.timeout(900)
def test_c5_majority_8_ranks_sweep(dtype):
    # C5: 8-rank majority-allreduce at 64 KiB, 1 MiB, 16 MiB, 256 MiB and 1 GiB buckets
    es = 4 if dtype == "fp32" else 2
    counts = [(1 << lg) // es for lg in (16, 20, 24, 28, 30)]
    _all_ok(run("gpu_config", 8, kind=MAJORITY, counts=counts, dtype_name=dtype, rounds=2,
                timeout=600))


# ---- partial semantics with a straggler ---------------------------

def _check_straggler(outs, world, kind, async_=3, seed=6545343):
    acts = ffref.activators(seed, world, 64)
    for r, o in enumerate(outs):
        assert o["delay_requested_s"] >= 2 * o["T_s"], o
        if r == world - 1:
            assert o["delay_achieved_s"] >= o["delay_requested_s"], o
        for t, c, uniform in o["rounds"]:
            assert uniform, (r, t)
            if kind == MAJORITY:
                want = world if acts[t - 1] == world - 1 else world - 1
            else:
                want = world if t % (async_ + 1) == 0 else world - 1
            assert c == want, (r, t, c, want, acts[t - 1])
        if kind == MAJORITY:   # the activator of every asynchronous round: libc rand_r
            for e in o["log"]:
                assert e["activator"] == acts[e["round"] - 1], e


def test_majority_straggler_c4_20pct():
    # BASELINE C4 as stated: 8 ranks, the 25 559 081-float ResNet-50 gradient, one rank
    # 20 % of a round late.  A 0.2 T delay races the round (the straggler may or may not
    # make it), so: rounds the straggler activates (rand_r draw, ffrand_allreduce.c:88)
    # wait for it and take all P; every other round takes P - 1 or P per element, the same
    # bits on every rank (rsgd.c:87,100 contributor counting).  Per element, not per bucket:
    # a round another rank activates joins the straggler passively, and its bucket is read
    # as it stands at that moment -- possibly while the straggler's own copy into it is
    # still running, so part of the bucket holds the fresh 1.0s and part the zeros.  The
    # reference has the same race: the activated progress thread moves sb -> rb
    # (ffallreduce.c:125-127) while the op's memcpy into sb
    # (opt_esgd_majority_imagenet_imbalance.py:302, before ffschedule_post at :305) may
    # be in flight.  Every rank then reduces the same snapshot.
    world = 8
    outs = run("gpu_straggler", world, kind=MAJORITY, count=25559081, rounds=8, delay_frac=0.2, timeout=420)
    acts = ffref.activators(6545343, world, 64)
    for r, o in enumerate(outs):
        # the straggler's ACHIEVED delay (a spin to the deadline, then its late gradient
        # written; measured barrier -> post) is the 0.2 T asked for plus that write, within
        # 10 % or 100 us; the on-time ranks post at once
        want = 0.2 * o["T_s"]
        if r == world - 1:
            assert want <= o["delay_achieved_s"] <= want + o["fill_s"] + max(0.1 * want, 100e-6), o
        else:
            assert o["delay_achieved_s"] < want, o
        for (t, c, uniform), (lo, hi, crc) in zip(o["rounds"], o["slices"]):
            if acts[t - 1] == world - 1:
                assert uniform and c == world, (r, t, c)
            else:
                assert world - 1 <= lo <= hi <= world, (r, t, lo, hi)
            assert crc == outs[0]["slices"][t - 4][2], (r, t)   # same bits on every rank
        for e in o["log"]:
            assert e["activator"] == acts[e["round"] - 1], e


@pytest.mark.parametrize("world,count,rounds", [(4, 1 << 20, 12), (8, 25559081, 8)])
@pytest.mark.timeout(900)
def test_majority_straggler_excluded(world, count, rounds):
    # the last rank is >= 2 T late every round: rounds another rank activates take P - 1
    # fresh gradients, rounds the straggler activates wait for it and take P
    outs = run("gpu_straggler", world, kind=MAJORITY, count=count, rounds=rounds, timeout=420)
    _check_straggler(outs, world, MAJORITY)


def test_solo_straggler_excluded():
    # solo, async 3: asynchronous rounds take P - 1, every 4th (synchronous) round P
    outs = run("gpu_straggler", 4, kind=SOLO, count=1 << 20, rounds=9, async_=3)
    _check_straggler(outs, 4, SOLO)


# ---- the RCCL transport between ranks on different GPUs ------------------------------

def _devices():
    import esgd
    return esgd.device_count()


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.timeout(900)
def test_rccl_transport_multi_gpu(world):
    # grouped ncclSend/ncclRecv over xGMI + the tree kernel on a side stream; RCCL
    # refuses two ranks on one GPU, so this runs only where the box has `world` GPUs
    if _devices() < world:
        pytest.skip(f"needs {world} GPUs (RCCL refuses ranks sharing a GPU)")
    for kind in (ALLREDUCE, SOLO, MAJORITY):
        verdicts = run("gpu_allreduce", world, count=1000003, rounds=2, kind=kind, transport="rccl")
        assert all(all(v) for v in verdicts), (kind, verdicts)
    _all_ok(run("gpu_config", world, kind=SOLO, counts=[64 << 20], rounds=2, transport="rccl", timeout=420))
    # bf16 on the wire: the same bits as the IPC wire rounds (oracle's bf16 tree of the
    # rounded inputs, widened); a 5-element bucket is one ragged shard (16-B stage pitch)
    for kw in (dict(count=1000003), dict(count=5), dict(count=1000003, buf="host", kind=MAJORITY)):
        verdicts = run("gpu_allreduce", world, rounds=2, wire=True, transport="rccl", **kw)
        assert all(all(v) for v in verdicts), (kw, verdicts)


@pytest.mark.timeout(600)
def test_largest_ff_bucket_2_ranks():
    # ff.h's int count: 2^31 - 1 fp32 = 8 GiB per rank, two ranks (16 GiB exported over
    # IPC from the arena), shards moved in 1 GiB pieces; round 1 never finished creating it
    outs = run("gpu_big", 2, count=(1 << 31) - 1, rounds=2, timeout=600)
    for o in outs:
        assert o["ok"], o
        assert o["create_s"] < 30, o


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_wire_bf16_device(world):
    # ESGD_SCHED_WIRE_BF16: fp32 buckets, bf16 copies exchanged;
    # every rank holds the oracle's bf16 tree of the rounded inputs, widened.  Ragged tails
    # (100003 = 8 k + 3 elements), in place, pieces of 64 KiB (> 16 gather segments at
    # P = 8), a bucket smaller than one 16-B vector per shard.
    for kw in (dict(count=100003), dict(count=100003, in_place=True),
               dict(count=300007, piece_bytes=65536), dict(count=17)):
        verdicts = run("gpu_allreduce", world, rounds=2, wire=True, **kw)
        assert all(all(v) for v in verdicts), (kw, verdicts)


def test_wire_bf16_host_and_partial_kinds():
    # host buckets (the reference's contract) and solo / majority schedules over the wire;
    # every rank posts behind a barrier, so each round is the full tree
    for world, kw in ((2, dict(count=262147, buf="host")), (2, dict(count=262147, buf="host", in_place=True)),
                      (4, dict(count=65536, kind=SOLO)), (4, dict(count=65539, kind=MAJORITY)),
                      (3, dict(count=(8 << 20) + 5, kind=MAJORITY))):
        verdicts = run("gpu_allreduce", world, rounds=3, wire=True, **kw)
        assert all(all(v) for v in verdicts), (world, kw, verdicts)


def test_wire_bf16_c3_size():
    # C3's 256 MiB fp32 bucket per rank over the wire at P = 2 (head / middle / tail
    # slices checked by gpu_config's digest path is not needed: the whole bucket is compared)
    verdicts = run("gpu_allreduce", 2, rounds=1, wire=True, count=(256 << 20) // 4, timeout=400)
    assert all(all(v) for v in verdicts), verdicts


STRESS = {"p3-one-launch": (3, 65536, "device"), "p3-five-launch": (3, (1 << 20) + 3, "device"),
          "p8-one-launch": (8, 65536, "device"), "p3-host-kernel-copy": (3, 65536, "host"),
          "p3-host-dma": (3, (1 << 20) + 3, "host")}


@pytest.mark.parametrize("case", sorted(STRESS))
@pytest.mark.parametrize("kind", [SOLO, MAJORITY])
def test_activation_stress(kind, case):
    # 600 steps per rank, random delays, no barriers: every round's result carries exactly
    # round t's bucket of every rank (int32 tags), the limiter cadence / majority activator
    # sequence hold, and peers' activations really carried ranks through rounds
    world, count, buf = STRESS[case]
    rounds, async_, seed = 600, 3, 34495645   # seed of rand_allreduce_correctness.c:64
    outs = run("gpu_stress", world, kind=kind, count=count, rounds=rounds, async_=async_, seed=seed,
               buf=buf, timeout=400)
    acts = ffref.activators(seed, world, rounds)
    for o in outs:
        assert o["nbad"] == 0, o["bad"]
        log = o["log"]
        assert [e["round"] for e in log] == list(range(1, rounds + 1))
        if kind == SOLO:
            assert [e["sync"] for e in log] == [t % (async_ + 1) == 0 for t in range(1, rounds + 1)]
        else:
            assert [e["activator"] for e in log] == acts
    assert sum(o["stats"]["auto_rounds"] for o in outs) > 0   # the stress exercised auto-joins


@pytest.mark.parametrize("kind", [SOLO, MAJORITY])
def test_activation_stress_many_schedules(kind):
    # four schedules driven like the wrapper's per-tensor ops, random delays, no barriers:
    # every round of every schedule takes exactly its generation of every rank's bucket
    world, rounds, async_, seed = 3, 200, 3, 34495645
    outs = run("gpu_stress_multi", world, kind=kind, rounds=rounds, async_=async_, seed=seed, timeout=400)
    for o in outs:
        assert o["nbad"] == 0, o["bad"]
        for i, log in enumerate(o["logs"]):
            assert [e["round"] for e in log] == list(range(1, rounds + 1))
            if kind == MAJORITY:
                assert [e["activator"] for e in log] == ffref.activators(seed + i, world, rounds)
    assert sum(o["auto_rounds"] for o in outs) > 0


@pytest.mark.parametrize("world", [3, 8])
@pytest.mark.parametrize("kind", [SOLO, MAJORITY])
def test_activation_stress_wire_bf16(kind, world):
    # the same stress over the bf16 wire (the optimizer's wire="bf16" path): small
    # integer tags that bf16 carries exactly
    rounds, async_, seed = 400, 3, 34495645
    outs = run("gpu_stress", world, kind=kind, count=(1 << 18) + 3, rounds=rounds, async_=async_, seed=seed,
               wire=True, timeout=400)
    for o in outs:
        assert o["nbad"] == 0, o["bad"]
        assert [e["round"] for e in o["log"]] == list(range(1, rounds + 1))
    assert sum(o["stats"]["auto_rounds"] for o in outs) > 0


@pytest.mark.parametrize("case", ["p3-one-launch", "p3-five-launch", "p8-one-launch", "p3-host-kernel-copy",
                                  "p3-host-dma"])
@pytest.mark.parametrize("kind", [SOLO, MAJORITY])
def test_fresh_only_stress(kind, case):
    # ESGD_SCHED_FRESH_ONLY under stress, gradients written in the wrapper's racy order:
    # every rank sees the same result for every round, and each rank's share of it is
    # exactly its tag if it had posted the round before joining it, else 0
    world, count, buf = STRESS[case]
    rounds = 600
    outs = run("gpu_stress_fresh", world, kind=kind, count=count, rounds=rounds, buf=buf, timeout=400)
    bits = outs[0]["bits"]
    for o in outs:
        assert not o["torn"], o["torn"]
        assert o["vals"] == outs[0]["vals"]
    for t in range(1, rounds + 1):
        v = outs[0]["vals"][t - 1]
        for q in range(world):
            share = (v >> (bits * q)) & ((1 << bits) - 1)
            want = t % (1 << bits) if outs[q]["fresh"][t - 1] else 0
            assert share == want, (t, q, share, want, [o["fresh"][t - 1] for o in outs])
    assert sum(o["stats"]["auto_rounds"] for o in outs) > 0


@pytest.mark.parametrize("world,batch", [(3, None), (4, [64, 0, 5, 2]), (8, None)])
@pytest.mark.parametrize("kind", [SOLO, MAJORITY])
def test_pipelined_stress_batched(kind, world, batch):
    # eight HOLD | FRESH_ONLY schedules posted all at once every step under random delays
    # (shared launches of rounds that peers' activations make due in different orders,
    # one five-launch size among them); a rank's share is its tag iff it had posted the
    # round, never torn, the same bits on every rank
    outs = run("gpu_stress_pipelined", world, kind=kind, rounds=120, batch=batch, timeout=400)
    _check_pipelined(outs, world)
    assert sum(o["auto_rounds"] for o in outs) > 0


def _check_pipelined(outs, world):
    # a rank's share of every round is its tag iff it had posted the round, never torn,
    # the same bits on every rank
    bits = outs[0]["bits"]
    for o in outs:
        assert not o["torn"], o["torn"]
        assert o["vals"] == outs[0]["vals"]
    for i in range(len(outs[0]["vals"])):
        for t in range(1, len(outs[0]["vals"][i]) + 1):
            v = outs[0]["vals"][i][t - 1]
            for q in range(world):
                want = t % (1 << bits) if outs[q]["fresh"][i][t - 1] else 0
                assert (v >> (bits * q)) & ((1 << bits) - 1) == want, (i, t, q, v, want)


@pytest.mark.parametrize("kind", [SOLO, MAJORITY])
def test_pipelined_stress_refused_exports_p8(kind):
    # round 4's r04zp configuration: 8 ranks, the batched per-tensor stress, the first
    # chunk export of ranks 4-7 refused -- through the real path now (ESGD_TEST fail_exports
    # writes the seal, then refuses the runtime call): the refused chunks are quarantined,
    # the published shards move, the peers map the moved chunks and read their seals
    world = 8
    outs = run("gpu_stress_pipelined", world, kind=kind, rounds=60, fail_exports=[0, 0, 0, 0, 1, 1, 1, 1],
               timeout=400)
    _check_pipelined(outs, world)


@pytest.mark.parametrize("kind", [SOLO, MAJORITY])
def test_schedule_churn_under_stress(kind):
    # temporary schedules (16 KiB .. 64 MiB) created, used and deleted every 20 steps
    # while a persistent schedule runs under the activation stress
    world, rounds = 3, 240
    outs = run("gpu_stress_churn", world, kind=kind, rounds=rounds, timeout=400)
    bits = outs[0]["bits"]
    for o in outs:
        assert not o["torn"], o["torn"]
        assert o["vals"] == outs[0]["vals"]
        assert o["churn_ok"] and all(o["churn_ok"]), o["churn_ok"]
    for t in range(1, rounds + 1):
        v = outs[0]["vals"][t - 1]
        for q in range(world):
            want = t % (1 << bits) if outs[q]["fresh"][t - 1] else 0
            assert (v >> (bits * q)) & ((1 << bits) - 1) == want, (t, q)


@pytest.mark.parametrize("kind", [SOLO, MAJORITY])
def test_stress_one_thread_per_schedule(kind):
    # three schedules driven concurrently from three threads per rank
    world, rounds = 3, 200
    outs = run("gpu_stress_threads", world, kind=kind, rounds=rounds, timeout=400)
    bits = outs[0]["bits"]
    for o in outs:
        assert not o["errs"], o["errs"]
    for i in range(len(outs[0]["res"])):
        for o in outs:
            assert not o["res"][i]["torn"], (i, o["res"][i]["torn"])
            assert o["res"][i]["vals"] == outs[0]["res"][i]["vals"], i
        for t in range(1, rounds + 1):
            v = outs[0]["res"][i]["vals"][t - 1]
            for q in range(world):
                want = t % (1 << bits) if outs[q]["res"][i]["fresh"][t - 1] else 0
                assert (v >> (bits * q)) & ((1 << bits) - 1) == want, (i, t, q)


# ---- cross-GPU hand-offs (run only where every rank has a GPU of its own) -------------

def _ngpu():
    import esgd
    return esgd.device_count()


CANARY = [("ipc", "one_launch"), ("ipc", "five_launch"), ("rccl", "rccl")]


def _canary_report(outs):
    lines = []
    for o in outs:
        for b in o["bad"]:
            lines.append(f"rank {o['rank']} device {o['device']} ({o['devices']}) transport {o['transport']} "
                         f"path {o['path']} strict {o['strict']} count {o['count']} round {b['round']}: "
                         f"{b['nbad']} bad, first at {b['first']} got {b['got']} want {b['want']}")
    return "\n".join(lines)


@pytest.mark.parametrize("strict", [0, 1])
def test_cross_gpu_canary(strict):
    # The first multi-rank test of the suite (conftest.py orders it): 2 ranks on distinct
    # devices, a tiny and a 16 MiB bucket, over IPC one-launch, IPC five-launch and RCCL,
    # relaxed and strict hand-offs (ESGD_STRICT_HANDOFFS).  A failure names the devices,
    # transport, round and first bad element with its value and the oracle's.
    if _ngpu() < 2:
        pytest.skip("needs >= 2 GPUs (ranks on distinct devices); the worker runs on one GPU in "
                    "test_canary_worker_on_a_shared_gpu")
    report = []
    for count in (4099, (4 << 20) + 3):
        for transport, path in CANARY:
            if transport == "rccl" and strict:
                continue   # the strict switch concerns the one-launch kernel only
            outs = run("gpu_canary", 2, count=count, transport=transport, path=path, strict=strict)
            assert all(len(set(o["devices"].split(","))) == 2 for o in outs), outs
            rep = _canary_report(outs)
            if rep:
                report.append(rep)
    assert not report, "\n".join(report)


def test_canary_worker_on_a_shared_gpu():
    # the canary's worker and report, exercised where both ranks share a GPU (IPC only:
    # RCCL refuses two ranks on one device); bit-exact in every case, strict and relaxed
    for count in (4099, (4 << 20) + 3):
        for transport, path in CANARY[:2]:
            for strict in (0, 1):
                outs = run("gpu_canary", 2, count=count, transport=transport, path=path, strict=strict)
                assert not _canary_report(outs), _canary_report(outs)
                assert all(o["rounds"] == 3 for o in outs), outs


@pytest.mark.parametrize("strict", [0, 1])
@pytest.mark.parametrize("flags", [0, 1, 2])
@pytest.mark.parametrize("path", sorted(SMALL))
def test_writer_then_post_visibility_across_gpus(path, flags, strict):
    # every rank rewrites its bucket on a producer stream right before posting; each
    # round's every element must match the oracle (mp_workers.gpu_visibility); relaxed and
    # strict hand-offs (ESGD_STRICT_HANDOFFS) of the one-launch kernel
    n = _ngpu()
    if n < 2:
        pytest.skip("needs >= 2 GPUs (ranks on distinct devices)")
    if strict and path != "one_launch":
        pytest.skip("the strict switch concerns the one-launch kernel only")
    for world in sorted({2, min(n, 8)}):
        count = 65536 + 3 if path == "one_launch" else (1 << 20) + 3
        outs = run("gpu_visibility", world, count=count, small_bytes=SMALL[path], flag_mode=flags,
                   strict=strict)
        for o in outs:
            assert not o["bad"], (world, o)
            assert len(set(o["devices"].split(","))) == world, o


@pytest.mark.parametrize("fails", [1, 2])
def test_schedules_survive_refused_exports(fails):
    # The runtime sometimes refuses to export a fresh process's first chunk
    # (hipErrorInvalidValue, round 3).  ESGD_TEST fail_exports=N fails each rank's first N chunk
    # exports the same way: buffers the schedule owns (published shard, host-bucket
    # staging) move to fresh chunks, a caller's device bucket in a refused chunk is
    # shadowed, and every round is still bit-exact
    old = os.environ.get("ESGD_TEST")
    os.environ["ESGD_TEST"] = f"fail_exports={fails}"
    try:
        for kw in (dict(count=4099), dict(count=300007, small_bytes=0), dict(count=70001, buf="host")):
            verdicts = run("gpu_allreduce", 2, rounds=2, **kw)
            assert all(all(v) for v in verdicts), (kw, verdicts)
    finally:
        if old is None:
            os.environ.pop("ESGD_TEST", None)
        else:
            os.environ["ESGD_TEST"] = old


POST_IO_CASES = {
    "batched": dict(count=4099),
    "batched_tiny": dict(count=17),
    "one_launch_per_round": dict(count=4099, batch=0),
    "five_launch": dict(count=300007, small_bytes=0),
    "dst_is_src": dict(count=100003, separate_dst=False),
    "mixed_with_plain_posts": dict(count=4099, plain_ranks=(1,)),
    "shadowed_rank": dict(count=4099, shadow_ranks=(1,)),
    "int32_no_divisor": dict(count=4099, dtype_name="int32"),
}


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", list(POST_IO_CASES))
def test_post_io_rounds_read_src_and_write_dst(case, world):
    # esgd_schedule_post_io: the round's snapshot reads src / divisor (the deep500 op's
    # copy-in fused) and its phases write dst (the copy-out fused) -- in shared launches,
    # one launch per round, five-launch rounds, beside a shadowed rank or a rank posting
    # through its send bucket; the oracle's bits every round
    outs = run("gpu_post_io", world, **POST_IO_CASES[case])
    for o in outs:
        assert all(o["verdicts"]), o["verdicts"]
        assert all(o["fresh"]), o["fresh"]


def test_post_io_round_carried_through_before_the_post():
    # solo, rank 1 posts late: rounds rank 0's activation carries it through do not take
    # rank 1's data (fresh 0, dst untouched, result in rb, its share zero); synchronous
    # rounds do; every rank the oracle's bits of that contributor set
    outs = run("gpu_post_io_late", 2, steps=9)
    for o in outs:
        for step in o:
            assert step["ok"] and step["untouched"], step
    for a, b in zip(outs[0], outs[1]):
        assert a["digest"] == b["digest"], (a, b)
    assert any(not st["fresh"][1] for st in outs[0][1:]), outs[0]   # the late path was taken


@pytest.mark.parametrize("count,in_place", [(4099, False), (4099, True), ((1 << 21) + 7, False)],
                         ids=["one_launch", "one_launch_in_place", "five_launch"])
@pytest.mark.parametrize("world", [2, 3])
def test_post_iov_pieces_packed_and_unpacked_by_the_round(world, count, in_place):
    # the fused optimizer's pack (/ P) and unpack as the round's own copy-in / copy-out
    # (esgd_schedule_post_iov): the oracle's bits in every piece
    outs = run("gpu_post_iov", world, count=count, in_place=in_place)
    for o in outs:
        assert all(o["ok"]), o["ok"]
        assert all(o["fresh"]), o["fresh"]


SWEEPS_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "bin",
                          "libesgd_sweeps.so")


@pytest.mark.skipif(not os.path.exists(SWEEPS_LIB), reason="tools/bin/libesgd_sweeps.so not built (make sweeps)")
def test_batched_rounds_progress_beside_a_kernel_holding_the_gpu():
    # forward progress of k_round_batch: a kernel on another stream holds all
    # but two CUs' wave slots for 6 s, and the two ranks' shared launches compete for the
    # rest; each rank's launch must finish its 5 rounds on the workgroups that fit, bit for
    # bit, well before the hog leaves -- whichever rank's workgroups the GPU dispatches
    # first (workers give their slots back after 2 ms at a closed gate and the agent block
    # folds what they left).  The later rounds, bit for bit too, start once the launch's
    # last workgroups could be dispatched.  ESGD_TIMEOUT_S = 10: every bounded wait of the
    # test together stays under the harness limit, itself under gpurun's 180 s of silence.
    old = os.environ.get("ESGD_TIMEOUT_S")
    os.environ["ESGD_TIMEOUT_S"] = "10"
    try:
        outs = run("gpu_residency", 2, timeout=150)
    finally:
        if old is None:
            os.environ.pop("ESGD_TIMEOUT_S", None)
        else:
            os.environ["ESGD_TIMEOUT_S"] = old
    for o in outs:
        assert all(o["ok"]) and len(o["ok"]) == 30, o
        assert o["first_round_s"] < 0.25 * o["hog_s"], o


@pytest.mark.skipif(not os.path.exists(SWEEPS_LIB), reason="tools/bin/libesgd_sweeps.so not built (make sweeps)")
def test_late_peer_after_a_timeout_never_succeeds_with_a_stale_sum():
    # the failure contract: rank 1's GPU runs the round
    # 3 s late, rank 0's GPU flag wait gives up at 1.5 s.  Rank 0 fails; rank 1 fails as well
    # or returns the oracle's sum -- for one-launch, batched and five-launch rounds of every
    # kind.  (Before round 6 rank 1 returned success with rank 0's shard folded from its
    # stale bucket.)
    cases = [(k, p) for p in ("batched", "one", "five") for k in ("allreduce", "solo", "majority")]
    old = os.environ.get("ESGD_TIMEOUT_S")
    os.environ["ESGD_TIMEOUT_S"] = "1.5"
    try:
        outs = run("gpu_late_peer_after_timeout", 2, cases=cases, delay_s=3.0, timeout=140)
    finally:
        if old is None:
            os.environ.pop("ESGD_TIMEOUT_S", None)
        else:
            os.environ["ESGD_TIMEOUT_S"] = old
    _check_late_peer(outs)


def _check_late_peer(outs):
    *on_time, late = outs
    for i, c1 in enumerate(late):
        cs = [r[i] for r in on_time]
        assert all(c["first_round_ok"] for c in cs) and c1["first_round_ok"], (cs, c1)
        assert all(c["failed"] for c in cs), cs                  # the ranks that timed out
        assert c1["failed"] or c1["result"] == "oracle", c1      # never a stale sum
        assert c1["result"] != "WRONG", c1
        # the late rank's outcome came from the GPU's flag protocol, not its host wait limit
        assert c1["gpu_failure"] or c1["result"] == "oracle", c1


@pytest.mark.skipif(not os.path.exists(SWEEPS_LIB), reason="tools/bin/libesgd_sweeps.so not built (make sweeps)")
def test_late_peer_among_four_ranks():
    # the same contract at P = 4, the last rank late: three ranks time out (or see a peer's
    # error word) and fail; the late rank fails through their error words.  Allreduce only:
    # every rank joins each of its rounds (a solo / majority round may complete without the
    # late rank, which is its semantics, not a failure)
    old = os.environ.get("ESGD_TIMEOUT_S")
    os.environ["ESGD_TIMEOUT_S"] = "1.5"
    try:
        outs = run("gpu_late_peer_after_timeout", 4, cases=[("allreduce", "batched"), ("allreduce", "five")],
                   delay_s=3.0, timeout=140)
    finally:
        if old is None:
            os.environ.pop("ESGD_TIMEOUT_S", None)
        else:
            os.environ["ESGD_TIMEOUT_S"] = old
    _check_late_peer(outs)


@pytest.mark.parametrize("delete_first", [False, True])
def test_finalize_with_rounds_held_in_the_shared_launch(delete_first):
    # rounds every rank launched into a held shared launch (batch_hold) are sent by the
    # schedule deletion / finalize while the schedules are alive, pair up and land
    outs = run("gpu_finalize_held", 2, delete_first=delete_first, timeout=120)
    for o in outs:
        assert o["launched_before_finalize"] == 0, o   # they really were held
        assert all(o["ok"]), o


def test_second_job_after_ipc_mappings_closed_is_refused():
    outs = run("gpu_reinit", 2)
    for o in outs:
        assert o["ok"], o
        assert o["err"] and "fresh process" in o["err"], o


@pytest.mark.parametrize("bypass", [
    None,
    # opt-in (ESGD_DIAGNOSTIC_TESTS=1): a probe of the runtime, not of this library
    pytest.param("2", marks=[pytest.mark.diagnostic, pytest.mark.xfail(
        strict=False, reason="ROCm dmabuf IPC: after an exported allocation is freed, one "
        "rank's re-exported bucket is mapped by every importer as another rank's "
        "(profiles/r03/ipc_reexport_decoded_r03k.txt); production never frees exported memory")]),
])
def test_ipc_reexport_sequence_bitexact(bypass):
    # the sequence behind round 2's wrong sums ("IPC arena"): 8 ranks, a
    # 16 MiB bucket exported, mapped by every peer, its schedule deleted and the bucket
    # freed, then a 256 MiB bucket exported and mapped.  Production (the arena: exported
    # memory never freed) must be bit-exact.  ESGD_TEST arena_bypass=2 (every bucket its own
    # hipMalloc, freed after every rank closed its peer mappings) is the driver-level
    # diagnostic: it failed in 5 of 7 runs this round, always the same way -- all 64 bytes
    # of every handle distinct (exporter VA + pid), yet every importer of ONE rank's new
    # bucket reads a different rank's bucket (decoded per element: the tree sum with that
    # rank's input replaced by the other's).  So it is expected to fail, not required to.
    counts = [(16 << 20) // 4, (256 << 20) // 4]
    env = {} if bypass is None else {"ESGD_TEST": f"arena_bypass={bypass}"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        _all_ok(run("gpu_config", 8, kind=MAJORITY, counts=counts, rounds=2, timeout=300,
                    close_before_free=bypass is not None, detail=bypass is not None))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
