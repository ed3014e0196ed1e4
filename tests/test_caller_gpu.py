"""The drop-in callers on the GPU: the deep500 op ABI (host buckets, the reference's
contract; device buckets with the wrapper's division fused) and the PyTorch
EagerSGDOptimizer, multi-rank (one GPU per rank where the box has them).

Known answers: the plain allreduce equals the oracle tree of every rank's gradient
(evaluation/allreduce.c:59-63 in fp32 form).  Solo and majority rounds are made
deterministic by the order in which ranks call the op (mp_workers.late_ranks):
majority -- the drawn activator (rand_r(6545343) % P, ffrand_allreduce.c:88) calls last,
so its round takes every fresh gradient (rand_allreduce_correctness.c:78-98's answer);
solo -- rank 0 calls first and activates, the others are carried through the round with
a zeroed send bucket, so the round is the oracle tree of (x0, 0, ..., 0) and their late
gradients are dropped, as the wrapper's zeroing after the wait does
(opt_esgd_solo_imagenet_imbalance.py:311-314).
"""
import pytest

from mp_workers import run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["allreduce", "solo", "majority"])
def test_deep500_op_host_path(mode):
    outs = run("op_host", 2, mode=mode, steps=4, count=5000)
    for o in outs:
        assert o["cuda"] and o["report"] == 4 * 5000 * 4
        assert all(o["ok"]) and len(o["ok"]) == 3, o


@pytest.mark.parametrize("on_time", [0, 1])
@pytest.mark.parametrize("count", [100003, 25559081])
def test_deep500_op_device_late_gradient_dropped(on_time, count):
    # solo, async 3: rounds 2, 3 (and 5..7) asynchronous -> the on-time rank's x / P only;
    # round 4 and 8 synchronous -> every rank.  A late gradient carried into the next round
    # (the race of the unfused copy-out / zeroing) would break the asynchronous rounds'
    # answer.  Either rank late; a one-launch bucket and the ResNet-50 fused bucket (five
    # launches)
    outs = run("op_device_late", 2, async_=3, steps=9, count=count, on_time=on_time)
    for o in outs:
        assert all(o["ok"]), o
        assert o["sync_rounds"] == [r % 4 == 0 for r in range(2, 10)]


VARIANTS = {"blocking": dict(pipeline=False), "pipelined": dict(pipeline=True), "fused": dict(fuse=True)}


@pytest.mark.parametrize("variant", list(VARIANTS))
@pytest.mark.parametrize("mode", ["allreduce", "solo", "majority"])
def test_eager_sgd_optimizer(mode, variant):
    # one blocking round per tensor (the reference's op chain), every tensor's round posted
    # before the first wait (pipeline=True, the default), or every gradient packed into
    # one bucket (fuse=True): the same bits
    outs = run("optimizer_step", 2, mode=mode, steps=3, **VARIANTS[variant])
    for o in outs:
        assert all(o["ok"]) and o["ok"], o["ok"]
        assert o["bytes"] > 0
    if mode == "allreduce":   # synchronous averaging keeps the replicas identical
        assert outs[0]["params_digest"] == outs[1]["params_digest"]


@pytest.mark.parametrize("variant", ["per_tensor", "fused_buckets"])
def test_eager_sgd_optimizer_rounds_posted_during_backward(variant):
    # overlap=True: each tensor's round posted from its post-accumulate-grad hook while
    # backward still runs (TF's dataflow order for the reference's ops), waited for in
    # apply_gradients -- the same rounds, so the oracle's bits and identical replicas;
    # fused_buckets: fuse=True in buckets of ~4 KiB (this model: several), each bucket's
    # fused round posted once its last gradient exists
    kw = dict(fuse=True, bucket_mb=4096 / (1 << 20)) if variant == "fused_buckets" else {}
    outs = run("optimizer_step", 2, mode="allreduce", steps=3, overlap=True, **kw)
    for o in outs:
        assert all(o["ok"]) and o["ok"], o["ok"]
        assert o["bytes"] > 0
    assert outs[0]["params_digest"] == outs[1]["params_digest"]


@pytest.mark.parametrize("fuse", [False, True])
@pytest.mark.parametrize("mode", ["allreduce", "solo", "majority"])
def test_eager_sgd_optimizer_wire_bf16(mode, fuse):
    # EagerSGDOptimizer(wire="bf16"): fp32 gradients, bf16 copies between the ranks
    # (ESGD_SCHED_WIRE_BF16); same contributors as the fp32 test, bf16 convention
    outs = run("optimizer_step", 2, mode=mode, steps=3, fuse=fuse, wire="bf16")
    for o in outs:
        assert all(o["ok"]) and o["ok"], o["ok"]
    if mode == "allreduce":
        assert outs[0]["params_digest"] == outs[1]["params_digest"]


def test_void_forward_keeps_going_on_a_lost_peer():
    # the reference's void allreducef_forward has no error channel; under
    # esgd_op_on_error(ESGD_OP_ON_ERROR_LOCAL) a lost peer no longer aborts the job: the
    # step gets this rank's own gradient and the op keeps the failure's status
    outs = run("op_void_peer_lost", 2, timeout=120)
    assert all(o["first_ok"] for o in outs), outs
    o = outs[0]
    assert o["own"] and o["status"] != 0 and o["elapsed"] < 30, o


@pytest.mark.parametrize("packed,host", [(False, False), (True, False), (False, True)])
def test_op_result_ordered_on_the_callers_default_stream(packed, host):
    # torch's default stream is handed to the op as stream 0: the op's copy-in, copy-out
    # and events must then run on the legacy default stream, NOT the library's own
    # non-blocking stream -- a read queued on the caller's stream right after the op
    # returns (g[:m].cpu() here, the optimizer's step in training) must see the reduced
    # bucket.  Round 3's ResNet-50 example diverged across ranks before this was so.
    # Steps follow the reference's random-straggler pattern with no barrier between them
    # (resnet_run_loop_solo_imagenet_300.py:290-294): every step's result must be the tree
    # of some contributor subset, the same on every rank.
    outs = run("op_device_pattern", 2, packed=packed, host=host, count=(1 << 22) + 5 if host else 25559081,
               timeout=240)
    for t in range(len(outs[0])):
        assert outs[0][t]["contributors"] is not None and outs[1][t]["contributors"] is not None, (t, outs)
        assert outs[0][t]["contributors"] == outs[1][t]["contributors"], (t, outs)
        assert outs[0][t]["digest"] == outs[1][t]["digest"], t


@pytest.mark.parametrize("world", [2, 3])
def test_group_post_wait_same_bits_as_single_ops(world):
    # the optimizer's per-tensor step through ONE post and ONE wait call
    # (allreducef_forward_cuda_post_many_io / _wait_many; aligned tensors, and unaligned ones
    # that go the copy-in way) against one forward_cuda_div per op: the oracle's bits,
    # ragged and tiny tensors and a five-launch size among them
    outs = run("op_group", world)
    for o in outs:
        assert all(o["ok"]) and o["ok"], o["ok"]
        assert o["errs"]["post_many_over_posted"] == -2, o["errs"]   # ESGD_INVALID_ARG
        assert o["errs"]["drained_op0"], o["errs"]


def test_registered_torch_op_in_a_traced_module():
    # esgd::allreducef (torch.library) inside a torch.fx GraphModule, 2 ranks on the GPU:
    # the oracle's bits of grad_r / P, one graph node per tensor, zero input gradients
    # (the reference op's empty backward, opt_esgd_solo_imagenet_imbalance.py:321-326)
    outs = run("op_torch_registered", 2)
    for o in outs:
        assert o["nodes"] == 3, o
        assert all(o["ok"]) and len(o["ok"]) == 12, o
