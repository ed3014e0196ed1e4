"""Round protocol of the partial allreduces, multi-process on CPU (gloo rendezvous,
control plane only: ESGD_BUF_NONE moves no data).

Reference behaviour checked (paths under /root/reference/eager-SGD-modules/fflib2):
  * limiter cadence — src/colls/ffsolo_limiter.c:4-35 / evaluation/limiter.c: rounds
    1..async asynchronous, round async+1 synchronous, repeating;
  * solo activation — the first rank to post an asynchronous round activates it for
    everyone (src/colls/ffactivation.c:11-106); late ranks join with what they hold;
  * majority activator — rand_r(&seed) % P with the same seed everywhere
    (src/colls/ffrand_allreduce.c:83-103), pinned against libc via the oracle;
  * plain allreduce — every round synchronous, every rank fresh.
"""
import os

import pytest

from mp_workers import run
from oracle import ffref

ALLREDUCE, SOLO, MAJORITY = 0, 1, 2
pytestmark = pytest.mark.slow


def test_allreduce_every_round_sync_and_fresh():
    outs = run("cp_rounds", 2, kind=ALLREDUCE, rounds=6)
    for o in outs:
        assert [e["round"] for e in o["log"]] == list(range(1, 7))
        assert all(e["sync"] and e["fresh"] for e in o["log"])
        assert o["roles"] == [2] * 6


@pytest.mark.parametrize("async_", [1, 2, 3])
def test_limiter_cadence(async_):
    outs = run("cp_rounds", 2, kind=SOLO, rounds=3 * (async_ + 1), async_=async_, barrier_each=True)
    for o in outs:
        got = [e["sync"] for e in o["log"]]
        want = [t % (async_ + 1) == 0 for t in range(1, 3 * (async_ + 1) + 1)]
        assert got == want


def test_solo_first_poster_activates():
    world, rounds = 3, 8
    outs = run("cp_rounds", world, kind=SOLO, rounds=rounds, async_=100, first_poster_rotates=True)
    for r, o in enumerate(outs):
        for e in o["log"]:
            t = e["round"]
            assert e["activator"] == t % world
            assert e["fresh"] == (r == t % world)   # the others joined on the activation
        roles = o["roles"]
        assert [roles[t - 1] for t in range(1, rounds + 1)] == [1 if r == t % world else 0
                                                                  for t in range(1, rounds + 1)]


def test_solo_straggler_bounded_by_limiter():
    # rank 1 is 0.25 s late every round; rank 0 runs the asynchronous rounds alone and
    # blocks only at the synchronous one (every 4th) — bounded staleness.
    async_, rounds = 3, 8
    outs = run("cp_rounds", 2, kind=SOLO, rounds=rounds, async_=async_, straggler=1, delay=0.25)
    fast, slow = outs[0]["log"], outs[1]["log"]
    for e in fast:
        assert e["fresh"]
        if not e["sync"]:
            assert e["activator"] == 0
    for e in slow:
        assert e["fresh"] == e["sync"], e   # the straggler is fresh only on sync rounds
    assert outs[1]["stats"]["auto_rounds"] == rounds - rounds // (async_ + 1)


@pytest.mark.parametrize("world,seed", [(2, 6545343), (4, 6545343), (3, 34495645)])
def test_majority_activator_is_rand_r(world, seed):
    rounds = 16
    outs = run("cp_rounds", world, kind=MAJORITY, rounds=rounds, seed=seed, barrier_each=True)
    want = ffref.activators(seed, world, rounds)
    for r, o in enumerate(outs):
        assert [e["activator"] for e in o["log"]] == want
        assert [o["roles"][t] for t in range(rounds)] == [1 if a == r else 0 for a in want]
        for e in o["log"]:
            if e["activator"] == r:
                assert e["fresh"]


def test_test_polling_equivalent_to_wait():
    outs = run("cp_rounds", 2, kind=SOLO, rounds=6, async_=2, use_test=True)
    for o in outs:
        assert [e["round"] for e in o["log"]] == list(range(1, 7))
        assert o["stats"]["completed"] == 6 and o["stats"]["waited"] == 6


@pytest.mark.parametrize("world", [2, 3])
def test_ordered_transport_same_issue_order_everywhere(world):
    # RCCL matches operations by issue order: the ticket ring must give every rank the
    # same (schedule, round) sequence even when ranks post buckets in different orders.
    logs = run("cp_ordered", world, nsched=4, rounds=5)
    assert len(logs[0]) == 4 * 5
    assert all(l == logs[0] for l in logs), logs
    for sid in range(4):   # rounds of one schedule appear in order
        rs = [r for s, r in logs[0] if s == sid]
        assert rs == sorted(rs) == list(range(1, 6))


@pytest.mark.parametrize("world", [2, 3])
def test_failed_creation_fails_every_rank(world):
    # registration is voted (engine.cpp sched_create): one rank's failure is every
    # rank's failure, with no rank left waiting for a peer's publication
    # the last rank creates a MAJORITY schedule where the others create a SOLO one: every
    # rank sees every rank's creation signature after the vote and fails the same way
    outs = run("cp_create_failure", world, bad_rank=world - 1)
    for r, o in enumerate(outs):
        assert o["err"] is not None, (r, o)
        assert "creation order must match" in o["err"], o["err"]
        assert "kind 2" in o["err"] and "kind 1" in o["err"], o["err"]
        assert o["recovered_s"] < 30


@pytest.mark.parametrize("world", [2, 3])
def test_connect_failure_fails_every_creation(world):
    # creation costs two barriers: a rank whose connect fails fails its creation, and its
    # peers fail theirs at the connect vote, not after the timeout
    outs = run("cp_connect_failure", world, bad_rank=world - 1)
    bad = outs[-1]
    assert bad["create_err"] and "fail_connect" in bad["create_err"], bad
    for o in outs[:-1]:
        assert o["create_err"] and "another rank failed to register" in o["create_err"], o
        assert o["t_fail"] < 5, o


def test_wait_fresh_bit_survives_run_ahead():
    outs = run("cp_fresh_queue", 2, rounds=300)
    assert outs[0]["joined"] == 300, outs[0]["joined"]
    fresh = outs[0]["fresh"]
    assert fresh[0] is True and not any(fresh[1:]), [i + 1 for i, f in enumerate(fresh) if f]


def test_delete_while_rounds_in_flight():
    # sched_delete vs a progress pass holding the registry copy
    outs = run("cp_churn_inflight", 2, rounds=300, churn=40)
    for o in outs:
        assert not o["errs"], o
        assert o["completed"] == 300


def test_stale_segment_of_a_dead_job_is_not_joined():
    # a crashed run's /dev/shm/esgd-<job> (same job id) holds old barrier
    # counts; ranks > 0 must not attach to it.  Make a real one: a rank 0 of a 2-rank job
    # that is killed while it waits for its peer in the init barrier (the file is
    # published, never unlinked).
    import signal
    import subprocess
    import sys
    import time
    import uuid

    from conftest import PKG
    job = "stale-" + uuid.uuid4().hex[:12]
    path = "/dev/shm/esgd-" + job
    code = ("import sys; sys.path.insert(0, %r); from esgd import comm; "
            "comm.init(job_id=%r, rank=0, world=2)") % (PKG, job)
    p = subprocess.Popen([sys.executable, "-c", code], env=dict(os.environ, ESGD_TIMEOUT_S="120"))
    try:
        t0 = time.time()
        while not os.path.exists(path) and time.time() - t0 < 60:
            time.sleep(0.05)
        assert os.path.exists(path), "rank 0 never published its segment"
    finally:
        p.send_signal(signal.SIGKILL)
        p.wait()
    assert os.path.exists(path)          # the crash left it behind
    try:
        outs = run("cp_stale_segment", 2, job=job, timeout=120)
        assert outs == [True, True]
    finally:
        if os.path.exists(path):
            os.unlink(path)


def test_hold_until_release():
    outs = run("cp_hold", 2, hold_s=0.3)
    for o in outs:
        assert "release() the round" in o["double_wait"], o
    assert outs[0]["round2_s"] >= 0.25, outs[0]      # rank 1 joined only after its release
    assert [e["round"] for e in outs[1]["log"]] == [1, 2]


def test_lost_peer_fails_the_round_instead_of_hanging():
    outs = run("cp_peer_lost", 3, timeout=120)
    for o in outs[:-1]:
        assert o["error"] and ("timed out" in o["error"] or "joined" in o["error"]), o
        assert 1.5 <= o["elapsed_s"] <= 15, o


# ---- ranks in different PID namespaces (one container per GPU sharing /dev/shm) -------

def _unshare_ok():
    import subprocess
    try:
        return subprocess.run(["unshare", "-p", "-f", "--kill-child", "true"], capture_output=True,
                              timeout=10).returncode == 0
    except Exception:
        return False


_RANK = ("import sys; sys.path.insert(0, %r); from esgd import comm; "
         "comm.init(job_id=%r, rank=%d, world=2); "
         "s = comm.Schedule(comm.ALLREDUCE, None, None, 0, buf=comm.BUF_NONE)\n"
         "for _ in range(3):\n    s.post(); s.wait()\n"
         "s.delete(); comm.finalize(); print('rank done')")


def _rank_cmd(job, rank, ns):
    import sys

    from conftest import PKG
    cmd = [sys.executable, "-c", _RANK % (PKG, job, rank)]
    return (["unshare", "-p", "-f", "--kill-child"] + cmd) if ns else cmd


@pytest.mark.skipif(not _unshare_ok(), reason="needs unshare -p (PID namespaces)")
def test_creator_in_another_pid_namespace_is_joined():
    # rank 0 in its own PID namespace -- its pid means nothing to rank 1, which
    # must still attach (creator liveness = rank 0's init-barrier heartbeat there)
    import subprocess
    import uuid
    job = "pidns-" + uuid.uuid4().hex[:12]
    env = dict(os.environ, ESGD_TIMEOUT_S="30")
    p0 = subprocess.Popen(_rank_cmd(job, 0, True), env=env, stdout=subprocess.PIPE, text=True)
    p1 = subprocess.Popen(_rank_cmd(job, 1, False), env=env, stdout=subprocess.PIPE, text=True)
    out0, _ = p0.communicate(timeout=90)
    out1, _ = p1.communicate(timeout=90)
    assert p0.returncode == 0 and "rank done" in out0
    assert p1.returncode == 0 and "rank done" in out1


@pytest.mark.skipif(not _unshare_ok(), reason="needs unshare -p (PID namespaces)")
def test_stale_segment_from_another_pid_namespace_is_not_joined():
    # a crashed rank 0 of another PID namespace left its segment behind: its heartbeat
    # stops, so once it is stale a new job with the same id does not attach to it
    import signal
    import subprocess
    import time
    import uuid
    job = "pidns-stale-" + uuid.uuid4().hex[:12]
    path = "/dev/shm/esgd-" + job
    env = dict(os.environ, ESGD_TIMEOUT_S="60")
    p = subprocess.Popen(_rank_cmd(job, 0, True), env=env)
    try:
        t0 = time.time()
        while not os.path.exists(path) and time.time() - t0 < 60:
            time.sleep(0.05)
        assert os.path.exists(path), "rank 0 never published its segment"
    finally:
        p.send_signal(signal.SIGKILL)
        p.wait()
    try:
        assert os.path.exists(path)
        time.sleep(2.5)          # past the 2 s heartbeat window
        env = dict(os.environ, ESGD_TIMEOUT_S="30")
        p1 = subprocess.Popen(_rank_cmd(job, 1, False), env=env, stdout=subprocess.PIPE, text=True)
        time.sleep(1.0)          # rank 1 meets the stale file first
        p0 = subprocess.Popen(_rank_cmd(job, 0, False), env=env, stdout=subprocess.PIPE, text=True)
        out0, _ = p0.communicate(timeout=90)
        out1, _ = p1.communicate(timeout=90)
        assert p0.returncode == 0 and "rank done" in out0
        assert p1.returncode == 0 and "rank done" in out1
    finally:
        if os.path.exists(path):
            os.unlink(path)


def test_creation_cost_161_schedules():
    # two node barriers per creation: the per-tensor wrapper's 161 buckets
    # cost a fraction of a millisecond each, once per job (generous bound for a loaded CI box)
    outs = run("cp_create_many", 4, n=161)
    worst = max(o["create_ms_per_schedule"] for o in outs)
    assert worst < 20, worst


@pytest.mark.parametrize("kind", [1, 2])
def test_post_group_same_rounds_as_single_posts(kind):
    # esgd_schedule_post_group (the per-tensor optimizer's one call for all its ops): the
    # same roles, rounds and activators as posting the schedules one by one in that order
    world, n, rounds = 3, 12, 20
    outs = run("cp_post_group", world, n=n, rounds=rounds, kind=kind)
    for o in outs:
        for i, log in enumerate(o["logs"]):
            assert [e["round"] for e in log] == list(range(1, rounds + 1))
            if kind == 2:   # majority: the libc draw of each schedule's seed
                assert [e["activator"] for e in log] == ffref.activators(6545343 + i, world, rounds)
    if kind == 2:
        for t in range(rounds):
            for i in range(n):
                act = ffref.activators(6545343 + i, world, rounds)[t]
                for r, o in enumerate(outs):
                    assert o["roles"][t][i] == (1 if act == r else 0), (t, i, r)


def test_progress_thread_profile_counts_joins():
    # esgd_comm_profile (the bench's per-step host breakdown): 5 schedules x 10 rounds
    # joined once each, time spent inside busy passes, no data-plane launches (BUF_NONE)
    outs = run("cp_profile", 2, n=5, rounds=10)
    for o in outs:
        assert o["joins"] == 50, o
        assert o["passes"] >= 1 and o["pass_ns"] > 0 and o["join_ns"] > 0, o
        assert o["launches"] == 0 and o["flush_ns"] == 0, o
