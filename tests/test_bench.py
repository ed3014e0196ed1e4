"""bench.py's host logic on the CPU (no device): a bare `bench.py --gpus N` must start
its own N ranks through torch.distributed.run -- before anything in the parent loads the
HIP library -- and exit with their status (the reference's launcher
starts its ranks the same way, test_scripts_imagenet/daint_eagersgd_imagenet.sh:2-5); the
line's device-derived labels, the CPU baseline's core list and pinned harness, and the
straggler's deadline wait (round 6)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

PROBE = r"""
import json, os, subprocess, sys
sys.path.insert(0, {root!r})
seen = {{}}
def fake_run(cmd, env=None, **kw):
    seen["cmd"] = cmd
    seen["env"] = {{k: env.get(k) for k in ("HSA_ENABLE_IPC_MODE_LEGACY", "ESGD_BENCH_SELF_LAUNCHED")}}
    class R: returncode = 7
    return R()
subprocess.run = fake_run
import bench
sys.argv = ["bench.py"] + {args!r}
try:
    bench.main()
except SystemExit as e:
    seen["exit"] = e.code
seen["hip_loaded"] = any(m.startswith("esgd") for m in sys.modules)
print(json.dumps(seen))
"""


def _probe(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    out = subprocess.run([sys.executable, "-c", PROBE.format(root=ROOT, args=args)], env=e, capture_output=True,
                         text=True, timeout=120, cwd=ROOT)
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_bare_multi_gpu_bench_launches_its_ranks():
    r = _probe(["--gpus", "4", "--steps", "3", "--warmup", "1"])
    cmd = r["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"], cmd
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-6:] == ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    assert os.path.basename(cmd[cmd.index("--master-port") + 2]) == "bench.py"
    assert r["env"] == {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "ESGD_BENCH_SELF_LAUNCHED": "1"}
    assert r["exit"] == 7                 # the launcher's status is the bench's
    assert not r["hip_loaded"]            # decided before the HIP library is touched


def test_launcher_started_ranks_do_not_relaunch():
    # under torch.distributed.run (WORLD_SIZE set) every process is a rank: no relaunch.
    # Without a device the rank then stops at its device check, never at the launcher.
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", HIP_VISIBLE_DEVICES=""),
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert "torch.distributed.run" not in r.stderr
    assert r.returncode != 0 and "no HIP device" in (r.stderr + r.stdout)
    assert r.stdout == ""                 # a rank's stdout carries the JSON line or nothing


QUIET = r"""
import os, sys
sys.path.insert(0, {root!r})
import bench
print("python chatter before")
bench._quiet_stdout()
print("python chatter after", flush=True)
os.write(1, b"[Gloo] Rank 1 is connected to 1 peer ranks\n")   # native code on fd 1
bench.emit({{"metric": "m", "value": 1.0}})
"""


def test_rank_stdout_carries_only_the_json_line():
    # gloo / RCCL print to fd 1 from native code; under a launcher that stdout is the
    # job's, which the driver parses for the line
    r = subprocess.run([sys.executable, "-c", QUIET.format(root=ROOT)], capture_output=True, text=True,
                       timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "python chatter before"
    assert [json.loads(x) for x in lines[1:]] == [{"metric": "m", "value": 1.0}]
    assert "[Gloo]" in r.stderr and "chatter after" in r.stderr


def test_run_labels_follow_the_devices():
    # the line says what ran -- ranks sharing one GPU are a rehearsal
    import bench
    assert bench.run_labels(2, [0, 0], "ipc") == {
        "parallelism": "dp2 (2 ranks on one GPU: rehearsal)",
        "transport": "ipc pull (reduce-scatter tree kernel + all-gather) in one GPU's HBM"}
    one = bench.run_labels(8, list(range(8)), "ipc")
    assert one["parallelism"] == "dp8 (one rank per GPU)" and one["transport"].endswith("over xGMI")
    mixed = bench.run_labels(4, [0, 0, 1, 1], "ipc")
    assert mixed["parallelism"] == "dp4 (4 ranks on 2 GPUs, shared)" and "shared GPUs" in mixed["transport"]
    assert bench.run_labels(2, [0, 1], "rccl")["transport"].startswith("rccl p2p")


def test_baseline_cpus_one_thread_per_physical_core():
    # the CPU baseline's core list: 2 cores per simulated rank, never two SMT siblings
    import bench
    allowed = sorted(os.sched_getaffinity(0))
    cores = bench._baseline_cpus(1)
    if cores is None:
        pytest.skip("fewer than 2 physical cores here")
    assert len(cores) == 2 and len(set(cores)) == 2 and set(cores) <= set(allowed)

    def siblings(c):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                return f.read().strip()
        except OSError:
            return str(c)
    assert siblings(cores[0]) != siblings(cores[1])
    assert bench._baseline_cpus(10 ** 6) is None      # more than the host has: unpinned


def test_pinned_c1_harness_is_correct_and_pinned():
    # the oracle's C1-shaped harness with its threads on given cores: the every-rank result
    # is the tree's; pinning changes only placement
    import bench
    from oracle import ffref
    cores = bench._baseline_cpus(2)
    if cores is None:
        pytest.skip("fewer than 4 physical cores here")
    t, ok = ffref.time_c1(2, 4096, 3, cpus=cores)
    assert ok and t > 0


def test_wait_until_reaches_its_deadline():
    # the straggler's delay (mp_workers.wait_until): asleep but for the last 2 ms, never early
    import time

    from mp_workers import wait_until
    for d in (0.0005, 0.01):
        t0 = time.perf_counter()
        wait_until(t0 + d)
        el = time.perf_counter() - t0
        assert d <= el < d + 0.02, (d, el)
