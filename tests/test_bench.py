"""bench.py's launcher logic on the CPU (no device): a bare `bench.py --gpus N` must start
its own N ranks through torch.distributed.run -- before anything in the parent loads the
HIP library -- and exit with their status (the reference's launcher
starts its ranks the same way, test_scripts_imagenet/daint_eagersgd_imagenet.sh:2-5)."""
import json
import os
import subprocess
import sys

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
