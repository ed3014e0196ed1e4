"""A C program that only includes ff.h and links libesgd.so (the drop-in boundary),
run as P processes with launcher-style environment, checking the reference
evaluation programs' known answers (see tests/c/ff_known_answers.c)."""
import os
import subprocess
import uuid

import pytest

from conftest import LIB, ROOT

pytestmark = pytest.mark.gpu


def build(tmp_path):
    exe = str(tmp_path / "ff_known_answers")
    subprocess.check_call(["gcc", "-O2", "-std=c11", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "ff_known_answers.c"), "-o", exe,
                           LIB, "-Wl,-rpath," + os.path.dirname(LIB)])
    return exe


def _gpus():
    import esgd
    return esgd.device_count()


# (world, transport): the IPC data plane at 1, 2 and 4 ranks; RCCL at one rank (its
# FFCOLL_BUFFERS rounds resize the staging on the progress thread from the arena, no
# hipFree there) and, where every rank has a GPU of its own, at two
@pytest.mark.parametrize("world,transport", [(1, "ipc"), (2, "ipc"), (4, "ipc"), (1, "rccl"), (2, "rccl")])
def test_c_caller_known_answers(tmp_path, world, transport):
    if transport == "rccl" and world > 1 and _gpus() < world:
        pytest.skip("RCCL refuses two ranks on one GPU")
    exe = build(tmp_path)
    job = uuid.uuid4().hex
    procs = []
    for r in range(world):
        # ffinit picks device LOCAL_RANK % device_count: one GPU per rank on a full node
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   ESGD_JOB_ID=job, ESGD_TIMEOUT_S="60", ESGD_TRANSPORT=transport,
                   ESGD_DEBUG=os.environ.get("ESGD_DEBUG", "0"))
        procs.append(subprocess.Popen([exe, "10007", "4"], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=180)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "Correctness check passed" in outs[0]
