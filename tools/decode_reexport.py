"""Decode the wrong sums of the IPC re-export diagnostic (test_ipc_reexport_sequence_bitexact[2]
run with ESGD_IPC_TRACE=1; gpu_config's detail lines).

For every mismatch line it finds which substitution of ONE rank's input by another rank's
reproduces the wrong value under the tree order ("i<-j": rank i's contribution was rank j's
data), or which single input the value equals ("=xj": a gathered shard read raw from rank j),
and lists each rank's exported chunks from the trace.

    python tools/decode_reexport.py gpurun_out/r03k/reexport_*.log
"""
import collections
import re
import sys

import numpy as np

LINE = re.compile(r"\[r(\d+)\] count=(\d+) t=(\d+) slice@(\d+): \d+ bad, first \d+ got (\S+) want (\S+); "
                  r"last \d+; inputs there \[([^\]]*)\]")
TRACE = re.compile(r"esgd-ipc pid (\d+) (\w+) peer (-?\d+) ptr (0x[0-9a-f]+) bytes (\d+) handle ([0-9a-f]+)")


def tree(v):
    v = [np.float32(a) for a in v]
    s = 1
    while s < len(v):
        for j in range(0, len(v) - s, 2 * s):
            v[j] = np.float32(v[j + s] + v[j])
        s *= 2
    return v[0]


def decode(path):
    pattern = collections.Counter()
    exports, opens, handles = {}, {}, set()
    text = open(path).read()
    for m in LINE.finditer(text):
        rank, _, t, sl, got, _, inputs = m.groups()
        x = np.array([float(a) for a in inputs.split(",")], np.float32)
        got = np.float32(float(got))
        tags = []
        for i in range(len(x)):
            for j in range(len(x)):
                if i != j:
                    y = x.copy()
                    y[i] = x[j]
                    if tree(y) == got:
                        tags.append(f"{i}<-{j}")
            if x[i] == got:
                tags.append(f"=x{i}")
        pattern[(int(t), int(sl), f"r{rank}" if sl == "0" else "all ranks", tuple(tags))] += 1
    for m in TRACE.finditer(text):
        pid, what, peer, ptr, nbytes, h = m.groups()
        if what == "export":
            exports.setdefault(pid, []).append((ptr, int(nbytes)))
            handles.add(h)
        elif what == "open":
            opens.setdefault(pid, set()).add(int(peer))
    world = len(exports)
    rank_of = {pid: (set(range(world)) - peers).pop() for pid, peers in opens.items() if len(peers) == world - 1}
    print(f"== {path}")
    print(f"   {sum(len(v) for v in exports.values())} exports, {len(handles)} distinct handles")
    for pid in sorted(exports, key=lambda p: rank_of.get(p, 99)):
        print(f"   rank {rank_of.get(pid)} pid {pid} exported {exports[pid]}")
    for k, v in sorted(pattern.items()):
        print(f"   round {k[0]} slice@{k[1]} {k[2]}: {' '.join(k[3]) or 'no single substitution'} (x{v})")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        decode(p)
