"""Generate the committed golden vectors under tests/golden/ (run from the repo root:
`python tests/golden/gen_golden.py`).

Everything here is produced by the build's own oracle (oracle/ffref.c, a CPU
restatement of fflib2) or by this host's libc — never by reference code, which may
not be executed in this pipeline.  Files are .npz (no pickle) and
JSON, each well under 1 MiB.

  tree_f32_p{2,4,8}.npz   inputs x[P][n] and every rank's recursive-doubling result
                          (src/colls/ffallreduce.c:138-171) for gaussian and special
                          (subnormal, +-0, +-inf, cancellation) fp32 inputs
  known_int32.npz         allreduce of to_reduce[j] = i + j (evaluation/allreduce.c:49-63)
  tree_bf16_p8.npz        bf16 extension (parity unpinned: no bf16 in the reference)
  rand_r.json             libc rand_r sequences for the seeds the reference uses
                          (6545343: opt_esgd_majority_imagenet_imbalance.py:252;
                           34495645: evaluation/rand_allreduce_correctness.c:64)
"""
from __future__ import annotations

import ctypes
import ctypes.util
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ffref  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
N = 4099  # ragged: not a multiple of 4 (fp32 vector width) or 1024 (VSUM strip)


def special_inputs(P: int, n: int, rng: np.random.Generator) -> np.ndarray:
    x = rng.standard_normal((P, n)).astype(np.float32)
    tiny = np.float32(np.finfo(np.float32).smallest_subnormal)
    for r in range(P):
        x[r, 0:16] = tiny * (r + 1)                       # subnormal sums
        x[r, 16:32] = np.float32(-0.0) if r % 2 else np.float32(0.0)   # signed zeros
        x[r, 32] = np.float32(np.inf) if r == 0 else np.float32(1.0)   # +inf survives
        x[r, 33] = np.float32(-np.inf) if r == P - 1 else np.float32(2.0)
        x[r, 34:64] = np.float32(1e30) * (1 if r % 2 == 0 else -1)     # cancellation
        x[r, 64:96] = np.float32(2.0 ** 24) if r == 0 else np.float32(1.0)  # rounding
        x[r, 96:128] = np.float32(3.4e38) / P                            # near overflow
    return x


def main():
    rng = np.random.default_rng(0x5EEDE56D)
    for P in (2, 4, 8):
        g = rng.standard_normal((P, N)).astype(np.float32)
        s = special_inputs(P, N, rng)
        out = {}
        for name, x in (("gauss", g), ("special", s)):
            rb = ffref.allreduce_rd(list(x))
            out[f"{name}_x"] = x
            out[f"{name}_rb"] = np.stack(rb)
        np.savez_compressed(os.path.join(OUT, f"tree_f32_p{P}.npz"), **out)

    ki = {}
    for P in (1, 2, 4, 8):
        for it in (0, 7):
            x = np.stack([np.arange(it, it + N, dtype=np.int32) for _ in range(P)])
            ki[f"p{P}_i{it}_x"] = x
            ki[f"p{P}_i{it}_rb"] = np.stack(ffref.allreduce_rd(list(x)))
    np.savez_compressed(os.path.join(OUT, "known_int32.npz"), **ki)

    xb = ffref.f32_to_bf16(rng.standard_normal((8, N)).astype(np.float32))
    np.savez_compressed(os.path.join(OUT, "tree_bf16_p8.npz"), x=xb, out=ffref.tree_sum_bf16(list(xb)))

    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.rand_r.argtypes = [ctypes.POINTER(ctypes.c_uint)]
    seqs = {}
    for seed in (6545343, 34495645, 0, 1, 0xFFFFFFFF):
        s = ctypes.c_uint(seed)
        seqs[str(seed)] = [int(libc.rand_r(ctypes.byref(s))) for _ in range(64)]
    with open(os.path.join(OUT, "rand_r.json"), "w") as f:
        json.dump({"source": "host libc rand_r (glibc)", "draws": 64, "sequences": seqs}, f,
                  indent=1)
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main()
