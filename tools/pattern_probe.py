"""Probe: the deep500 op with the reference's random-straggler pattern and no barriers
between steps (tests/mp_workers.op_device_pattern); prints, per configuration, the steps
whose result differed between the two ranks and each step's contributor set."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    import mp_workers as m
    for packed in (False, True):
        for barrier in (False, True):
            for rep in range(2):
                outs = m.run("op_device_pattern", 2, packed=packed, barrier=barrier, timeout=200)
                bad = [t for t in range(len(outs[0])) if outs[0][t]["digest"] != outs[1][t]["digest"]]
                print(json.dumps({"packed": packed, "barrier": barrier, "rep": rep, "diverged_steps": bad,
                                  "r0": [(o["t"], o["late"], o["contributors"]) for o in outs[0]],
                                  "r1": [(o["t"], o["late"], o["contributors"]) for o in outs[1]]}), flush=True)


if __name__ == "__main__":
    main()
