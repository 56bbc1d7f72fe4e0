"""BASELINE configs[0] on one host: the reference's Python Environment.step() beside the
drop-in (shippingenv_amd.shipping, host stepper and, with a GPU, the kernel), in one process,
interleaved, best of R medians of 10 runs each. Build container only: it imports the
reference from /root/reference (with the cv2 stub of tests/golden) to time it.

    python tools/time_config1_vs_reference.py [--reps 15] [--json out.json]

The workload is bench.py's run_config1: random.seed(0), the five DEFAULT_PORTS, 100 steps
of moves uniform over N, E, S, W from random.Random(1), reset on done.
"""
import argparse
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PORTS = [[41, 40], [60, 22], [78, 29], [49, 72], [62, 72]]  # utils/constants.py:57-63


def runner(env_mod, map_path, moves):
    def once():
        random.seed(0)
        env = env_mod.Environment(map_path)
        for p in PORTS:
            env.add_port(list(p))
        env.reset()
        pick = random.Random(1)
        t0 = time.perf_counter()
        for _ in range(100):
            try:
                _, _, done, _ = env.step([env_mod.ActionType.MOVE_SHIP, moves[pick.randrange(4)]])
            except ValueError:
                continue
            if done:
                env.reset()
        return (time.perf_counter() - t0) * 1e3
    return once


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=15)
    p.add_argument("--json")
    a = p.parse_args()
    sys.path.insert(0, ROOT)
    from shippingenv_amd.shipping import ShipMove, environment as ours

    legs = {}
    os.environ["SHIPENV_STEPPER"] = "host"
    mv = [ShipMove.NORTH, ShipMove.EAST, ShipMove.SOUTH, ShipMove.WEST]
    legs["dropin_host"] = runner(ours, "mapa_mundi_binario.jpg", mv)
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden", "cv2stub"))
    sys.path.insert(0, REF)
    from shipping import environment as ref  # noqa: E402  the reference package
    from shipping.type import ShipMove as RM  # noqa: E402

    legs["reference"] = runner(ref, os.path.join(REF, "mapa_mundi_binario.jpg"),
                               [RM.NORTH, RM.EAST, RM.SOUTH, RM.WEST])
    for f in legs.values():
        f()
    best = {k: float("inf") for k in legs}
    for _ in range(a.reps):
        for k, f in legs.items():
            best[k] = min(best[k], statistics.median(f() for _ in range(10)))
    out = {"workload": "BASELINE configs[0]: 1 env x 100 steps, default ports, uniform moves",
           "ms_per_100_steps": {k: round(v, 4) for k, v in best.items()},
           "ratio_dropin_over_reference": round(best["dropin_host"] / best["reference"], 3),
           "host": os.uname().nodename, "basis": f"best of {a.reps} medians of 10 runs, interleaved"}
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
