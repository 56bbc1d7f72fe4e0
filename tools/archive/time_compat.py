"""Config 1 (BASELINE.json configs[0]): one env, 100 steps through the drop-in
shipping.Environment, as the survey timed the reference:
random.seed(0) before construction, the five DEFAULT_PORTS, moves uniform over
N, E, S, W from random.Random(1), reset on done.

    python tools/time_compat.py [--reps R] [--oracle]

Prints one JSON line: ms per 100 steps (median over R repetitions) and the per-call
split. --oracle swaps the GPU stepper for the C oracle (test infrastructure: a CPU
timing of the same host logic, never the product path).
"""
import argparse
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

DEFAULT_PORTS = [[41, 40], [60, 22], [78, 29], [49, 72], [62, 72]]  # utils/constants.py:57-63


def run_once(Environment, ShipMove, ActionType):
    random.seed(0)
    env = Environment("mapa_mundi_binario.jpg")
    for p in DEFAULT_PORTS:
        env.add_port(list(p))
    env.reset()
    moves = [ShipMove.NORTH, ShipMove.EAST, ShipMove.SOUTH, ShipMove.WEST]
    pick = random.Random(1)
    t0 = time.perf_counter()
    for _ in range(100):
        try:
            _, _, done, _ = env.step([ActionType.MOVE_SHIP, moves[pick.randrange(4)]])
        except ValueError:  # "Move is out of range" (:284): the survey's driver skipped it
            continue
        if done:
            env.reset()
    return (time.perf_counter() - t0) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--oracle", action="store_true")
    a = ap.parse_args()
    from shippingenv_amd.shipping import environment
    from shippingenv_amd.shipping import ShipMove

    if a.oracle:
        from oracle_stepper import OracleStepper

        environment._set_stepper_factory(OracleStepper)
    run_once(environment.Environment, ShipMove, environment.ActionType)  # warm-up (map, library)
    ms = [run_once(environment.Environment, ShipMove, environment.ActionType) for _ in range(a.reps)]
    print(json.dumps({"workload": "config 1: 1 env x 100 steps through shipping.Environment",
                      "stepper": "oracle (CPU)" if a.oracle else "GPU (se_step_replay)",
                      "ms_per_100_steps": round(statistics.median(ms), 4),
                      "min_ms": round(min(ms), 4), "reps": a.reps}))


if __name__ == "__main__":
    main()
