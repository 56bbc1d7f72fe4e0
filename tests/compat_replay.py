"""Replay a compat_seed*.json script (tests/golden/make_compat_golden.py) against
shippingenv_amd.shipping.Environment and assert every result, Python type and
the global `random` stream match what the reference produced."""
import json
import os
import random

import numpy as np

from conftest import GOLDEN


def load_script(seed):
    with open(os.path.join(GOLDEN, f"compat_seed{seed}.json")) as f:
        return json.load(f)


def tname(v):
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, np.floating):
        return "np.float64"
    if isinstance(v, np.integer):
        return "np.int"
    if isinstance(v, int):
        return "int"
    if isinstance(v, float):
        return "float"
    if v is None:
        return "None"
    return type(v).__name__


def snap(env):
    st = env._build_state()["ship"]
    pos = st["position"]
    return {
        "position": [int(pos[0]), int(pos[1])] if len(pos) else [],
        "fuel": float(st["fuel"]), "fuel_type": tname(st["fuel"]),
        "cargo_field": float(st["cargo"]),
        "cargo": int(env.cargo),
        "origin": st["origin_port_index"], "dest": st["destination_port_index"],
        "aliases_port": any(pos is p for p in env.port_positions),
    }


def replay(script, max_events=None):
    from shippingenv_amd.maps import BUILTIN_MAP
    from shippingenv_amd.shipping import Environment

    random.seed(script["seed"])
    env = Environment(BUILTIN_MAP)
    n = 0
    for k, ev in enumerate(script["events"]):
        if max_events is not None and k >= max_events:
            break
        op = ev["op"]
        where = f"seed {script['seed']} event {k} {ev}"
        if op == "add_ports":
            for p in ev["ports"]:
                env.add_port(list(p))
            assert env.port_fuel == ev["port_fuel"] and env.port_cargo == ev["port_cargo"], where
        elif op == "reset":
            env.reset()
            assert snap(env) == ev["after"], where
        elif op == "set_fuel":
            env.fuel = ev["value"] if ev["value_type"] != "float" else float(ev["value"])
        elif op == "sample_action":
            try:
                a = env.sample_action()
                got = [a[0], list(a[1]) if isinstance(a[1], tuple) else a[1]]
                assert ev["exc"] is None and got == ev["result"], where
            except Exception as e:  # noqa: BLE001
                assert ev["exc"] == [type(e).__name__, str(e)], (where, e)
        elif op == "step":
            act = ev["action"]
            action = [act[0], tuple(act[1]) if isinstance(act[1], list) else act[1]]
            try:
                _, reward, done, info = env.step(action)
                got = {"exc": None, "reward": float(reward), "reward_type": tname(reward),
                       "done": bool(done), "done_type": tname(done)}
                want = {k2: ev[k2] for k2 in got}
                assert got == want, (where, got)
                assert info == {}
            except AssertionError:
                raise
            except Exception as e:  # noqa: BLE001
                assert ev["exc"] == [type(e).__name__, str(e)], (where, e)
            if "after" in ev:
                assert snap(env) == ev["after"], (where, snap(env))
            n += 1
        if "probe" in ev:
            assert random.random() == ev["probe"], f"random stream diverged at {where}"
    return n
