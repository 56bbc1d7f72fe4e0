"""Golden sample_action decisions of the reference Environment.

TEST INFRASTRUCTURE, build container only (imports /root/reference with the cv2
stub of cv2stub/). For random ship states on the default map (ports on and off
the ship's cell, destination set or None, cargo 0 or not, fuel 0 or not, one port
with an empty cargo stock) it records what sample_action()
(shipping/environment.py:245-263) returned or raised. The category of the result
is a function of the state alone; the value is drawn through `random`. The test
tests/test_rollout_cpu.py requires the oracle's sample_action to return the same
category and a value in the same support.

    python tests/golden/make_sample_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "cv2stub"))
sys.path.insert(0, REF)

from shipping import Environment  # noqa: E402

MAP = os.path.join(REF, "mapa_mundi_binario.jpg")
DEFAULT_PORTS = [[41, 40], [60, 22], [78, 29], [49, 72], [62, 72]]  # utils/constants.py:57-63


def main(n_states=1500, seed=7):
    random.seed(seed)
    env = Environment(MAP)
    for p in DEFAULT_PORTS:
        env.add_port(list(p))
    env.port_cargo[4] = 0  # randint(1, 0) raises ValueError from sample_action
    rng = random.Random(seed + 1)
    water = [(x, y) for x in range(100) for y in range(100) if env.np_game[x, y] != 0]
    out = []
    for _ in range(n_states):
        if rng.random() < 0.45:
            pos = list(DEFAULT_PORTS[rng.randrange(5)])
        else:
            pos = list(water[rng.randrange(len(water))])
        dest = None if rng.random() < 0.3 else rng.randrange(5)
        origin = None if rng.random() < 0.2 else rng.randrange(5)
        cargo = 0 if rng.random() < 0.5 else rng.randint(1, 80)
        fuel = 0 if rng.random() < 0.2 else round(rng.uniform(0.5, 250.0), 3)
        env.ship_position = pos
        env.destination_port_index = dest
        env.origin_port_index = origin
        env.cargo = cargo
        env.fuel = fuel
        rec = {"x": pos[0], "y": pos[1], "dest": dest, "origin": origin, "cargo": cargo,
               "fuel": fuel}
        try:
            t, v = env.sample_action()
            if isinstance(v, (list, tuple)):
                rec["out"] = {"type": int(t), "a": int(v[0]), "b": int(v[1])}
            else:
                rec["out"] = {"type": int(t), "a": int(v), "b": 0}
        except Exception as e:  # noqa: BLE001 - the reference's exception is the datum
            rec["out"] = {"raise": type(e).__name__}
        out.append(rec)
    doc = {"ports": DEFAULT_PORTS, "port_fuel": list(env.port_fuel),
           "port_cargo": list(env.port_cargo), "states": out}
    path = os.path.join(HERE, "sample_golden.json")
    with open(path, "w") as f:
        json.dump(doc, f)
    cats = {}
    for r in out:
        k = r["out"].get("raise") or r["out"]["type"]
        cats[k] = cats.get(k, 0) + 1
    print(path, cats)


if __name__ == "__main__":
    main()
