"""Golden table of the reference's own action decode (utils/preprocessing.py:111-137).

TEST INFRASTRUCTURE, build container only (it imports /root/reference with the cv2 stub).
For P = 5 (utils/constants.py:57-63, the default ports) and P = 64, it calls the
reference's ``map_action_to_env_action(agent_action, env)`` on a reference Environment for
every agent index from -6 to A + 2 (A = ``get_action_space_size(env)``) and records what
it returns, [ActionType, value] with a move's value as (dx, dy), or the exception it raises
(IndexError for indices below -4: Python list indexing of the four moves). Output:
``decode_golden.json``:

    {"P": {"5": {"A": 259, "rows": [[index, type, a, b] | [index, "IndexError"], ...]}, "64": ...}}

tests/test_reference_quirks.py pins the kernel's decode and the golden tapes' agent_idx
column to this table (CPU), and tests/test_gpu_parity.py replays the golden records as
agent indices taken from it through the production agent-path kernel
(se_step_agent_replay).

    python tests/golden/make_decode_golden.py
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
from utils.constants import DEFAULT_PORTS  # noqa: E402
from utils.preprocessing import get_action_space_size, map_action_to_env_action  # noqa: E402


def table(ports):
    random.seed(0)
    env = Environment(os.path.join(REF, "mapa_mundi_binario.jpg"))
    for p in ports:
        env.add_port(list(p))
    A = get_action_space_size(env)
    rows = []
    for idx in range(-6, A + 3):
        try:
            t, v = map_action_to_env_action(idx, env)
        except IndexError:
            rows.append([idx, "IndexError"])
            continue
        if isinstance(v, tuple):
            rows.append([idx, int(t), int(v[0]), int(v[1])])
        else:
            rows.append([idx, int(t), int(v), 0])
    return {"A": A, "rows": rows}


def main():
    water = None
    random.seed(1)
    env = Environment(os.path.join(REF, "mapa_mundi_binario.jpg"))
    water = [(x, y) for x in range(100) for y in range(100) if env.np_game[x, y] == 1]
    ports64 = random.Random(5).sample(water, 64)
    out = {"source": "utils/preprocessing.py:111-137 map_action_to_env_action, :93-108 get_action_space_size",
           "P": {"5": table(DEFAULT_PORTS), "64": table(ports64)}}
    with open(os.path.join(HERE, "decode_golden.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print({k: (v["A"], len(v["rows"])) for k, v in out["P"].items()})


if __name__ == "__main__":
    main()
