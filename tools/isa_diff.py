"""Compare two gfx950 device assembly files kernel by kernel.

    hipcc <build flags> --cuda-device-only -S -o before.s shippingenv_amd/csrc/shipenv.hip
    ... edit ...
    hipcc <build flags> --cuda-device-only -S -o after.s  shippingenv_amd/csrc/shipenv.hip
    python tools/isa_diff.py before.s after.s

Prints the kernels only in one file and the kernels whose instruction stream differs
(comments, directives and the per-function label numbering normalised away). Used to show
that deleting dead compile-time variants left the product kernels' code unchanged.
"""
from __future__ import annotations

import re
import sys


def functions(path):
    funcs = {}
    cur = None
    body = []
    for line in open(path):
        m = re.match(r"^(_Z\w+|\w+):\s*(;.*)?$", line)
        if m and not line.startswith("."):
            if cur:
                funcs[cur] = body
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            funcs[cur] = body
            cur, body = None, []
            continue
        s = line.split(";", 1)[0].strip()
        if not s or s.startswith(".loc") or s.startswith(".file") or s.startswith(".cfi"):
            continue
        s = re.sub(r"\.LBB\d+_(\d+)", r".LBB_\1", s)
        s = re.sub(r"\.Ltmp\d+", ".Ltmp", s)
        s = re.sub(r"\.Lfunc_end\d+", ".Lfunc_end", s)
        body.append(s)
    if cur:
        funcs[cur] = body
    return funcs


def main(a, b):
    fa, fb = functions(a), functions(b)
    only_a = sorted(set(fa) - set(fb))
    only_b = sorted(set(fb) - set(fa))
    diff = sorted(k for k in set(fa) & set(fb) if fa[k] != fb[k])
    same = len(set(fa) & set(fb)) - len(diff)
    print(f"identical: {same}")
    for k in only_a:
        print(f"only in {a}: {k} ({len(fa[k])} lines)")
    for k in only_b:
        print(f"only in {b}: {k} ({len(fb[k])} lines)")
    for k in diff:
        print(f"DIFFERS: {k} ({len(fa[k])} vs {len(fb[k])} lines)")
    return 1 if diff else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))
