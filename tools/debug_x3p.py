"""Round-6 debugging aid: the pipelined fp32 policy (no q_out) against the first masked
argmax of the q_out kernel's own Q rows."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
if len(sys.argv) > 1:
    from shippingenv_amd import _native
    _native.LIB_PATH = os.path.abspath(sys.argv[1])
from test_gpu_policy import make, valid_bool, first_masked_argmax, _OPEN

for n in (32,):
    env, model, pol = make(n, steps=0, scale=20.0)
    q_out = torch.empty((env.n, env.action_space_size), dtype=torch.float32, device=env.device)
    full = pol.act(0.0, 5, q_out=q_out, precision="f32").cpu().numpy().copy()
    q = q_out.cpu().numpy(); valid = valid_bool(env)
    comp = pol.act(0.0, 5, precision="f32").cpu().numpy()
    a = np.arange(q.shape[1])
    for hsel in (0, 1):
        m = valid & (((a % 8) // 4) == hsel)[None, :]
        print("half", hsel, first_masked_argmax(q, m)[:8])
    print("comp", comp[:8], "full", full[:8])
    print("valid actions env0", np.nonzero(valid[0])[0])
    print("q env0 valid", q[0][valid[0]])
    while _OPEN:
        _OPEN.pop().close()
