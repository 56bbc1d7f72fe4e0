"""Which load / init order of torch's HIP runtime and libshipenv_hip.so lets se_create
see the GPU (diagnostic for the compat path: Environment(<jpeg>) loads the library
for the map decode before anything touches the GPU)."""
import ctypes as C
import sys

import numpy as np
import torch

order = sys.argv[1]
sys.path.insert(0, ".")
from shippingenv_amd import _native as N  # noqa: E402


def create(lib):
    h = C.c_void_p()
    water = np.ones((100, 100), np.uint8)
    px = np.array([1], np.int32)
    rc = lib.se_create(C.byref(h), 0, 1, 0, 100, 100, water.ctypes.data_as(C.c_void_p), 1,
                       px.ctypes.data_as(C.c_void_p), px.ctypes.data_as(C.c_void_p),
                       px.ctypes.data_as(C.c_void_p), px.ctypes.data_as(C.c_void_p), 0, 0)
    return rc, lib.se_last_error().decode()


if order == "torch_first":
    print(torch.cuda.is_available())
    lib = N.lib()
elif order == "lib_first":
    lib = N.lib()
    print(torch.cuda.is_available())
elif order == "jpeg_first":
    from shippingenv_amd.maps import load_water
    load_water("mapa_mundi_binario.jpg")
    lib = N.lib()
    print(torch.cuda.is_available())
elif order == "env_jpeg":
    from shippingenv_amd.shipping import Environment
    env = Environment("mapa_mundi_binario.jpg")
    env.add_port([41, 40]); env.add_port([60, 22])
    env.reset()
    print(order, "reset ok")
    sys.exit(0)
elif order == "env_builtin":
    from shippingenv_amd.maps import BUILTIN_MAP
    from shippingenv_amd.shipping import Environment
    env = Environment(BUILTIN_MAP)
    env.add_port([41, 40]); env.add_port([60, 22])
    env.reset()
    print(order, "reset ok")
    sys.exit(0)
elif order == "lib_first_tensor":
    lib = N.lib()
    torch.zeros(1, device="cuda")
print(order, create(lib))
