"""shippingenv_amd — MI355X-native batched ShippingEnv.

The hot path of VanshJP/ShippingEnv (shipping/environment.py Environment.step /
reset) as gfx950 HIP kernels behind a C-ABI (include/shipenv.h):

* ``shippingenv_amd.vec.VecEnv`` — N environments per GPU on torch tensors;
* ``shippingenv_amd.shipping`` — the reference's ``shipping`` package surface
  (Environment, add_port, reset, step, sample_action, ...) on the same kernels;
  the directory ``shippingenv_amd/dropin`` on ``sys.path`` makes it ``import shipping``;
* ``VecEnv.observe`` / ``VecEnv.valid_mask`` — the reference's
  ``utils.preprocessing`` row layout and DQN validity, batched;
* ``shippingenv_amd.policy`` / ``shippingenv_amd.dqn`` — the fused DQN policy and
  the vectorised DQN training loop;
* ``shippingenv_amd.maps`` — the map loader (``_initialize_map``);
* ``shippingenv_amd.dist`` — one process per GPU, env sharding, RCCL stats.
"""

__version__ = "0.1.0"
