"""The DQN policy step fused on the GPU (include/shipenv.h se_policy).

``DQNNetwork`` has the reference's module layout (agents/dqn.py:21-33: fc1, fc2,
fc3 nn.Linear), so a reference state_dict loads into it unchanged; training stays
in torch. ``QPolicy`` packs its weights for the fused kernel (bf16 MFMA, f32
accumulation), which computes for every env of a VecEnv the observation row,
Q = DQNNetwork(obs), the first maximum over the valid actions and epsilon-greedy
exploration (choose_action, :177-203) in one launch, without writing Q to HBM.
``act(precision="f32")`` runs the same step with the network in fp32 (bf16 MFMA on
3-way operand splits, or f32 MFMA), the precision the reference's agent evaluates it in.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn

from . import _native as N

HIDDEN = 128  # DQNNetwork's hidden_size default (agents/dqn.py:24); the fused kernel's width


class DQNNetwork(nn.Module):
    """agents/dqn.py:21-33: fc1 -> relu -> fc2 -> relu -> fc3."""

    def __init__(self, input_size: int, output_size: int, hidden_size: int = HIDDEN):
        super().__init__()
        self.fc1 = nn.Linear(input_size, hidden_size)
        self.fc2 = nn.Linear(hidden_size, hidden_size)
        self.fc3 = nn.Linear(hidden_size, output_size)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = torch.relu(self.fc1(x))
        x = torch.relu(self.fc2(x))
        return self.fc3(x)


def _ptr(t):
    return C.c_void_p(t.data_ptr())


class QPolicy:
    """choose_action for every env of `env` (a VecEnv) with the weights of `model`."""

    def __init__(self, env, model: DQNNetwork | None = None):
        self.env = env
        self._h = C.c_void_p()
        N.check(N.lib().se_qnet_create(C.byref(self._h), env._h))
        self.model = model if model is not None else DQNNetwork(env.obs_size, env.action_space_size)
        self.model.to(env.device)
        self.actions = torch.empty(env.n, dtype=torch.int32, device=env.device)
        self.set_weights()

    def set_weights(self, model: DQNNetwork | None = None):
        """Pack the current weights (after an optimizer step, or se_set_ports)."""
        if model is not None:
            self.model = model.to(self.env.device)
        m = self.model
        if m.fc1.out_features != HIDDEN or m.fc2.out_features != HIDDEN:
            raise ValueError(f"the fused policy is built for hidden_size {HIDDEN}")
        if m.fc1.in_features != self.env.obs_size or m.fc3.out_features != self.env.action_space_size:
            raise ValueError("network shape does not match the environment (6+4P -> ... -> 4+P+250)")
        self._w = [p.detach().to(self.env.device, torch.float32).contiguous() for p in (
            m.fc1.weight, m.fc1.bias, m.fc2.weight, m.fc2.bias, m.fc3.weight, m.fc3.bias)]
        N.check(N.lib().se_qnet_set_weights(self._h, *[_ptr(t) for t in self._w], self.env._stream()))

    def repack(self, bump: torch.Tensor | None = None):
        """Repack the same weight tensors after their values changed in place (an optimizer
        step); bump (device int32 [1]) is advanced by one on the stream (se_qnet_repack)."""
        N.check(N.lib().se_qnet_repack(self._h, _ptr(bump) if bump is not None else None, self.env._stream()))

    def act_record(self, replay, epsilon: float = 0.0, t: int = 0, precision: str = "bf16"):
        """act() plus the replay ring's remember(state, action) in the same launch
        (se_policy_record / se_policy_record_f32; replay: shippingenv_amd.dqn.ReplayBuffer).
        precision as act()."""
        if precision not in ("bf16", "f32"):
            raise ValueError("precision must be 'bf16' or 'f32'")
        fn = N.lib().se_policy_record if precision == "bf16" else N.lib().se_policy_record_f32
        N.check(fn(self._h, replay._h, _ptr(self.actions), float(epsilon), int(t) & 0xFFFFFFFF,
                   self.env._stream()))
        replay._act = self.actions
        return self.actions

    def act(self, epsilon: float = 0.0, t: int = 0, q_out: torch.Tensor | None = None,
            precision: str = "bf16"):
        """int32 actions [n] in the agent-index encoding (VecEnv.step input).
        q_out: optional f32 [n, >= A] to receive the Q rows (testing / inspection).
        precision: "bf16" (se_policy: bf16 weights and activations on bf16 MFMA, f32
        accumulation) or "f32" (se_policy_f32: the network in fp32 as agents/dqn.py runs
        it; fc2 and fc3 on bf16 MFMA with every f32 operand split into three bf16 parts,
        about 4x the bf16 policy's time)."""
        if precision not in ("bf16", "f32"):
            raise ValueError("precision must be 'bf16' or 'f32'")
        fn = N.lib().se_policy if precision == "bf16" else N.lib().se_policy_f32
        ldq = 0 if q_out is None else q_out.stride(0)
        N.check(fn(self._h, _ptr(self.actions), float(epsilon), int(t) & 0xFFFFFFFF,
                   None if q_out is None else _ptr(q_out), ldq, self.env._stream()))
        return self.actions

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            torch.cuda.synchronize(self.env.device)
            N.lib().se_qnet_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
