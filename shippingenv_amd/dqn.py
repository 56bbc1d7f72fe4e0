"""Vectorised DQN training on the device (agents/dqn.py DQNAgent).

One ``VecDQNAgent.step()`` is one iteration of the reference's training loop
(agents/dqn.py:276-300) for every env of an auto-reset VecEnv at once:

* choose_action (:177-203): ``se_policy``, the fused MFMA policy step (policy.py).
* env.step, then remember (:117-123): ``se_replay_begin`` / ``se_step`` /
  ``se_replay_end``, which append to the device replay ring (include/shipenv.h).
* the loop's episode breaks: a step that raised (:304-309) or ``max_steps``
  (:281). ``se_replay_end`` marks these envs and ``se_reset`` restarts them.
* update() (:206-245): ``se_qtrain_step_replay`` (FusedUpdate, csrc/qtrain.h) draws the
  minibatch from the ring (the transitions ``se_replay_sample`` would pick), computes the
  MSE to r + gamma * max target Q * (1 - done), the backward pass and Adam in two f32 MFMA
  kernels, and rewrites the policy's bf16 weights. Then comes the epsilon decay.
  ``fused=False`` runs the same update with torch autograd and torch.optim.Adam on the
  minibatch ``se_replay_sample`` writes.

The fused update is two launches, issued eagerly: a HIP graph replay of them measured
5-6 us slower per update (the graph launch's own gap; tools/diag/update_forms.py). The
torch path (about 50 small kernels) is captured in one HIP graph after ``graph_warmup``
eager updates; ``graph=True`` / ``False`` forces either form on either path.

Differences from the single-env reference, by construction:
* The batch holds distinct transitions, like random.sample; see se_replay_sample.
* A raised step is stored flagged and never sampled.
* The target network is synchronised every ``target_update_every`` updates instead
  of every ``target_update_freq`` episodes. With N envs, episodes end N at a time.
* ``len(memory)`` counts ring slots.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _native as N
from .policy import HIDDEN, DQNNetwork, QPolicy

# utils/constants.py TrainingDefaults (DQN_*): the reference's defaults
DQN_BATCH_SIZE = 32
DQN_MEMORY_SIZE = 2000
DQN_GAMMA = 0.95
DQN_EPSILON = 1.0
DQN_EPSILON_MIN = 0.01
DQN_EPSILON_DECAY = 0.995
DQN_LEARNING_RATE = 0.001
MAX_STEPS_PER_EPISODE = 1000

_DEBUG = os.environ.get("SHIPENV_DEBUG") == "1"


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class MiniBatch:
    """The static minibatch tensors se_replay_sample writes (graph-replay safe)."""

    def __init__(self, batch, width, device):
        f32 = dict(dtype=torch.float32, device=device)
        self.obs = torch.zeros((batch, width), **f32)
        self.next_obs = torch.zeros((batch, width), **f32)
        self.act = torch.zeros(batch, dtype=torch.int64, device=device)
        self.rew = torch.zeros(batch, **f32)
        self.done = torch.zeros(batch, **f32)
        self.weight = torch.zeros(batch, **f32)
        self.batch = batch


class ReplayBuffer:
    """DQNAgent.memory (agents/dqn.py:86) on the device: a ring of `capacity` compact
    transitions of one VecEnv (se_replay_*)."""

    def __init__(self, env, capacity: int):
        self.env = env
        self._h = C.c_void_p()
        N.check(N.lib().se_replay_create(C.byref(self._h), env._h, int(capacity)))

    def __len__(self):
        return self.size

    @property
    def size(self) -> int:
        s = C.c_int64()
        N.check(N.lib().se_replay_size(self._h, C.byref(s), None))
        return s.value

    @property
    def capacity(self) -> int:
        c = C.c_int64()
        N.check(N.lib().se_replay_size(self._h, None, C.byref(c)))
        return c.value

    def begin(self, actions: torch.Tensor):
        """remember's state and action, before env.step(actions)."""
        self._act = actions  # kept alive until the launch has run
        N.check(N.lib().se_replay_begin(self._h, _ptr(actions), self.env._stream()))

    def end(self, cut: torch.Tensor | None = None, max_steps: int = 0, reset: bool = False):
        """reward, done and next_state, after env.step; cut[i] = 1 where the episode must restart.
        reset: also restart those episodes in the same pass (se_replay_end_reset: what
        env.reset(cut) would do, one launch instead of two)."""
        fn = N.lib().se_replay_end_reset if reset else N.lib().se_replay_end
        N.check(fn(self._h, _ptr(cut), int(max_steps), self.env._stream()))

    def step_end(self, actions: torch.Tensor, cut: torch.Tensor, max_steps: int = 0):
        """env.step(actions) then end(cut, max_steps, reset=True) in one launch
        (se_step_record: the step kernel writes the record and restarts the cut envs)."""
        env = self.env
        a = actions
        if not (type(a) is torch.Tensor and a.dtype is torch.int32 and a.is_cuda and a.is_contiguous()
                and a.numel() == env.n and a.data_ptr() % 16 == 0):
            a = env._dev(actions, torch.int32)
        N.check(N.lib().se_step_record(self._h, _ptr(a), _ptr(cut), int(max_steps), env._stream()))
        env._keep = a

    def sample(self, out: MiniBatch, t: int = 0, t_dev: torch.Tensor | None = None) -> MiniBatch:
        """update()'s minibatch (agents/dqn.py:213-224) into `out`; the sampler key is t, or
        the device counter t_dev (uint32 viewed as int32) when given."""
        N.check(N.lib().se_replay_sample(self._h, out.batch, _ptr(t_dev), int(t) & 0xFFFFFFFF,
                                         _ptr(out.obs), _ptr(out.next_obs), _ptr(out.act),
                                         _ptr(out.rew), _ptr(out.done), _ptr(out.weight),
                                         self.env._stream()))
        return out

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            torch.cuda.synchronize(self.env.device)
            N.lib().se_replay_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class SeMlp(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("w1", "b1", "w2", "b2", "w3", "b3")]


def _linear_params(model):
    ps = [model.fc1.weight, model.fc1.bias, model.fc2.weight, model.fc2.bias, model.fc3.weight, model.fc3.bias]
    for p in ps:
        if p.dtype != torch.float32 or not p.is_contiguous() or not p.is_cuda:
            raise ValueError("the fused update needs contiguous f32 device parameters")
    return ps


def _mlp(tensors):
    return SeMlp(*[t.data_ptr() for t in tensors])


class FusedUpdate:
    """update()'s loss, backward and Adam step (agents/dqn.py:226-242) fused on f32 MFMA
    (se_qtrain_*: two kernels per update). The parameters stay the torch modules' tensors,
    updated in place. Adam's exp_avg / exp_avg_sq live here."""

    def __init__(self, env, model, target_model, max_batch: int, lr: float,
                 betas=(0.9, 0.999), eps: float = 1e-8):
        if model.fc1.out_features != HIDDEN or model.fc2.out_features != HIDDEN:
            raise ValueError(f"the fused update is built for hidden_size {HIDDEN}")
        self.env, self.lr, self.betas, self.eps = env, float(lr), tuple(map(float, betas)), float(eps)
        self.params = _linear_params(model)
        self.target = _linear_params(target_model)
        self.exp_avg = [torch.zeros_like(p) for p in self.params]
        self.exp_avg_sq = [torch.zeros_like(p) for p in self.params]
        self._structs = [_mlp(t) for t in (self.params, self.target, self.exp_avg, self.exp_avg_sq)]
        self._h = C.c_void_p()
        N.check(N.lib().se_qtrain_create(C.byref(self._h), env._h, int(max_batch)))
        N.check(N.lib().se_qtrain_bind(self._h, *[C.byref(x) for x in self._structs], env._stream()))

    def pack(self, which: int):
        """Rebuild the kernel's image of the online (0) or target (1) network."""
        N.check(N.lib().se_qtrain_pack(self._h, int(which), self.env._stream()))

    def step(self, b: MiniBatch, gamma: float, step_dev: torch.Tensor, loss_out: torch.Tensor):
        N.check(N.lib().se_qtrain_step(self._h, b.batch, _ptr(b.obs), _ptr(b.next_obs), _ptr(b.act),
                                       _ptr(b.rew), _ptr(b.done), _ptr(b.weight), float(gamma),
                                       self.lr, self.betas[0], self.betas[1], self.eps,
                                       _ptr(step_dev), _ptr(loss_out), self.env._stream()))

    def step_policy(self, b: MiniBatch, gamma: float, step_dev: torch.Tensor, loss_out: torch.Tensor, policy):
        """step(), then policy.repack(bump=step_dev), in the same two launches
        (se_qtrain_step_policy): the policy's images are written by the Adam kernel and the
        counter is advanced by the first kernel. policy: a QPolicy packed from `model`."""
        N.check(N.lib().se_qtrain_step_policy(self._h, policy._h, b.batch, _ptr(b.obs), _ptr(b.next_obs),
                                              _ptr(b.act), _ptr(b.rew), _ptr(b.done), _ptr(b.weight),
                                              float(gamma), self.lr, self.betas[0], self.betas[1], self.eps,
                                              _ptr(step_dev), _ptr(loss_out), self.env._stream()))

    def step_replay(self, memory, batch: int, gamma: float, ctr: torch.Tensor, loss_out: torch.Tensor,
                    policy=None, t: int | None = None):
        """memory.sample(t_dev=ctr) then step_policy(..., step_dev=ctr) (step() without a
        policy), in two launches (se_qtrain_step_replay): the first draws its minibatch rows
        from the ring itself. ctr: device int32 [2], both entries the updates taken so far.
        t: the caller's copy of ctr[0] (eager calls: the first kernel then does not wait on
        the device counter); None reads it on the device (graph capture). t must equal
        ctr[0] exactly: the first kernel writes ctr[1] = t + 1, which becomes Adam's step
        count and the next ctr[0], so a stale t would rewind the counter. SHIPENV_DEBUG=1
        checks it (one host sync per call)."""
        if ctr.dtype != torch.int32 or ctr.numel() < 2 or not ctr.is_contiguous():
            raise ValueError("ctr must be a contiguous int32 device tensor of 2 entries")
        if t is not None and _DEBUG and not torch.cuda.is_current_stream_capturing():
            dev_t = int(ctr[0].item())
            if dev_t != int(t):
                raise ValueError(f"step_replay: t = {t} but ctr[0] = {dev_t} (t must be ctr[0])")
        N.check(N.lib().se_qtrain_step_replay(self._h, None if policy is None else policy._h, memory._h,
                                              int(batch), float(gamma), self.lr, self.betas[0],
                                              self.betas[1], self.eps, _ptr(ctr), -1 if t is None else int(t),
                                              _ptr(loss_out), self.env._stream()))

    # ---- data parallel (one learner per GPU): the update split at the gradient exchange
    def grad_size(self) -> int:
        """Floats in the gradient vector of grad() / apply() (layout: grad_layout)."""
        return int(N.lib().se_qtrain_grad_size(self._h))

    def grad(self, b: MiniBatch, gamma: float, out: torch.Tensor):
        """This rank's gradient sums and {sum w d^2, sum w} into `out` (se_qtrain_grad);
        no parameter changes."""
        if out.dtype != torch.float32 or not out.is_contiguous() or out.numel() < self.grad_size():
            raise ValueError("out must be a contiguous float32 device tensor of grad_size() floats")
        N.check(N.lib().se_qtrain_grad(self._h, b.batch, _ptr(b.obs), _ptr(b.next_obs), _ptr(b.act),
                                       _ptr(b.rew), _ptr(b.done), _ptr(b.weight), float(gamma), _ptr(out),
                                       self.env._stream()))

    def apply(self, grad: torch.Tensor, step_dev: torch.Tensor, loss_out: torch.Tensor, policy=None):
        """One Adam step from `grad` summed over the ranks (se_qtrain_apply); with `policy`,
        its bf16 images are rewritten too. step_dev: Adam steps taken before this one (the
        caller advances it)."""
        if grad.dtype != torch.float32 or not grad.is_contiguous() or grad.numel() < self.grad_size():
            raise ValueError("grad must be a contiguous float32 device tensor of grad_size() floats")
        N.check(N.lib().se_qtrain_apply(self._h, None if policy is None else policy._h, _ptr(grad),
                                        self.lr, self.betas[0], self.betas[1], self.eps, _ptr(step_dev),
                                        _ptr(loss_out), self.env._stream()))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            torch.cuda.synchronize(self.env.device)
            N.lib().se_qtrain_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def grad_layout(action_size: int, in_size: int) -> dict:
    """Offsets (floats) of the data-parallel gradient vector (csrc/qtrain.h Grad): the
    six dynamic columns of dW1 ([128][6]; the port columns are db1 x port on every rank),
    db1, dW2, db2, dW3 and db3 (rows padded to a multiple of 32), then {sum w d^2, sum w}."""
    rows3 = (action_size + 31) // 32 * 32
    lay = {"w1d": 0, "b1": 768, "w2": 896, "b2": 896 + 128 * 128}
    lay["w3"] = lay["b2"] + 128
    lay["b3"] = lay["w3"] + rows3 * 128
    lay["lw"] = lay["b3"] + rows3
    lay["size"] = lay["lw"] + 2
    lay["rows3"] = rows3
    return lay


def dqn_loss(model, target_model, b: MiniBatch, gamma: float) -> torch.Tensor:
    """update()'s loss (agents/dqn.py:226-234) over the minibatch; weight-0 rows (no
    valid transition found) are left out of the mean, which is nn.MSELoss when all
    weights are 1."""
    q = model(b.obs).gather(1, b.act.unsqueeze(1)).squeeze(1)
    with torch.no_grad():
        next_q = target_model(b.next_obs).max(1)[0]
        target_q = b.rew + gamma * next_q * (1 - b.done)
    d = q - target_q
    return (b.weight * d * d).sum() / b.weight.sum().clamp_min(1.0)


class VecDQNAgent:
    """DQNAgent (agents/dqn.py:36-245) over every env of an auto-reset VecEnv."""

    def __init__(self, env, learning_rate: float = DQN_LEARNING_RATE, gamma: float = DQN_GAMMA,
                 epsilon: float = DQN_EPSILON, epsilon_min: float = DQN_EPSILON_MIN,
                 epsilon_decay: float = DQN_EPSILON_DECAY, memory_size: int | None = None,
                 batch_size: int = DQN_BATCH_SIZE, target_update_every: int = 1000,
                 hidden_size: int = HIDDEN, max_steps: int = MAX_STEPS_PER_EPISODE,
                 updates_per_step: int = 1, graph: bool | None = None, graph_warmup: int = 3,
                 fused: bool = True, model: DQNNetwork | None = None,
                 data_parallel: bool = False, process_group=None, precision: str = "bf16"):
        if not env.auto_reset:
            raise ValueError("VecDQNAgent needs an auto-reset VecEnv (finished episodes restart in se_step)")
        self.env = env
        self.state_size, self.action_size = env.obs_size, env.action_space_size
        self.gamma, self.epsilon = float(gamma), float(epsilon)
        self.epsilon_min, self.epsilon_decay = float(epsilon_min), float(epsilon_decay)
        self.learning_rate, self.batch_size = float(learning_rate), int(batch_size)
        self.target_update_every, self.max_steps = int(target_update_every), int(max_steps)
        self.updates_per_step = int(updates_per_step)
        if precision not in ("bf16", "f32"):
            raise ValueError("precision must be 'bf16' or 'f32'")
        # the acting network's precision: "f32" evaluates it in fp32 as agents/dqn.py:198-200
        # does (se_policy_f32, about 7x the policy time); the update is f32 either way
        self.precision = precision
        dev = env.device
        self.model = (model if model is not None else
                      DQNNetwork(self.state_size, self.action_size, hidden_size)).to(dev)
        self.target_model = DQNNetwork(self.state_size, self.action_size, hidden_size).to(dev)
        self.fused = bool(fused)
        self.trainer = None
        self.update_target_model()
        if self.fused:  # se_qtrain: the update on f32 MFMA, Adam state on the device
            self.trainer = FusedUpdate(env, self.model, self.target_model, self.batch_size,
                                       self.learning_rate)
            self.optimizer = None
        else:  # torch autograd + Adam (capturable: eager and graph replays run the same kernels)
            self.optimizer = torch.optim.Adam(self.model.parameters(), lr=self.learning_rate,
                                              capturable=True)
        cap = memory_size if memory_size is not None else max(DQN_MEMORY_SIZE, 4 * env.n)
        self.memory = ReplayBuffer(env, cap)
        self.policy = QPolicy(env, self.model)
        self.batch = MiniBatch(self.batch_size, self.state_size, dev)
        self.cut = torch.zeros(env.n, dtype=torch.uint8, device=dev)
        self.t = 0         # vector steps taken (policy exploration counter)
        self.updates = 0   # update() calls that trained
        # updates taken so far, twice: [0] the sampler key, [1] the fused update's Adam count
        # (se_qtrain_step_replay advances [1], then copies it into [0])
        self._ctr = torch.zeros(2, dtype=torch.int32, device=dev)
        self.use_graph = (not self.fused) if graph is None else bool(graph)
        self.graph_warmup = int(graph_warmup)
        self._graph = None
        self._loss = torch.zeros((), dtype=torch.float32, device=dev)
        # data parallel (opt-in): every rank steps its own envs into its own ring; the update
        # sums the ranks' gradients (all-reduce, RCCL) and takes the same Adam step everywhere.
        # Every rank of the group must construct its agent and update in lockstep (the
        # construction and every update issue collectives), so it is never switched on
        # implicitly: independent per-rank learners stay collective-free.
        self.group = process_group
        self.data_parallel = bool(data_parallel)
        self._grad = None
        self._graphs = None
        if self.data_parallel:
            if not self.fused:
                raise ValueError("data_parallel needs the fused update (fused=True)")
            self._grad = torch.zeros(self.trainer.grad_size(), dtype=torch.float32, device=dev)
            self._broadcast_params()

    def update_target_model(self):
        """agents/dqn.py:109-111 (an in-place copy: the graph keeps the same tensors)."""
        with torch.no_grad():
            for d, s in zip(self.target_model.parameters(), self.model.parameters()):
                d.copy_(s)
        if self.trainer is not None:
            self.trainer.pack(1)

    def _broadcast_params(self):
        """Rank 0's initial weights on every rank (DDP's start), then the kernel images.
        Every rank must hold as many envs and ring slots: the rings then fill in step, so all
        ranks begin updating (and all-reducing) at the same iteration."""
        import torch.distributed as dist

        def agree(vals):
            t = torch.tensor(vals, dtype=torch.int64, device=self.env.device)
            lo, hi = -t.clone(), t.clone()
            dist.all_reduce(lo, op=dist.ReduceOp.MAX, group=self.group)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
            return torch.equal(-lo, hi)

        if not agree([self.env.n, self.memory.capacity, self.batch_size, self.env.P]):
            raise ValueError("data-parallel ranks need the same env count, memory size, batch size "
                             "and port count")
        # the exchanged gradient leaves out dW1's port columns: every rank rebuilds them as
        # db1 x its own port block, so the ports (positions and stocks) must be the same too
        e = self.env
        if not agree([int(v) for v in (*e.port_x, *e.port_y, *e.port_fuel, *e.port_cargo)]):
            raise ValueError("data-parallel ranks need the same ports (positions and stocks)")
        src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
        with torch.no_grad():
            for p in self.model.parameters():
                dist.broadcast(p.data, src, group=self.group)
        self.update_target_model()
        self.trainer.pack(0)
        self.policy.repack()

    # ------------------------------------------------------------------ update
    def _grad_body(self):  # data parallel, before the exchange
        self.memory.sample(self.batch, t_dev=self._ctr)
        self.trainer.grad(self.batch, self.gamma, self._grad)

    def _apply_body(self):  # data parallel, after the exchange
        self.trainer.apply(self._grad, self._ctr, self._loss, self.policy)
        self._ctr.add_(1)

    def _exchange(self):
        from .dist import allreduce_gradient

        allreduce_gradient(self._grad, self.group)

    def _update_body(self):
        if self.fused:  # _ctr = Adam steps taken so far
            # the minibatch draw, the update, the policy's new images and the counter's
            # advance: two launches (the batch buffers are not written)
            # eager: the host's update count is ctr[0], so T1 need not load it first
            t = None if torch.cuda.is_current_stream_capturing() else self.updates
            self.trainer.step_replay(self.memory, self.batch_size, self.gamma, self._ctr, self._loss,
                                     self.policy, t=t)
            return
        self.memory.sample(self.batch, t_dev=self._ctr)
        loss = dqn_loss(self.model, self.target_model, self.batch, self.gamma)
        self.optimizer.zero_grad(set_to_none=False)
        loss.backward()
        self.optimizer.step()
        self._loss.copy_(loss.detach())
        # the next choose_action sees the new weights; the update counter advances in the same launch
        self.policy.repack(bump=self._ctr)
        self._ctr[1:].copy_(self._ctr[:1])

    def _capture_one(self, body):
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(self.env.device)
        side.wait_stream(torch.cuda.current_stream(self.env.device))
        with torch.cuda.stream(side), torch.cuda.graph(g, stream=side):
            body()
        torch.cuda.current_stream(self.env.device).wait_stream(side)
        return g

    def _capture(self):
        for p in self.model.parameters():  # static gradient buffers for the graph (torch path)
            if p.grad is None and not self.fused:
                p.grad = torch.zeros_like(p)
        if self.data_parallel:  # two graphs; the all-reduce runs eagerly between them
            self._graphs = (self._capture_one(self._grad_body), self._capture_one(self._apply_body))
            self._graph = self._graphs
        else:
            self._graph = self._capture_one(self._update_body)

    def update(self):
        """agents/dqn.py:206-245. Returns the loss as a device scalar (no host sync), or
        None while the memory holds fewer than batch_size transitions."""
        if self.memory.size < self.batch_size:
            return None
        if self.use_graph and self._graph is None and self.updates >= self.graph_warmup:
            self._capture()  # capturing records the update; it runs on replay below
        if self.data_parallel:
            if self._graphs is not None:
                self._graphs[0].replay()
                self._exchange()
                self._graphs[1].replay()
            else:
                self._grad_body()
                self._exchange()
                self._apply_body()
        elif self._graph is not None:
            self._graph.replay()
        else:
            self._update_body()
        self.updates += 1
        if self.epsilon > self.epsilon_min:
            self.epsilon *= self.epsilon_decay
        if self.target_update_every > 0 and self.updates % self.target_update_every == 0:
            self.update_target_model()
        return self._loss

    # ------------------------------------------------------------------ acting
    def choose_actions(self, deterministic: bool = False) -> torch.Tensor:
        """choose_action (agents/dqn.py:177-203) for every env."""
        return self.policy.act(0.0 if deterministic else self.epsilon, self.t, precision=self.precision)

    def step(self):
        """One training-loop iteration for every env; returns the last update's loss (or None)."""
        # choose_action + remember(state, action): one launch (se_policy_record)
        a = self.policy.act_record(self.memory, self.epsilon, self.t, precision=self.precision)
        # env.step, remember's reward / next_state, and the episodes that raised or reached
        # max_steps start over (env.reset(cut)): one launch (se_step_record)
        self.memory.step_end(a, self.cut, self.max_steps)
        loss = None
        for _ in range(self.updates_per_step):
            loss = self.update()
        self.t += 1
        return loss

    def train(self, steps: int):
        """`steps` vector steps; returns the final loss as a float (one sync), or None."""
        loss = None
        for _ in range(int(steps)):
            loss = self.step()
        return None if loss is None else float(loss)

    def close(self):
        for obj in (getattr(self, "policy", None), getattr(self, "memory", None),
                    getattr(self, "trainer", None)):
            if obj is not None:
                obj.close()


__all__ = ["DQNNetwork", "FusedUpdate", "MiniBatch", "ReplayBuffer", "VecDQNAgent", "dqn_loss", "grad_layout"]
