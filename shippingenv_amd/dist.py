"""One process per GPU: environment sharding and the episode-statistics all-reduce.

Envs are independent (no env reads another's state; the map and ports are
read-only, shipping/environment.py:345,354 never decrement port stocks), so the
path shards with no data-path collective: rank r owns global env ids
[r*n, (r+1)*n). Every random draw is keyed by (seed, global env id), so a
shard's trajectories are identical to the same ids in a single-GPU run
(tests/test_gpu_parity.py::test_shard_invariance). The one collective is a
SUM all-reduce of three doubles {sum of returns, episodes, sum of lengths}
(backend "nccl", which is RCCL on ROCm): latency-bound, off the step path.
Data-parallel DQN training (shippingenv_amd.dqn.VecDQNAgent with several ranks) adds the
one exchange its update has: a SUM all-reduce of the gradient vector per update.
"""
from __future__ import annotations

import os

import torch

STATS_FIELDS = ("sum_return", "episodes", "sum_len")


def shard_bounds(n_global, world, rank):
    """Contiguous shard of rank `rank`: (first global id, count). Shard starts are
    multiples of 4 because envs 4k..4k+3 share their Philox draw blocks."""
    if n_global % (4 * world):
        raise ValueError("n_global must be a multiple of 4 * world_size")
    per = n_global // world
    return rank * per, per


def init_from_env(backend=None, gpu=None):
    """Initialise torch.distributed from RANK / WORLD_SIZE / LOCAL_RANK (as torchrun sets
    them; MASTER_ADDR defaults to 127.0.0.1) or run single-process. One process per GPU:
    local rank r drives GPU r, unless `gpu` names the device (a caller rehearsing several
    ranks on fewer GPUs passes it, with backend "gloo": RCCL refuses two ranks on one GPU).
    Backend: "nccl" (RCCL) on GPUs, "gloo" on CPU, unless given. Returns (rank, world,
    local_rank, device)."""
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        dev = local if gpu is None else int(gpu)
        if not 0 <= dev < torch.cuda.device_count():
            raise RuntimeError(f"local rank {local} has no GPU (device {dev} of {torch.cuda.device_count()})")
        torch.cuda.set_device(dev)
        device = torch.device("cuda", dev)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if device.type == "cuda" else "gloo"
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return rank, world, local, device


def reduce_episode_stats(stats, group=None):
    """SUM-all-reduce a f64[3] {sum_return, episodes, sum_len} tensor in place."""
    import torch.distributed as dist

    if stats.dtype != torch.float64 or stats.numel() != 3:
        raise ValueError("episode stats are a float64 tensor of 3 entries")
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.SUM, group=group)
    return stats


def allreduce_gradient(grad, group=None):
    """SUM-all-reduce a data-parallel DQN gradient vector in place (se_qtrain_grad's sums
    and {sum w d^2, sum w}; shippingenv_amd.dqn.grad_layout). Summing, not averaging: the
    update divides by the global weight sum, so ranks may hold different numbers of valid
    transitions. One 200-odd-KB message per update: on xGMI that is latency, not link
    bandwidth."""
    import torch.distributed as dist

    if grad.dtype != torch.float32 or grad.dim() != 1:
        raise ValueError("the gradient vector is a 1-D float32 tensor")
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return grad


def summarize(stats):
    s = [float(v) for v in stats.tolist()]
    eps = s[1]
    return {"episodes": eps, "mean_return": s[0] / eps if eps else None,
            "mean_len": s[2] / eps if eps else None}


class ShardedVecEnv:
    """This rank's shard of a multi-GPU environment set (a VecEnv with global ids)."""

    def __init__(self, n_per_rank, gpu=None, backend=None, **kw):
        from .vec import VecEnv

        self.rank, self.world, self.local, self.device = init_from_env(backend, gpu)
        first, count = shard_bounds(n_per_rank * self.world, self.world, self.rank)
        self.first = first
        self.env = VecEnv(count, env_id_base=first, device=self.device, **kw)

    def __getattr__(self, name):
        env = self.__dict__.get("env")  # absent if VecEnv construction failed in __init__
        if name == "env" or env is None:
            raise AttributeError(name)
        return getattr(env, name)

    def global_episode_stats(self):
        return reduce_episode_stats(self.env.episode_stats().clone())
