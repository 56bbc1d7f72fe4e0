"""Benchmark: batched ShippingEnv step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n ENVS_PER_GPU]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py launches its own N
ranks (spawn_ranks: N fresh child processes, one per GPU, RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set; the parent makes no GPU call), forwards rank 0's line and
exits non-zero if any rank fails. Under torchrun the ranks are torchrun's.

A "step" is one se_step launch over all envs of the GPU (one pass of the hot
path over one batch). Workload for `value`: BASELINE config 3 — N = 2^20 envs
per GPU, full step (moves, cargo pickup/delivery, rewards), the reference's 5
default ports, synthetic agent actions (90 % move, 5 % take cargo, 3 % take
fuel, 2 % select; Philox-generated, resident in HBM before timing). Config 4
(64 random ports, auto-reset with ballot-compacted done list and per-wave
episode-return reduction, RCCL all-reduce of the stats) is measured in the same
run and reported under "config4". Weak scaling: every rank owns 2^20 envs with
global ids rank*2^20 + i.

Rank 0 prints ONE JSON line on stdout; progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

# algorithmic bytes per env-step for this build's field widths (DESIGN.md "Roofline"):
#   state x,y,origin,dest u8 + cargo i32 + fuel f64 = 16 B, read and written;
#   action i32 4 B read; reward f32 4 B, done u8 1 B, err i8 1 B written.
BYTES_STEP = 16 + 16 + 4 + 4 + 1 + 1  # 42
# + ep_return f32, read and written. Since round 5 the running length is an episode-start
# stamp (se_state.ep_start) read and written only for the ~1 in 240 envs that finish, like
# the done-list records (excluded); it was ep_len i32 read and written per env (58 B).
BYTES_STEP_AUTO = BYTES_STEP + 4 + 4  # 50
# the survey's canonical widths (x, y, origin, dest, cargo i32; fuel f64): 66 / 82 B
CANONICAL_STEP, CANONICAL_STEP_AUTO = 66, 82


LITERAL_STEPS, LITERAL_WARMUP = 1000, 10  # "Warm-up 10 steps, time 1000 steps"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--n", type=int, default=1 << 20, help="envs per GPU")
    p.add_argument("--seed", type=int, default=2026)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-config4", action="store_true")
    p.add_argument("--preroll3", type=int, default=1000,
                   help="config 3 workload setup: untimed steps from reset to the steady state mix the "
                        "survey's 1000-step definition measures; 0 = time from reset (the from-reset "
                        "figure is reported beside it either way)")
    p.add_argument("--preroll4", type=int, default=1000,
                   help="config 4 workload setup: untimed steps from reset to the steady episode mix "
                        "(episodes of ~240 steps end in every step), before the warm-up")
    p.add_argument("--large-n", type=int, default=1 << 24,
                   help="extra HBM-resident run (working set beyond the 256 MiB MALL); 0 = skip")
    p.add_argument("--dqn-steps", type=int, default=50,
                   help="config 5: timed DQN policy + step iterations at N envs/GPU (fp32 policy, then "
                        "bf16); 0 = skip")
    p.add_argument("--preroll5", type=int, default=300,
                   help="config 5: untimed policy + step iterations from reset (eps 1.0) before the legs")
    p.add_argument("--train-steps", type=int, default=30,
                   help="timed vectorised DQN training iterations (policy, step, replay, update); 0 = skip")
    p.add_argument("--train-batch", type=int, default=8192, help="DQN minibatch per update")
    p.add_argument("--config1", type=int, default=1, help="time BASELINE configs[0] (N = 1 drop-in API); 0 = skip")
    p.add_argument("--rollouts", type=int, default=20,
                   help="timed se_rollout launches (MCTS random rollouts, 2^20 x 100 steps); 0 = skip")
    return p.parse_args()


REHEARSAL_ENV = "SHIPENV_REHEARSE"  # "1": every rank on GPU 0 over gloo (launch rehearsal, never a measurement)


class Dist:
    """torch.distributed glue (shippingenv_amd.dist): barrier, max over ranks, stats all-reduce.
    Backend "nccl" (RCCL) with local rank r on GPU r. SHIPENV_REHEARSE=1 rehearses the N-rank
    launch on a box with fewer GPUs: every rank on GPU r % device_count over gloo (RCCL refuses
    two ranks on one GPU); the line then says "rehearsal" in its dist object."""

    def __init__(self, want):
        from shippingenv_amd import dist as D

        self.D = D
        self.rehearsal = os.environ.get(REHEARSAL_ENV) == "1"
        gpu, backend = None, None
        if self.rehearsal and torch.cuda.is_available():
            gpu = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
            backend = "gloo"
        self.rank, self.world, self.local, self.dev = D.init_from_env(backend, gpu)
        if self.world != want:
            raise SystemExit(f"--gpus {want} but WORLD_SIZE={self.world}")
        import torch.distributed as tdist

        self.pg = tdist if self.world > 1 else None
        self.info = {"world_size": tdist.get_world_size() if self.pg else 1,
                     "backend": tdist.get_backend() if self.pg else None,
                     "device": str(self.dev),
                     "launcher": os.environ.get("SHIPENV_LAUNCHER", "torchrun" if self.world > 1 else None)}
        if self.rehearsal:
            self.info["rehearsal"] = "all ranks on one GPU over gloo: a launch rehearsal, not scaling data"

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def max(self, v):
        if not self.pg:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.dev)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


def spawn_ranks(n, argv, script=None, env=None, grace_s=30.0):
    """Run `script argv` as N fresh processes, rank r with RANK = LOCAL_RANK = r (GPU r),
    WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free MASTER_PORT, as torchrun would. The
    parent makes no GPU or HIP call (it only imports torch, which initialises nothing).
    Rank 0's JSON line is forwarded to stdout (its other stdout lines to stderr); every
    rank's stderr is inherited. If a rank exits non-zero the others get `grace_s` seconds, then SIGTERM
    (SIGKILL 10 s later): a rank left waiting in a collective for a dead peer would hang.
    Returns 0 if every rank succeeded, else the first non-zero exit status (1 for a signal)."""
    import socket
    import subprocess
    import tempfile

    script = os.path.abspath(script or __file__)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), SHIPENV_LAUNCHER="bench.spawn_ranks")
    out0 = tempfile.TemporaryFile(mode="w+b")
    procs = []
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
            procs.append(subprocess.Popen([sys.executable, script, *argv], env=e,
                                          stdout=out0 if r == 0 else subprocess.DEVNULL))
        first_bad, t_bad = None, None
        while True:
            codes = [p.poll() for p in procs]
            for r, c in enumerate(codes):
                if c not in (None, 0) and first_bad is None:
                    first_bad, t_bad = (r, c), time.monotonic()
                    log(f"[launcher] rank {r} exited with status {c}")
            if all(c is not None for c in codes):
                break
            if first_bad is not None and time.monotonic() - t_bad > grace_s:
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                for p in procs:
                    try:
                        p.wait(10)
                    except subprocess.TimeoutExpired:
                        p.kill()
                break
            time.sleep(0.05)
    finally:
        for p in procs:  # an exception or signal in the parent: no orphaned ranks
            if p.poll() is None:
                p.kill()
                p.wait()
    codes = [p.returncode for p in procs]
    bad = [c for c in codes if c != 0]
    if bad:
        log(f"[launcher] rank exit statuses {codes}")
        c = first_bad[1] if first_bad else bad[0]
        return c if c > 0 else 1
    out0.seek(0)
    # the driver reads one JSON line: rank 0's other stdout text (a library's own chatter,
    # e.g. gloo's "[Gloo] Rank 0 is connected to ...") goes to stderr
    for line in out0.read().decode().splitlines(keepends=True):
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
    sys.stdout.flush()
    return 0


def make_actions(env, steps):
    acts = torch.empty((steps, env.n), dtype=torch.int32, device=env.device)
    for t in range(steps):
        env.gen_actions(t, out=acts[t])
    return acts


def timed_loop(env, acts, first, steps, dist, reduce_every=0, counter=None, step_seq=False):
    """K back-to-back launches bracketed by barrier + synchronize on both sides; wall
    time is the max over ranks. Two HIP events on the launch stream give the GPU time per
    launch (roofline.kernel_ms): one right before launch 1, one after launch K, over K
    launches. The first is taken by the GPU when it reaches it, so the ~20 us that launch 1's
    command takes to reach an idle queue ("The short run") is not in it;
    the few microseconds between the event and launch 1's dispatch are (a conservative
    basis: the kernel time it gives is at most the trace's launch average plus those).

    One VecEnv.step call per step, the drop-in's per-step API; step_seq=True issues the
    same launches with VecEnv.step_seq (se_step_seq_mark: the launch loop in native code,
    which records the launch-1 event itself, split only where a stats all-reduce goes
    between two steps). On a box whose Python issue rate is slower than an 8 us kernel
    (BENCH r04a: step_py 10.5 us per launch by events) only step_seq keeps the queue full."""
    stream = torch.cuda.current_stream(env.device)
    ef, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(2))
    for e in (ef, e1):  # the HIP events exist before the clock starts (torch creates them lazily)
        e.record(stream)
    # the step's action rows as views made before the clock starts: indexing the
    # [steps, n] table inside the loop is harness work (1.4 us of host time per step,
    # tools/archive/diag/host_step_cost.py), not the step's
    if not step_seq:
        chunks = [acts[first + k] for k in range(steps)]
    else:  # runs that end where an all-reduce follows; the first run records ef right before
        # its launch 1 from native code (se_step_seq_mark, mark_after = 0): splitting the run
        # after launch 1 for a Python record cost ~0.7 us per step over the driver's 20, and a
        # native record there 0.2-0.4 (tools/archive/diag/wall_forms.py, profiles/r04/wall_forms*)
        cuts = sorted({0, steps} | ({k for k in range(reduce_every, steps, reduce_every)}
                                    if reduce_every else set()))
        chunks = [acts[first + a:first + b] for a, b in zip(cuts, cuts[1:])]
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = 0
    for c in chunks:
        if step_seq:
            if done == 0:
                env.step_seq(c, mark=ef, mark_after=0)
            else:
                env.step_seq(c)
            done += c.shape[0]
        else:
            if done == 0:
                ef.record(stream)
            env.step(c)
            done += 1
        if reduce_every and done % reduce_every == 0:
            # episode-return aggregation over the GPUs (RCCL all-reduce of 3 doubles), in
            # place in the env's stats buffer: a torch copy_ of the 24 bytes first went
            # through a blit whose host side stalled the queue ~40 us (kernel trace r03)
            dist.D.reduce_episode_stats(env.episode_stats())
            if counter is not None:
                counter[0] += 1
    e1.record(stream)
    torch.cuda.synchronize()
    dist.barrier()
    wall = dist.max(time.perf_counter() - t0)
    k_ms = ef.elapsed_time(e1) / steps
    return wall, k_ms


def run_config(n, ports, auto, args, dist, label, preroll=0, step_seq=False):
    """One leg: reset, `preroll` untimed steps of workload setup (actions generated one row
    at a time), W warm-up steps, then the K timed steps from rows resident in HBM.
    Auto-reset legs all-reduce the episode statistics (RCCL) every min(100, K // 2) steps
    inside the timed region; the count is returned in `info`."""
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(n, seed=args.seed, ports=ports, env_id_base=dist.rank * n, device=dist.dev,
                 auto_reset=auto)
    total = args.warmup + args.steps
    log(f"[{label}] rank {dist.rank}: n={n} P={env.P} auto_reset={auto}; pre-roll {preroll}, "
        f"generating {total} action rows")
    acts = make_actions(env, total)
    env.reset()
    if preroll:
        row = torch.empty(n, dtype=torch.int32, device=env.device)
        for t in range(preroll):  # action rows of their own (t offset past the timed rows)
            env.step(env.gen_actions(1_000_000 + t, out=row))
    for k in range(args.warmup):  # the timed leg's own issue path (and kernel) warmed up
        if step_seq:
            env.step_seq(acts[k:k + 1])
        else:
            env.step(acts[k])
    if auto:  # the stats path runs inside the timed region: load its kernels now
        dist.D.reduce_episode_stats(env.episode_stats().clone())
    torch.cuda.synchronize()
    if auto:
        env.clear_stats()
    every = max(1, min(100, args.steps // 2)) if auto else 0
    count = [0]
    wall, k_ms = timed_loop(env, acts, args.warmup, args.steps, dist, reduce_every=every, counter=count,
                            step_seq=step_seq)
    stats = None
    if auto:
        s = env.episode_stats().clone()
        dist.D.reduce_episode_stats(s)
        stats = s.cpu().tolist()
    env.close()
    del acts
    torch.cuda.empty_cache()
    # allreduces_in_timed_region counts the reduce_episode_stats calls; collectives_in_timed_region
    # the RCCL all-reduces they issued (none at world size 1, dist.reduce_episode_stats)
    info = {"preroll_steps": preroll, "allreduce_every": every, "allreduces_in_timed_region": count[0],
            "collectives_in_timed_region": count[0] if dist.world > 1 else 0,
            "collective_backend": dist.info.get("backend") if dist.world > 1 else None}
    return wall, k_ms, stats, info


def run_config1(args):
    """BASELINE configs[0]: one env, 100 steps through the drop-in shipping.Environment, as
    the survey timed the reference: random.seed(0), the five DEFAULT_PORTS,
    moves uniform over N, E, S, W from random.Random(1), reset on done; median of 10 runs.
    Timed on the drop-in's default stepper (the step kernels' per-env code compiled for the
    host: one C call per step), on SHIPENV_STEPPER=gpu (the resident stepper wave: one mailbox
    command per step, csrc/server.h) and on SHIPENV_STEPPER=gpu with SHIPENV_GPU_SERVER=0 (one
    launch and one stream synchronise per step)."""
    import random
    import statistics

    from shippingenv_amd.shipping import ShipMove, environment

    ports = [[41, 40], [60, 22], [78, 29], [49, 72], [62, 72]]  # utils/constants.py:57-63
    moves = [ShipMove.NORTH, ShipMove.EAST, ShipMove.SOUTH, ShipMove.WEST]

    def once():
        random.seed(0)
        env = environment.Environment("mapa_mundi_binario.jpg")
        for p in ports:
            env.add_port(list(p))
        env.reset()
        pick = random.Random(1)
        t0 = time.perf_counter()
        for _ in range(100):
            try:
                _, _, done, _ = env.step([environment.ActionType.MOVE_SHIP, moves[pick.randrange(4)]])
            except ValueError:  # "Move is out of range" (:284)
                continue
            if done:
                env.reset()
        return (time.perf_counter() - t0) * 1e3

    ms = {}
    prev = {k: os.environ.get(k) for k in ("SHIPENV_STEPPER", "SHIPENV_GPU_SERVER")}
    try:
        for kind, server in (("host", "1"), ("gpu", "1"), ("gpu_launch", "0")):
            os.environ["SHIPENV_STEPPER"] = kind.split("_")[0]
            os.environ["SHIPENV_GPU_SERVER"] = server
            once()
            ms[kind] = statistics.median(once() for _ in range(10))
    finally:
        for k, v in prev.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return {"workload": "BASELINE configs[0]: 1 env x 100 steps through shipping.Environment "
                        "(the reference's API) on its default host stepper",
            "ms_per_100_steps": round(ms["host"], 4),
            "ms_per_100_steps_gpu_stepper": round(ms["gpu"], 4),
            "ms_per_100_steps_gpu_launch_per_step": round(ms["gpu_launch"], 4),
            "gpu_stepper_note": "SHIPENV_STEPPER=gpu: the resident stepper wave (se_server_call, csrc/server.h); "
                                "gpu_launch_per_step: SHIPENV_GPU_SERVER=0, one se_step_replay launch + synchronise",
            "reference_python_ms_per_100_steps": 0.98,
            "reference_note": "survey container, 1 core (BASELINE.md); the reference cannot run on the GPU box. "
                              "Same-host comparison in the build container: profiles/r03/config1_vs_reference.json"}


def run_rollouts(n, args, dist):
    """MCTS random rollouts (agents/mcts.py:211-238, se_rollout): one rollout of up to
    100 counted steps from each of the n envs of the config-3 set, after 50 policy
    steps; rollout ids are fresh per launch. Rate = counted env-steps / time."""
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(n, seed=args.seed, env_id_base=dist.rank * n, device=dist.dev)
    env.reset()
    for t in range(50):
        env.step(env.gen_actions(t))
    src = torch.arange(n, dtype=torch.int32, device=env.device)
    for k in range(2):  # warm (and load the reduction kernel used after timing)
        _, steps, _ = env.rollout(src, max_steps=100, rollout_base=(dist.rank * 1000 + k) * n)
        int(steps.sum().item())
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(env.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kept = []  # counted steps per launch, summed after the timed region
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for k in range(args.rollouts):
        kept.append(env.rollout(src, max_steps=100, rollout_base=(dist.rank * 1000 + 2 + k) * n)[1])
    e1.record(stream)
    torch.cuda.synchronize()
    dist.barrier()
    wall = dist.max(time.perf_counter() - t0)
    total = float(sum(int(s.sum().item()) for s in kept))
    env.close()
    k_ms = e0.elapsed_time(e1) / args.rollouts
    steps_launch = total / args.rollouts
    achieved = ROLLOUT_VALU_PER_STEP * steps_launch / (k_ms * 1e-3) / 1e9
    return {
        "workload": "se_rollout: 2^20 rollouts/GPU from config-3 states, max 100 counted steps "
                    "(sample_action + step, retries uncounted), Philox per rollout",
        "launches": args.rollouts,
        "value": round(total * dist.world / wall, 1),
        "unit": "rollout env-steps/s",
        "ms_per_launch": round(wall / args.rollouts * 1e3, 4),
        "kernel_ms": round(k_ms, 4),
        "mean_steps_per_rollout": round(total / (args.rollouts * n), 2),
        # rollout_kernel is bound by instruction issue (one rollout per lane: Philox draws,
        # sample_action and the step's select chain; 20 VGPRs, no HBM stream to speak of):
        # achieved = the VALU wave instructions per counted step of the committed PMC pass
        # (profiles/r06/rollout/summary.json, SQ_INSTS_VALU / counted steps) x this launch's
        # counted steps / its time, against one wave64 VALU instruction per 2 cycles per SIMD
        "roofline": {"bound": "valu-issue", "achieved": round(achieved, 1), "peak": VALU_ISSUE_PEAK_G,
                     "unit": "G wave-instr/s", "frac": round(achieved / VALU_ISSUE_PEAK_G, 4), "traffic": None,
                     "valu_wave_instr_per_step": ROLLOUT_VALU_PER_STEP,
                     "source": "profiles/r06/rollout/summary.json (SQ counters, kernel trace)"},
    }


ROLLOUT_VALU_PER_STEP = 2.9451  # SQ_INSTS_VALU per counted env-step, profiles/r06/rollout/summary.json
VALU_ISSUE_PEAK_G = 1024 * 2.4 / 2  # 1024 SIMDs x 2.4 GHz, one wave64 VALU per 2 cycles (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TFLOPS = 157.3  # v_mfma_f32_32x32x2_f32, MI355X_MICROARCH.md
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, no sparsity)


def policy_step_loop(env, pol, prec, eps, t0_key, steps, dist, every):
    """`steps` iterations of policy + step (the config-5 consumer loop), bracketed by barrier +
    synchronize, with the episode-statistics all-reduce every `every` steps inside the region.
    Returns (wall max over ranks, events ms per iteration, all-reduces)."""
    stream = torch.cuda.current_stream(env.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    count = 0
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for k in range(steps):
        env.step(pol.act(eps, t0_key + k, precision=prec))
        if every and (k + 1) % every == 0:
            dist.D.reduce_episode_stats(env.episode_stats())
            count += 1
    e1.record(stream)
    torch.cuda.synchronize()
    dist.barrier()
    wall = dist.max(time.perf_counter() - t0)
    return wall, e0.elapsed_time(e1) / steps, count


def run_config5(n, args, dist):
    """BASELINE configs[4] / SURVEY 8(d) config 5: N envs per GPU (global ids rank*N + i),
    auto-reset on done (default 5 ports), the DQN rollout consumer (agents/dqn.py:177-204:
    DQNNetwork 26->128->128->259 forward + the first maximum over the valid actions +
    epsilon-greedy, fused in se_policy_f32 / se_policy) then se_step, and the RCCL SUM
    all-reduce of {sum of returns, episodes, sum of lengths} every min(100, K // 2) steps
    inside the timed region. `value` evaluates the network in fp32, the reference's own
    precision (se_policy_f32, split-bf16 MFMA); the bf16 policy's figure is beside it. Also: the
    env kernel alone (se_step over the same auto-reset shard) and the unfused torch policy."""
    from shippingenv_amd.policy import DQNNetwork, QPolicy
    from shippingenv_amd.vec import VecEnv

    K = args.dqn_steps
    env = VecEnv(n, seed=args.seed, env_id_base=dist.rank * n, device=dist.dev, auto_reset=True)
    env.reset()
    torch.manual_seed(args.seed)
    model = DQNNetwork(env.obs_size, env.action_space_size).to(env.device)
    pol = QPolicy(env, model)
    eps = 0.1
    every = max(1, min(100, K // 2))
    stream = torch.cuda.current_stream(env.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # pre-roll at the agent's initial exploration rate (DQN_EPSILON = 1.0,
    # utils/constants.py:33): random valid actions take the ships out of their origin ports.
    # A random-init network's greedy choice at a port is almost never a move (4 of ~250
    # valid actions), so from reset at eps 0.1 no ship leaves port and no episode ends in
    # the timed steps (BENCH r04a: 0 episodes). After it, ships at sea move greedily, burn
    # fuel and finish episodes, so the all-reduced returns are the consumer's real ones.
    for t in range(args.preroll5):
        env.step(pol.act(1.0, 200_000 + t))
    legs = {}
    for i, prec in enumerate(("f32", "bf16")):
        for t in range(5):  # warm-up: both kernels and the stats path loaded
            env.step(pol.act(eps, 100_000 * i + t, precision=prec))
        dist.D.reduce_episode_stats(env.episode_stats().clone())
        torch.cuda.synchronize()
        env.clear_stats()
        wall, e2e_ms, count = policy_step_loop(env, pol, prec, eps, 100_000 * i + 5, K, dist, every)
        s = env.episode_stats().clone()
        dist.D.reduce_episode_stats(s)
        st = s.cpu().tolist()
        # the policy launch alone on the state the loop left (fresh draws)
        e0.record(stream)
        for t in range(K):
            pol.act(eps, 500_000 + 100_000 * i + t, precision=prec)
        e1.record(stream)
        torch.cuda.synchronize()
        legs[prec] = {"value": round(n * dist.world * K / wall, 1),
                      "ms_per_step": round(wall / K * 1e3, 4),
                      "e2e_kernel_ms": round(e2e_ms, 4),
                      "policy_ms": round(e0.elapsed_time(e1) / K, 4),
                      "allreduces_in_timed_region": count,
                      "collectives_in_timed_region": count if dist.world > 1 else 0,
                      "episodes": st[1],
                      "mean_return": st[0] / st[1] if st[1] else None}
    # the env kernel alone: se_step over the same shard, the policy's last actions each step
    acts = pol.act(0.0, 999_999).clone()
    for _ in range(3):
        env.step(acts)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(K):
        env.step(acts)
    e1.record(stream)
    torch.cuda.synchronize()
    step_ms = e0.elapsed_time(e1) / K
    # unfused torch reference path, fp32 as agents/dqn.py runs it (a few iterations)
    A = env.action_space_size
    shifts = torch.arange(7, -1, -1, device=env.device, dtype=torch.uint8)

    def torch_policy():
        with torch.no_grad():
            q = model(env.observe())
            bits = ((env.valid_mask().unsqueeze(-1) >> shifts) & 1).flatten(1)[:, :A].bool()
            return q.masked_fill(~bits, float("-inf")).argmax(1).to(torch.int32)

    torch_policy()
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(5):
        torch_policy()
    e1.record(stream)
    torch.cuda.synchronize()
    torch_ms = e0.elapsed_time(e1) / 5
    # greedy decisions of both modes against fp32 torch on these states
    # (agents/dqn.py:198-204: the first maximum of the fp32 network's Q over the valid actions)
    a16 = pol.act(0.0, 3000).clone()
    a32 = pol.act(0.0, 3000, precision="f32").clone()
    mask = env.valid_mask()
    dis16 = dis32 = 0
    with torch.no_grad():
        obs_all = env.observe()
        for i in range(0, n, 1 << 17):
            q = model(obs_all[i:i + (1 << 17)])
            bits = ((mask[i:i + (1 << 17)].unsqueeze(-1) >> shifts) & 1).flatten(1)[:, :A].bool()
            ref = q.masked_fill(~bits, float("-inf")).argmax(1).to(torch.int32)
            dis16 += int((a16[i:i + (1 << 17)] != ref).sum())
            dis32 += int((a32[i:i + (1 << 17)] != ref).sum())
    del obs_all, mask
    # FLOPs per env the kernels' algorithm evaluates: fc1 over the 6 dynamic inputs (the
    # constant port block is folded into the bias), fc2, and fc3 over the compact rows (the
    # actions some env can ever take, in 32-row tiles). The reference network's
    # count (all A rows, all 6 + 4P inputs) is reported beside it as a count, not a rate.
    cmax = min(max(int(v) for v in env.port_cargo), 49)
    fmax = min(max(int(v) for v in env.port_fuel), 199)
    rows3 = 32 * ((4 + env.P + cmax + fmax + 31) // 32)
    flop_env = 2 * (6 * 128 + 128 * 128 + rows3 * 128)
    flop_ref = 2 * (env.obs_size * 128 + 128 * 128 + 128 * A)  # the reference network's MACs x 2
    # the MFMA FLOPs se_policy_f32 executes per env: fc2 and fc3 six bf16 products each, fc1 two
    # split-bf16 32x32x16 MFMAs per row tile (x3_fc1_slot: 24 of their 32 k slots used)
    x3_flop_env = 6 * 2 * (128 * 128 + rows3 * 128) + 4 * 2 * (32 * 32 * 16 * 2) // 32
    pol32_ms, pol_ms = legs["f32"]["policy_ms"], legs["bf16"]["policy_ms"]
    achieved32 = flop_env * n / (pol32_ms * 1e-3) / 1e12
    achieved = flop_env * n / (pol_ms * 1e-3) / 1e12
    # what the kernel issues per 32 envs at most: fc1 (the port block folded into the bias,
    # one k-step per row tile), fc2, and fc3 over the compact rows
    mfma_tile = 4 + 32 + 8 * ((4 + env.P + cmax + fmax + 31) // 32)
    pol.close()
    env.close()
    f32 = legs["f32"]
    return {
        "workload": "BASELINE configs[4]: N envs/GPU (global ids rank*N + i), auto-reset, default 5 ports; "
                    "per step the fused DQN policy (obs + DQNNetwork 26->128->128->259 + masked first argmax "
                    "+ eps-greedy 0.1; fp32 by 3-way bf16 splits on bf16 MFMA, se_policy_f32) then se_step; RCCL SUM all-reduce "
                    "of {sum return, episodes, sum len} every min(100, K // 2) steps in the timed region; "
                    "random-init weights; untimed pre-roll of preroll_steps policy steps from reset at "
                    "eps 1.0 (the agent's initial exploration rate). "
                    "bf16: the same loop on the bf16 policy (se_policy)",
        "value": f32["value"],
        "unit": "env-steps/s (policy + step, end to end)",
        "precision": "fp32 (the reference's network precision, agents/dqn.py:198-204)",
        "n_gpus": dist.world,
        "global_envs": n * dist.world,
        "steps": K,
        "ms_per_step": f32["ms_per_step"],
        "e2e_kernel_ms": f32["e2e_kernel_ms"],
        "policy_ms": f32["policy_ms"],
        "preroll_steps": args.preroll5,
        "allreduce_every": every,
        "allreduces_in_timed_region": f32["allreduces_in_timed_region"],
        "collectives_in_timed_region": f32["collectives_in_timed_region"],
        "episodes": f32["episodes"],
        "mean_return": f32["mean_return"],
        "env_kernel": {"value": round(n * dist.world / (step_ms * 1e-3), 1), "kernel_ms": round(step_ms, 5),
                       "unit": "env-steps/s (se_step alone, auto-reset shard, events)"},
        "bf16": legs["bf16"],
        "greedy_disagreement_vs_fp32_torch": {"bf16": round(dis16 / n, 5), "f32": round(dis32 / n, 6),
                                              "states": n,
                                              "note": "greedy actions on the config-5 states vs the first "
                                                      "masked argmax of the fp32 torch DQNNetwork"},
        "torch_unfused_policy_ms": round(torch_ms, 4),
        # se_policy_f32 (round 5) evaluates the fp32 network on bf16 MFMA with 3-way operand
        # splits: six bf16 products per f32 product for fc2 and fc3, fc1 as two split-bf16 MFMAs
        # per row tile (qpolicy.h policy_x3_kernel, x3_fc1_slot). Its roofline is the bf16 MFMA peak over the MFMA FLOPs
        # the fp32-faithful algorithm executes; the f32-equivalent rate (the network's own
        # FLOPs) is beside it against the f32 MFMA peak, which the split datapath exceeds.
        "roofline": {"bound": "mfma (bf16, fp32 by 3-way operand splits)",
                     "achieved": round(x3_flop_env * n / (pol32_ms * 1e-3) / 1e12, 1),
                     "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(x3_flop_env * n / (pol32_ms * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS, 4),
                     "flop_per_env": x3_flop_env, "traffic": None,
                     "f32_equivalent": {"achieved": round(achieved32, 2), "peak": F32_MFMA_PEAK_TFLOPS,
                                        "frac": round(achieved32 / F32_MFMA_PEAK_TFLOPS, 4),
                                        "flop_per_env": flop_env},
                     "reference_network_flop_per_env": flop_ref,
                     "note": "se_policy_f32 (includes its per-call repack of the split image); flop_per_env = "
                             "6 x (fc2 + fc3 over its 32-row tiles) bf16 MFMA FLOPs + fc1's 8 split-bf16 MFMAs per 32 envs; "
                             "f32_equivalent: the FLOPs the fused step evaluates (fc1's 6 dynamic inputs, fc2, "
                             "fc3's compact rows) against the f32 MFMA peak",
                     # the policy-alone launches (policy_ms's basis) in the committed kernel trace
                     "committed_trace": committed_trace("config5_policy_f32_alone")},
        "roofline_bf16": {"bound": "mfma", "achieved": round(achieved, 1), "peak": BF16_DENSE_PEAK_TFLOPS,
                          "unit": "TFLOP/s", "frac": round(achieved / BF16_DENSE_PEAK_TFLOPS, 4),
                          "flop_per_env": flop_env, "traffic": None,
                          "executed_mfma_per_32_envs": mfma_tile,
                          "note": "at most executed_mfma_per_32_envs v_mfma_f32_32x32x16_bf16 per 32 envs "
                                  "(fc1 pads K to 16)",
                          "committed_trace": committed_trace("config5_policy_bf16_alone")},
    }


def run_dqn_train(n, args, dist):
    """the vectorised DQN training loop (shippingenv_amd.dqn.VecDQNAgent).
    One iteration for all N envs: fused policy + replay begin, se_step (auto-reset) +
    replay end, cut and reset of the cut envs, then one update: two launches
    (se_qtrain_step_replay) for the minibatch draw from the ring, DQNNetwork forward and
    backward at batch B, Adam, and the policy repack. Random-init weights; the reference's hyperparameters
    (gamma 0.95, lr 1e-3, epsilon decay 0.995), with B = --train-batch per GPU.
    Several GPUs: data parallel, one learner per rank on its own envs and ring; each
    update is the sampler + the gradient sums, a SUM all-reduce of the gradient vector
    (RCCL), then Adam + the policy images, so the global minibatch is B x ranks."""
    from shippingenv_amd.dqn import VecDQNAgent
    from shippingenv_amd.vec import VecEnv

    env = VecEnv(n, seed=args.seed, env_id_base=dist.rank * n, device=dist.dev, auto_reset=True)
    env.reset()
    torch.manual_seed(args.seed)
    agent = VecDQNAgent(env, batch_size=args.train_batch, memory_size=4 * n,
                        data_parallel=dist.world > 1)
    for _ in range(6):  # warm-up iterations
        agent.step()
    stream = torch.cuda.current_stream(env.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.train_steps):
        loss = agent.step()
    e1.record(stream)
    torch.cuda.synchronize()
    dist.barrier()
    wall = dist.max(time.perf_counter() - t0)
    kern_ms = e0.elapsed_time(e1) / args.train_steps
    e0.record(stream)
    for _ in range(args.train_steps):
        agent.update()
    e1.record(stream)
    torch.cuda.synchronize()
    upd_ms = e0.elapsed_time(e1) / args.train_steps
    # algorithmic f32 FLOPs of one fused update per sample (csrc/qtrain.h): online fc1 (6
    # dynamic inputs; the constant port block is folded), fc2, the gathered q; target fc1,
    # fc2, fc3 over all A rows; backward dH2 and dW3 (row gathers), dW2, dH1 and dW1 (6 cols)
    H, Aa = 128, env.action_space_size
    flop = 2 * (6 * H + H * H + H) + 2 * (6 * H + H * H + H * Aa) + 2 * (2 * H + 2 * H * H + 6 * H)
    upd_tf = flop * args.train_batch / (upd_ms * 1e-3) / 1e12
    out = {
        "workload": "8f row 3: vectorised DQN training, N envs/GPU (auto-reset, default ports): "
                    "fused policy + se_step + device replay ring + one two-launch update "
                    f"(B = {args.train_batch}) per iteration; random-init weights",
        "value": round(n * dist.world * args.train_steps / wall, 1),
        "unit": "env-steps/s (training loop)",
        "ms_per_step": round(wall / args.train_steps * 1e3, 4),
        "stream_ms_per_step": round(kern_ms, 4),
        "update_ms": round(upd_ms, 4),
        "updates_per_s": round(1e3 / upd_ms, 1),
        "update_roofline": {"bound": "mfma (f32 arithmetic; T1's forward on split-bf16 MFMA, its backward on f32 MFMA)",
                            "achieved": round(upd_tf, 2), "peak": F32_MFMA_PEAK_TFLOPS,
                            "unit": "TFLOP/s", "frac": round(upd_tf / F32_MFMA_PEAK_TFLOPS, 4),
                            "flop_per_sample": flop,
                            "note": "whole update: 2 kernels (T1 also draws the minibatch from the ring and advances the counter, T2 also rewrites the policy images); peak = the f32 MFMA peak, the precision the update computes in"},
        "batch": args.train_batch,
        "global_batch": args.train_batch * dist.world,
        "data_parallel": (f"dp{dist.world}: gradient SUM all-reduce of {agent._grad.numel()} f32 per update"
                          if agent.data_parallel else None),
        "replay_capacity": agent.memory.capacity,
        "final_loss": float(loss),
        "epsilon": agent.epsilon,
    }
    agent.close()
    env.close()
    return out


KERNEL_MS_BASIS = ("HIP events on the launch stream, one right before launch 1 and one after launch K, over K "
                   "launches (this run)")


def roofline(bytes_per_step, n, k_ms, canonical):
    """The roofline object of one leg. achieved = this build's algorithmic bytes per
    env-step (42 / 50 B) x n / the per-launch kernel time; the
    survey's canonical field widths (66 / 82 B) are given as a byte count only: the
    kernel does not move them, so no rate is derived from them."""
    achieved = bytes_per_step * n / (k_ms * 1e-3) / 1e9
    return {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBPS, 4),
        "traffic": None,
        "bytes_per_env_step": bytes_per_step,
        "canonical_bytes_per_env_step": canonical,
        "kernel_ms": round(k_ms, 5),
        "kernel_ms_basis": KERNEL_MS_BASIS,
    }


def pmc_traffic(key="step_kernel_bytes_per_launch"):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get(key), os.path.relpath(path, ROOT)


TRACE_SUMMARY = os.path.join("profiles", "rocprof_legs.json")  # condensed from a profiles/r0*/kt_legs*.json


def committed_trace(key):
    """A leg's kernel-trace average from the committed rocprofv3 summary (tools/trace_driver.sh
    -> tools/kt_legs.py -> profiles/rocprof_legs.json), with the commit and date of the code
    it was traced on. It is NOT a figure of this run: it goes under its own key
    ("committed_trace") beside the live events figure, so a stale trace shows as such."""
    path = os.path.join(ROOT, TRACE_SUMMARY)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    leg = d.get(key)
    if not leg:
        return None
    return {"avg_us": leg["avg_us_timed"], "frac": leg.get("frac_from_trace"), "source": TRACE_SUMMARY,
            "traced_code": d.get("traced_code"), "trace": d.get("trace")}


def cpu_threads():
    """Host threads for the threaded CPU leg: the job's CPU share (OMP_NUM_THREADS is
    16 on the GPU box, whose nproc counts the whole machine), else the affinity set."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return max(1, min(16, len(os.sched_getaffinity(0))))


def cpu_baseline(n_workload, ports_seed, budget_s):
    """The C restatement (oracle, Philox mode) on bounded samples of the same workload
    (single-thread and over the host's cores, in the same run):
      - 1 thread on 2^16 of the envs, as many whole steps as fit half the budget;
      - T threads (cpu_threads()) on all n envs, each stepping a quad-aligned slice
        (ctypes releases the GIL), as many whole steps as fit the other half.
    The threaded figure is `value`; the single-thread one rides along."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    from shippingenv_amd.maps import builtin_water
    from shippingenv_amd.vec import DEFAULT_PORTS, draw_port_stocks

    water = builtin_water()
    pf, pc = draw_port_stocks(5, ports_seed)
    world = O.OracleWorld(water, [p[0] for p in DEFAULT_PORTS], [p[1] for p in DEFAULT_PORTS], pf, pc)

    def timed(n, threads, budget):
        st = O.OracleState(n)
        O.reset(world, st, seed=ports_seed, epoch=0)
        acts = [O.gen_actions(n, 5, ports_seed, 0, t) for t in range(16)]
        steps, spent = 0, 0.0
        with ThreadPoolExecutor(threads) as pool:
            while spent < budget:
                t0 = time.perf_counter()
                if threads == 1:
                    O.step(world, st, actions=acts[steps % 16], seed=ports_seed, t=steps)
                else:
                    O.step_threaded(world, st, acts[steps % 16], pool, threads, seed=ports_seed, t=steps)
                spent += time.perf_counter() - t0
                steps += 1
        return n * steps / spent, steps, spent

    n1 = min(n_workload, 1 << 16)
    v1, s1, t1 = timed(n1, 1, budget_s / 2)
    threads = cpu_threads()
    vt, st_, tt = timed(n_workload, threads, budget_s / 2)
    return {
        "value": round(vt, 1),
        "unit": "env-steps/s",
        "cores": threads,
        "kind": "port",
        "single_thread_value": round(v1, 1),
        "sample": f"oracle/shipenv_oracle.c (Philox mode, same action mix): {threads} threads on "
                  f"{n_workload} envs x {st_} steps ({tt:.1f} s); 1 thread on {n1} envs x {s1} steps "
                  f"({t1:.1f} s) -> single_thread_value. Reference Python measured in the build "
                  "container: 1.0-1.2e5 env-steps/s on 1 core (BASELINE.md)",
    }


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's plain `python3 bench.py --gpus N`: launch the N ranks here
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    dist = Dist(args.gpus)
    from shippingenv_amd.maps import builtin_water
    from shippingenv_amd.vec import random_water_ports

    n = args.n
    # config 3 from reset first (ships at their origin ports, cargo rising: the first steps'
    # state mix; DESIGN.md section 5, "The short run"), then the headline leg in steady
    # state, its K steps issued by VecEnv.step_seq (the native launch loop, whose kernel has
    # a trace name of its own), then the same steady leg with one VecEnv.step call per step
    el3r, k3r, _, _ = run_config(n, None, False, args, dist, "config3-from-reset", preroll=0)
    el3, k3, _, info3 = run_config(n, None, False, args, dist, "config3", preroll=args.preroll3,
                                   step_seq=True)
    value = n * dist.world * args.steps / el3
    el3p, k3p, _, _ = run_config(n, None, False, args, dist, "config3-step-py", preroll=args.preroll3)
    # SURVEY 8(d) config 3 to the letter: se_reset, warm-up 10, time 1000 steps (whatever K is)
    lit = argparse.Namespace(**vars(args))
    lit.steps, lit.warmup = LITERAL_STEPS, LITERAL_WARMUP
    el3l, k3l, _, _ = run_config(n, None, False, lit, dist, "config3-literal", preroll=0, step_seq=True)
    out = {
        "metric": "env-steps/sec at N=2^20 parallel envs per GPU (config 3: full step, 5 default ports; "
                  "K steps in the steady state after a 1000-step pre-roll; config3_literal: the survey's "
                  "1000 steps from reset)",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el3 / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64+int (fuel f64; reward computed in f64, stored f32 after one rounding; positions/cargo int)",
        "data": "synthetic (Philox agent actions resident in HBM; reference map and ports)",
        "config": {
            "workload": "BASELINE configs[2]: N=2^20 envs/GPU, full step, default 5 ports; steady state "
                        f"mix as in the survey's 1000-step run: {args.preroll3} untimed pre-roll steps from "
                        "reset before the warm-up (from_reset: the same leg timed right after reset); "
                        "the K timed steps issued by VecEnv.step_seq (se_step_seq, the native launch loop: "
                        "its kernel, step_kernel<..., true>, is the trace row of exactly these launches; "
                        "step_py: the same leg with one VecEnv.step call per step); "
                        f"roofline.kernel_ms: {KERNEL_MS_BASIS}",
            "preroll_steps": args.preroll3,
            "envs_per_gpu": n,
            "global_envs": n * dist.world,
            "ports": 5,
            "parallelism": f"env-shard dp{dist.world} (no data-path collective)",
        },
        "roofline": roofline(BYTES_STEP, n, k3, CANONICAL_STEP),
        "from_reset": {"value": round(n * dist.world * args.steps / el3r, 1),
                       "ms_per_step": round(el3r / args.steps * 1e3, 5),
                       "kernel_ms": round(k3r, 5),
                       "frac": roofline(BYTES_STEP, n, k3r, CANONICAL_STEP)["frac"]},
        "step_py": {"value": round(n * dist.world * args.steps / el3p, 1),
                    "ms_per_step": round(el3p / args.steps * 1e3, 5),
                    "kernel_ms": round(k3p, 5),
                    "frac": roofline(BYTES_STEP, n, k3p, CANONICAL_STEP)["frac"]},
        "config3_literal": {"workload": f"SURVEY 8(d) config 3 as written: se_reset, warm-up {LITERAL_WARMUP}, "
                                        f"{LITERAL_STEPS} timed steps (VecEnv.step_seq), N=2^20 envs/GPU",
                            "steps": LITERAL_STEPS, "warmup": LITERAL_WARMUP,
                            "value": round(n * dist.world * LITERAL_STEPS / el3l, 1),
                            "ms_per_step": round(el3l / LITERAL_STEPS * 1e3, 5),
                            "kernel_ms": round(k3l, 5),
                            "frac": roofline(BYTES_STEP, n, k3l, CANONICAL_STEP)["frac"]},
        "dist": dist.info,
    }
    for key, obj in (("config3", out["roofline"]), ("config3_from_reset", out["from_reset"]),
                     ("config3_step_py", out["step_py"]), ("config3_literal", out["config3_literal"])):
        obj["committed_trace"] = committed_trace(key)
    traffic, src = pmc_traffic()
    if traffic:
        out["roofline"]["traffic"] = traffic
        out["roofline"]["traffic_source"] = src

    if not args.no_config4:
        ports64 = random_water_ports(builtin_water(), 64, seed=3)
        el4, k4, stats, info4 = run_config(n, ports64, True, args, dist, "config4", preroll=args.preroll4)
        t4, src4 = pmc_traffic("step_kernel_auto_bytes_per_launch")
        out["config4"] = {
            "workload": "BASELINE configs[3]: N=2^20 envs/GPU, 64 random ports, auto-reset, "
                        "ballot-compacted done list (per-wave segments), per-wave return reduction, RCCL all-reduce "
                        "of the stats every min(100, steps // 2) steps inside the timed region; steady episode "
                        f"mix: {args.preroll4} untimed pre-roll steps from reset before the warm-up; "
                        f"roofline.kernel_ms: {KERNEL_MS_BASIS}",
            "value": round(n * dist.world * args.steps / el4, 1),
            "ms_per_step": round(el4 / args.steps * 1e3, 5),
            "roofline": roofline(BYTES_STEP_AUTO, n, k4, CANONICAL_STEP_AUTO),
            "episodes": stats[1],
            "mean_return": stats[0] / stats[1] if stats and stats[1] else None,
            "mean_len": stats[2] / stats[1] if stats and stats[1] else None,
        } | info4
        out["config4"]["roofline"]["committed_trace"] = committed_trace("config4")
        if t4:
            out["config4"]["roofline"]["traffic"] = t4
            out["config4"]["roofline"]["traffic_source"] = src4

    if args.config1 and dist.world == 1:
        out["config1"] = run_config1(args)

    if args.rollouts:
        out["rollouts"] = run_rollouts(n, args, dist)

    if args.dqn_steps:
        out["config5"] = run_config5(n, args, dist)

    if args.train_steps:  # N > 1: data parallel (gradient all-reduce per update)
        try:
            out["dqn_train"] = run_dqn_train(n, args, dist)
        except Exception as e:  # noqa: BLE001 - keep the headline line whatever this leg does
            log(f"[dqn_train] failed: {type(e).__name__}: {e}")
            out["dqn_train"] = {"error": f"{type(e).__name__}: {e}"[:400]}

    if args.large_n and dist.world == 1:
        # the config-3 step at 2^24 envs: from reset, then in the headline's steady state
        # (the same pre-roll); 100 timed steps each
        small = argparse.Namespace(**vars(args))
        small.steps, small.warmup = 100, 5
        elr, kr, _, _ = run_config(args.large_n, None, False, small, dist, "large-n-from-reset")
        el, k, _, _ = run_config(args.large_n, None, False, small, dist, "large-n", preroll=args.preroll3)
        out["large_n"] = {
            "envs": args.large_n,
            "note": "working set beyond the 256 MiB Infinity Cache: traffic reaches HBM; steady state "
                    f"after {args.preroll3} untimed pre-roll steps as the headline (from_reset: timed "
                    "right after reset, where most ships carry cargo and draw the loss gate)",
            "preroll_steps": args.preroll3,
            "value": round(args.large_n * small.steps / el, 1),
            "roofline": roofline(BYTES_STEP, args.large_n, k, CANONICAL_STEP)
            | {"committed_trace": committed_trace("large_n")},
            "from_reset": {"value": round(args.large_n * small.steps / elr, 1),
                           "kernel_ms": round(kr, 5),
                           "frac": roofline(BYTES_STEP, args.large_n, kr, CANONICAL_STEP)["frac"],
                           "committed_trace": committed_trace("large_n_from_reset")},
        }
        if not args.no_config4:
            # config 4 at the same size in its steady episode mix (the same pre-roll): the
            # auto-reset step with the traffic beyond the Infinity Cache
            ports64 = random_water_ports(builtin_water(), 64, seed=3)
            el4b, k4b, st4b, _ = run_config(args.large_n, ports64, True, small, dist, "large-n-config4",
                                            preroll=args.preroll4)
            t4b, src4b = pmc_traffic("step_kernel_auto_big_bytes_per_launch")
            out["large_n"]["config4"] = {
                "value": round(args.large_n * small.steps / el4b, 1),
                "ms_per_step": round(el4b / small.steps * 1e3, 5),
                "roofline": roofline(BYTES_STEP_AUTO, args.large_n, k4b, CANONICAL_STEP_AUTO)
                | {"committed_trace": committed_trace("large_n_config4")},
                "episodes": st4b[1],
                "preroll_steps": args.preroll4,
            }
            if t4b:
                out["large_n"]["config4"]["roofline"]["traffic"] = t4b
                out["large_n"]["config4"]["roofline"]["traffic_source"] = src4b
        tb, srcb = pmc_traffic("step_kernel_big_bytes_per_launch")
        if tb:
            out["large_n"]["roofline"]["traffic"] = tb
            out["large_n"]["roofline"]["traffic_source"] = srcb

    if dist.rank == 0 and dist.world == 1 and not args.no_cpu:
        log("[cpu] timing the C restatement")
        out["cpu_baseline"] = cpu_baseline(n, args.seed, args.cpu_seconds)

    if dist.rank == 0:
        print(json.dumps(out), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
