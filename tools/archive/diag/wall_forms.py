"""Where the headline's wall time beyond its kernels goes (diagnostic).

Runs bench.py's timed_loop (config 3, N = 2^20, after a 1000-step pre-roll, K = 20,
VecEnv.step_seq) `reps` times in a fresh child process per HIP runtime setting, so each
setting is read at runtime initialisation:
  default            the image's defaults
  dev_kernarg        HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory)
  spin               hipSetDeviceFlags(hipDeviceScheduleSpin) before the first HIP call
  dev_kernarg+spin   both
  active_wait        ROC_ACTIVE_WAIT_TIMEOUT=2000 (the host spins up to 2 ms on a signal before
                     it sleeps on the interrupt)
and, inside each child, three loop forms rotated: `events` (bench.py's native-issue loop, an
event after launch 1 and after launch K), `bare` (the K launches in one native call, no event)
and `py` (bench.py's loop with one VecEnv.step call per step).

    python tools/diag/wall_forms.py [--reps 15] [--settings default,spin]
One JSON line per (setting, form): median / min wall us per step, events us per launch.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SETTINGS = {
    "default": {},
    "dev_kernarg": {"HIP_FORCE_DEV_KERNARG": "1"},
    "spin": {"SHIPENV_DIAG_SPIN": "1"},
    "dev_kernarg+spin": {"HIP_FORCE_DEV_KERNARG": "1", "SHIPENV_DIAG_SPIN": "1"},
    "active_wait": {"ROC_ACTIVE_WAIT_TIMEOUT": "2000"},
}


def child(reps, K):
    if os.environ.get("SHIPENV_DIAG_SPIN") == "1":
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
        if rc:
            raise SystemExit(f"hipSetDeviceFlags -> {rc}")
    import importlib.util
    import time

    import torch

    sys.path.insert(0, ROOT)
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    from shippingenv_amd.vec import VecEnv

    dist = b.Dist(1)
    n = 1 << 20
    env = VecEnv(n, seed=2026, device=dist.dev)
    acts = b.make_actions(env, 64 + K)
    env.reset()
    row = torch.empty(n, dtype=torch.int32, device=env.device)
    for t in range(1000):
        env.step(env.gen_actions(1_000_000 + t, out=row))
    for k in range(5):
        env.step_seq(acts[k:k + 1])
    torch.cuda.synchronize()
    res = {"events": {"wall": [], "events": []}, "bare": {"wall": []}, "py": {"wall": [], "events": []}}
    forms = ("events", "bare", "py")
    for rep in range(reps):
        first = (rep * 3) % 64
        for form in forms[rep % 3:] + forms[:rep % 3]:
            if form in ("events", "py"):
                wall, k_ms = b.timed_loop(env, acts, first, K, dist, step_seq=form == "events")
                res[form]["events"].append(round(k_ms * 1e3, 3))
            else:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                env.step_seq(acts[first:first + K])
                torch.cuda.synchronize()
                wall = time.perf_counter() - t0
            res[form]["wall"].append(round(wall / K * 1e6, 3))
    out = {}
    for form, r in res.items():
        out[form] = {"wall_us_median": statistics.median(r["wall"]), "wall_us_min": min(r["wall"]),
                     "events_us_median": statistics.median(r["events"]) if r.get("events") else None,
                     "wall": r["wall"]}
    print(json.dumps(out), flush=True)
    env.close()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=15)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--settings", default=",".join(SETTINGS))
    p.add_argument("--child", action="store_true")
    a = p.parse_args()
    if a.child:
        child(a.reps, a.steps)
        return
    for rnd in range(2):  # two rounds, so box drift shows
        for name in a.settings.split(","):
            env = dict(os.environ, **SETTINGS[name])
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--reps", str(a.reps),
                                "--steps", str(a.steps)], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode:
                print(json.dumps({"setting": name, "round": rnd, "rc": r.returncode, "err": r.stderr[-600:]}))
                sys.exit(r.returncode)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            for form, v in d.items():
                print(json.dumps({"setting": name, "round": rnd, "form": form, **v}), flush=True)


if __name__ == "__main__":
    main()
