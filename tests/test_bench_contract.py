"""bench.py's roofline object keeps the keys the driver's contract names (no GPU needed)."""
import importlib.util
import os

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_roofline_object_has_the_contract_keys():
    b = _bench()
    r = b.roofline(b.BYTES_STEP, 1 << 20, 0.0085, b.CANONICAL_STEP)
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    # achieved = algorithmic bytes per launch / launch time; frac = achieved / peak
    assert abs(r["achieved"] - b.BYTES_STEP * (1 << 20) / 8.5e-6 / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-4
    assert r["kernel_ms"] == 0.0085


def test_no_roofline_rate_above_its_peak():
    """Every GB/s figure in the object is a rate the kernel moves: the survey's canonical
    widths appear as a byte count only (canonical_achieved exceeded 8 TB/s)."""
    b = _bench()
    for k_ms in (0.0085, 0.004):  # the second would put a 66 B rate above the peak
        r = b.roofline(b.BYTES_STEP, 1 << 20, k_ms, b.CANONICAL_STEP)
        assert "canonical_achieved" not in r
        assert r["canonical_bytes_per_env_step"] == 66
        assert [key for key in r if key.endswith("achieved")] == ["achieved"]
    assert b.KERNEL_MS_BASIS in b.roofline(b.BYTES_STEP, 1, 1.0, 66)["kernel_ms_basis"]


def test_committed_trace_summary_covers_every_leg():
    """bench.py prints each leg's committed kernel-trace average (committed_trace) from
    profiles/rocprof_legs.json, a file outside the gpurun-ignored profiles/r0* directories, so
    the GPU box's run sees it; every timed leg must be in it, with a frac below 1."""
    b = _bench()
    for key in ("config3", "config3_from_reset", "config3_step_py", "config4", "large_n",
                "large_n_from_reset"):
        r = b.committed_trace(key)
        assert r is not None, key
        assert 0 < r["frac"] < 1 and r["avg_us"] > 0, key
    assert not b.TRACE_SUMMARY.startswith(os.path.join("profiles", "r0"))


def test_committed_trace_is_labelled_as_such():
    """the committed trace figures go under their own key with the code they were
    traced on, and kernel_ms_basis names only what this run measured."""
    b = _bench()
    r = b.committed_trace("config3")
    assert r["traced_code"] and r["source"] == b.TRACE_SUMMARY
    assert "rocprof" not in b.KERNEL_MS_BASIS and "this run" in b.KERNEL_MS_BASIS


CHILD = r'''
import json, os, sys, time
rank = int(os.environ["RANK"])
mode = sys.argv[1]
if mode == "ok":
    if rank == 0:
        # a library's own chatter on stdout (gloo prints "[Gloo] Rank 0 is connected ...")
        print("[Gloo] Rank 0 is connected to 2 peer ranks.", flush=True)
        print(json.dumps({"rank": rank, "world": int(os.environ["WORLD_SIZE"]),
                          "local": int(os.environ["LOCAL_RANK"]), "argv": sys.argv[1:],
                          "master": [os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"]],
                          "launcher": os.environ.get("SHIPENV_LAUNCHER")}))
    else:
        print("not for the driver")  # a non-zero rank's stdout is dropped
elif mode == "fail":
    sys.exit(3 if rank == 1 else 0)
elif mode == "hang":  # rank 1 dies, rank 0 waits forever (a collective with a dead peer)
    if rank == 1:
        sys.exit(5)
    time.sleep(600)
'''


def _child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return str(p)


def test_spawn_ranks_forwards_rank0_line_only(tmp_path, capsys):
    import json

    import torch

    b = _bench()
    rc = b.spawn_ranks(3, ["ok", "--steps", "7"], script=_child(tmp_path))
    out = capsys.readouterr().out.strip().splitlines()
    assert rc == 0 and len(out) == 1
    d = json.loads(out[0])
    assert d["rank"] == 0 and d["world"] == 3 and d["local"] == 0
    assert d["argv"] == ["ok", "--steps", "7"]
    assert d["master"][0] == "127.0.0.1" and int(d["master"][1]) > 0
    assert d["launcher"] == "bench.spawn_ranks"
    assert not torch.cuda.is_initialized()  # the parent made no GPU call


def test_spawn_ranks_fails_when_a_rank_fails(tmp_path, capsys):
    b = _bench()
    assert b.spawn_ranks(2, ["fail"], script=_child(tmp_path)) == 3
    assert capsys.readouterr().out == ""


def test_spawn_ranks_ends_ranks_left_waiting(tmp_path, capsys):
    import time

    b = _bench()
    t0 = time.monotonic()
    assert b.spawn_ranks(2, ["hang"], script=_child(tmp_path), grace_s=1.0) == 5
    assert time.monotonic() - t0 < 60
    assert capsys.readouterr().out == ""


def test_main_spawns_without_touching_the_gpu(tmp_path, monkeypatch, capsys):
    """`bench.py --gpus 2` with no WORLD_SIZE: main() hands its own arguments to N children
    and never reaches torch.cuda or torch.distributed in the parent."""
    import sys

    import torch

    b = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(b, "__file__", _child(tmp_path))

    def boom(*a, **k):
        raise AssertionError("the launcher parent touched the GPU")

    for name in ("is_available", "device_count", "synchronize", "set_device", "init", "current_device"):
        monkeypatch.setattr(torch.cuda, name, boom)
    monkeypatch.setattr(b, "Dist", boom)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    # the child script reads argv[1] as its mode: "--gpus" is not a mode, so every rank
    # falls through and exits 0 with no line
    try:
        b.main()
    except SystemExit as e:
        assert e.code == 0
    else:
        raise AssertionError("main() must exit with the launcher's status")
    assert capsys.readouterr().out == ""
