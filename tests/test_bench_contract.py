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
    """bench.py prints each leg's committed kernel-trace average (roofline.rocprof_trace) from
    profiles/rocprof_legs.json, a file outside the gpurun-ignored profiles/r0* directories, so
    the GPU box's run sees it; every timed leg must be in it, with a frac below 1."""
    b = _bench()
    for key in ("config3", "config3_from_reset", "config3_step_py", "config4", "large_n",
                "large_n_from_reset"):
        r = b.rocprof_leg(key)
        assert r is not None, key
        assert 0 < r["frac"] < 1 and r["avg_us"] > 0, key
    assert not b.TRACE_SUMMARY.startswith(os.path.join("profiles", "r0"))
