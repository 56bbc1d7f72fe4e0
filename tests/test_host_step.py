"""The host-compiled step (se_host_step_replay / se_host_reset_to: the step kernels' own
per-env code, replay_env in csrc/shipenv.hip, built for the host) against the reference's
golden records, and the drop-in shipping.Environment on it against the reference's seeded
traces. No GPU: this is the product's N = 1 path (the default stepper of the drop-in);
tests/test_compat_gpu.py checks it against the kernel bit for bit."""
import os

import numpy as np
import pytest

from compat_replay import load_script, replay
from conftest import golden_files, load_golden

FIELDS = ("x", "y", "fuel", "cargo", "origin", "dest")


def _u8(v):
    return np.where(np.asarray(v) < 0, 255, v).astype(np.uint8)


def _world(z, with_ports):
    sl = slice(None) if with_ports else slice(0, 0)
    return (z["port_x"][sl], z["port_y"][sl], z["port_fuel"][sl], z["port_cargo"][sl])


def _tape(z, sel):
    from shippingenv_amd.vec import TAPE_DTYPE

    tape = np.zeros(len(sel), TAPE_DTYPE)
    for f in ("u_fuel", "u_gate", "u_type", "beta", "arrive_dest"):
        tape[f] = z[f][sel]
    return tape


def host_replay(z, sel, water, with_ports=True):
    from shippingenv_amd.shipping._host import host_step_replay

    state = {f: (_u8(z["pre_" + f][sel]) if f in ("origin", "dest") else z["pre_" + f][sel]) for f in FIELDS}
    return host_step_replay(water, *_world(z, with_ports), state, z["act_type"][sel], z["act_a"][sel],
                            z["act_b"][sel], _tape(z, sel))


@pytest.mark.parametrize("path", golden_files(), ids=os.path.basename)
def test_host_replay_matches_reference(path, water):
    z = load_golden(path)
    checked = 0
    for kind, with_ports in ((0, True), (2, False)):
        sel = np.nonzero(z["kind"] == kind)[0]
        if not len(sel):
            continue
        got = host_replay(z, sel, water, with_ports)
        for f in FIELDS:
            want = z["post_" + f][sel]
            g = got[f]
            if f in ("origin", "dest"):
                g = np.where(g == 255, -1, g.astype(np.int32))
            if f == "fuel":
                np.testing.assert_array_equal(g.view(np.int64), want.view(np.int64), err_msg="fuel bits")
            else:
                np.testing.assert_array_equal(g.astype(np.int64), want, err_msg=f)
        np.testing.assert_array_equal(got["reward"], z["reward"][sel].astype(np.float32))
        np.testing.assert_array_equal(got["reward64"], z["reward"][sel])  # the reference's f64 reward
        np.testing.assert_array_equal(got["done"].astype(np.int32), z["done"][sel])
        np.testing.assert_array_equal(got["err"].astype(np.int32), z["err"][sel])
        checked += len(sel)
    assert checked > 1000


@pytest.mark.parametrize("path", golden_files("tape"), ids=os.path.basename)
def test_host_resets_match_reference(path, water):
    from shippingenv_amd.shipping._host import host_reset_to

    z = load_golden(path)
    sel = np.nonzero(z["kind"] == 1)[0]
    got = host_reset_to(water, *_world(z, True), z["reset_origin"][sel], z["reset_dest"][sel])
    for f in FIELDS:
        want = z["post_" + f][sel]
        g = got[f].view(np.int64) if f == "fuel" else got[f].astype(np.int64)
        np.testing.assert_array_equal(g, want.view(np.int64) if f == "fuel" else want, err_msg=f)


def test_host_replay_need_draw_leaves_state(water):
    """A move whose tape lacks u_fuel answers SE_ERR_NEED_DRAW and changes nothing (the
    drop-in's draw protocol), like se_step_replay."""
    z = load_golden(golden_files("tape")[0])
    sel = np.nonzero((z["kind"] == 0) & (z["act_type"] == 1) & (z["err"] == 0))[0][:64]
    from shippingenv_amd.shipping._host import host_step_replay
    from shippingenv_amd.vec import TAPE_DTYPE

    state = {f: (_u8(z["pre_" + f][sel]) if f in ("origin", "dest") else z["pre_" + f][sel]) for f in FIELDS}
    tape = np.zeros(len(sel), TAPE_DTYPE)
    tape["u_fuel"] = tape["u_gate"] = tape["u_type"] = tape["beta"] = np.nan
    tape["arrive_dest"] = -1
    got = host_step_replay(water, *_world(z, True), state, z["act_type"][sel], z["act_a"][sel],
                           z["act_b"][sel], tape)
    assert (got["err"] == 10).all()
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], np.asarray(state[f], got[f].dtype))
    assert (got["reward"] == 0).all() and (got["done"] == 0).all()


@pytest.fixture()
def host_backend(monkeypatch):
    from shippingenv_amd.shipping import environment

    environment._set_stepper_factory(None)
    monkeypatch.setenv("SHIPENV_STEPPER", "host")
    yield


@pytest.mark.parametrize("seed", range(6))
def test_dropin_host_stepper_matches_reference_traces(host_backend, seed):
    """The drop-in on its default (host) stepper reproduces the reference's seeded
    traces, RNG stream included (tests/golden/compat_seed*.json)."""
    assert replay(load_script(seed)) > 600


def test_stepper_kind_is_explicit(monkeypatch):
    from shippingenv_amd.shipping import environment

    monkeypatch.setenv("SHIPENV_STEPPER", "cpu")
    with pytest.raises(ValueError):
        environment.stepper_kind()
    monkeypatch.delenv("SHIPENV_STEPPER")
    assert environment.stepper_kind() == "host"
