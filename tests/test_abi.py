"""The C ABI library loads and exports exactly what include/dronerl.h
declares (CPU only: no compute call is made without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "dronerl.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dr_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_abi():
    names = declared_functions()
    for must in ("dr_create", "dr_destroy", "dr_reset", "dr_step", "dr_get_state",
                 "dr_set_state", "dr_set_reset_uniforms", "dr_last_error", "dr_gae",
                 "dr_ppo_loss", "dr_clip_adam", "dr_permutation", "dr_policy_sample"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from drone_rl_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "build libdronerl.so first (__graft_entry__.build)"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dr_[a-z0-9_]+)", out))
    declared = set(declared_functions())
    assert declared <= exported, declared - exported
    # the ctypes binding covers the whole declared ABI
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)


def test_library_loads_and_validates_without_gpu():
    from drone_rl_amd import _lib
    L = _lib.lib()
    assert L.dr_abi_version() == _lib.ABI_VERSION == 16
    # argument validation happens before any HIP call
    cfg = _lib.dr_config(num_envs=0)
    h = ctypes.c_void_p()
    rc = L.dr_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc == _lib.DR_ERR_INVALID
    assert "num_envs" in _lib.last_error()
    assert L.dr_step(None, None, None, None, None, None, None) == _lib.DR_ERR_INVALID
    assert L.dr_rollout(None, 4, None, None, None, None, None) == _lib.DR_ERR_INVALID
    assert L.dr_rollout_random(None, 4, 7, 0, 0.0, 1.0, None, None, None, None,
                               None) == _lib.DR_ERR_INVALID
    assert L.dr_gae(0, 0, None, None, None, None, None, 0.99, 0.95, None, None,
                    None) == _lib.DR_ERR_INVALID
    with pytest.raises(_lib.DroneRLError):
        _lib.check(L.dr_reset(None, None, None))


def test_oracle_not_linked_by_product():
    """The product library must not depend on the oracle."""
    from drone_rl_amd import _lib
    out = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "oracle" not in out
    for dirpath, _, files in os.walk(os.path.join(ROOT, "drone_rl_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", txt, re.M), f


def test_v5_v7_entry_points_validate_without_gpu():
    """The minibatch-gather, paired first-layer and deferred-finish entry
    points reject bad arguments before any HIP call."""
    from drone_rl_amd import _lib
    L = _lib.lib()
    bad = _lib.DR_ERR_INVALID
    assert L.dr_gather_minibatch(4, None, 15, None, None, None, None, None, None, None,
                                 None) == bad
    assert L.dr_linear_tanh2(4, 15, 6, None, None, None, None, None, None, None, None,
                             None) == bad
    assert L.dr_first_layer_backward2(4, 15, 256, None, None, None, None, None, None, None,
                                      None, None, None, 0, None, 0, None) == bad
    f = _lib.dr_grad_finish()
    assert L.dr_grad_finish_clip_adam(None, 10, None, None, None, None, 1e-3, 0.9, 0.999,
                                      1e-5, 0.5, 1, None, None, 0, None) == bad
    # an empty descriptor has nothing to finish
    assert L.dr_grad_finish_workspace_bytes(ctypes.byref(f)) > 0
    buf = (ctypes.c_float * 16)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    assert L.dr_grad_finish_clip_adam(ctypes.byref(f), 10, p, p, p, p, 1e-3, 0.9, 0.999,
                                      1e-5, 0.5, 1, None, p, 4096, None) == bad
    assert "nothing to finish" in _lib.last_error()
    # a head segment without its outputs is refused
    f.head_workspace, f.head_m, f.head_hd = p, 64, 256
    assert L.dr_grad_finish_clip_adam(ctypes.byref(f), 10, p, p, p, p, 1e-3, 0.9, 0.999,
                                      1e-5, 0.5, 1, None, p, 4096, None) == bad
    assert "head" in _lib.last_error()
