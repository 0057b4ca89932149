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
    assert L.dr_abi_version() == _lib.ABI_VERSION == 7
    # argument validation happens before any HIP call
    cfg = _lib.dr_config(num_envs=0)
    h = ctypes.c_void_p()
    rc = L.dr_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc == _lib.DR_ERR_INVALID
    assert "num_envs" in _lib.last_error()
    assert L.dr_step(None, None, None, None, None, None, None) == _lib.DR_ERR_INVALID
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
