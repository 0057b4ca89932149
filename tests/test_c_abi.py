"""The C ABI used from plain C (what a non-Python host would bind)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "c", "abi_demo.c")


def _compile(out):
    cmd = ["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
           "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include", SRC, "-o", out,
           "-L" + os.path.join(ROOT, "drone_rl_amd"), "-ldronerl", "-L/opt/rocm/lib",
           "-lamdhip64", "-lm", "-Wl,-rpath," + os.path.join(ROOT, "drone_rl_amd"),
           "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_header_compiles_as_c_and_links(tmp_path):
    _compile(str(tmp_path / "abi_demo"))


@pytest.mark.gpu
def test_c_program_steps_envs(tmp_path):
    exe = str(tmp_path / "abi_demo")
    _compile(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "c abi ok" in r.stdout
