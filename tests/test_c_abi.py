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


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_ctypes_structs_match_the_header(tmp_path):
    """The ctypes mirrors in drone_rl_amd/_lib.py have the C layout of
    include/dronerl.h (size and every field offset)."""
    import ctypes

    from drone_rl_amd import _lib
    src = tmp_path / "layout.c"
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "dronerl.h"',
             "int main(void) {"]
    for cname, cls in (("dr_config", _lib.dr_config), ("dr_grad_finish", _lib.dr_grad_finish)):
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["return 0;", "}"]
    src.write_text("\n".join(lines))
    exe = str(tmp_path / "layout")
    subprocess.run(["gcc", "-std=c11", "-D__HIP_PLATFORM_AMD__",
                    "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include", str(src),
                    "-o", exe], check=True, capture_output=True, text=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run(
        [exe], check=True, capture_output=True, text=True).stdout.split("\n") if l)
    for cname, cls in (("dr_config", _lib.dr_config), ("dr_grad_finish", _lib.dr_grad_finish)):
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)
