"""Repository hygiene (CPU): history stays source-only.  Built libraries,
executables and code objects travel to the GPU box with the tree but are
never tracked (round 5 tracked four unbundled gfx950 code objects under
ciruela_amd/ by accident)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


def _tracked():
    if not shutil.which("git") or not os.path.isdir(os.path.join(ROOT, ".git")):
        pytest.skip("not a git checkout")
    out = subprocess.check_output(["git", "-C", ROOT, "ls-files", "-z"])
    return [p for p in out.decode().split("\0") if p]


def test_no_tracked_elf():
    elves = []
    for rel in _tracked():
        path = os.path.join(ROOT, rel)
        if not os.path.isfile(path):
            continue
        with open(path, "rb") as f:
            if f.read(4) == b"\x7fELF":
                elves.append(rel)
    assert elves == [], elves


def test_no_tracked_build_outputs_in_package_or_bin():
    bad = [p for p in _tracked()
           if (p.startswith("ciruela_amd/") or p.startswith("bin/") or p.startswith("build/"))
           and not (p.endswith(".py") or p.startswith("ciruela_amd/csrc/"))]
    assert bad == [], bad


def test_sanitizer_drivers_not_in_default_target():
    """`make` builds the library, CLI, load drivers and oracle; the ASan and
    TSan drivers are `make asan` / `make tsan` (build() asks for them)."""
    mk = open(os.path.join(ROOT, "Makefile")).read()
    all_line = next(l for l in mk.splitlines() if l.startswith("all:"))
    assert "asan" not in all_line and "tsan" not in all_line
    for t in ("asan:", "tsan:", "sanitizers:"):
        assert any(l.startswith(t) for l in mk.splitlines()), t
