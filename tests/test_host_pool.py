"""The host worker pool behind the staged paths' readers and copies
(ciruela_amd/csrc/pool.hpp) under ThreadSanitizer, g++ on the header alone:
concurrent callers of random width over random item counts, every item
processed exactly once per call, no call left waiting (tools/pool_stress.cpp)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


def test_worker_pool_tsan(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    exe = str(tmp_path / "pool_stress")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread",
                    "-I" + os.path.join(ROOT, "ciruela_amd", "csrc"),
                    os.path.join(ROOT, "tools", "pool_stress.cpp"), "-o", exe, "-lpthread"],
                   check=True)
    p = subprocess.run([exe, "8", "300"], capture_output=True, timeout=300)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert b"ok" in p.stdout and b"WARNING: ThreadSanitizer" not in p.stderr
