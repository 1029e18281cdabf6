"""The striped multi-device scan's progress (ciruela_amd/csrc/stripes.hpp,
used by hash_files in scan.cpp) under ASan + UBSan, g++ on the header alone:
after every batch of every device the prefix handed to the emitter equals
the true complete prefix of the global block order -- a batch inside the
first open stripe and the last stripe's completion included -- and it is
reported exactly when it grows (tools/stripe_prefix_fuzz.cpp).  The GPU
side (CIR_DEBUG_SPLIT=2, the index written in many pieces while the scan
runs) is test_gpu_parity.py::test_split_scan_streams_within_stripes."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


def test_stripe_prefix_sanitized(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    exe = str(tmp_path / "stripe_prefix_fuzz")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all",
                    "-I" + os.path.join(ROOT, "ciruela_amd", "csrc"),
                    os.path.join(ROOT, "tools", "stripe_prefix_fuzz.cpp"), "-o", exe], check=True)
    for seed in (1, 2, 3):
        p = subprocess.run([exe, "400", str(seed)], capture_output=True, timeout=120)
        assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
        assert p.stdout.startswith(b"ok ")
