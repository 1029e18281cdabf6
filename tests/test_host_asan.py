"""The library's host code under AddressSanitizer + UBSan, and under
ThreadSanitizer, on the GPU (tools/host_asan_driver.cpp, built by `make asan` and
`make tsan` with the sanitizers on the host translation units only, against the
production device code): random rounds
of every host-path entry point -- descriptor batches, batch and asynchronous
verify, hash_memory / hash_file / check_file at block sizes up to 2^32-1
(files that grow included), scans whole and streamed, the rewrite, the
registries -- through a plain, a three-state (CIR_DEBUG_SPLIT) and a
one-shot context, with four more threads calling into one context at once
every fifth round, each GPU digest checked against the library's host
hashers.  A memory error, undefined behaviour or a data race in the
library's sources fails the run (tools/tsan_hip.supp drops TSan's reports
inside the uninstrumented HIP and HSA runtimes)."""
import os
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.gpu
def test_host_code_under_asan_and_ubsan():
    exe = os.path.join(ROOT, "build", "host_asan_driver")
    assert os.path.exists(exe), "build/host_asan_driver missing: run make asan"
    # leaks: the HIP runtime keeps allocations to the end; link order: the
    # sanitizer runtime is linked into the executable, not preloaded
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([exe, "24", "7"], capture_output=True, timeout=300, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-6000:])
    assert p.stdout.strip() == b"ok 24 rounds"


@pytest.mark.gpu
def test_host_code_under_tsan():
    exe = os.path.join(ROOT, "build", "host_tsan_driver")
    assert os.path.exists(exe), "build/host_tsan_driver missing: run make tsan"
    supp = os.path.join(ROOT, "tools", "tsan_hip.supp")
    env = dict(os.environ, TSAN_OPTIONS="suppressions=%s report_thread_leaks=0" % supp)
    p = subprocess.run([exe, "15", "5"], capture_output=True, timeout=300, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-6000:])
    assert p.stdout.strip() == b"ok 15 rounds"
    assert b"WARNING: ThreadSanitizer" not in p.stderr, p.stderr[-6000:]
