"""The asynchronous verify's queue (ciruela_amd/csrc/verify_queue.hpp: the
bounded queue, its worker, forget and expiry behind cir_verify_submit /
poll / wait / forget / limits) on the host with a test hasher in place of
the GPU batch, g++ on the header alone, under ThreadSanitizer and under
ASan + UBSan (tools/verify_queue_stress.cpp):
  * deterministic states with the hasher held closed: a non-blocking submit
    without room is CIR_EAGAIN and takes nothing, a blocking one waits until
    the worker frees room, 0-byte blocks always fit, a block larger than the
    bound is taken alone; forget of a pending ticket (releasing its waiter),
    of a finished one and of an unknown one; expiry keeps the newest
    max_results outcomes; a failed batch reports its code to every ticket;
    two hash types never share a batch; a bound larger than memory still
    verifies (arenas stay at most 128 MiB), a block whose own arena cannot
    be allocated is CIR_ENOMEM;
  * random traffic from 2-5 threads, blocking and not, with forgets and
    polls: every outcome right, the peak within the bound, nothing held at
    the end, and a queue destroyed with work queued drains it.
The same entry points on the GPU, against the oracle:
test_gpu_parity.py::test_verify_async_*."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_verify_queue_sanitized(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    exe = str(tmp_path / "verify_queue_stress")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=" + san,
                    "-fno-sanitize-recover=all",
                    "-I" + os.path.join(ROOT, "ciruela_amd", "csrc"),
                    "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tools", "verify_queue_stress.cpp"), "-o", exe,
                    "-lpthread"], check=True)
    # (a queue bound past what can be allocated must come back as CIR_ENOMEM:
    # the sanitizers' allocators return null for it instead of aborting)
    env = dict(os.environ, ASAN_OPTIONS="allocator_may_return_null=1",
               TSAN_OPTIONS="allocator_may_return_null=1")
    p = subprocess.run([exe, "6", "7"], capture_output=True, timeout=300, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert p.stdout.startswith(b"ok ") and b"WARNING: ThreadSanitizer" not in p.stderr
