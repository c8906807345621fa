"""The batch front end's host thread pool (`ppls_amd/csrc/aq_host_pool.h`, used by aq_integrate_batch's
staging and unpacking) built alone with g++ and run under ThreadSanitizer and without it: each piece of
every run executes exactly once, across runs with late-waking workers, and the pool shuts down cleanly."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "host_pool_check.cpp")
INC = os.path.join(ROOT, "ppls_amd", "csrc")


@pytest.mark.parametrize("san", [None, "thread"])
def test_host_pool_each_piece_once(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "host_pool_check")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", "-I", INC, SRC, "-o", exe]
    if san:
        cmd.insert(1, "-fsanitize=" + san)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode and san:
        pytest.skip("sanitizer runtime unavailable: " + r.stderr[-400:])
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, "600" if san else "3000"], capture_output=True, text=True, timeout=300, env=env)
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    assert r.stdout.startswith("ok ")
