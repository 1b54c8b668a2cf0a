"""CPU: AddressSanitizer + UBSan builds of the host-side native code.

SURVEY.md §5 "Race detection / sanitizers": the C oracle (oracle/pathsim_oracle.c)
and the native log writer (csrc/dps_log.cpp) are rebuilt with
-fsanitize=address,undefined and driven by tests/native/*_main.* (random
graphs, both denominators, k beyond the target count; float formatting
round-trips, multi-thread multi-part log writes, argument rejection).
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(shutil.which("make") is None, reason="make not available")


def _run(target_dir, binary, *args):
    subprocess.run(["make", "-s", "asan"], cwd=target_dir, check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(target_dir, binary), *args], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_oracle_asan():
    assert "oracle asan ok" in _run(os.path.join(REPO, "oracle"), "_asan/oracle_asan")


def test_log_writer_asan(tmp_path):
    out = _run(os.path.join(REPO, "distributed-pathsim_amd", "csrc"), "build_asan/log_asan",
               str(tmp_path / "asan.log"))
    assert "log asan ok" in out
