"""Sanitizer runs on the host code: the kernel's state machine compiled for the
host (tests/hostsim, csrc/fjsp_env.h) and the parity oracle (oracle/fjsp_oracle.c), built
together with AddressSanitizer + UndefinedBehaviorSanitizer (no recovery: the first report
aborts), step 256 envs x 400 steps side by side with random and masked-random actions and
auto-resets, plus a stress configuration, and must agree byte for byte.  GPU code is not
sanitized (no GPU ASan on this pool)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-ffp-contract=off", "-fsanitize=address,undefined",
       "-fno-sanitize-recover=all"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_hostsim_and_oracle_under_asan_ubsan(tmp_path):
    obj = tmp_path / "oracle.o"
    exe = tmp_path / "san_main"
    subprocess.run(["gcc", *SAN, "-c", os.path.join(REPO, "oracle", "fjsp_oracle.c"), "-o", str(obj)], check=True)
    subprocess.run(["g++", *SAN, "-std=c++17", "-Wno-unknown-pragmas", os.path.join(REPO, "tests", "hostsim", "san_main.cpp"),
                    str(obj), "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="abort_on_error=1:detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), "256", "400"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "OK" in r.stdout and "mismatches" in r.stdout
    print(r.stdout)
