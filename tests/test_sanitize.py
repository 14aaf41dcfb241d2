"""CPU sanitizer runs (the committed record is profiles/r02/sanitize_r02.log):
the oracle, and the reference libsecp256k1 where its tree exists, under ASan + UBSan driven by
oracle/sanitize_main.c; and, when `make -C eges_amd/csrc asan` has been run, libeges's host code
under the same sanitizers through tools/sanitize_host.cpp (host-only paths here, no GPU)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_oracle_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize", "N=12", "NO_REPLAY=1"], capture_output=True,
                       text=True, env=ENV, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout and "ERROR: AddressSanitizer" not in r.stderr


def test_libeges_host_code_under_asan_ubsan():
    exe = os.path.join(ROOT, "tools", "asan", "sanitize_host")
    if not os.path.exists(exe):
        pytest.skip("host-ASan build absent (make -C eges_amd/csrc asan)")
    env = dict(ENV, HIP_VISIBLE_DEVICES="-1")  # host-only paths, whatever the machine has
    r = subprocess.run([exe, "3000"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
