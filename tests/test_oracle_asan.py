"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

The reference's Debug build compiles its core with -fsanitize=address,undefined
(reference CMakeLists.txt:97-105).  Our host-side restatement of that core (oracle/cog_oracle.c)
deliberately reproduces u8 wrap-around and flat-DeckObs scans; this test runs it
over the golden trace scenarios (oracle/gen_golden.py traces(): stored-mask driver with
auto-resets, B-start seeds, 2/3/4 players, selected-mask loop) built with both sanitizers and
-fno-sanitize-recover, and checks that nothing is reported and that every output record hashes
the same as in the plain build (oracle/asan_harness.c, `make -C oracle asan`).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
ASAN_ENV = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0",
                UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def harness():
    r = subprocess.run(["make", "-s", "-C", ORACLE, "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("no sanitizer toolchain: " + r.stderr[-400:])
    return os.path.join(ORACLE, "_asan", "harness"), os.path.join(ORACLE, "_asan", "harness_asan")


def test_sanitizer_is_live(harness):
    _, asan = harness
    r = subprocess.run([asan, "--selftest"], capture_output=True, text=True, env=ASAN_ENV, timeout=60)
    assert r.returncode != 0
    assert "runtime error" in r.stderr or "AddressSanitizer" in r.stderr


def test_oracle_clean_under_asan_ubsan(harness):
    plain, asan = harness
    p = subprocess.run([plain], capture_output=True, text=True, timeout=300)
    a = subprocess.run([asan], capture_output=True, text=True, env=ASAN_ENV, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert a.returncode == 0, a.stderr[-2000:]
    assert "runtime error" not in a.stderr and "AddressSanitizer" not in a.stderr, a.stderr[-2000:]
    lines = a.stdout.split("\n")
    assert len([ln for ln in lines if ln.strip()]) == 7
    assert a.stdout == p.stdout                            # same outputs, every step, every record
    resets = {ln.split()[0]: int(ln.split()[2]) for ln in lines if ln.strip()}
    assert resets["stored_hard_ms30"] > 0 and resets["stored_medium_ms40_bstart"] > 0   # auto-resets ran
