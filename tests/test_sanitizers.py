"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer and ThreadSanitizer (SURVEY
§5: the reference's one concurrency primitive is the CAS loop of log.clj:5-11; the oracle's is the
pthread pool over cluster chunks). A fuzz batch runs in a child process with the sanitizer
runtime preloaded; any report fails the test."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
BUILD = ROOT / "oracle" / "build"


def runtime(name):
    out = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True)
    p = out.stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.parametrize("kind,lib,rt", [("asan", "libraftref_asan.so", "libasan.so"),
                                         ("tsan", "libraftref_tsan.so", "libtsan.so")])
def test_oracle_fuzz_under_sanitizer(kind, lib, rt):
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "sanitize"], check=True)
    pre = runtime(rt)
    if pre is None:
        pytest.skip(f"{rt} not available")
    env = dict(os.environ, LD_PRELOAD=pre,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0")
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "sanitize_driver.py"),
                        str(BUILD / lib), "7"], env=env, capture_output=True, text=True,
                       timeout=600)
    report = r.stderr[-4000:]
    assert r.returncode == 0 and "sanitize driver ok" in r.stdout, report
    for marker in ("AddressSanitizer", "runtime error:", "ThreadSanitizer"):
        assert marker not in r.stderr, report
