"""Tier-1 native test of the C++ coordinator under ThreadSanitizer and
AddressSanitizer+UBSan (host code only; SURVEY.md §5 "Race detection")."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENG = os.path.join(ROOT, "csrc", "engine")
SRCS = [os.path.join(ENG, f) for f in ("controller.cc", "wire.cc", "timeline.cc")] + \
    [os.path.join(ENG, "tests", "test_controller.cpp")]


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_controller_under_sanitizer(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "test_controller")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}",
                        "-fno-omit-frame-pointer", "-I", ENG, *SRCS, "-o", exe, "-lpthread"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1",
               ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "4"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_ring_under_sanitizer(tmp_path, san):
    """CPU ring data plane (csrc/engine/ring.cc): 4 ranks as threads over loopback."""
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "test_ring")
    srcs = [os.path.join(ENG, f) for f in ("ring.cc", "wire.cc")] + \
        [os.path.join(ENG, "tests", "test_ring.cpp")]
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}",
                        "-fno-omit-frame-pointer", "-I", ENG, *srcs, "-o", exe, "-lpthread"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1",
               ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "4"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr
