"""Host-side sanitizer run of native code.  GPU ASan is not available on this
pool, so the pure-C++ CSV formatting core is built with -fsanitize=address,undefined and
fuzzed (tools/csv_fuzz.cpp); the same header is compiled into fairify_amd/_C."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_csv_format_core_asan_ubsan(tmp_path):
    exe = str(tmp_path / "csv_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-I" + os.path.join(ROOT, "fairify_amd", "csrc"), os.path.join(ROOT, "tools", "csv_fuzz.cpp"), "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    r = subprocess.run([exe, "50000"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "csv_fuzz: ok" in r.stdout


def _build(tmp_path, name, san, extra=()):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-pthread", *extra,
           "-I" + os.path.join(ROOT, "fairify_amd", "csrc"), os.path.join(ROOT, "tools", "exact_tsan.cpp"), "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_exact_checker_and_csv_core_thread_sanitizer(tmp_path):
    """The BaB runtime's native exact confirmation (csrc/exact_host.h), shared by 8 host threads,
    and the CSV core under -fsanitize=thread; a deliberately racy build must be reported."""
    exe = _build(tmp_path, "exact_tsan", "thread")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([exe, "8", "2000"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout and "ThreadSanitizer" not in r.stderr
    bad = _build(tmp_path, "exact_tsan_selftest", "thread", ["-DFA_TSAN_SELFTEST"])
    r = subprocess.run([bad, "8", "200"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 66 and "data race" in r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_exact_checker_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "exact_asan", "address,undefined", ["-fno-sanitize-recover=all"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    r = subprocess.run([exe, "8", "2000"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
