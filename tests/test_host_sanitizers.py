"""Host C++ under AddressSanitizer+UBSan and ThreadSanitizer.  GPU sanitizers are
not available on this pool; the native host code (draw generator, multithreaded CSV loader) is
built into a standalone driver with each sanitizer and run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "tests", "native", "host_sanity.cpp"),
        os.path.join(ROOT, "csrc", "host", "datagen.cpp"), os.path.join(ROOT, "csrc", "host", "csv_loader.cpp")]


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_host_code_under_sanitizer(tmp_path, san):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "host_sanity")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}", "-pthread",
           "-I", os.path.join(ROOT, "csrc", "host")] + SRCS + ["-o", exe]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0 and "cannot find" in (p.stderr or ""):
        pytest.skip(f"sanitizer runtime for {san} not installed")
    assert p.returncode == 0, p.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, str(tmp_path / "s.csv")], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "host_sanity ok" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr[-3000:]
