"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
section 5): tests/cpp/oracle_sanitize.c drives every oracle entry point; the
oracle sources are compiled into it with the sanitizers, so any out-of-bounds
access, use of uninitialised heap memory through ASan's allocator, signed
overflow or other UB aborts the run.  Host code only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(not shutil.which("gcc"), reason="no gcc")
def test_oracle_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_sanitize")
    cmd = ["gcc", "-std=c11", "-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(HERE, "cpp", "oracle_sanitize.c"), os.path.join(ROOT, "oracle", "uwvk_oracle.c"),
           os.path.join(ROOT, "oracle", "uwvk_small_oracle.c"), "-o", exe, "-lm", "-lpthread"]
    subprocess.run(cmd, check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "status 0" in r.stdout, r.stdout + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
