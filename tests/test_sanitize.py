"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5,
race detection / sanitizers row): tests/sanitize_driver.cpp linked with the
C oracle (oracle/csg_oracle.c) and the host writers (csrc/csg_io.cpp), built
with -fsanitize=address,undefined (no recovery) and run on a synthetic scene
with the edge cases of both.  GPU code is not sanitized (not available on the
GPU pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
def test_oracle_and_writers_clean_under_asan_ubsan(tmp_path):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
    obj = str(tmp_path / "oracle.o")
    subprocess.run(["gcc", "-c", "-std=c11", "-ffp-contract=off", "-fopenmp"] + san +
                   [os.path.join(ROOT, "oracle", "csg_oracle.c"), "-o", obj], check=True)
    exe = str(tmp_path / "sanitize_driver")
    subprocess.run(["g++", "-std=c++17", "-fopenmp", f'-DSAN_TMPDIR="{tmp_path}"'] + san +
                   [os.path.join(ROOT, "tests", "sanitize_driver.cpp"),
                    os.path.join(ROOT, "constructionsceneposeestimation_amd", "csrc", "csg_io.cpp"), obj,
                    "-lz", "-lm", "-o", exe], check=True)
    # (verify_asan_link_order=0: the environment may preload a library of its own)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="2")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize driver ok" in r.stdout
    for name in ("a.png", "b.png", "m.npy", "d.csv", "p.txt", "l.json", "l2.json"):
        assert (tmp_path / name).stat().st_size > 0
