"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 "race /
memory checks"; GPU sanitizers are not available on this pool): tests/sanitize/san_main.cpp
drives the C oracle (oracle/reacher_ref.c, OpenMP) and the product's host-only C++
(reacherdistilation_amd/csrc/gym_seed.cpp), built with -fsanitize=address,undefined and no
recovery, so any report fails the run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
       "-fopenmp"]


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None, reason="needs gcc/g++")
def test_host_code_under_asan_ubsan(tmp_path):
    ref_o, gym_o, exe = tmp_path / "ref.o", tmp_path / "gym.o", tmp_path / "san"
    subprocess.check_call(["gcc", *SAN, "-std=c11", "-c", os.path.join(ROOT, "oracle", "reacher_ref.c"),
                           "-o", str(ref_o)])
    subprocess.check_call(["g++", *SAN, "-std=c++17", "-c",
                           os.path.join(ROOT, "reacherdistilation_amd", "csrc", "gym_seed.cpp"), "-o", str(gym_o)])
    subprocess.check_call(["g++", *SAN, "-std=c++17", os.path.join(ROOT, "tests", "sanitize", "san_main.cpp"),
                           str(ref_o), str(gym_o), "-lm", "-o", str(exe)])
    env = dict(os.environ, OMP_NUM_THREADS="2",
               # the sanitizer runtime need not be first in the library list here; leaks are
               # reported at exit like any other error
               ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "san ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
