"""Host code under AddressSanitizer + UBSan (CPU only): the C front end
(parser, dedup, patterns tree) and the C++ flattener build both images,
through the image cache, and two bounds-checked host walks of them agree at
every position of the shipped stream plus a synthetic tail
(tests/sanitize/host_check.cpp)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "patternmatching_amd", "csrc")
DATA = os.path.join(REPO, "tests", "golden", "data")
HARNESS = os.path.join(REPO, "tests", "sanitize", "host_check.cpp")


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    if not shutil.which("g++") or not shutil.which("gcc") or not os.path.exists(HARNESS):
        pytest.skip("no host compiler or harness")
    d = tmp_path_factory.mktemp("asan")
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-g", "-O1"]
    inc = ["-I" + os.path.join(REPO, "include"), "-I" + CSRC]
    obj = str(d / "pm_dict.o")
    subprocess.run(["gcc", "-std=gnu11", *san, *inc, "-c", os.path.join(CSRC, "host", "pm_dict.c"), "-o", obj],
                   check=True)
    exe = str(d / "host_check")
    subprocess.run(["g++", "-std=c++17", *san, *inc, HARNESS, os.path.join(CSRC, "pm_flatten.cpp"), obj, "-o", exe],
                   check=True)
    return exe


@pytest.mark.parametrize("dicts", [["et.dict"], ["snort.dict", "et.dict"]])
def test_host_code_clean_under_asan_ubsan(host_check, dicts, tmp_path):
    # verify_asan_link_order=0: the environment may preload a library of its
    # own ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([host_check, str(tmp_path), os.path.join(DATA, "dictionaries_generated.stream")]
                       + [os.path.join(DATA, x) for x in dicts], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.startswith("ok"), r.stdout
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
