"""AddressSanitizer + UBSan runs of host code (CPU only; GPU sanitizers are
not available on this pool and no GPU call is made here).

* The front door: trajopt-1_amd/host/tests/json_fuzz.cpp, built with
  -fsanitize=address,undefined (host Makefile target `san`), feeds seeded
  mutations of valid TrajOptRequest documents through Json::parse and
  ConstructProblem -- every input constructs or throws, with no memory or UB
  error.
* The oracle: its known-answer tests (oracle/tests/kat_main.cpp) built with the
  same sanitizers (oracle Makefile target `build/kat_san`).
"""
import os
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
HOST = REPO / "trajopt-1_amd" / "host"
LIB = REPO / "trajopt-1_amd" / "lib"

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _have_asan():
    r = subprocess.run(["g++", "-fsanitize=address,undefined", "-x", "c++", "-", "-o", "/dev/null"],
                       input="int main(){return 0;}", capture_output=True, text=True)
    return r.returncode == 0


pytestmark = pytest.mark.skipif(not _have_asan(), reason="no libasan / libubsan for g++ in this image")


@pytest.fixture(scope="module")
def built():
    import __graft_entry__

    import fcntl

    __graft_entry__.build()
    jobs = str(min(8, os.cpu_count() or 1))
    with open(REPO / ".build.lock", "w") as lock:  # (parallel pytest workers)
        fcntl.flock(lock, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", str(HOST), "-j", jobs, "san"], check=True, capture_output=True, text=True)
        subprocess.run(["make", "-C", str(REPO / "oracle"), "-j", jobs, "build/kat_san"], check=True,
                       capture_output=True, text=True)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True, env=ENV, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_front_door_json_fuzz_under_sanitizers(built, seed):
    out = _run([str(LIB / "json_fuzz_san"), str(seed), "4000"])
    assert "constructed" in out


def test_oracle_kats_under_sanitizers(built):
    out = _run([str(REPO / "oracle" / "build" / "kat_san")])
    assert "fail=0" in out
