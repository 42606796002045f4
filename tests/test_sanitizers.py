"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer.

The CPU oracle (oracle/, C) and libotmatch's host C++ (the C ABI, JSON,
report(), the request reader, batcher, formatter, tile math, synthetic inputs) are rebuilt with
-fsanitize=address,undefined (`make asan` in oracle/ and reporter_amd/csrc/,
clang for both so one ASan runtime serves the process; GPU sanitizers are not
available on this pool, so device code is not instrumented).  The CPU test
modules then run in a child process with that runtime preloaded and the
sanitized builds selected (OTM_LIB / OTM_ORACLE_LIB).  Any ASan or UBSan
report aborts the child (halt_on_error) and is written to the log this test
reads.
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_LIB = os.path.join(ROOT, "reporter_amd", "lib", "asan", "libotmatch.so")
ASAN_ORACLE = os.path.join(ROOT, "oracle", "build", "asan", "libotm_oracle.so")
MODULES = ["tests/test_golden.py", "tests/test_host.py", "tests/test_formatter.py", "tests/test_batcher.py",
           "tests/test_tiles.py", "tests/test_fast_request.py", "tests/test_transport.py"]


def _runtime():
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return rt[-1] if rt else None


@pytest.mark.slow
def test_host_code_is_clean_under_asan_and_ubsan(tmp_path):
    rt = _runtime()
    if rt is None:
        pytest.skip("clang ASan runtime not found")
    jobs = str(min(8, os.cpu_count() or 2))
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "reporter_amd", "csrc"), "asan", "-j", jobs])
    # the builds really are instrumented
    for lib in (ASAN_LIB, ASAN_ORACLE):
        syms = subprocess.run(["nm", "-D", lib], capture_output=True, text=True).stdout
        assert "__asan_report_load" in syms and "__ubsan_handle" in syms, lib
    log = str(tmp_path / "san")
    env = dict(os.environ)
    env.update(LD_PRELOAD=rt, OTM_LIB=ASAN_LIB, OTM_ORACLE_LIB=ASAN_ORACLE,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:log_path=" + log,
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:log_path=" + log)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu"] + MODULES,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1500)
    reports = "".join(open(f).read() for f in glob.glob(log + "*"))
    assert not reports, reports[:4000]
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout


TSAN_LIB = os.path.join(ROOT, "reporter_amd", "lib", "tsan", "libotmatch.so")
TSAN_MODULES = ["tests/test_batcher.py", "tests/test_formatter.py", "tests/test_host.py", "tests/test_fast_request.py"]


@pytest.mark.slow
def test_host_threads_are_clean_under_tsan(tmp_path):
    """The host C++ under ThreadSanitizer (`make tsan`): the batcher's thread
    team, the formatter's threads and the host pool (OTM_HOST_THREADS=4), with
    the runtime preloaded into a child pytest; any data race report fails."""
    rts = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.tsan-x86_64.so"))
    if not rts:
        pytest.skip("clang TSan runtime not found")
    jobs = str(min(8, os.cpu_count() or 2))
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "reporter_amd", "csrc"), "tsan", "-j", jobs])
    syms = subprocess.run(["nm", "-D", TSAN_LIB], capture_output=True, text=True).stdout
    assert "__tsan_write" in syms or "__tsan_read" in syms
    log = str(tmp_path / "tsan")
    env = dict(os.environ)
    env.update(LD_PRELOAD=rts[-1], OTM_LIB=TSAN_LIB, OTM_HOST_THREADS="4",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0:log_path=" + log)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu"]
                       + TSAN_MODULES, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1500)
    reports = "".join(open(f).read() for f in glob.glob(log + "*"))
    assert not reports, reports[:4000]
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout
