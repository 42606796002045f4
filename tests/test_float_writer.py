"""The float text of every response (otm::json::put_float, reporter_amd/csrc/
json.cpp) against json.dumps of the same double -- float.__repr__'s shortest
round-trip digits and its fixed / exponent switch, as the reference's
json.dumps writes them (py/reporter_service.py:215).  A small native harness
(tests/native/float_writer.cpp) is compiled against json.cpp with g++."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "reporter_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not found")
def test_put_float_is_json_dumps(tmp_path):
    exe = str(tmp_path / "float_writer")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", CSRC, os.path.join(ROOT, "tests", "native", "float_writer.cpp"),
                           os.path.join(CSRC, "json.cpp"), "-o", exe])
    out = subprocess.run([exe, "60000"], capture_output=True, text=True, check=True).stdout.split("\n")
    n = 0
    for line in out:
        if not line:
            continue
        h, s = line.split()
        assert s == json.dumps(float.fromhex(h)), line
        n += 1
    assert n == 60000
