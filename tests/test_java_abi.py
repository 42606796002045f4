"""The committed Java hosts against the C ABI they bind, with
no JDK and no GPU: tests/native/abi_java_layouts.c, compiled here with gcc
against libotmatch.so, prints every struct the Java MemoryLayouts describe
(size and field offsets) and drives the native formatter + batcher the way
OtmBatcher.java / OtmJni's batcher calls do.

* layouts: parsed out of integration/java/.../OtmMatcher.java and
  OtmBatcher.java (the FFM MemoryLayouts, explicit padding included) and
  compared field by field with the C compiler's offsetof / sizeof; every
  member also sits at its natural alignment, which FFM's structLayout
  requires (it throws at class initialisation otherwise);
* batcher: the C program's forwarded records equal the Python face's
  (reporter_amd.batcher over the same library calls) on the same stream;
* compact: an otm_batch_compact filled as OtmMatcher.matchCompact fills it is
  refused without an engine (OTM_EINVAL) -- the call reads the struct the
  layout describes and returns without touching a device."""
import json
import os
import re
import shutil
import subprocess

import pytest

from reporter_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "integration", "java", "org", "opentraffic", "reporter")
SIZES = {"JAVA_BYTE": 1, "JAVA_SHORT": 2, "JAVA_CHAR": 2, "JAVA_INT": 4, "JAVA_FLOAT": 4, "JAVA_LONG": 8,
         "JAVA_DOUBLE": 8, "ADDRESS": 8}
# Java layout constant -> C struct (include/otmatch.h)
STRUCTS = {"BATCH_COMPACT": "otm_batch_compact", "RESULTS": "otm_results", "TRACE_RESULT": "otm_trace_result",
           "SEGMENT": "otm_segment", "REPORT_REC": "otm_report_rec", "RESULT": "otm_result",
           "FORWARD": "otm_forward", "BATCHER_CFG": "otm_batcher_cfg"}


def split_top(args):
    out, depth, cur = [], 0, ""
    for ch in args:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def java_layouts():
    """{NAME: (size, {field: offset})} from the FFM structLayout declarations."""
    out = {}
    for fn in ("OtmMatcher.java", "OtmBatcher.java"):
        src = open(os.path.join(JAVA, fn)).read()
        for m in re.finditer(r"static final MemoryLayout (\w+)\s*=\s*MemoryLayout\.structLayout\(", src):
            i, depth = m.end(), 1
            j = i
            while depth:
                depth += {"(": 1, ")": -1}.get(src[j], 0)
                j += 1
            off, fields = 0, {}
            for el in split_top(src[i:j - 1]):
                pm = re.fullmatch(r"MemoryLayout\.paddingLayout\((\d+)\)", el)
                if pm:
                    off += int(pm.group(1))
                    continue
                vm = re.fullmatch(r'ValueLayout\.(\w+)\.withName\("(\w+)"\)', el)
                assert vm, "unparsed layout element %r in %s" % (el, m.group(1))
                size = SIZES[vm.group(1)]
                assert off % size == 0, "%s.%s misaligned (FFM would throw)" % (m.group(1), vm.group(2))
                fields[vm.group(2)] = off
                off += size
            out[m.group(1)] = (off, fields)
    return out


@pytest.fixture(scope="module")
def c_run(tmp_path_factory):
    gcc = shutil.which("gcc")
    if not gcc:
        pytest.skip("no gcc")
    exe = str(tmp_path_factory.mktemp("abi") / "abi_java_layouts")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run([gcc, "-O1", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "abi_java_layouts.c"), "-L", libdir, "-lotmatch",
                    "-Wl,-rpath," + libdir, "-Wl,--allow-shlib-undefined", "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, check=True).stdout
    return json.loads(out)


def test_java_layouts_match_the_c_structs(c_run):
    jl = java_layouts()
    assert set(STRUCTS) <= set(jl), set(STRUCTS) - set(jl)
    for jname, cname in STRUCTS.items():
        size, fields = jl[jname]
        c = c_run["layouts"][cname]
        assert size == c["size"], "%s: Java %d bytes, C %d" % (jname, size, c["size"])
        assert fields == c["fields"], "%s field offsets differ: Java %s C %s" % (jname, fields, c["fields"])


def stream():
    """The C program's stream (make_stream in abi_java_layouts.c)."""
    msgs, ts, m = [], [], 0
    for k in range(48):
        for v in range(6):
            t = 1500000000 + 10 * k + v
            if m % 37 == 36:
                msgs.append("not json %d" % m)
            else:
                msgs.append('{"timestamp":%d,"id":"veh%d","accuracy":%d,"latitude":%.6f,"longitude":%.6f}'
                            % (t, v, 5 + v, 37.75 + 0.001 * k + 0.01 * v, -122.40 - 0.0005 * k))
            ts.append(t * 1000)
            m += 1
    return msgs, ts


def test_c_host_batcher_equals_python_face(c_run):
    from reporter_amd.batcher import Batcher
    from reporter_amd.formatter import Formatter

    def handler(bodies):
        out = []
        for b in bodies:
            n = b.count(b'"lat"')
            out.append((200, '{"shape_used":%d}' % (n - 12 if n > 12 else 0)))
        return out

    msgs, ts = stream()
    bt = Batcher(handler=handler, threads=3)
    f = Formatter(",json,id,latitude,longitude,timestamp,accuracy")
    half = len(msgs) // 2
    bt.process_raw(f, msgs[:half], ts[:half], nthreads=2)
    bt.process_raw(f, msgs[half:], ts[half:], nthreads=2)
    bt.flush()
    want = sorted(bt.forwarded())
    bt.close()
    st = bt.stats()
    cb = c_run["batcher"]
    assert cb["rc"] == 0 and cb["close_rc"] == 0
    got = sorted((s, k, b) for s, k, b in cb["forwarded"])
    assert len(got) > 100 and got == want
    for k in ("records", "requests", "raw_messages", "raw_dropped", "stored_batches"):
        assert cb["stats"][k] == st[k], k
    assert cb["stats"]["raw_dropped"] == 7


def test_compact_batch_refused_without_engine(c_run):
    assert c_run["compact"]["rc_without_engine"] == -1  # OTM_EINVAL


def test_java_sources_bind_only_declared_calls():
    """Every downcall the FFM classes create and every otm_* call the JNI shim
    makes is a function include/otmatch.h declares (the library exporting each
    is tests/test_host.py's check); the binary and stream paths are bound."""
    from test_host import header_functions
    declared = set(header_functions())
    used = set()
    for fn in ("OtmMatcher.java", "OtmBatcher.java"):
        used |= set(re.findall(r'fn\("(otm_[a-z0-9_]+)"', open(os.path.join(JAVA, fn)).read()))
    jni = open(os.path.join(ROOT, "integration", "jni", "otmatch_jni.c")).read()
    used_jni = set(re.findall(r"\b(otm_[a-z0-9_]+)\s*\(", jni))
    assert used <= declared and used_jni <= declared
    for need in ("otm_match_compact", "otm_host_alloc", "otm_batcher_create", "otm_batcher_process_raw",
                 "otm_batcher_take", "otm_batcher_close", "otm_formatter_create"):
        assert need in used, need
        assert need in used_jni or need == "otm_host_alloc", need
    # every native method OtmJni.java declares has its JNI function in the shim
    natives = re.findall(r"native\s+[\w\[\]]+\s+(\w+)\(", open(os.path.join(JAVA, "OtmJni.java")).read())
    for nm in natives:
        assert "Java_org_opentraffic_reporter_OtmJni_%s(" % nm in jni, nm
