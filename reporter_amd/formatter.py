"""Formatter: the reference's raw-message formatter, native.

Python face of libotmatch's otm_formatter_* (include/otmatch.h), which
restates src/main/java/org/opentraffic/reporter/Formatter.java in C++
(reporter_amd/csrc/formatter.cpp).  Mirrors its interface: GetFormatter(spec)
from the --formatter string (Reporter.java:33-43), format(message) returning
(key, point) or raising where the Java throws -- KeyedFormattingProcessor
(:30-37) drops those messages.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import lib


def pack_messages(messages):
    """[bytes | str] -> (flat uint8 buffer, int64 offsets)."""
    mb = [m.encode("utf-8") if isinstance(m, str) else bytes(m) for m in messages]
    off = np.zeros(len(mb) + 1, np.int64)
    if mb:
        np.cumsum([len(m) for m in mb], out=off[1:])
    buf = np.frombuffer(b"".join(mb) or b"\0", np.uint8)
    return buf, off


class Formatter(object):
    def __init__(self, spec):
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = lib().otm_formatter_create(spec.encode("utf-8"), C.byref(h), err, 512)
        if rc != 0:
            raise ValueError(err.value.decode("utf-8", "replace") or "formatter spec rejected")
        self.h = h

    @classmethod
    def GetFormatter(cls, spec):  # noqa: N802 (the reference's name)
        return cls(spec)

    def __del__(self):
        if getattr(self, "h", None):
            lib().otm_formatter_destroy(self.h)
            self.h = None

    def format_many(self, messages, nthreads=1):
        """dict of arrays: ok, lat, lon, accuracy, time, and keys (list of str, None where dropped)."""
        buf, off = pack_messages(messages)
        r = _lib.Formatted()
        rc = lib().otm_format(self.h, len(off) - 1, buf.ctypes.data, off.ctypes.data, nthreads, C.byref(r))
        if rc != 0:
            raise RuntimeError("otm_format failed (%d)" % rc)
        try:
            n = r.n

            def arr(p, ct, dt):
                return np.ctypeslib.as_array(C.cast(p, C.POINTER(ct)), (n,)).astype(dt) if n else np.zeros(0, dt)
            ok = arr(r.ok, C.c_uint8, np.uint8).astype(bool)
            koff = np.ctypeslib.as_array(C.cast(r.key_off, C.POINTER(C.c_int64)), (n + 1,)).copy()
            kb = C.string_at(r.keys, int(koff[-1])) if n else b""
            keys = [kb[koff[i]:koff[i + 1]].decode("utf-8", "surrogateescape") if ok[i] else None for i in range(n)]
            return {"ok": ok, "keys": keys, "lat": arr(r.lat, C.c_float, np.float32),
                    "lon": arr(r.lon, C.c_float, np.float32), "accuracy": arr(r.accuracy, C.c_int32, np.int32),
                    "time": arr(r.time, C.c_int64, np.int64)}
        finally:
            lib().otm_formatted_free(C.byref(r))

    def format(self, message):
        """Formatter.format: (key, (lat, lon, accuracy, time)); ValueError where the reference throws."""
        r = self.format_many([message])
        if not r["ok"][0]:
            raise ValueError("message not formattable")
        return r["keys"][0], (r["lat"][0], r["lon"][0], int(r["accuracy"][0]), int(r["time"][0]))
