"""Batcher: the reference's Kafka Streams batching processor, native.

Python face of libotmatch's otm_batcher_* (include/otmatch.h), which restates
BatchingProcessor (src/main/java/org/opentraffic/reporter/BatchingProcessor.java)
and Batch (Batch.java) in C++.  Mirrors the processor's interface: process()
per formatted record (key, Point, record timestamp), close(), and the records
it forwards downstream (context.forward(key, response), :70-71).

The matcher is the engine (GPU batches of every key that is ready), or any
/report handler: a callable taking a list of request bodies and returning
(code, body) pairs -- the HttpClient.POST of Batch.java:63 -- or None when the
call failed as a whole (every request then gets HttpClient's null response).
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import lib


class KeyBlock(object):
    """Record keys packed for otm_batcher_process (char* array + lengths), so a
    caller replaying a stream can pay the conversion once."""

    def __init__(self, keys):
        kb = [k.encode("utf-8") if isinstance(k, str) else k for k in keys]
        self.n = len(kb)
        self._keep = kb
        self.arr = (C.c_char_p * self.n)(*kb)
        self.lens = (C.c_size_t * self.n)(*[len(k) for k in kb])


class Batcher(object):
    def __init__(self, engine=None, handler=None, json_path=False, max_batch=0, native_handler=None, **cfg):
        """native_handler: (callback address, context address) of a C
        otm_report_fn, called by the batcher without Python in between."""
        if engine is None and handler is None and native_handler is None:
            raise ValueError("engine or handler required")
        L = lib()
        c = _lib.BatcherCfg()
        L.otm_batcher_defaults(C.byref(c))
        for k, v in cfg.items():
            setattr(c, k, v)
        c.max_batch = max_batch
        c.json_path = 1 if json_path else 0
        self._handler = handler
        ctx = None
        if native_handler is not None:
            self._cb = _lib.REPORT_FN(native_handler[0])
            ctx = native_handler[1]
        else:
            self._cb = _lib.REPORT_FN(self._call) if handler is not None else _lib.REPORT_FN()
        h = C.c_void_p()
        rc = L.otm_batcher_create(engine.h if engine is not None else None, C.byref(c), self._cb, ctx, C.byref(h))
        if rc != 0:
            raise RuntimeError("otm_batcher_create failed (%d)" % rc)
        self.h = h

    def _call(self, ctx, n, reqs, lens, resps, resp_lens, codes):
        bodies = [C.string_at(reqs[i], lens[i]) for i in range(n)]
        out = self._handler(bodies)
        if out is None:
            return 1  # the whole call failed (a transport failure: null responses)
        for i, (code, body) in enumerate(out):
            b = body.encode("utf-8") if isinstance(body, str) else body
            resps[i] = _lib.malloc_bytes(b)
            resp_lens[i] = len(b)
            codes[i] = code
        return 0

    def close_handle(self):
        if getattr(self, "h", None):
            lib().otm_batcher_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close_handle()

    def process(self, keys, lat, lon, accuracy, time, ts_ms):
        """Records in stream order (BatchingProcessor.process); keys: strings,
        bytes or a KeyBlock."""
        kb = keys if isinstance(keys, KeyBlock) else KeyBlock(keys)
        n, arr, lens = kb.n, kb.arr, kb.lens
        lat = np.ascontiguousarray(lat, np.float32)
        lon = np.ascontiguousarray(lon, np.float32)
        acc = np.ascontiguousarray(accuracy, np.int32)
        tm = np.ascontiguousarray(time, np.int64)
        ts = np.ascontiguousarray(ts_ms, np.int64)
        rc = lib().otm_batcher_process(self.h, n, arr, lens, lat.ctypes.data, lon.ctypes.data, acc.ctypes.data,
                                       tm.ctypes.data, ts.ctypes.data)
        if rc != 0:
            raise RuntimeError("otm_batcher_process failed (%d)" % rc)

    def process_raw(self, formatter, messages, ts_ms, nthreads=1):
        """Raw messages through the formatter into the batcher (the
        KeyedFormattingProcessor -> BatchingProcessor topology, Reporter.java:95-103)."""
        from .formatter import pack_messages
        buf, off = pack_messages(messages)
        ts = np.ascontiguousarray(ts_ms, np.int64)
        if len(ts) != len(off) - 1:
            raise ValueError("one record timestamp per message")
        rc = lib().otm_batcher_process_raw(self.h, formatter.h, len(ts), buf.ctypes.data, off.ctypes.data,
                                           ts.ctypes.data, nthreads)
        if rc != 0:
            raise RuntimeError("otm_batcher_process_raw failed (%d)" % rc)

    def flush(self):
        if lib().otm_batcher_flush(self.h) != 0:
            raise RuntimeError("otm_batcher_flush failed")

    def close(self):
        """BatchingProcessor.close: relaxed reports of every stored batch."""
        if lib().otm_batcher_close(self.h) != 0:
            raise RuntimeError("otm_batcher_close failed")

    def forwarded(self):
        """[(seq, key, body)] forwarded since the last call."""
        out = []
        buf = (_lib.Forward * 4096)()
        while True:
            n = lib().otm_batcher_take(self.h, buf, 4096)
            for i in range(n):
                f = buf[i]
                key = _lib.take(f.key, f.key_len).decode("utf-8")
                body = _lib.take(f.body, f.body_len).decode("utf-8")
                out.append((f.seq, key, body))
            if n < 4096:
                return out

    def stats(self):
        s = _lib.BatcherStats()
        lib().otm_batcher_get_stats(self.h, C.byref(s))
        return {n: getattr(s, n) for n in _lib.BATCHER_STATS}

    def batch(self, key):
        """(points [(lat, lon, accuracy, time)], max_separation) stored for key, or None."""
        kb = key if isinstance(key, bytes) else key.encode("utf-8")
        ms = C.c_float()
        n = lib().otm_batcher_batch(self.h, kb, len(kb), 0, None, None, None, None, C.byref(ms))
        if n < 0:
            return None
        la, lo = np.zeros(n, np.float32), np.zeros(n, np.float32)
        ac, tm = np.zeros(n, np.int32), np.zeros(n, np.int64)
        lib().otm_batcher_batch(self.h, kb, len(kb), n, la.ctypes.data, lo.ctypes.data, ac.ctypes.data,
                                tm.ctypes.data, C.byref(ms))
        return list(zip(la.tolist(), lo.tolist(), ac.tolist(), tm.tolist())), ms.value
