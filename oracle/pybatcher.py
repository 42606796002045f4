"""Serial restatement of the reference's Kafka Streams batcher (TEST INFRASTRUCTURE).

The checker for libotmatch's otm_batcher (reporter_amd/csrc/batcher.cpp): the
same semantics, written straight from the Java, one record at a time, with
the matcher called synchronously -- exactly how the reference runs.  Only
tests/ import it.

  Batch               src/main/java/org/opentraffic/reporter/Batch.java:16-84
  Point.Serder        src/main/java/org/opentraffic/reporter/Point.java:29,39-45
  BatchingProcessor   src/main/java/org/opentraffic/reporter/BatchingProcessor.java:19-133

Java float arithmetic is reproduced with numpy float32; DecimalFormat
("###.######", HALF_EVEN, JDK 8+ exact-value rounding) with decimal.Decimal.
One deliberate divergence, shared with the native batcher: where the reference
would throw a NullPointerException in clean() (a popped key with no stored
batch), the key is counted and skipped.  Math.cos is the platform libm here;
the JVM's may differ in the last ulp (only a distance exactly at a gate could
notice).
"""
import json
import math
from collections import deque
from decimal import ROUND_HALF_EVEN, Context, Decimal

import numpy as np

f32 = np.float32
RAD_PER_DEG = math.pi / 180.0
METERS_PER_DEG = 20037581.187 / 180.0


def decimal6(v):
    """DecimalFormat("###.######") of a float (Point.java:29)."""
    d = Decimal(float(f32(v))).quantize(Decimal("0.000001"), rounding=ROUND_HALF_EVEN, context=Context(prec=400))
    s = format(d, "f")
    neg = s.startswith("-")
    if neg:
        s = s[1:]
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    if s.startswith("0.") and len(s) > 1:
        s = s[1:]
    return ("-" if neg else "") + s


class Point(object):
    __slots__ = ("lat", "lon", "accuracy", "time")

    def __init__(self, lat, lon, accuracy, time):
        self.lat, self.lon, self.accuracy, self.time = f32(lat), f32(lon), int(accuracy), int(time)


def distance(a, b):
    """Batch.distance (Batch.java:34-38)."""
    x = float(f32(a.lon - b.lon)) * METERS_PER_DEG * math.cos(float(f32(f32(0.5) * f32(a.lat + b.lat))) * RAD_PER_DEG)
    y = float(f32(a.lat - b.lat)) * METERS_PER_DEG
    return math.sqrt(x * x + y * y)


def find_value(node, name):
    """Jackson JsonNode.findValue: a node's own fields first, then depth-first."""
    if isinstance(node, dict):
        if name in node:
            return node[name]
        for v in node.values():
            r = find_value(v, name)
            if r is not None:
                return r
    elif isinstance(node, list):
        for v in node:
            r = find_value(v, name)
            if r is not None:
                return r
    return None


class Batch(object):
    def __init__(self, p=None):
        self.max_separation = f32(0.0)
        self.points = [] if p is None else [p]

    def update(self, p):
        if self.points:
            self.max_separation = f32(max(float(self.max_separation), distance(p, self.points[0])))
        self.points.append(p)

    def body(self, key):
        parts = ['{"lat":%s,"lon":%s,"time":%d,"accuracy":%d}' % (decimal6(p.lat), decimal6(p.lon), p.time,
                                                                  p.accuracy) for p in self.points]
        # HttpClient.POST sends it through new StringEntity(body) (HttpClient.java:26):
        # ISO-8859-1, '?' for a character above U+00FF (one per code point: a Java
        # surrogate pair is one Python character)
        return ('{"uuid":"' + key + '","trace":[' + ",".join(parts) + "]}").encode("latin-1", "replace")

    def report(self, key, post, min_dist, min_size, min_elapsed):
        if (float(self.max_separation) < min_dist or len(self.points) < min_size or
                self.points[-1].time - self.points[0].time < min_elapsed):
            return None
        response = post(self.body(key))
        try:
            node = json.loads(response)
            su = find_value(node, "shape_used")
            trim_to = len(self.points) if su is None else int(su)
            if trim_to < 0 or trim_to > len(self.points):
                raise IndexError(trim_to)
            del self.points[:trim_to]
            self.max_separation = f32(0.0)
            for i in range(1, len(self.points)):
                self.max_separation = f32(max(float(self.max_separation), distance(self.points[i], self.points[0])))
        except Exception:
            self.max_separation = f32(0.0)
            self.points = []
        return response


class BatchingProcessor(object):
    REPORT_TIME, REPORT_COUNT, REPORT_DIST, SESSION_GAP = 60, 10, 500, 60000

    def __init__(self, post):
        """post(body_bytes) -> response str (the HttpClient.POST of Batch.java:63)."""
        self.post = post
        self.store = {}
        self.time_to_key = deque()
        self.forwarded = []  # (seq, key, response)
        self.null_batch_in_clean = 0
        self.requests = 0
        self._seq = 0

    def _post(self, body):
        self.requests += 1
        return self.post(body)

    def process(self, key, point, ts):
        self.clean(key, ts)
        batch = self.store.pop(key, None)
        if batch is None:
            batch = Batch(point)
        else:
            batch.update(point)
            result = batch.report(key, self._post, self.REPORT_DIST, self.REPORT_COUNT, self.REPORT_TIME)
            if result is not None:
                self.forwarded.append((self._seq, key, result))
        if batch.points:
            self.store[key] = batch
        # else: time_to_key.remove(iter) -- removes nothing in the reference
        self._seq += 1

    def clean(self, key, ts):
        while self.time_to_key and ts - self.time_to_key[0][0] > self.SESSION_GAP:
            _, k = self.time_to_key.popleft()
            b = self.store.get(k)
            if b is None:  # the reference's store.get returns null here -> NullPointerException
                self.null_batch_in_clean += 1
                continue
            b.report(k, self._post, 0, 2, 0)
        self.time_to_key.append((ts, key))

    def close(self):
        # in-memory store = TreeMap: String.compareTo order, i.e. UTF-16 code units
        for k in sorted(self.store, key=lambda x: x.encode("utf-16-be", "surrogatepass")):
            self.store[k].report(k, self._post, 0, 2, 0)
