"""Drop-in for the `valhalla` module py/reporter_service.py imports (:21).

reporter_service.py calls exactly three things of the Valhalla 2.2.7 Python
binding: valhalla.Configure(conf_path) (:279), valhalla.SegmentMatcher()
once per worker thread (:52) and SegmentMatcher.Match(json_str) (:112).  Put
this module ahead of the real binding on sys.path (as `valhalla`, or import
reporter_amd.valhalla and alias it) and the service runs unmodified on the
GPU engine: Configure creates one engine (graph + distance index in HBM) for
the process, every SegmentMatcher shares it (the engine is thread-safe), and
Match returns the {"segments":[...]} JSON of otm_match_json.  A matcher error
raises, and report() turns it into its 500 body (:239-240).

Configure takes the engine config file (include/otmatch.h,
otm_engine_create): {"otm":{"graph":...},"meili":{"default":{...}}}.
"""
import threading

from .engine import Engine

_lock = threading.Lock()
_engine = None


def Configure(path):  # noqa: N802 -- the binding's name (py/reporter_service.py:279)
    # A second Configure does not close the engine earlier SegmentMatchers
    # hold (a Match may be running on it): each matcher keeps its engine
    # alive, and the old engine is freed when the last of them goes away.
    global _engine
    with _lock:
        _engine = Engine(config_path=path)


def _current():
    if _engine is None:
        raise RuntimeError("valhalla.Configure was not called")
    return _engine


class SegmentMatcher(object):
    """valhalla.SegmentMatcher() (py/reporter_service.py:52)."""

    def __init__(self):
        self._eng = _current()

    def Match(self, s):  # noqa: N802 -- the binding's name (:112)
        code, body = self._eng.match_json(s)
        if code != 200:
            raise RuntimeError(body)
        return body
