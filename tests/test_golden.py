"""Golden vectors from the reference itself (tests/golden/make_golden.py).

Both restatements of reporter_service.py's request path -- the CPU oracle (C)
and the product's host layer in libotmatch.so (C++) -- must reproduce every
recorded (status, body, stderr) of the real reporter_service.py, byte for
byte.  CPU only: no matcher runs here (the recorded cases feed canned Match
outputs, as the reference run did through its stub `valhalla` module).
"""
import json
import os

import pytest

from reporter_amd import engine as E

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ENV_KEYS = ("REPORT_LEVELS", "TRANSITION_LEVELS", "THRESHOLD_SEC")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


REPORT_CASES = load("report_cases.json")
REQUEST_CASES = load("request_cases.json")


@pytest.fixture
def clean_env(monkeypatch):
    for k in ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


def _cases():
    return [c for c in REPORT_CASES if c["match_output"] is not None]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: "%s-%s" % (c["name"], "_".join(sorted(c["env"]))))
def test_oracle_report_matches_reference(case, oracle):
    rc = oracle.report_cfg_from_env(case["env"])
    code, body, err = oracle.report_segments(case["request"], case["match_output"], rc)
    assert code == case["code"]
    assert body == case["body"]
    assert err == case["stderr"]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: "%s-%s" % (c["name"], "_".join(sorted(c["env"]))))
def test_product_report_matches_reference(case, clean_env, capfd):
    for k, v in case["env"].items():
        clean_env.setenv(k, v)
    code, body = E.report_segments(case["request"], case["match_output"])
    assert code == case["code"]
    assert body == case["body"]
    out, err = capfd.readouterr()
    assert err == case["stderr"]


def test_matcher_input_is_python_redump(oracle):
    """report() hands Match json.dumps(trace, separators=(',',':'))
    (py/reporter_service.py:112); the oracle's redump reproduces it."""
    for c in REPORT_CASES[:120]:
        if c["match_input"] is None:
            continue
        ok, red = oracle.json_redump(c["request"])
        assert ok and red == c["match_input"]


@pytest.mark.parametrize("case", [c for c in REQUEST_CASES if "path" not in c], ids=lambda c: c["body_hex"][:40])
def test_request_errors(case, oracle, clean_env):
    body = bytes.fromhex(case["body_hex"])
    if case["response"].startswith('{"stats"'):
        pytest.skip("valid request: covered by the matcher tests")
    code, resp, _ = oracle.report_segments(body, '{"segments":[]}')
    assert (code, resp) == (case["code"], case["response"])
    code, resp = E.report_segments(body, '{"segments":[]}')
    assert (code, resp) == (case["code"], case["response"])


def test_action_routing(oracle):
    """parse_trace's action check (py/reporter_service.py:92-96) on the oracle's
    full request path (the matcher is not reached for these)."""
    for c in REQUEST_CASES:
        if "path" not in c:
            continue
        # every recorded case is rejected before the matcher is reached
        code, resp = oracle.handle_request(None, c["body"], path=c["path"])
        assert (code, resp) == (c["code"], c["response"])


def test_env_parsing_quirks(clean_env):
    """make_thread_locals (py/reporter_service.py:55-62): strtobool on
    THRESHOLD_SEC, int() on the level lists.  The product reads them where the
    reference's worker threads would (engine creation / report_segments)."""
    for c in load("env_cases.json"):
        for k in ENV_KEYS:
            clean_env.delenv(k, raising=False)
        for k, v in c["env"].items():
            clean_env.setenv(k, v)
        code, body = E.report_segments('{"uuid":"a","trace":[{"time":1},{"time":2}]}', '{"segments":[]}')
        if "error" in c:
            msg = c["error"].split(": ", 1)[1]
            assert code == 500 and body == '{"error":"%s"}' % msg
        else:
            assert code == 200


def test_decode_polyline6(oracle):
    for c in load("decode_cases.json"):
        assert oracle.decode_polyline6(c["encoded"]) == c["decoded"]


def test_synthesize_gps_restatement():
    """reporter_amd.tracegen.synthesize_gps restates py/generate_test_trace.py:31-73."""
    from reporter_amd import tracegen
    for c in load("synth_cases.json"):
        got = tracegen.synthesize_gps(c["edges"], c["shape"], uuid=c["uuid"], now=c["now"])
        assert got == (c["result"] if not isinstance(c["result"], list) else tuple(c["result"]))
