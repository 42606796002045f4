"""Restatement of the reference's raw-message Formatter (TEST INFRASTRUCTURE).

The checker for libotmatch's otm_formatter (reporter_amd/csrc/formatter.cpp),
written independently from the Java it restates; only tests/ import it.

  Formatter.GetFormatter / formatSV / formatJSON
      src/main/java/org/opentraffic/reporter/Formatter.java:36-51, 97-109, 111-124
  KeyedFormattingProcessor.process (drop on any exception)
      src/main/java/org/opentraffic/reporter/KeyedFormattingProcessor.java:30-37

Java library behaviour restated here (no JVM exists in this container, so
this is parity against the documented behaviour, pinned only by the
reference's own format examples -- Reporter.java:35-43, README.md:23-27):
  String.split(regex)        java.util.regex -> Python re (ASCII classes),
                             Pattern.split with limit 0
  DecimalFormat.parse        "###.######", Locale.US, JDK 8 (prefix parse,
                             grouping ',' ignored, 'E' exponent, Long vs Double)
  Double.parseDouble         FloatingDecimal grammar -> float() / float.fromhex
  Double.toString            shortest repr digits, JDK >= 19 rules
  joda DateTimeFormat        y M d H m s S patterns, UTC, default year 2000
  Jackson JsonNode           readTree (first value), get, asText/asLong/asDouble
  Kafka StringDeserializer   new String(bytes, UTF8) of JDK 8 (java_utf8_decode)
  Kafka StringSerializer     String.getBytes(UTF8): an unpaired surrogate -> '?'
"""
import json
import math
import re
import unicodedata
from decimal import Decimal

import numpy as np

f32 = np.float32
LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1
INT_MIN, INT_MAX = -(1 << 31), (1 << 31) - 1


def java_digit(ch):
    """Character.digit(ch, 10) in JDK 8 (Unicode 6.2): BMP decimal digits
    (the two blocks Unicode 7.0 added excluded); -1 otherwise."""
    o = ord(ch)
    if o > 0xFFFF or 0x0DE6 <= o <= 0x0DEF or 0xA9F0 <= o <= 0xA9F9:
        return -1
    return unicodedata.decimal(ch, -1) if unicodedata.category(ch) == "Nd" else -1


def java_utf8_decode(b):
    """new String(bytes, UTF_8) in JDK 8 (sun.nio.cs.UTF_8 ArrayDecoder, REPLACE),
    as a Python str.  Differs from bytes.decode('utf-8', 'replace') on encoded
    surrogates: JDK 8 replaces a whole ED A0..BF xx sequence (or a truncated
    ED A0..BF) with ONE U+FFFD, Python with one per byte."""
    R = "\ufffd"
    out = []
    i, n = 0, len(b)
    while i < n:
        c = b[i]
        i += 1
        if c < 0x80:
            out.append(chr(c))
            continue
        if 0xC2 <= c <= 0xDF:
            if i >= n:
                out.append(R)
                break
            if b[i] & 0xC0 != 0x80:
                out.append(R)
            else:
                out.append(chr(((c & 0x1F) << 6) | (b[i] & 0x3F)))
                i += 1
            continue
        if 0xE0 <= c <= 0xEF:
            if n - i >= 2:
                c2, c3 = b[i], b[i + 1]
                bad2 = (c == 0xE0 and 0x80 <= c2 <= 0x9F) or c2 & 0xC0 != 0x80
                if bad2 or c3 & 0xC0 != 0x80:
                    out.append(R)
                    i += 0 if bad2 else 1
                    continue
                cp = ((c & 0xF) << 12) | ((c2 & 0x3F) << 6) | (c3 & 0x3F)
                out.append(R if 0xD800 <= cp <= 0xDFFF else chr(cp))
                i += 2
                continue
            if i < n and ((c == 0xE0 and 0x80 <= b[i] <= 0x9F) or b[i] & 0xC0 != 0x80):
                out.append(R)
                continue
            out.append(R)
            break
        if 0xF0 <= c <= 0xF7:
            def bad_second(x):
                return c > 0xF4 or (c == 0xF0 and not 0x90 <= x <= 0xBF) or (c == 0xF4 and not 0x80 <= x <= 0x8F) \
                    or x & 0xC0 != 0x80
            if n - i >= 3:
                c2, c3, c4 = b[i], b[i + 1], b[i + 2]
                cp = ((c & 7) << 18) | ((c2 & 0x3F) << 12) | ((c3 & 0x3F) << 6) | (c4 & 0x3F)
                if any(x & 0xC0 != 0x80 for x in (c2, c3, c4)) or not 0x10000 <= cp <= 0x10FFFF:
                    out.append(R)
                    if bad_second(c2):
                        pass
                    elif c3 & 0xC0 != 0x80:
                        i += 1
                    else:
                        i += 2
                    continue
                out.append(chr(cp))
                i += 3
                continue
            if c > 0xF4 or (i < n and bad_second(b[i])):
                out.append(R)
                continue
            i += 1
            if i < n and b[i] & 0xC0 != 0x80:
                out.append(R)
                continue
            out.append(R)
            break
        out.append(R)
    return "".join(out)


def java_serialize_key(s):
    """Kafka StringSerializer's String.getBytes(UTF8), read back: an unpaired
    surrogate (a JSON \\ud800 escape the Formatter kept) becomes '?'."""
    return "".join("?" if 0xD800 <= ord(ch) <= 0xDFFF else ch for ch in s)


def java_latin1(s):
    """String.getBytes(ISO_8859_1) (httpcore StringEntity's default charset,
    HttpClient.java:26): above U+00FF -> '?' (a supplementary character, one
    surrogate pair in Java, is one '?')."""
    return bytes(ord(ch) if ord(ch) <= 0xFF else 0x3F for ch in s)


class Drop(Exception):
    """The reference throws; KeyedFormattingProcessor drops the message."""


class SpecError(Exception):
    """GetFormatter throws (or the restatement does not support the spec)."""


# ------------------------------------------------------------ java.lang
def d2i(d):
    if math.isnan(d):
        return 0
    if d >= INT_MAX:
        return INT_MAX
    if d <= INT_MIN:
        return INT_MIN
    return int(d)


def d2l(d):
    if math.isnan(d):
        return 0
    if d >= 9223372036854775807.0:
        return LONG_MAX
    if d <= -9223372036854775808.0:
        return LONG_MIN
    return int(d)


def java_trim(s):
    a, b = 0, len(s)
    while a < b and ord(s[a]) <= 32:
        a += 1
    while b > a and ord(s[b - 1]) <= 32:
        b -= 1
    return s[a:b]


def parse_long(s, lo=LONG_MIN, hi=LONG_MAX):
    """Long.parseLong / Integer.parseInt (digits by Character.digit)."""
    neg = s[:1] == "-"
    body = s[1:] if s[:1] in ("-", "+") else s
    if not body:
        raise ValueError(s)
    v = 0
    for ch in body:
        d = java_digit(ch)
        if d < 0:
            raise ValueError(s)
        v = v * 10 + d
    v = -v if neg else v
    if v < lo or v > hi:
        raise ValueError(s)
    return v


_DEC_RE = re.compile(r"([+-]?)((?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?)[fFdD]?\Z")
_HEX_RE = re.compile(r"([+-]?)0[xX]((?:[0-9a-fA-F]+\.?|[0-9a-fA-F]*\.[0-9a-fA-F]+)[pP][+-]?[0-9]+)[fFdD]?\Z")


def parse_double(s):
    """Double.parseDouble."""
    s = java_trim(s)
    m = re.match(r"([+-]?)(NaN|Infinity)\Z", s)
    if m:
        if m.group(2) == "NaN":
            return math.nan
        return -math.inf if m.group(1) == "-" else math.inf
    m = _HEX_RE.match(s)
    if m:
        body = m.group(2)
        v = float.fromhex("0x" + body)
        return -v if m.group(1) == "-" else v
    m = _DEC_RE.match(s)
    if m:
        v = float(m.group(2))
        return -v if m.group(1) == "-" else v
    raise ValueError(s)


def double_to_string(d):
    """Double.toString."""
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "-Infinity" if d < 0 else "Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    t = Decimal(repr(abs(d))).normalize().as_tuple()  # shortest round-trip digits
    digits = "".join(map(str, t.digits))
    x = len(digits) + t.exponent - 1  # value = d.ddd x 10^x
    if len(digits) == 1:  # one digit competes with the closest two-digit decimal
        m2, _, e2 = ("%.1e" % abs(d)).partition("e")
        digits = m2.replace(".", "").rstrip("0") or "0"
        x = int(e2)
    sign = "-" if d < 0 else ""
    a = abs(d)
    if 1e-3 <= a < 1e7:
        if x >= 0:
            ipart = (digits + "0" * (x + 1))[:x + 1]
            fpart = digits[x + 1:] or "0"
            return sign + ipart + "." + fpart
        return sign + "0." + "0" * (-x - 1) + digits
    return sign + digits[0] + "." + (digits[1:] or "0") + "E" + str(x)


# -------------------------------------------------------- DecimalFormat
def decimal_format_parse(text):
    """DecimalFormat("###.######", Locale.US).parse(text).floatValue()."""
    if text.startswith("�"):
        return f32(math.nan)
    i, neg = 0, False
    if text.startswith("-"):
        neg, i = True, 1
    if text[i:i + 1] == "∞":
        return f32(-math.inf if neg else math.inf)
    sig = ""          # significant digits
    int_digits = None  # significant digits before the point (None: no point yet)
    lead_frac_zeros = 0
    saw_digit = False
    exponent = 0
    n = len(text)
    while i < n:
        ch = text[i]
        dg = java_digit(ch)
        if dg >= 0:
            saw_digit = True
            if dg == 0 and not sig:
                if int_digits is not None:
                    lead_frac_zeros += 1
            else:
                sig += str(dg)
        elif ch == ".":
            if int_digits is not None:
                break
            int_digits = len(sig)
        elif ch == ",":
            if int_digits is not None:
                break
        elif ch == "E":
            j = i + 1
            eneg = text[j:j + 1] == "-"
            j += eneg
            ed = ""
            while j < n and java_digit(text[j]) >= 0:
                ed += str(java_digit(text[j]))
                j += 1
            m = (None, "-" if eneg else "", ed) if ed else None
            if m:
                ev = int(m[2])
                if ev <= (1 << 63) - (0 if m[1] else 1):
                    ev = -ev if m[1] else ev
                    exponent = ((ev + (1 << 31)) % (1 << 32)) - (1 << 31)  # (int) narrowing
            break
        else:
            break
        i += 1
    if not saw_digit:
        raise Drop("ParseException")
    if int_digits is None:
        int_digits = len(sig)
    # decimalAt as a Java int
    decimal_at = int_digits - lead_frac_zeros + exponent
    decimal_at = ((decimal_at + (1 << 31)) % (1 << 32)) - (1 << 31)
    sig = sig.rstrip("0")
    if not sig:
        return f32(-0.0) if neg else f32(0.0)
    if len(sig) <= decimal_at <= 19:
        iv = int(sig + "0" * (decimal_at - len(sig)))
        if (-iv if neg else iv) >= LONG_MIN and (-iv if neg else iv) <= LONG_MAX:
            v = -iv if neg else iv
            return _int_to_f32(v)
    d = float(Decimal(("-" if neg else "") + "0." + sig + "E" + str(decimal_at)))
    with np.errstate(over="ignore"):
        return f32(d)  # (float) of a double beyond float range is +-Infinity


def _int_to_f32(v):
    """(float) of a long: one rounding, to nearest even."""
    if v == 0:
        return f32(0.0)
    a = abs(v)
    if a < (1 << 24):
        r = float(a)
    else:
        shift = a.bit_length() - 24
        q, rem = divmod(a, 1 << shift)
        half = 1 << (shift - 1)
        if rem > half or (rem == half and q & 1):
            q += 1
        r = float(q << shift)
    return f32(-r if v < 0 else r)


# ------------------------------------------------------------- regex
def java_regex_to_python(p):
    """The supported java.util.regex subset as a Python pattern (re.ASCII)."""
    out = []
    i = 0
    while i < len(p):
        c = p[i]
        if c == "\\":
            if i + 1 >= len(p):
                raise SpecError("separator regex ends in a backslash")
            e = p[i + 1]
            if e in "dDsSwW":
                out.append("\\" + e)
                i += 2
            elif e in "tnrfae":
                out.append({"t": "\\t", "n": "\\n", "r": "\\r", "f": "\\f", "a": "\\x07", "e": "\\x1b"}[e])
                i += 2
            elif e == "x" and re.match(r"[0-9a-fA-F]{2}", p[i + 2:i + 4]):
                out.append(re.escape(chr(int(p[i + 2:i + 4], 16))))
                i += 4
            elif e == "u" and re.match(r"[0-9a-fA-F]{4}", p[i + 2:i + 6]):
                out.append(re.escape(chr(int(p[i + 2:i + 6], 16))))
                i += 6
            elif e.isalnum():
                raise SpecError("unsupported escape")
            else:
                out.append(re.escape(e))
                i += 2
            continue
        if c == ".":
            out.append("[^\\n\\r\\u0085\\u2028\\u2029]")
            i += 1
            continue
        if c == "[":
            j = p.find("]", i + 2)
            if j < 0:
                raise SpecError("unclosed class")
            body = p[i + 1:j]
            if "[" in body or "&&" in body or body in ("", "^"):
                raise SpecError("unsupported class")
            out.append("[" + body + "]")
            i = j + 1
            continue
        if c in "|()^$*+?{":
            raise SpecError("unsupported metacharacter")
        out.append(re.escape(c))
        i += 1
        if i < len(p) and p[i] in "*+?{":
            m = re.match(r"[*+?]|\{[0-9]+(,[0-9]*)?\}", p[i:])
            if not m:
                raise SpecError("bad repetition")
            out.append(m.group(0))
            i += len(m.group(0))
            if i < len(p) and p[i] in "?+":
                raise SpecError("lazy/possessive")
    pat = "".join(out)
    # quantifiers after classes / escapes
    return pat


def compile_split(regex):
    # quantifiers directly after escapes / classes are handled by re itself:
    # translate atom by atom, then append whatever quantifier follows
    atoms = []
    i = 0
    p = regex
    while i < len(p):
        j = i
        if p[j] == "\\":
            j += 2
            if p[i + 1] == "x":
                j += 2
            elif p[i + 1] == "u":
                j += 4
        elif p[j] == "[":
            j = p.find("]", j + 2) + 1
            if j == 0:
                raise SpecError("unclosed class")
        else:
            j += 1
        atom = java_regex_to_python(p[i:j])
        i = j
        m = re.match(r"[*+?]|\{[0-9]+(,[0-9]*)?\}", p[i:])
        q = ""
        if m:
            q = m.group(0)
            i += len(q)
            if i < len(p) and p[i] in "?+":
                raise SpecError("lazy/possessive")
        atoms.append((atom, q))
    def lo(q):
        if q in ("*", "?"):
            return 0
        m = re.match(r"\{([0-9]+)", q)
        return int(m.group(1)) if m else 1
    if all(lo(q) == 0 for _, q in atoms):
        raise SpecError("separator regex can match the empty string")
    return re.compile("".join(a + q for a, q in atoms), re.ASCII)


def java_split(rx, text):
    """Pattern.split(text, 0) for a pattern that cannot match empty."""
    parts = []
    index = 0
    for m in rx.finditer(text):
        parts.append(text[index:m.start()])
        index = m.end()
    if index == 0:
        return [text]
    parts.append(text[index:])
    while parts and parts[-1] == "":
        parts.pop()
    return parts


# ------------------------------------------------------------- joda
_NUMERIC = set("cCxyYdhHmsSeDFwWkK")


def compile_time_pattern(pattern):
    toks = []
    i, n = 0, len(pattern)
    while i < n:
        c = pattern[i]
        if c.isascii() and c.isalpha():
            j = i
            while j + 1 < n and pattern[j + 1] == c:
                j += 1
            toks.append(("F", c * (j - i + 1)))
            i = j + 1
            continue
        lit, in_lit = "", False
        while i < n:
            d = pattern[i]
            if d == "'":
                if i + 1 < n and pattern[i + 1] == "'":
                    lit += "'"
                    i += 2
                    continue
                in_lit = not in_lit
            elif not in_lit and d.isascii() and d.isalpha():
                break
            else:
                lit += d
            i += 1
        toks.append(("L", lit))
    out = []
    for k, (kind, tok) in enumerate(toks):
        if kind == "L":
            if tok:
                out.append(("L", tok, 0))
            continue
        nxt_numeric = k + 1 < len(toks) and toks[k + 1][0] == "F" and (
            toks[k + 1][1][0] in _NUMERIC or (toks[k + 1][1][0] == "M" and len(toks[k + 1][1]) <= 2))
        c, ln = tok[0], len(tok)
        if c == "y":
            if ln == 2:
                raise SpecError("yy")
            out.append(("y", ln, ln if nxt_numeric else 9))
        elif c == "M":
            if ln > 2:
                raise SpecError("MMM")
            out.append(("M", ln, 2))
        elif c in "dHms":
            out.append((c, ln, 2))
        elif c == "S":
            out.append(("S", ln, min(ln, 18)))
        else:
            raise SpecError("letter " + c)
    return out


def _days_in_month(y, m):
    if m == 2:
        return 29 if (y % 4 == 0 and y % 100 != 0) or y % 400 == 0 else 28
    return [31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31][m - 1]


def _epoch_days(y, m, d):
    # days since 1970-01-01 in the proleptic Gregorian calendar (any year)
    def days_before_year(yy):  # days from 0000-01-01 to yy-01-01
        yy -= 1
        return 365 * (yy + 1) + yy // 4 - yy // 100 + yy // 400 + 1
    cum = [0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334]
    leap = (y % 4 == 0 and y % 100 != 0) or y % 400 == 0
    doy = cum[m - 1] + (1 if leap and m > 2 else 0) + d - 1
    return days_before_year(y) + doy - days_before_year(1970)


def parse_time(fmt, text):
    pos = 0
    saved = []
    rank = {"y": 0, "M": 1, "d": 2, "H": 3, "m": 4, "s": 5, "S": 6}
    for kind, a, b in fmt:
        if kind == "L":
            if text[pos:pos + len(a)].lower() != a.lower():
                raise Drop("literal")
            pos += len(a)
            continue
        if kind == "S":
            m = re.match(r"[0-9]{1,%d}" % b, text[pos:])
            if not m:
                raise Drop("fraction")
            ds = m.group(0)
            saved.append((6, int((ds + "000")[:3])))
            pos += len(ds)
            continue
        pat = r"[+-]?[0-9]{1,%d}" % b if kind == "y" else r"[0-9]{1,%d}" % b
        m = re.match(pat, text[pos:])
        if not m:
            raise Drop("number")
        saved.append((rank[kind], int(m.group(0))))
        pos += len(m.group(0))
    if pos != len(text):
        raise Drop("trailing")
    saved.sort(key=lambda t: t[0])  # stable
    y, mo, d, H, mi, s, ms = 1970, 1, 1, 0, 0, 0, 0
    if saved and saved[0][0] in (1, 2):
        y = 2000
    for r, v in saved:
        if r == 0:
            if not -292275054 <= v <= 292278993:
                raise Drop("year")
            y, mo, d, H, mi, s, ms = v, 1, 1, 0, 0, 0, 0
        elif r == 1:
            if not 1 <= v <= 12:
                raise Drop("month")
            mo, d, H, mi, s, ms = v, 1, 0, 0, 0, 0
        elif r == 2:
            if not 1 <= v <= _days_in_month(y, mo):
                raise Drop("day")
            d, H, mi, s, ms = v, 0, 0, 0, 0
        elif r == 3:
            if not 0 <= v <= 23:
                raise Drop("hour")
            H, mi, s, ms = v, 0, 0, 0
        elif r == 4:
            if not 0 <= v <= 59:
                raise Drop("minute")
            mi, s, ms = v, 0, 0
        elif r == 5:
            if not 0 <= v <= 59:
                raise Drop("second")
            s, ms = v, 0
        else:
            ms = v
    millis = _epoch_days(y, mo, d) * 86400000 + H * 3600000 + mi * 60000 + s * 1000 + ms
    q = abs(millis) // 1000
    return -q if millis < 0 else q


# ----------------------------------------------------------- Jackson
class _Big(int):
    pass


def _no_constants(name):
    raise ValueError(name)


_DECODER = json.JSONDecoder(parse_constant=_no_constants)


def read_tree(s):
    i = 0
    while i < len(s) and s[i] in " \t\n\r":
        i += 1
    try:
        v, _ = _DECODER.raw_decode(s, i)
    except ValueError:
        raise Drop("JsonParseException")
    return v


def as_text(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return double_to_string(v)
    if isinstance(v, str):
        return v
    if v is None:
        return "null"
    return ""


def as_long(v):
    if isinstance(v, bool):
        return 1 if v else 0
    if isinstance(v, int):
        if LONG_MIN <= v <= LONG_MAX:
            return v
        low = v & ((1 << 64) - 1)  # BigInteger.longValue
        return low - (1 << 64) if low >= (1 << 63) else low
    if isinstance(v, float):
        return d2l(v)
    if isinstance(v, str):
        s = java_trim(v)
        if not s:
            return 0
        if s[0] == "+":
            s = s[1:]
            body = s
        else:
            body = s[1:] if s[0] == "-" else s
        if any(not ("0" <= c <= "9") for c in body):
            try:
                return d2l(parse_double(s))
            except ValueError:
                return 0
        try:
            return parse_long(s)
        except ValueError:
            return 0
    return 0


def as_double(v):
    if isinstance(v, bool):
        return 1.0 if v else 0.0
    if isinstance(v, int):
        return float(v)
    if isinstance(v, float):
        return v
    if isinstance(v, str):
        s = java_trim(v)
        if not s:
            return 0.0
        try:
            return parse_double(s)
        except ValueError:
            return 0.0
    return 0.0


# ------------------------------------------------------------ Formatter
class Formatter(object):
    def __init__(self, spec):
        """Formatter.GetFormatter."""
        if not spec:
            raise SpecError("empty spec")
        split_on, rest = spec[0], spec[1:]
        args = java_split(compile_split(split_on), rest)
        if not args:
            raise SpecError("too few arguments")
        pattern = None
        if args[0] == "sv":
            if len(args) < 7:
                raise SpecError("too few arguments")
            self.sv = True
            self.rx = compile_split(args[1])
            try:
                self.idx = [parse_long(a, INT_MIN, INT_MAX) for a in args[2:7]]
            except ValueError:
                raise SpecError("NumberFormatException")
            pattern = args[7] if len(args) > 7 else None
        elif args[0] == "json":
            if len(args) < 6:
                raise SpecError("too few arguments")
            self.sv = False
            self.keys = args[1:6]
            pattern = args[6] if len(args) > 6 else None
        else:
            raise SpecError("Unsupported raw format parser")
        self.time_fmt = compile_time_pattern(pattern) if pattern is not None else None

    def format(self, message):
        """Formatter.format: bytes -> (key, lat, lon, accuracy, time); Drop if the reference throws."""
        if isinstance(message, bytes):
            message = java_utf8_decode(message)
        return self._sv(message) if self.sv else self._json(message)

    def _sv(self, msg):
        parts = java_split(self.rx, msg)
        u, la, lo, t, a = self.idx
        for k in (u, la, lo, t, a):
            if k < 0 or k >= len(parts):
                raise Drop("ArrayIndexOutOfBoundsException")
        lat = decimal_format_parse(parts[la])
        lon = decimal_format_parse(parts[lo])
        if self.time_fmt is not None:
            time = parse_time(self.time_fmt, parts[t])
        else:
            try:
                time = parse_long(parts[t])
            except ValueError:
                raise Drop("NumberFormatException")
        av = float(decimal_format_parse(parts[a]))
        acc = 0 if math.isnan(av) else d2i(av if math.isinf(av) else float(math.ceil(av)))
        return parts[u], lat, lon, acc, time

    def _json(self, msg):
        node = read_tree(msg)
        if not isinstance(node, dict):
            raise Drop("NullPointerException")
        uk, lak, lok, tk, ak = self.keys
        for k in (uk, lak, lok, tk, ak):
            if k not in node:
                raise Drop("NullPointerException")
        lat = decimal_format_parse(as_text(node[lak]))
        lon = decimal_format_parse(as_text(node[lok]))
        if self.time_fmt is not None:
            time = parse_time(self.time_fmt, as_text(node[tk]))
        else:
            time = as_long(node[tk])
        d = as_double(node[ak])
        if math.isnan(d):
            acc = 0
        elif math.isinf(d):
            acc = d2i(d)
        else:
            acc = d2i(float(math.ceil(d)))
        return java_serialize_key(as_text(node[uk])), lat, lon, acc, time
