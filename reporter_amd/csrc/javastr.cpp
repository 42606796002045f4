// javastr.cpp -- JDK 8 charset steps on the /report transport (javastr.h).
//
// Restated from the published behaviour of openjdk-8's sun.nio.cs.UTF_8 and
// ISO_8859_1 coders on the String(byte[], charset) / String.getBytes(charset)
// paths (the ArrayDecoder / ArrayEncoder fast paths, CodingErrorAction.REPLACE),
// which the reference reaches through Kafka's StringDeserializer /
// StringSerializer and httpcore's StringEntity (HttpClient.java:26).  No JVM
// exists in this image: the cases in tests/test_transport.py are worked by
// hand from those rules and checked against an independent Python restatement
// (oracle/pyformatter.py java_utf8_decode).
#include "javastr.h"

#include <cstdint>

#include "json.h"

namespace otm {
namespace jstr {

namespace {

constexpr char16_t kRepl = 0xFFFD;
inline bool cont(unsigned b) { return (b & 0xC0) == 0x80; }
inline bool surrogate(uint32_t c) { return c >= 0xD800 && c <= 0xDFFF; }

}  // namespace

std::u16string utf8_decode(std::string_view s) {
  std::u16string o;
  o.reserve(s.size());
  const size_t sl = s.size();
  size_t sp = 0;
  auto at = [&](size_t i) { return (unsigned)(unsigned char)s[i]; };
  while (sp < sl) {
    const unsigned b1 = at(sp++);
    if (b1 < 0x80) {
      o.push_back((char16_t)b1);
    } else if (b1 >= 0xC2 && b1 <= 0xDF) {  // 110xxxxx 10xxxxxx (C0/C1 fall to the last branch)
      if (sp < sl) {
        const unsigned b2 = at(sp);
        if (!cont(b2)) {
          o.push_back(kRepl);  // b2 is read again
        } else {
          o.push_back((char16_t)(((b1 & 0x1F) << 6) | (b2 & 0x3F)));
          ++sp;
        }
        continue;
      }
      o.push_back(kRepl);
      return o;
    } else if (b1 >= 0xE0 && b1 <= 0xEF) {  // 1110xxxx 10xxxxxx 10xxxxxx
      if (sp + 1 < sl) {
        const unsigned b2 = at(sp), b3 = at(sp + 1);
        const bool overlong = b1 == 0xE0 && (b2 & 0xE0) == 0x80;
        if (overlong || !cont(b2) || !cont(b3)) {
          o.push_back(kRepl);
          sp += (overlong || !cont(b2)) ? 0 : 1;  // malformedN: length 1 or 2 from b1
          continue;
        }
        const uint32_t c = ((b1 & 0x0F) << 12) | ((b2 & 0x3F) << 6) | (b3 & 0x3F);
        o.push_back(surrogate(c) ? kRepl : (char16_t)c);  // a surrogate: one U+FFFD for all 3 bytes
        sp += 2;
        continue;
      }
      // truncated at the end: at most one byte follows
      if (sp < sl && ((b1 == 0xE0 && (at(sp) & 0xE0) == 0x80) || !cont(at(sp)))) {
        o.push_back(kRepl);  // that byte is read again
        continue;
      }
      o.push_back(kRepl);
      return o;
    } else if (b1 >= 0xF0 && b1 <= 0xF7) {  // 11110xxx + 3 continuation bytes
      if (sp + 2 < sl) {
        const unsigned b2 = at(sp), b3 = at(sp + 1), b4 = at(sp + 2);
        const uint32_t uc = ((b1 & 0x07) << 18) | ((b2 & 0x3F) << 12) | ((b3 & 0x3F) << 6) | (b4 & 0x3F);
        if (!cont(b2) || !cont(b3) || !cont(b4) || uc < 0x10000 || uc > 0x10FFFF) {
          o.push_back(kRepl);
          // malformedN(4)
          if (b1 > 0xF4 || (b1 == 0xF0 && (b2 < 0x90 || b2 > 0xBF)) || (b1 == 0xF4 && (b2 & 0xF0) != 0x80) ||
              !cont(b2))
            sp += 0;
          else if (!cont(b3))
            sp += 1;
          else
            sp += 2;
          continue;
        }
        const uint32_t v = uc - 0x10000;
        o.push_back((char16_t)(0xD800 + (v >> 10)));
        o.push_back((char16_t)(0xDC00 + (v & 0x3FF)));
        sp += 3;
        continue;
      }
      // truncated at the end: at most two bytes follow
      if (b1 > 0xF4 ||
          (sp < sl && ((b1 == 0xF0 && (at(sp) < 0x90 || at(sp) > 0xBF)) ||
                       (b1 == 0xF4 && (at(sp) & 0xF0) != 0x80) || !cont(at(sp))))) {
        o.push_back(kRepl);
        continue;
      }
      ++sp;
      if (sp < sl && !cont(at(sp))) {
        o.push_back(kRepl);
        continue;
      }
      o.push_back(kRepl);
      return o;
    } else {  // 80..C1, F8..FF
      o.push_back(kRepl);
    }
  }
  return o;
}

std::string utf8_encode(std::u16string_view s) {
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    const uint32_t c = s[i];
    if (c < 0x80) {
      o.push_back((char)c);
    } else if (c < 0x800) {
      o.push_back((char)(0xC0 | (c >> 6)));
      o.push_back((char)(0x80 | (c & 0x3F)));
    } else if (surrogate(c)) {
      if (c <= 0xDBFF && i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
        const uint32_t uc = 0x10000 + ((c - 0xD800) << 10) + ((uint32_t)s[i + 1] - 0xDC00);
        o.push_back((char)(0xF0 | (uc >> 18)));
        o.push_back((char)(0x80 | ((uc >> 12) & 0x3F)));
        o.push_back((char)(0x80 | ((uc >> 6) & 0x3F)));
        o.push_back((char)(0x80 | (uc & 0x3F)));
        ++i;
      } else {
        o.push_back('?');
      }
    } else {
      o.push_back((char)(0xE0 | (c >> 12)));
      o.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (c & 0x3F)));
    }
  }
  return o;
}

std::string latin1_encode(std::u16string_view s) {
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    const uint32_t c = s[i];
    if (c <= 0xFF) {
      o.push_back((char)c);
      continue;
    }
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) ++i;
    o.push_back('?');
  }
  return o;
}

namespace {
bool ascii(std::string_view s) {
  for (char c : s)
    if ((unsigned char)c >= 0x80) return false;
  return true;
}
}  // namespace

bool kafka_key(std::string_view raw, std::string* out) {
  if (ascii(raw)) return false;
  std::string w = utf8_encode(utf8_decode(raw));
  if (w.size() == raw.size() && std::string_view(w) == raw) return false;
  *out = std::move(w);
  return true;
}

bool wtf8_key(std::string_view s, std::string* out) {
  bool any = false;
  for (size_t i = 0; i + 2 < s.size(); ++i)
    if ((unsigned char)s[i] == 0xED && (unsigned char)s[i + 1] >= 0xA0) {
      any = true;
      break;
    }
  if (!any) return false;
  out->clear();
  for (size_t i = 0; i < s.size();) {
    if (i + 2 < s.size() && (unsigned char)s[i] == 0xED && (unsigned char)s[i + 1] >= 0xA0 &&
        (unsigned char)s[i + 1] <= 0xBF && cont((unsigned char)s[i + 2])) {
      out->push_back('?');
      i += 3;
    } else {
      out->push_back(s[i++]);
    }
  }
  return true;
}

std::string key_on_wire(std::string_view key) {
  if (ascii(key)) return std::string(key);
  return latin1_encode(utf8_decode(key));
}

bool wire_key_plain(std::string_view w) {
  bool hi = false;
  for (char ch : w) {
    const unsigned char c = (unsigned char)ch;
    if (c < 0x20 || c == '"' || c == '\\') return false;
    if (c >= 0x80) hi = true;
  }
  // bytes.decode('utf-8'): Latin-1 bytes that happen to be well-formed UTF-8
  // ("\xC3\xA9" for the key "Ã©") decode; anything else is a 400
  return !hi || json::utf8_error(w).empty();
}

int compare(std::string_view a, std::string_view b) {
  if (ascii(a) && ascii(b)) return a.compare(b) < 0 ? -1 : (a == b ? 0 : 1);
  const std::u16string x = utf8_decode(a), y = utf8_decode(b);
  return x.compare(y) < 0 ? -1 : (x == y ? 0 : 1);
}

}  // namespace jstr
}  // namespace otm
