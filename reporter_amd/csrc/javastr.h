// javastr.h -- the Java String <-> bytes conversions on the /report transport.
//
// The reference's bytes pass through three JDK 8 charset steps before the
// service sees them (openjdk-8, Dockerfile:17-21,31):
//   * Kafka's StringDeserializer (kafka-clients 0.10.2.1, pom.xml:14) turns a
//     record key into a String: new String(bytes, "UTF8"), malformed input
//     replaced by U+FFFD (JDK 8 sun.nio.cs.UTF_8.Decoder, ArrayDecoder path);
//   * StringSerializer writes a String back: getBytes("UTF8"), an unpaired
//     surrogate replaced by '?' (UTF_8.Encoder, ArrayEncoder path);
//   * HttpClient.POST sends the /report body through new StringEntity(body)
//     (HttpClient.java:26), whose default content type is text/plain with
//     ISO-8859-1 (httpcore 4.4, httpclient 4.5.3 at pom.xml:50): every
//     character above U+00FF -- a surrogate pair counts as one -- becomes '?'.
// The uuid is the record key, appended to the body unescaped (Batch.java:55),
// so a key with a character in U+0080..U+00FF reaches reporter_service.py as
// a lone Latin-1 byte and its body.decode('utf-8') fails
// (py/reporter_service.py:99): a 400, not a match.
#pragma once
#include <string>
#include <string_view>

namespace otm {
namespace jstr {

// new String(bytes, UTF_8) of JDK 8 (REPLACE): UTF-16 code units
std::u16string utf8_decode(std::string_view b);
// String.getBytes(UTF_8) of JDK 8 (REPLACE): unpaired surrogates -> '?'
std::string utf8_encode(std::u16string_view s);
// String.getBytes(ISO_8859_1) of JDK 8 (REPLACE): above U+00FF -> '?', a
// surrogate pair -> one '?'
std::string latin1_encode(std::u16string_view s);

// A record key as the Java host holds it, written back out: the key bytes
// through StringDeserializer and StringSerializer.  Returns false (and leaves
// *out alone) when that is the key itself -- every well-formed UTF-8 key.
bool kafka_key(std::string_view raw, std::string* out);
// Generalised UTF-8 (a surrogate code point encoded as ED A0..BF 80..BF, as a
// JSON \uD800 escape decodes) -> the bytes StringSerializer writes for that
// String: each surrogate sequence becomes '?'.  false when there is none.
bool wtf8_key(std::string_view s, std::string* out);
// The key's bytes inside the /report body as HttpClient sends them
// (latin1_encode(utf8_decode(key))).
std::string key_on_wire(std::string_view key);
// True when a body carrying this wire key parses as the batcher's own bytes
// would: valid UTF-8 (body.decode('utf-8')) and nothing json.loads reads
// differently inside a string (no '"', '\\' or control character).
bool wire_key_plain(std::string_view wire);
// String.compareTo of two keys given as UTF-8 (UTF-16 code unit order):
// TreeMap order of the batcher's store (BatchingProcessor.java:120-130)
int compare(std::string_view a, std::string_view b);

}  // namespace jstr
}  // namespace otm
