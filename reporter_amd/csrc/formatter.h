// formatter.h -- the reference's raw-message Formatter, native.
//
// Restates src/main/java/org/opentraffic/reporter/Formatter.java (GetFormatter
// :36-51, formatSV :97-109, formatJSON :111-124) with the Java library
// semantics it leans on: String.split (java.util.regex, limit 0),
// DecimalFormat("###.######", Locale.US).parse (JDK 8), joda-time
// DateTimeFormat patterns (2.9.9, UTC), Jackson 2.8 JsonNode.asText / asLong /
// asDouble, Math.ceil and Java's narrowing casts.  A message whose formatting
// throws is dropped, as KeyedFormattingProcessor.process (:30-37) logs and
// drops it.
//
// Supported subsets (anything else fails loudly at create time, never per
// message): separator regexes of literals, escapes, . \d \s \w (and negations),
// [classes] and greedy * + ? {n,m} quantifiers that cannot match empty;
// time patterns of y (not yy), M/MM, d, H, m, s, S and literals.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace otm {

struct FormattedPoint {
  float lat = 0.0f, lon = 0.0f;
  int32_t accuracy = 0;
  int64_t time = 0;
};

class Formatter {
 public:
  // Formatter.GetFormatter; false + *err on a spec the reference rejects or
  // this restatement does not support
  bool init(const std::string& spec, std::string* err);
  // Formatter.format; false where the reference throws (message dropped)
  bool format(std::string_view msg, std::string* key, FormattedPoint* pt) const;

  struct Re;  // compiled separator regex
  struct TimeTok {
    char field;  // 0 = literal, else y M d H m s S
    int len;     // token length (S: fraction digits, y: min digits)
    int max_digits;
    std::string lit;
  };

 private:
  bool sv_ = true;
  std::vector<std::shared_ptr<Re>> re_;
  int uuid_i_ = 0, lat_i_ = 0, lon_i_ = 0, time_i_ = 0, acc_i_ = 0;
  std::string uuid_k_, lat_k_, lon_k_, time_k_, acc_k_;
  bool has_time_fmt_ = false;
  std::vector<TimeTok> time_fmt_;
  bool format_sv(std::string_view msg, std::string* key, FormattedPoint* pt) const;
  bool format_json(std::string_view msg, std::string* key, FormattedPoint* pt) const;
};

// pieces with their own tests
bool java_split(std::string_view regex, std::string_view text, std::vector<std::string_view>* parts, std::string* err);
bool decimal_format_parse(std::string_view text, float* out);  // DecimalFormat("###.######").parse(..).floatValue()
bool java_parse_double(std::string_view s, double* out);        // Double.parseDouble
bool java_parse_long(std::string_view s, int64_t* out);         // Long.parseLong
void java_double_to_string(double d, std::string* out);         // Double.toString (shortest digits)

}  // namespace otm
