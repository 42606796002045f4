// report.h -- reporter_service.py's request/response layer on the host.
#pragma once
#include <string>
#include <vector>

#include "json.h"
#include "otm_internal.h"
#include "otmatch.h"

namespace otm {

// parse_trace + handle_request validation (py/reporter_service.py:85-106,
// :218-234).  Returns 0 with *trace filled, or the HTTP code with *resp set.
int parse_request(const char* path, std::string_view body, json::Value* trace, std::string* resp);

// report() (py/reporter_service.py:110-215) over any matcher output, with
// Python value semantics.  Returns true and *resp, or false and *exc =
// str(exception).  *stderr_text gets "Speed exceeds 200kph\n" per invalid speed.
bool report_dom(const ReportConfig& rc, const json::Value& trace, json::Value* segments, std::string* resp,
                std::string* stderr_text, std::string* exc);

// Points of a parsed request for the matcher (the Match input contract).
struct TracePoints {
  std::vector<float> lat, lon, acc;
  std::vector<double> time;
};
bool extract_points(const json::Value& trace, TracePoints* out, std::string* err);
// The Java batcher's request bytes (Batch.java:52-61, Point.java:39-45) read
// straight into points, without a DOM: {"uuid":"<printable ASCII>","trace":[
// {"lat":n,"lon":n,"time":n[,"accuracy":n]}, ... >= 2 points]} with the keys
// in any order, each once, no whitespace, plain numbers (no exponent, ints of
// at most 18 digits).  Returns false (and the caller takes parse_request +
// extract_points) on anything else, so every accepted body gives exactly the
// points, uuid and outcome of the DOM path.
bool fast_request(std::string_view body, TracePoints* out, std::string* uuid);

// Typed writers over one trace of a results set.
void write_match_json(const otm_results& r, int32_t t, std::string* out);
// Full /report response for trace t; returns the HTTP code.  matcher_json:
// the "segment_matcher" value to write verbatim (the Match output passed
// through, mode added), or null for the typed segments of r.
int write_report_response(const otm_results& r, int32_t t, std::string* out,
                          const std::string* matcher_json = nullptr);
// A Match output (and the request's last time) as typed segment records for
// k_report: false with *why when a field has a JSON type the matcher never
// emits (Python's exceptions for those are the host report_dom's).
bool typed_segments(const json::Value& trace, const json::Value& match, std::vector<otm_segment>* out,
                    double* end_time, std::string* why);
const char* trace_error_text(int kind);

std::string error_body(const std::string& msg);

// Java DecimalFormat("###.######") of a float (Point.java:29,41-42)
void java_decimal6(float f, std::string* o);
// Batch.report's body (Batch.java:52-61, Point.java:39-45) with the uuid
// given as its bytes on the wire (javastr.h key_on_wire); *out is replaced
void encode_request(std::string_view wire_uuid, int n, const float* lat, const float* lon, const int64_t* time,
                    const int32_t* accuracy, std::string* out);

}  // namespace otm
