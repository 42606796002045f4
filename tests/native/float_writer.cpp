// Prints "<%a of d> <put_float(d)>" for random doubles (all bit patterns, and
// values over a wide exponent range) so tests/test_float_writer.py can compare
// the response writer's float text with json.dumps / float.__repr__.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "json.h"

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 100000;
  std::mt19937_64 g(7);
  for (int k = 0; k < n; ++k) {
    const uint64_t b = g();
    double d;
    if (k % 3 == 0) {
      std::memcpy(&d, &b, 8);
    } else {
      d = std::ldexp((double)(b >> 11), (int)(g() % 200) - 150);
      if (g() & 1) d = -d;
    }
    std::string s;
    otm::json::put_float(d, &s);
    std::printf("%a %s\n", d, s.c_str());
  }
  return 0;
}
