"""reporter_amd -- MI355X-native /report matcher for Open Traffic Reporter.

The product is libotmatch.so (HIP kernels for gfx950 behind a C ABI,
include/otmatch.h).  This package is its Python host face:

  Engine           one GPU + its HBM-resident graph (engine.py)
  valhalla         drop-in for the `valhalla` module reporter_service.py
                   imports (Configure / SegmentMatcher().Match)
  reporter_service the /report request handler on the native path
  synth            seeded synthetic graphs and traces (harness tooling)
"""
from .engine import Engine, OtmError, Results, encode_request, murmur2_partition, report_segments, write_config

__all__ = ["Engine", "OtmError", "Results", "encode_request", "murmur2_partition", "report_segments",
           "write_config"]
