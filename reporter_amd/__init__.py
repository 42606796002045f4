"""reporter_amd -- MI355X-native /report matcher for Open Traffic Reporter.

The product is libotmatch.so (HIP kernels for gfx950 behind a C ABI,
include/otmatch.h).  This package is its Python host face:

  Engine      one GPU + its HBM-resident graph and the /report path (engine.py):
              report / report_batch / submit+poll (handle_request,
              py/reporter_service.py:218-240), match_json (SegmentMatcher.Match,
              :112), match / match_device (binary batches)
  valhalla    drop-in for the `valhalla` module reporter_service.py imports
              (Configure / SegmentMatcher().Match)
  Batcher     the Kafka Streams batcher (BatchingProcessor + Batch), native (batcher.py)
  Formatter   the raw-message formatter (Formatter.java), native (formatter.py)
  flush       the RCCL reduce-scatter of per-segment speed histograms
  datastore   a rank's histogram flush body and POST
  synth, tracegen  seeded synthetic graphs and traces, config-1 requests (harness tooling)
"""
from .engine import (Engine, OtmError, RequestArena, Results, encode_request, murmur2_partition, report_segments,
                     write_config)

__all__ = ["Engine", "OtmError", "RequestArena", "Results", "encode_request", "murmur2_partition", "report_segments",
           "write_config"]
