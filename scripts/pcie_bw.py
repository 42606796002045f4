"""PCIe copy rates on the GPU box: pinned host <-> HBM with hipMemcpyAsync
(torch copies), one stream and three concurrent streams, H2D, D2H and both at
once.  The host-inclusive leg moves ~24 B/point in and ~15 B/point out."""
import json
import time

import torch

dev = torch.device("cuda", 0)
MB = 1 << 20
out = {}
for size_mb in (4, 8, 32):
    n = size_mb * MB
    h = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
    d = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(3)]
    ss = [torch.cuda.Stream(dev) for _ in range(3)]
    for mode in ("h2d", "d2h", "both"):
        for nstreams in (1, 3):
            reps = 20
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                for i in range(nstreams):
                    with torch.cuda.stream(ss[i]):
                        if mode in ("h2d", "both"):
                            d[i].copy_(h[i], non_blocking=True)
                        if mode in ("d2h", "both"):
                            h[(i + 1) % 3].copy_(d[(i + 1) % 3], non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            nbytes = reps * nstreams * n * (2 if mode == "both" else 1)
            out["%s_%dMB_%dstream" % (mode, size_mb, nstreams)] = round(nbytes / dt / 1e9, 1)
print(json.dumps(out, indent=1))
