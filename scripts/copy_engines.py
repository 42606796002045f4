#!/usr/bin/env python3
"""Which engine does the runtime pick for a pinned host->device copy?  Copies
the same 8 MB from four host buffers (torch pin_memory, hipHostMalloc default,
hipHostMalloc non-coherent, hipHostRegister'd malloc) on one stream, phase by
phase with a marker kernel between, so a rocprofv3 --kernel-trace
--memory-copy-trace run can attribute each phase's copies to SDMA (memory-copy
records) or to blit kernels (__amd_rocclr_copyBuffer)."""
import ctypes as C
import time

import numpy as np
import torch

hip = C.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
N = 8 << 20
dev = torch.empty(N, dtype=torch.uint8, device="cuda:0")
stream = torch.cuda.Stream()
bufs = {}
t = torch.empty(N, dtype=torch.uint8, pin_memory=True)
bufs["torch_pinned"] = t.data_ptr()
p = C.c_void_p()
assert hip.hipHostMalloc(C.byref(p), N, 0) == 0
bufs["hostmalloc_default"] = p.value
p2 = C.c_void_p()
assert hip.hipHostMalloc(C.byref(p2), N, 0x40000000) == 0  # hipHostMallocNonCoherent
bufs["hostmalloc_noncoherent"] = p2.value
a = np.empty(N + 4096, np.uint8)
base = (a.ctypes.data + 4095) // 4096 * 4096
assert hip.hipHostRegister(C.c_void_p(base), N, 0) == 0
bufs["hostregister"] = base
hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
raw = C.c_void_p()
assert hip.hipStreamCreateWithFlags(C.byref(raw), 1) == 0  # hipStreamNonBlocking, as the engine's streams
rdev = C.c_void_p()
assert hip.hipMalloc(C.byref(rdev), N) == 0
res = {}
for name, ptr in list(bufs.items()) + [("raw_stream_hostmalloc", bufs["hostmalloc_default"])]:
    if name.startswith("raw_stream"):
        torch.cuda.synchronize()
        torch.ones(1, device="cuda:0")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            assert hip.hipMemcpyAsync(rdev, C.c_void_p(ptr), N, 1, raw) == 0
        hip.hipStreamSynchronize(raw)
        res[name] = round(10 * N / (time.perf_counter() - t0) / 1e9, 1)
        # and copies right behind a kernel on that stream: the engine's pattern
        continue
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        torch.ones(1, device="cuda:0")  # phase marker kernel
    t0 = time.perf_counter()
    for _ in range(10):
        assert hip.hipMemcpyAsync(C.c_void_p(dev.data_ptr()), C.c_void_p(ptr), N, 1, C.c_void_p(stream.cuda_stream)) == 0
    stream.synchronize()
    res[name] = round(10 * N / (time.perf_counter() - t0) / 1e9, 1)
print('RESULT', res, flush=True)
