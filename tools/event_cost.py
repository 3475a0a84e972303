import ctypes, time
h = ctypes.CDLL("libamdhip64.so")
h.hipSetDevice(0)
s = ctypes.c_void_p()
h.hipStreamCreate(ctypes.byref(s))
a = ctypes.c_void_p(); b = ctypes.c_void_p()
h.hipEventCreateWithFlags(ctypes.byref(a), 0x20000000)
h.hipEventCreateWithFlags(ctypes.byref(b), 0x20000000)
ms = ctypes.c_float()
res = {}
for rep in range(3):
    t0 = time.perf_counter()
    for i in range(2000):
        h.hipEventRecord(a, s); h.hipEventRecord(b, s)
    t1 = time.perf_counter()
    h.hipStreamSynchronize(s)
    t2 = time.perf_counter()
    for i in range(2000):
        h.hipEventElapsedTime(ctypes.byref(ms), a, b)
    t3 = time.perf_counter()
    for i in range(2000):
        h.hipStreamSynchronize(s)
    t4 = time.perf_counter()
    res[rep] = {"record_pair_us": (t1 - t0) / 2000 * 1e6, "elapsed_us": (t3 - t2) / 2000 * 1e6, "idle_sync_us": (t4 - t3) / 2000 * 1e6}
print(res)
