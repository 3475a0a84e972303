// Host-link probe (C4): D2H into fresh pageable memory and H2D from pageable
// memory, the runtime's own staged copy against T host threads that each DMA
// into their own pinned double buffer and memcpy to/from the pageable side.
//   hipcc -O2 -std=c++17 -o tools/link_probe tools/link_probe.cpp -lpthread
//   ./tools/link_probe [MB]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <sys/mman.h>
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

static double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Worker {
  hipStream_t s;
  unsigned char *pin[2];
  hipEvent_t ev[2];
};

static std::vector<Worker> MakeWorkers(int T, size_t ch) {
  std::vector<Worker> w(T);
  for (auto &x : w) {
    CK(hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking));
    for (int k = 0; k < 2; k++) {
      CK(hipHostMalloc((void **)&x.pin[k], ch, hipHostMallocDefault));
      CK(hipEventCreateWithFlags(&x.ev[k], hipEventDisableTiming));
    }
  }
  return w;
}
static void FreeWorkers(std::vector<Worker> &w) {
  for (auto &x : w) {
    for (int k = 0; k < 2; k++) {
      CK(hipHostFree(x.pin[k]));
      CK(hipEventDestroy(x.ev[k]));
    }
    CK(hipStreamDestroy(x.s));
  }
}

// worker t handles chunks t, t+T, ...: DMA of chunk i+1 in flight while chunk i is memcpy'd
static void D2HThreaded(std::vector<Worker> &ws, unsigned char *dst, const unsigned char *src, size_t n, size_t ch) {
  const int T = (int)ws.size();
  const size_t nch = (n + ch - 1) / ch;
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      CK(hipSetDevice(0));
      Worker &w = ws[t];
      auto issue = [&](size_t c, int k) {
        const size_t off = c * ch, len = std::min(ch, n - off);
        CK(hipMemcpyAsync(w.pin[k], src + off, len, hipMemcpyDeviceToHost, w.s));
        CK(hipEventRecord(w.ev[k], w.s));
      };
      int k = 0;
      if ((size_t)t < nch) issue(t, 0);
      for (size_t c = t; c < nch; c += T, k ^= 1) {
        if (c + T < nch) issue(c + T, k ^ 1);
        CK(hipEventSynchronize(w.ev[k]));
        const size_t off = c * ch, len = std::min(ch, n - off);
        memcpy(dst + off, w.pin[k], len);
      }
    });
  for (auto &x : th) x.join();
}

static void H2DThreaded(std::vector<Worker> &ws, unsigned char *dst, const unsigned char *src, size_t n, size_t ch) {
  const int T = (int)ws.size();
  const size_t nch = (n + ch - 1) / ch;
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      CK(hipSetDevice(0));
      Worker &w = ws[t];
      int k = 0;
      bool used[2] = {false, false};
      for (size_t c = t; c < nch; c += T, k ^= 1) {
        if (used[k]) CK(hipEventSynchronize(w.ev[k]));
        const size_t off = c * ch, len = std::min(ch, n - off);
        memcpy(w.pin[k], src + off, len);
        CK(hipMemcpyAsync(dst + off, w.pin[k], len, hipMemcpyHostToDevice, w.s));
        CK(hipEventRecord(w.ev[k], w.s));
        used[k] = true;
      }
      CK(hipStreamSynchronize(w.s));
    });
  for (auto &x : th) x.join();
}


// the 2 MiB-aligned interior of [p, p+n)
static void Interior(void *p, size_t n, unsigned char **a, size_t *len) {
  uintptr_t b = ((uintptr_t)p + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
  uintptr_t e = ((uintptr_t)p + n) & ~(uintptr_t)((2u << 20) - 1);
  *a = (unsigned char *)b;
  *len = e > b ? e - b : 0;
}
static void Huge(void *p, size_t n) {
  unsigned char *a;
  size_t len;
  Interior(p, n, &a, &len);
  if (len) madvise(a, len, MADV_HUGEPAGE);
}
// fault the pages in on T threads (MADV_POPULATE_WRITE per slice, touch fallback)
static void Populate(void *p, size_t n, int T) {
  std::vector<std::thread> th;
  const size_t per = ((n + T - 1) / T + 4095) & ~(size_t)4095;
  uintptr_t base = (uintptr_t)p & ~(uintptr_t)4095;
  const size_t tot = (uintptr_t)p + n - base;
  for (int t = 0; t < T; t++)
    th.emplace_back([=] {
      const size_t off = (size_t)t * per;
      if (off >= tot) return;
      const size_t len = std::min(per, tot - off);
      if (madvise((void *)(base + off), len, MADV_POPULATE_WRITE) != 0)
        for (size_t i = 0; i < len; i += 4096) ((volatile unsigned char *)(base + off))[i] = 0;
    });
  for (auto &x : th) x.join();
}

int main(int argc, char **argv) {
  const size_t MB = argc > 1 ? (size_t)atol(argv[1]) : 256;
  const size_t n = MB << 20;
  unsigned char *d;
  CK(hipMalloc((void **)&d, n));
  CK(hipMemset(d, 0x5a, n));
  unsigned char *pin;
  CK(hipHostMalloc((void **)&pin, n, hipHostMallocDefault));
  CK(hipDeviceSynchronize());
  auto gbs = [&](double s) { return (double)n / s / 1e9; };
  // pinned DMA rates (the link itself)
  for (int r = 0; r < 3; r++) {
    double t0 = Now();
    CK(hipMemcpy(pin, d, n, hipMemcpyDeviceToHost));
    double t1 = Now();
    CK(hipMemcpy(d, pin, n, hipMemcpyHostToDevice));
    double t2 = Now();
    printf("pinned       D2H %6.1f GB/s  H2D %6.1f GB/s\n", gbs(t1 - t0), gbs(t2 - t1));
  }
  // the runtime's pageable copies into/out of fresh calloc memory (what the getters do today)
  for (int r = 0; r < 3; r++) {
    unsigned char *h = (unsigned char *)calloc(1, n);
    double t0 = Now();
    CK(hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
    double t1 = Now();
    CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
    double t2 = Now();
    printf("pageable     D2H %6.1f GB/s (fresh)  H2D %6.1f GB/s (warm)  first byte %d\n", gbs(t1 - t0), gbs(t2 - t1),
           h[12345]);
    free(h);
  }
  // single-thread memcpy rates: fresh destination, warm destination
  {
    unsigned char *h = (unsigned char *)calloc(1, n);
    double t0 = Now();
    memcpy(h, pin, n);
    double t1 = Now();
    memcpy(h, pin, n);
    double t2 = Now();
    printf("memcpy 1 thr  fresh %6.1f GB/s  warm %6.1f GB/s\n", gbs(t1 - t0), gbs(t2 - t1));
    free(h);
  }
  // fresh destinations: huge-page advice, parallel population, both
  for (int v = 0; v < 6; v++)
    for (int r = 0; r < 3; r++) {
      unsigned char *h = (unsigned char *)calloc(1, n + 64);
      unsigned char *dst = h + 4;  // MoonBit payloads start 8 bytes into a header'd block + the 4-byte count
      double t0 = Now();
      if (v == 1 || v == 3 || v == 5) Huge(dst, n);
      if (v == 2 || v == 3) Populate(dst, n, 8);
      double t1 = Now();
      if (v >= 4) {
        auto ws = MakeWorkers(8, 8u << 20);
        double ta = Now();
        D2HThreaded(ws, dst, d, n, 8u << 20);
        double tb = Now();
        printf("fresh v%d threaded T=8 D2H %6.1f GB/s (prep %.1f ms)\n", v, gbs(tb - ta + t1 - t0), (t1 - t0) * 1e3);
        FreeWorkers(ws);
      } else {
        CK(hipMemcpy(dst, d, n, hipMemcpyDeviceToHost));
        double t2 = Now();
        printf("fresh v%d %s%s D2H %6.1f GB/s total (prep %.1f ms, copy %.1f GB/s)\n", v, (v & 1) ? "huge " : "",
               v >= 2 ? "populate8 " : "", gbs(t2 - t0), (t1 - t0) * 1e3, gbs(t2 - t1));
      }
      if (dst[n - 1] != 0x5a || dst[0] != 0x5a) printf("MISMATCH\n");
      free(h);
    }
  // huge-page advice + T threads x chunk size
  for (size_t ch : {2u << 20, 4u << 20, 8u << 20, 16u << 20})
    for (int T : {4, 6, 8, 12, 16}) {
      auto ws = MakeWorkers(T, ch);
      double best = 0, sum = 0;
      for (int r = 0; r < 4; r++) {
        unsigned char *h = (unsigned char *)calloc(1, n + 64);
        unsigned char *dst = h + 4;
        double t0 = Now();
        Huge(dst, n);
        D2HThreaded(ws, dst, d, n, ch);
        double g = gbs(Now() - t0);
        best = std::max(best, g);
        sum += g;
        if (dst[n - 1] != 0x5a || dst[0] != 0x5a) printf("MISMATCH\n");
        free(h);
      }
      printf("huge threaded T=%2d ch=%2zuMB D2H best %6.1f mean %6.1f GB/s\n", T, ch >> 20, best, sum / 4);
      FreeWorkers(ws);
    }
  if (argc > 2) return 0;
  const int Ts[] = {2, 4, 8, 12, 16};
  const size_t CHs[] = {2u << 20, 4u << 20, 8u << 20};
  for (size_t ch : CHs)
    for (int T : Ts) {
      auto ws = MakeWorkers(T, ch);
      double best_d = 0, best_h = 0, warm_d = 0;
      for (int r = 0; r < 3; r++) {
        unsigned char *h = (unsigned char *)calloc(1, n);
        double t0 = Now();
        D2HThreaded(ws, h, d, n, ch);
        double t1 = Now();
        D2HThreaded(ws, h, d, n, ch);
        double t2 = Now();
        H2DThreaded(ws, d, h, n, ch);
        double t3 = Now();
        if (h[n - 1] != 0x5a || h[0] != 0x5a) printf("MISMATCH\n");
        best_d = std::max(best_d, gbs(t1 - t0));
        warm_d = std::max(warm_d, gbs(t2 - t1));
        best_h = std::max(best_h, gbs(t3 - t2));
        free(h);
      }
      printf("threaded T=%2d ch=%zuMB  D2H fresh %6.1f  warm %6.1f  H2D %6.1f GB/s\n", T, ch >> 20, best_d, warm_d,
             best_h);
      FreeWorkers(ws);
    }
  CK(hipHostFree(pin));
  CK(hipFree(d));
  return 0;
}
