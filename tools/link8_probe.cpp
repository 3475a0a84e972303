// 8 MB device -> host copies into a freshly allocated destination (the Arrow
// getter of one 1e6-row INT64 slice, the MoonBit decoders' cap): the runtime's
// pageable copy against pinned-bounce variants, destination from malloc or
// calloc each call (as a MoonBit runtime / the C harness allocate a Bytes).
//   hipcc -O2 -std=c++17 -o tools/link8_probe tools/link8_probe.cpp -lpthread
//   ./tools/link8_probe [MB] [iters]
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// persistent memcpy helpers (spin-waiting on a generation word)
struct Team {
  int n;
  std::vector<std::thread> th;
  std::atomic<uint64_t> gen{0};
  std::atomic<int> left{0};
  std::atomic<bool> stop{false};
  std::function<void(int)> job;
  explicit Team(int k) : n(k) {
    for (int i = 1; i < n; i++)
      th.emplace_back([this, i] {
        uint64_t seen = 0;
        while (!stop.load()) {
          uint64_t g = gen.load(std::memory_order_acquire);
          if (g == seen) {
            __builtin_ia32_pause();
            continue;
          }
          seen = g;
          job(i);
          left.fetch_sub(1);
        }
      });
  }
  void Run(std::function<void(int)> f) {
    job = f;
    left.store(n - 1);
    gen.fetch_add(1, std::memory_order_release);
    job(0);
    while (left.load() > 0) __builtin_ia32_pause();
  }
  ~Team() {
    stop = true;
    for (auto &t : th) t.join();
  }
};

int main(int argc, char **argv) {
  const size_t mb = argc > 1 ? atoi(argv[1]) : 8;
  const int iters = argc > 2 ? atoi(argv[2]) : 200;
  const size_t n = mb << 20;
  void *d = nullptr;
  CK(hipMalloc(&d, n));
  CK(hipMemset(d, 1, n));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned char *pin = nullptr;
  CK(hipHostMalloc((void **)&pin, n, hipHostMallocDefault));
  const size_t CH = 1 << 20;
  unsigned char *pin2[2];
  hipEvent_t ev[2];
  for (int k = 0; k < 2; k++) {
    CK(hipHostMalloc((void **)&pin2[k], CH, hipHostMallocDefault));
    CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
  }
  Team team4(4), team8(8);
  auto par_copy = [&](Team &t, unsigned char *dst, const unsigned char *src, size_t len) {
    t.Run([&](int i) {
      size_t part = (len / t.n + 4095) & ~(size_t)4095;
      size_t b = (size_t)i * part;
      if (b < len) memcpy(dst + b, src + b, std::min(part, len - b));
    });
  };
  // all threads copy each chunk as soon as its DMA lands (one stream, an
  // event per chunk): the copy-out of chunk c overlaps the DMA of c + 1..
  std::vector<hipEvent_t> cev(64);
  for (auto &e : cev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  auto fine = [&](Team &t, unsigned char *dst, size_t CHK) {
    const size_t nch = (n + CHK - 1) / CHK;
    for (size_t c = 0; c < nch; c++) {
      CK(hipMemcpyAsync(pin + c * CHK, (char *)d + c * CHK, std::min(CHK, n - c * CHK), hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(cev[c], s));
    }
    std::atomic<size_t> landed{0};
    t.Run([&](int i) {
      for (size_t c = 0; c < nch; c++) {
        if (i == 0) {
          while (hipEventQuery(cev[c]) == hipErrorNotReady) __builtin_ia32_pause();
          landed.store(c + 1, std::memory_order_release);
        } else {
          while (landed.load(std::memory_order_acquire) <= c) __builtin_ia32_pause();
        }
        const size_t len = std::min(CHK, n - c * CHK);
        size_t part = (len / t.n + 4095) & ~(size_t)4095;
        size_t b = (size_t)i * part;
        if (b < len) memcpy(dst + c * CHK + b, pin + c * CHK + b, std::min(part, len - b));
      }
    });
  };
  // the same pipeline with the chunk landings signalled by the stream itself:
  // after each chunk's DMA, hipStreamWriteValue32 stores the call's generation
  // into a coherent pinned flag, and the copy threads spin on plain loads of
  // their flags (no event queries).  per_thread: thread t copies chunks t,
  // t+T, ... whole; else every thread copies its slice of every chunk.
  unsigned *flags = nullptr;
  CK(hipHostMalloc((void **)&flags, 64 * sizeof(unsigned), hipHostMallocCoherent));
  memset(flags, 0, 64 * sizeof(unsigned));
  unsigned fgen = 0;
  auto flagged = [&](Team &t, unsigned char *dst, size_t CHK, bool per_thread) {
    const size_t nch = (n + CHK - 1) / CHK;
    const unsigned g = ++fgen;
    for (size_t c = 0; c < nch; c++) {
      CK(hipMemcpyAsync(pin + c * CHK, (char *)d + c * CHK, std::min(CHK, n - c * CHK), hipMemcpyDeviceToHost, s));
      CK(hipStreamWriteValue32(s, flags + c, g, 0));
    }
    t.Run([&](int i) {
      for (size_t c = per_thread ? i : 0; c < nch; c += per_thread ? t.n : 1) {
        while (__atomic_load_n(flags + c, __ATOMIC_ACQUIRE) != g) __builtin_ia32_pause();
        const size_t len = std::min(CHK, n - c * CHK);
        if (per_thread) {
          memcpy(dst + c * CHK, pin + c * CHK, len);
          continue;
        }
        size_t part = (len / t.n + 4095) & ~(size_t)4095;
        size_t b = (size_t)i * part;
        if (b < len) memcpy(dst + c * CHK + b, pin + c * CHK + b, std::min(part, len - b));
      }
    });
  };
  struct V {
    const char *name;
    std::function<void(unsigned char *)> f;
  };
  std::vector<V> vs = {
      {"runtime hipMemcpy", [&](unsigned char *dst) { CK(hipMemcpy(dst, d, n, hipMemcpyDeviceToHost)); }},
      {"pinned bounce + memcpy", [&](unsigned char *dst) {
         CK(hipMemcpyAsync(pin, d, n, hipMemcpyDeviceToHost, s));
         CK(hipStreamSynchronize(s));
         memcpy(dst, pin, n);
       }},
      {"pinned bounce + 4 thr", [&](unsigned char *dst) {
         CK(hipMemcpyAsync(pin, d, n, hipMemcpyDeviceToHost, s));
         CK(hipStreamSynchronize(s));
         par_copy(team4, dst, pin, n);
       }},
      {"pinned bounce + 8 thr", [&](unsigned char *dst) {
         CK(hipMemcpyAsync(pin, d, n, hipMemcpyDeviceToHost, s));
         CK(hipStreamSynchronize(s));
         par_copy(team8, dst, pin, n);
       }},
      {"1MB pipeline, 1 thr", [&](unsigned char *dst) {
         const size_t nch = (n + CH - 1) / CH;
         auto issue = [&](size_t c, int k) {
           CK(hipMemcpyAsync(pin2[k], (char *)d + c * CH, std::min(CH, n - c * CH), hipMemcpyDeviceToHost, s));
           CK(hipEventRecord(ev[k], s));
         };
         issue(0, 0);
         for (size_t c = 0; c < nch; c++) {
           if (c + 1 < nch) issue(c + 1, (c + 1) & 1);
           CK(hipEventSynchronize(ev[c & 1]));
           memcpy(dst + c * CH, pin2[c & 1], std::min(CH, n - c * CH));
         }
       }},
      {"pinned split DMA 2 + 4 thr", [&](unsigned char *dst) {
         // the second half's DMA overlaps the first half's copy-out
         const size_t h = n / 2;
         hipEvent_t e0 = ev[0];
         CK(hipMemcpyAsync(pin, d, h, hipMemcpyDeviceToHost, s));
         CK(hipEventRecord(e0, s));
         CK(hipMemcpyAsync(pin + h, (char *)d + h, n - h, hipMemcpyDeviceToHost, s));
         CK(hipEventSynchronize(e0));
         par_copy(team4, dst, pin, h);
         CK(hipStreamSynchronize(s));
         par_copy(team4, dst + h, pin + h, n - h);
       }},
      {"register + DMA + unregister", [&](unsigned char *dst) {
         CK(hipHostRegister(dst, n, hipHostRegisterDefault));
         void *dp = nullptr;
         CK(hipHostGetDevicePointer(&dp, dst, 0));
         CK(hipMemcpyAsync(dst, d, n, hipMemcpyDeviceToHost, s));
         CK(hipStreamSynchronize(s));
         CK(hipHostUnregister(dst));
       }},
      {"fine 8 chunks, 8 thr", [&](unsigned char *dst) { fine(team8, dst, n / 8); }},
      {"fine 16 chunks, 8 thr", [&](unsigned char *dst) { fine(team8, dst, n / 16); }},
      {"fine 32 chunks, 8 thr", [&](unsigned char *dst) { fine(team8, dst, n / 32); }},
      {"fine 16 chunks, 4 thr", [&](unsigned char *dst) { fine(team4, dst, n / 16); }},
      {"flag 8 chunks, 8 thr slices", [&](unsigned char *dst) { flagged(team8, dst, n / 8, false); }},
      {"flag 16 chunks, 8 thr slices", [&](unsigned char *dst) { flagged(team8, dst, n / 16, false); }},
      {"flag 8 chunks, 8 thr whole", [&](unsigned char *dst) { flagged(team8, dst, n / 8, true); }},
      {"flag 16 chunks, 8 thr whole", [&](unsigned char *dst) { flagged(team8, dst, n / 16, true); }},
      {"flag 32 chunks, 8 thr whole", [&](unsigned char *dst) { flagged(team8, dst, n / 32, true); }},
      {"flag 16 chunks, 4 thr whole", [&](unsigned char *dst) { flagged(team4, dst, n / 16, true); }},
  };
  for (int alloc = 0; alloc < 2; alloc++) {
    for (auto &v : vs) {
      double best = 1e9, tot = 0;
      for (int it = 0; it < iters; it++) {
        double t0 = Now();
        unsigned char *dst = alloc ? (unsigned char *)calloc(1, n + 8) : (unsigned char *)malloc(n + 8);
        v.f(dst + 8);
        double t1 = Now();
        if (dst[8] != 1 || dst[8 + n - 1] != 1) {
          fprintf(stderr, "bad copy\n");
          return 1;
        }
        free(dst);
        best = std::min(best, t1 - t0);
        tot += t1 - t0;
      }
      printf("%-7s %-28s %zu MB: best %6.1f GB/s  mean %6.1f GB/s (alloc + copy)\n", alloc ? "calloc" : "malloc",
             v.name, mb, n / best / 1e9, n / (tot / iters) / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
