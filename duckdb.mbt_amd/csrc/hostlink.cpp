// Device -> pageable host copies for the Arrow getters (C4 read-back; the
// reference's getters fill a MoonBit Bytes from libduckdb's host vectors,
// src/duckdb_native.c:2392-2422).
//
// A getter's destination is a freshly allocated Bytes object: pages that have
// never been touched.  The runtime's pageable D2H copies through its own pinned
// buffer and then faults every 4 KiB page of the destination on one host
// thread: 13-26 GB/s into fresh memory against 57 GB/s for the link itself
// (profiles/r02_link_probe.log).  Here the 2 MiB-aligned interior of the
// destination is advised MADV_HUGEPAGE (512x fewer faults), and T host
// threads each DMA 1-4 MiB chunks into their own pinned double buffer and copy
// them out, so page faults, memcpy and DMA overlap: ~40 GB/s into fresh memory
// with T=8 and 4 MiB chunks on the MI355X box.
//
// Only copies of >= 32 MiB take this path: glibc serves those from fresh
// mmaps (its mmap threshold tops out at 32 MiB), while smaller Bytes usually
// reuse warm heap pages, where the runtime's copy already runs at 20-38 GB/s
// and huge-page advice costs more than it saves (7 GB/s on recycled 8 MB
// buffers; profiles/r02_c4_probe.log).
//
// MBX_LINK_THREADS (default 8; 0 = the runtime's copy), MBX_LINK_MIN (bytes,
// default 32 MiB), MBX_LINK_HUGE=0 skips the huge-page advice (never given
// below 32 MiB).
#include "hostlink.h"
#include "knobs.h"

#include <hip/hip_runtime_api.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace mbx {
namespace {

constexpr size_t kMaxChunk = (size_t)4 << 20;
constexpr size_t kMinChunk = (size_t)256 << 10;
constexpr size_t kHugePage = (size_t)2 << 20;
constexpr int kFreshBytes = 32 << 20;  // glibc's largest mmap threshold

int EnvInt(const char *name, int dflt) {
  const char *v = Knob(name);
  return v && *v ? atoi(v) : dflt;
}

std::string HipErr(hipError_t e, const char *what) {
  return std::string("HIP error: ") + hipGetErrorString(e) + " at " + what;
}

class LinkPool {
 public:
  LinkPool(int device, int nthreads) : device_(device) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return;
    workers_.resize(nthreads);
    for (auto &w : workers_) {
      if (hipStreamCreateWithFlags(&w.s, hipStreamNonBlocking) != hipSuccess) {
        Fail(prev);
        return;
      }
      for (int k = 0; k < 2; k++) {
        if (hipHostMalloc((void **)&w.pin[k], kMaxChunk, hipHostMallocDefault) != hipSuccess) {
          Fail(prev);
          return;
        }
        if (hipEventCreateWithFlags(&w.ev[k], hipEventDisableTiming) != hipSuccess) {
          Fail(prev);
          return;
        }
      }
    }
    (void)hipSetDevice(prev);
    // the threads live for the rest of the process, parked on cv_go_ between copies
    for (int t = 0; t < nthreads; t++) std::thread([this, t] { Run(t); }).detach();
    ok_ = true;
  }
  bool ok() const { return ok_; }

  std::string Copy(uint8_t *dst, const uint8_t *src, size_t n) {
    std::lock_guard<std::mutex> call(call_mu_);  // one copy at a time per device
    const size_t T = workers_.size();
    size_t ch = (n / (2 * T) + 65535) & ~(size_t)65535;
    ch = std::min(kMaxChunk, std::max(kMinChunk, ch));
    std::unique_lock<std::mutex> lk(mu_);
    dst_ = dst;
    src_ = src;
    n_ = n;
    ch_ = ch;
    err_.clear();
    pending_ = (int)T;
    gen_++;
    cv_go_.notify_all();
    cv_done_.wait(lk, [&] { return pending_ == 0; });
    return err_;
  }

 private:
  struct Worker {
    hipStream_t s = nullptr;
    uint8_t *pin[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
  };

  void Fail(int prev) {
    (void)hipSetDevice(prev);
    ok_ = false;
  }

  void Run(int t) {
    (void)hipSetDevice(device_);
    uint64_t seen = 0;
    for (;;) {
      uint8_t *dst;
      const uint8_t *src;
      size_t n, ch;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_go_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        dst = dst_;
        src = src_;
        n = n_;
        ch = ch_;
      }
      std::string e = Part(workers_[t], t, dst, src, n, ch);
      std::lock_guard<std::mutex> lk(mu_);
      if (!e.empty() && err_.empty()) err_ = e;
      if (--pending_ == 0) cv_done_.notify_all();
    }
  }

  // chunks t, t+T, ...: chunk i+T's DMA is in flight while chunk i is copied out
  std::string Part(Worker &w, int t, uint8_t *dst, const uint8_t *src, size_t n, size_t ch) {
    const size_t T = workers_.size(), nch = (n + ch - 1) / ch;
    std::string err;
    auto issue = [&](size_t c, int k) {
      const size_t off = c * ch, len = std::min(ch, n - off);
      hipError_t e = hipMemcpyAsync(w.pin[k], src + off, len, hipMemcpyDeviceToHost, w.s);
      if (e == hipSuccess) e = hipEventRecord(w.ev[k], w.s);
      if (e != hipSuccess && err.empty()) err = HipErr(e, "LinkD2H chunk copy");
      return e == hipSuccess;
    };
    int k = 0;
    bool live = (size_t)t < nch && issue((size_t)t, 0);
    for (size_t c = t; live && c < nch; c += T, k ^= 1) {
      if (c + T < nch && !issue(c + T, k ^ 1)) break;
      hipError_t e = hipEventSynchronize(w.ev[k]);
      if (e != hipSuccess) {
        err = HipErr(e, "LinkD2H chunk wait");
        break;
      }
      const size_t off = c * ch;
      memcpy(dst + off, w.pin[k], std::min(ch, n - off));
    }
    // nothing may still be landing in a pinned buffer when the next copy starts
    hipError_t e = hipStreamSynchronize(w.s);
    if (e != hipSuccess && err.empty()) err = HipErr(e, "LinkD2H drain");
    return err;
  }

  int device_;
  bool ok_ = false;
  std::vector<Worker> workers_;
  std::mutex call_mu_, mu_;
  std::condition_variable cv_go_, cv_done_;
  uint64_t gen_ = 0;
  int pending_ = 0;
  uint8_t *dst_ = nullptr;
  const uint8_t *src_ = nullptr;
  size_t n_ = 0, ch_ = 0;
  std::string err_;
};

std::mutex g_pools_mu;
LinkPool *g_pools[64] = {};  // never freed: parked threads may outlive static destructors

LinkPool *Pool(int device, int nthreads) {
  if (device < 0 || device >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_pools_mu);
  if (!g_pools[device]) g_pools[device] = new LinkPool(device, nthreads);
  return g_pools[device]->ok() ? g_pools[device] : nullptr;
}

void AdviseHuge(void *p, size_t n) {
  const uintptr_t b = ((uintptr_t)p + kHugePage - 1) & ~(uintptr_t)(kHugePage - 1);
  const uintptr_t e = ((uintptr_t)p + n) & ~(uintptr_t)(kHugePage - 1);
  if (e > b) (void)madvise((void *)b, e - b, MADV_HUGEPAGE);
}

// ---------------------------------------------------------------------------
// Mid-size copies (2 MiB up to the pool's 32 MiB; the reference's getters hand
// out 8 MB per 1e6-row INT64 slice, duckdb_native.c:2392-2422).  At this size
// the per-call machinery is the limit, and which method wins depends on the
// box's host side, 2-3x apart between boxes of the same pool for the same
// method (profiles/r03_link8_probe*.log, r04_link8_probe_flags.log):
//   M_RUNTIME  the runtime's pageable copy (its own staging),
//   M_REGISTER page-lock the destination (hipHostRegister), one DMA straight
//              into it, unregister,
//   M_BOUNCE   one DMA into a per-device pinned bounce, then T host threads
//              copy their slices out (threads spin between calls, then sleep).
// So the library measures: per device and power-of-two size class, the first
// calls run each method for a block of kBlock calls, timed end to end (a
// block's first call, which pays the method's setup and cold pages, is not
// counted), and the class then keeps the method with the best median.  The bytes are the same whichever method runs.
// MBX_LINK_MID=0 keeps the runtime's copy; MBX_LINK_MID_MODE=0|1|2 (or
// duckdb_mbx_set_link_mode) pins one.  The mid path is part of the host copy
// machinery, so MBX_LINK_THREADS=0 turns it off too.
enum MidMethod { M_RUNTIME = 0, M_REGISTER = 1, M_BOUNCE = 2, M_COUNT = 3 };

class SpinTeam {  // T-1 helper threads + the caller; helpers spin kSpinUs after a job, then sleep
 public:
  explicit SpinTeam(int t) : n_(t) {
    for (int i = 1; i < n_; i++) std::thread([this, i] { Loop(i); }).detach();
  }
  void Run(const std::function<void(int)> &f) {
    job_ = &f;
    left_.store(n_ - 1, std::memory_order_release);
    {
      std::lock_guard<std::mutex> g(mu_);
      gen_.fetch_add(1, std::memory_order_acq_rel);
    }
    if (sleepers_.load(std::memory_order_acquire)) cv_.notify_all();
    f(0);
    while (left_.load(std::memory_order_acquire) > 0) __builtin_ia32_pause();
  }
  int size() const { return n_; }

 private:
  static constexpr int kSpinUs = 2000;
  void Loop(int i) {
    uint64_t seen = 0;
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      int k = 0;
      while (gen_.load(std::memory_order_acquire) == seen) {
        if ((++k & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSpinUs)) {
          std::unique_lock<std::mutex> lk(mu_);
          sleepers_.fetch_add(1);
          cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
          sleepers_.fetch_sub(1);
          break;
        }
        __builtin_ia32_pause();
      }
      seen = gen_.load(std::memory_order_acquire);
      (*job_)(i);
      left_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  const int n_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> left_{0}, sleepers_{0};
  const std::function<void(int)> *job_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_;
};

class MidLink {
 public:
  MidLink() {}

  // {"class_mib": [lo, hi], "calls": c, "kept": method, "trial_median_gbs": {...}} per class with calls
  std::string StatsJson() {
    std::lock_guard<std::mutex> call(mu_);
    static const char *names[M_COUNT] = {"runtime", "register", "bounce"};
    std::string j = "[";
    for (int c = 0; c < kClasses; c++) {
      Class &C = cls_[c];
      if (!C.calls) continue;
      if (j.size() > 1) j += ",";
      j += "{\"class_mib\":[" + std::to_string(2 << c) + "," + std::to_string(4 << c) + "],\"calls\":" +
           std::to_string(C.calls) + ",\"kept\":\"" + (C.best >= 0 ? names[C.best] : "runtime (no trial yet)") +
           "\",\"trial_median_gbs\":{";
      bool first = true;
      for (int m = 0; m < M_COUNT; m++) {
        if (C.gbs[m].empty() && !C.broken[m]) continue;
        std::vector<double> v = C.gbs[m];
        double med = 0;
        if (!v.empty()) {
          std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
          med = v[v.size() / 2] / 1e3;  // MB/s -> GB/s
        }
        j += std::string(first ? "" : ",") + "\"" + names[m] + "\":" + (C.broken[m] ? "\"refused\"" : std::to_string(med));
        first = false;
      }
      j += "}}";
    }
    return j + "]";
  }

  std::string Copy(void *dst, const void *src, size_t n, int forced) {
    std::lock_guard<std::mutex> call(mu_);
    int cls = 0;  // 2-4 MiB: 0, 4-8: 1, 8-16: 2, 16-32: 3
    for (size_t q = n >> 21; q > 1 && cls < kClasses - 1; q >>= 1) cls++;
    Class &C = cls_[cls];
    bool sample = false;
    int m = forced >= 0 && forced < M_COUNT ? forced : Pick(C, &sample);
    const auto t0 = std::chrono::steady_clock::now();
    std::string err = Run(m, dst, src, n);
    if (!err.empty() && m != M_RUNTIME) {  // a method the box refuses (e.g. registration): never again here
      C.broken[m] = true;
      m = M_RUNTIME;
      err = Run(m, dst, src, n);
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (err.empty()) C.Record(m, n / us, sample);
    return err;
  }

 private:
  static constexpr int kClasses = 4, kBlock = 5;  // trial calls per method (the first not counted)
  struct Class {
    std::vector<double> gbs[M_COUNT];  // (bytes/us = MB/s; only the order matters)
    bool broken[M_COUNT] = {false, false, false};
    uint64_t calls = 0;
    int best = -1;
    // one trial block per method, back to back (alternating methods call by
    // call disturbed them: on one box the runtime copy ran 6-8 GB/s between
    // bounce calls and 16 GB/s in a run of its own); a block's first call pays
    // the method's setup and cold pages and is not a sample
    void Record(int m, double rate, bool sample) {
      if (!sample) return;
      gbs[m].push_back(rate);
      double bm = -1;
      best = -1;
      for (int k = 0; k < M_COUNT; k++) {
        if (broken[k] || gbs[k].empty()) continue;
        std::vector<double> s = gbs[k];
        std::nth_element(s.begin(), s.begin() + s.size() / 2, s.end());
        if (s[s.size() / 2] > bm) bm = s[s.size() / 2], best = k;
      }
    }
  };
  // the method for call k of a class, and whether its rate is a trial sample
  int Pick(Class &C, bool *sample) {
    const uint64_t k = C.calls++;
    *sample = false;
    if (k < (uint64_t)M_COUNT * kBlock) {
      const int t = (int)(k / kBlock);
      if (!C.broken[t]) {
        *sample = k % kBlock != 0;
        return t;
      }
    }
    return C.best >= 0 ? C.best : M_RUNTIME;
  }
  std::string Run(int m, void *dst, const void *src, size_t n) {
    if (m == M_REGISTER) {
      const uintptr_t pg = 4096, b = (uintptr_t)dst & ~(pg - 1), e = ((uintptr_t)dst + n + pg - 1) & ~(pg - 1);
      hipError_t r = hipHostRegister((void *)b, e - b, hipHostRegisterDefault);
      if (r != hipSuccess) {
        (void)hipGetLastError();
        return HipErr(r, "LinkD2H hipHostRegister");
      }
      hipError_t c = hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
      r = hipHostUnregister((void *)b);
      if (c != hipSuccess) return HipErr(c, "LinkD2H registered copy");
      return r == hipSuccess ? "" : HipErr(r, "LinkD2H hipHostUnregister");
    }
    if (m == M_BOUNCE) {
      if (n > bounce_n_) {
        if (bounce_) (void)hipHostFree(bounce_);
        bounce_ = nullptr;
        bounce_n_ = 0;
        size_t b = (size_t)4 << 20;
        while (b < n) b <<= 1;
        hipError_t r = hipHostMalloc((void **)&bounce_, b, hipHostMallocDefault);
        if (r != hipSuccess) return HipErr(r, "LinkD2H bounce allocation");
        bounce_n_ = b;
        if (!stream_ && hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess)
          return "HIP error: LinkD2H bounce stream";
      }
      hipError_t r = hipMemcpyAsync(bounce_, src, n, hipMemcpyDeviceToHost, stream_);
      if (r == hipSuccess) r = hipStreamSynchronize(stream_);
      if (r != hipSuccess) return HipErr(r, "LinkD2H bounce DMA");
      if (!team_) team_.reset(new SpinTeam(8));
      const int T = team_->size();
      const size_t part = (n / T + 4095) & ~(size_t)4095;
      team_->Run([&](int i) {
        const size_t o = (size_t)i * part;
        if (o < n) memcpy((uint8_t *)dst + o, bounce_ + o, std::min(part, n - o));
      });
      return "";
    }
    hipError_t e = hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
    return e == hipSuccess ? "" : HipErr(e, "LinkD2H hipMemcpy");
  }
  std::mutex mu_;
  Class cls_[kClasses];
  uint8_t *bounce_ = nullptr;
  size_t bounce_n_ = 0;
  hipStream_t stream_ = nullptr;
  std::unique_ptr<SpinTeam> team_;
};

MidLink *g_mid[64] = {};  // never freed, as the pools

MidLink *Mid(int device) {
  if (device < 0 || device >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_pools_mu);
  if (!g_mid[device]) g_mid[device] = new MidLink();
  return g_mid[device];
}

}  // namespace

static std::atomic<int> g_link_mode{-1};

void SetLinkMode(int mode) { g_link_mode.store(mode >= 0 && mode < M_COUNT ? mode : -1); }

std::string LinkStatsJson() {
  std::string j = "[";
  for (int d = 0; d < 64; d++) {
    MidLink *m = nullptr;
    {
      std::lock_guard<std::mutex> lk(g_pools_mu);
      m = g_mid[d];
    }
    if (!m) continue;
    if (j.size() > 1) j += ",";
    j += "{\"device\":" + std::to_string(d) + ",\"mode\":" + std::to_string(g_link_mode.load()) +
         ",\"classes\":" + m->StatsJson() + "}";
  }
  return j + "]";
}

std::string LinkD2H(int device, void *dst, const void *src, size_t n) {
  // read per call (tests flip them); a device's pool keeps its first thread count
  const int threads = std::min(64, std::max(0, EnvInt("MBX_LINK_THREADS", 8)));
  const long min_bytes = std::max(1, EnvInt("MBX_LINK_MIN", kFreshBytes));
  const bool huge = EnvInt("MBX_LINK_HUGE", 1) != 0;
  if (n == 0) return "";
  if (threads > 0 && (long)n < min_bytes && n >= (size_t)2 << 20 && EnvInt("MBX_LINK_MID", 1) != 0) {
    MidLink *mid = Mid(device);
    const int mode = g_link_mode.load();
    if (mid) return mid->Copy(dst, src, n, mode >= 0 ? mode : EnvInt("MBX_LINK_MID_MODE", -1));
  }
  LinkPool *pool = threads > 0 && (long)n >= min_bytes ? Pool(device, threads) : nullptr;
  if (!pool) {
    hipError_t e = hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
    return e == hipSuccess ? "" : HipErr(e, "LinkD2H hipMemcpy");
  }
  if (huge && n >= (size_t)kFreshBytes) AdviseHuge(dst, n);
  return pool->Copy((uint8_t *)dst, (const uint8_t *)src, n);
}

}  // namespace mbx
