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
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
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

}  // namespace

std::string LinkD2H(int device, void *dst, const void *src, size_t n) {
  // read per call (tests flip them); a device's pool keeps its first thread count
  const int threads = std::min(64, std::max(0, EnvInt("MBX_LINK_THREADS", 8)));
  const long min_bytes = std::max(1, EnvInt("MBX_LINK_MIN", kFreshBytes));
  const bool huge = EnvInt("MBX_LINK_HUGE", 1) != 0;
  if (n == 0) return "";
  LinkPool *pool = threads > 0 && (long)n >= min_bytes ? Pool(device, threads) : nullptr;
  if (!pool) {
    hipError_t e = hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
    return e == hipSuccess ? "" : HipErr(e, "LinkD2H hipMemcpy");
  }
  if (huge && n >= (size_t)kFreshBytes) AdviseHuge(dst, n);
  return pool->Copy((uint8_t *)dst, (const uint8_t *)src, n);
}

}  // namespace mbx
