// rccl_combine.cpp — RCCL communicators of a sharded connection and the pack /
// combine kernels around its collectives (see rccl_combine.h, combine.h).
#include "rccl_combine.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>

#include "knobs.h"

#include "phys.h"

#include <algorithm>

namespace mbx {
namespace rc {

namespace {
// the RCCL entry points, resolved from librccl at first use
struct Api {
  bool ok = false;
  std::string why;
  decltype(&ncclCommInitAll) init = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllGather) allgather = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclGetErrorString) errstr = nullptr;
  decltype(&ncclGroupStart) gstart = nullptr;
  decltype(&ncclGroupEnd) gend = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommCount) count = nullptr;        // (evidence only: optional)
  decltype(&ncclCommUserRank) user_rank = nullptr;
  decltype(&ncclCommCuDevice) cu_device = nullptr;
};

const Api &GetApi() {
  static Api api;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = nullptr;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) {
      const char *e = dlerror();
      api.why = std::string("librccl not loadable: ") + (e ? e : "?");
      return;
    }
    api.init = (decltype(api.init))dlsym(h, "ncclCommInitAll");
    api.destroy = (decltype(api.destroy))dlsym(h, "ncclCommDestroy");
    api.allgather = (decltype(api.allgather))dlsym(h, "ncclAllGather");
    api.reduce = (decltype(api.reduce))dlsym(h, "ncclReduce");
    api.errstr = (decltype(api.errstr))dlsym(h, "ncclGetErrorString");
    api.gstart = (decltype(api.gstart))dlsym(h, "ncclGroupStart");
    api.gend = (decltype(api.gend))dlsym(h, "ncclGroupEnd");
    api.abort = (decltype(api.abort))dlsym(h, "ncclCommAbort");
    api.count = (decltype(api.count))dlsym(h, "ncclCommCount");
    api.user_rank = (decltype(api.user_rank))dlsym(h, "ncclCommUserRank");
    api.cu_device = (decltype(api.cu_device))dlsym(h, "ncclCommCuDevice");
    // a collective that could not be aborted would leave its wait unbounded:
    // without ncclCommAbort the combine is never started
    api.ok = api.init && api.destroy && api.allgather && api.reduce && api.errstr && api.gstart && api.gend &&
             api.abort;
    if (!api.ok) api.why = "librccl lacks an entry point the combine needs (ncclCommAbort included)";
  });
  return api;
}

std::string ErrText(const Api &a, ncclResult_t r) {
  return std::string("RCCL error: ") + (a.errstr ? a.errstr(r) : "?") + " (" + std::to_string((int)r) + ")";
}

double Since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

int InitTimeoutMs() {
  static const int ms = [] {
    const char *v = Knob("MBX_RCCL_INIT_TIMEOUT_MS");
    return v ? std::max(1, atoi(v)) : 30000;
  }();
  return ms;
}

// the lanes rank r sends in the check: distinct per rank and lane, with
// carries in their sums
int64_t CheckLane(int r, int j) {
  return (int64_t)((uint64_t)0x123456789abcdefULL * (uint64_t)(j + 1) + (uint64_t)(r + 1) * 0x9e3779b97f4a7c15ULL -
                   (uint64_t)j * (uint64_t)j);
}
}  // namespace

std::string ApiProblem() { return GetApi().ok ? std::string() : GetApi().why; }

Comms::~Comms() {
  if (comms.empty()) return;
  const Api &a = GetApi();
  for (auto c : comms)
    if (c && a.destroy) a.destroy(c);
}

bool IsLoopback(const Comms &c) { return c.loopback; }

std::shared_ptr<Comms> OpenLoopback(const std::vector<int> &devs) {
  auto c = std::make_shared<Comms>();
  c->devs = devs;
  c->loopback = true;
  return c;
}

// The multi-rank check the communicators are gated on: every rank sends
// CheckLane(r, .) through one grouped reduce (to rank 0) and one grouped
// all-gather; the sums (int64, wrapping) on rank 0 and every rank's gathered
// block are verified on the host, and RCCL's own rank count, rank and device
// of every communicator are read.  "" when all of it holds.
static std::string CheckComms(Comms &c, int timeout_ms) {
  const Api &a = GetApi();
  const int n = (int)c.devs.size();
  constexpr int L = 97;  // an odd lane count: 3 columns x 32 + the error word
  c.count.assign(n, -1), c.user_rank.assign(n, -1), c.cu_device.assign(n, -1);
  for (int i = 0; i < n; i++) {
    if (a.count) a.count(c.comms[i], &c.count[i]);
    if (a.user_rank) a.user_rank(c.comms[i], &c.user_rank[i]);
    if (a.cu_device) a.cu_device(c.comms[i], &c.cu_device[i]);
    if ((a.count && c.count[i] != n) || (a.user_rank && c.user_rank[i] != i))
      return "RCCL check: communicator " + std::to_string(i) + " reports rank " + std::to_string(c.user_rank[i]) +
             " of " + std::to_string(c.count[i]) + ", expected " + std::to_string(i) + " of " + std::to_string(n);
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  std::vector<hipStream_t> s(n, nullptr);
  std::vector<int64_t *> buf(n, nullptr);  // per rank: send L | reduce L | gather n L
  const size_t lanes = (size_t)(2 + n) * L;
  std::string err;
  for (int i = 0; i < n && err.empty(); i++) {
    std::vector<int64_t> host(lanes, -1);
    for (int j = 0; j < L; j++) host[j] = CheckLane(i, j);
    if (hipSetDevice(c.devs[i]) != hipSuccess || hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&buf[i], lanes * 8) != hipSuccess ||
        hipMemcpyAsync(buf[i], host.data(), lanes * 8, hipMemcpyHostToDevice, s[i]) != hipSuccess ||
        hipStreamSynchronize(s[i]) != hipSuccess)
      err = "RCCL check: HIP setup failed on device " + std::to_string(c.devs[i]);
  }
  std::vector<const int64_t *> sp(n);
  std::vector<int64_t *> rp(n), gp(n), xp(n, nullptr);
  for (int i = 0; i < n; i++) sp[i] = buf[i], rp[i] = buf[i] ? buf[i] + L : nullptr, gp[i] = buf[i] ? buf[i] + 2 * L : nullptr;
  if (err.empty() && !Collective(c, true, sp, rp, xp, s, L, &err)) {
  } else if (err.empty() && !Collective(c, false, sp, gp, xp, s, L, &err)) {
  }
  // bounded: a collective that never completes leaves this open failed
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n && err.empty();) {
    const hipError_t q = hipStreamQuery(s[i]);
    if (q == hipSuccess) {
      i++;
    } else if (q != hipErrorNotReady) {
      err = "RCCL check: stream error on device " + std::to_string(c.devs[i]);
    } else if (Since(t0) > timeout_ms * 1e3) {
      for (auto &x : c.comms)
        if (x) a.abort(x), x = nullptr;
      err = "RCCL check: the collectives did not complete within " + std::to_string(timeout_ms) + " ms";
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  for (int i = 0; i < n && err.empty(); i++) {
    std::vector<int64_t> back(lanes);
    if (hipSetDevice(c.devs[i]) != hipSuccess ||
        hipMemcpy(back.data(), buf[i], lanes * 8, hipMemcpyDeviceToHost) != hipSuccess) {
      err = "RCCL check: copy-back failed on device " + std::to_string(c.devs[i]);
      break;
    }
    for (int r = 0; r < n && err.empty(); r++)
      for (int j = 0; j < L && err.empty(); j++)
        if (back[2 * L + (size_t)r * L + j] != CheckLane(r, j))
          err = "RCCL check: all-gather lane " + std::to_string(j) + " of rank " + std::to_string(r) +
                " differs on rank " + std::to_string(i);
    if (i == 0)
      for (int j = 0; j < L && err.empty(); j++) {
        uint64_t sum = 0;
        for (int r = 0; r < n; r++) sum += (uint64_t)CheckLane(r, j);
        if (back[L + j] != (int64_t)sum) err = "RCCL check: reduce lane " + std::to_string(j) + " differs on rank 0";
      }
  }
  for (int i = 0; i < n; i++) {
    if (!s[i] && !buf[i]) continue;
    (void)hipSetDevice(c.devs[i]);
    if (s[i] && err.find("did not complete") == std::string::npos) (void)hipStreamSynchronize(s[i]);
    if (buf[i] && err.find("did not complete") == std::string::npos) (void)hipFree(buf[i]);
    if (s[i]) (void)hipStreamDestroy(s[i]);
  }
  (void)hipSetDevice(cur);
  return err;
}

// ncclCommInitAll over devs, then CheckComms; the result or why it failed
static std::shared_ptr<Comms> OpenChecked(const std::vector<int> &devs, std::string *note) {
  const Api &a = GetApi();
  if (!a.ok) {
    *note = a.why;
    return nullptr;
  }
  auto c = std::make_shared<Comms>();
  c->devs = devs;
  c->comms.assign(devs.size(), nullptr);
  const auto t0 = std::chrono::steady_clock::now();
  const ncclResult_t r = a.init(c->comms.data(), (int)devs.size(), devs.data());
  c->init_s = Since(t0) * 1e-6;
  if (r != ncclSuccess) {
    c->comms.clear();
    *note = "ncclCommInitAll: " + ErrText(a, r);
    return nullptr;
  }
  const auto t1 = std::chrono::steady_clock::now();
  const std::string err = CheckComms(*c, InitTimeoutMs());
  c->check_us = Since(t1);
  if (!err.empty()) {
    *note = err + ": host merge";
    c->dead = true;
    return nullptr;
  }
  return c;
}

struct Init {
  std::vector<int> devs;
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  bool abandoned = false;  // a waiter gave up: communicators that arrive later are destroyed
  std::shared_ptr<Comms> comms;
  std::string note;
  std::chrono::steady_clock::time_point t0;
};

namespace {
std::mutex g_mu;
std::map<std::vector<int>, std::weak_ptr<Init>> g_opens;  // opens in flight or alive, by device list
std::map<std::vector<int>, std::string> g_failed;        // device lists that failed: why

void Remember(const std::vector<int> &devs, const std::string &why) {
  std::lock_guard<std::mutex> g(g_mu);
  g_failed[devs] = why;
  g_opens.erase(devs);
}
}  // namespace

std::shared_ptr<Init> Prepare(const std::vector<int> &devs) {
  std::lock_guard<std::mutex> g(g_mu);
  auto f = g_failed.find(devs);
  if (f != g_failed.end()) {
    auto in = std::make_shared<Init>();
    in->devs = devs;
    in->done = true;
    in->note = f->second + " (an earlier open of these devices in this process)";
    return in;
  }
  auto w = g_opens.find(devs);
  if (w != g_opens.end())
    if (auto in = w->second.lock()) return in;
  auto in = std::make_shared<Init>();
  in->devs = devs;
  in->t0 = std::chrono::steady_clock::now();
  g_opens[devs] = in;
  // the helper thread holds the Init until it finishes: an init that never
  // completes (a bootstrap that cannot reach itself, a link down) leaves only
  // this thread behind, and the waiters take the host merge after the bound
  std::thread([in] {
    std::string note;
    auto c = OpenChecked(in->devs, &note);
    bool failed = !c;
    {
      std::lock_guard<std::mutex> g(in->mu);
      if (in->abandoned && c) {
        c.reset();  // nobody waits for them any more: destroyed here
        failed = true;
        note = "ncclCommInitAll completed after its waiters had given up";
      }
      in->comms = c;
      if (!c) in->note = note;
      in->done = true;
    }
    in->cv.notify_all();
    if (failed) Remember(in->devs, note);
  }).detach();
  return in;
}

std::shared_ptr<Comms> Wait(const std::shared_ptr<Init> &in, std::string *note, double *waited_ms) {
  const auto t = std::chrono::steady_clock::now();
  std::unique_lock<std::mutex> lk(in->mu);
  const int timeout_ms = InitTimeoutMs();
  const bool ok = in->done || in->cv.wait_until(lk, in->t0 + std::chrono::milliseconds(timeout_ms),
                                                [&] { return in->done; });
  if (waited_ms) *waited_ms = Since(t) * 1e-3;
  if (!ok) {
    in->abandoned = true;
    lk.unlock();
    const std::string why = "ncclCommInitAll + check did not complete within " + std::to_string(timeout_ms) + " ms";
    Remember(in->devs, why);
    *note = why + ": host merge";
    return nullptr;
  }
  if (!in->comms || in->comms->dead) {
    *note = in->note.empty() ? "RCCL communicators unavailable: host merge" : in->note;
    return nullptr;
  }
  return in->comms;
}

const char *InitState(const Init &in) {
  std::lock_guard<std::mutex> g(const_cast<Init &>(in).mu);
  if (!in.done) return "pending";
  return in.comms && !in.comms->dead ? "ready" : "failed";
}

void MarkDead(Comms &c, const std::string &why) {
  c.dead = true;
  if (!c.loopback) Remember(c.devs, why);
}

void Abort(Comms &c, const std::string &why) {
  const Api &a = GetApi();
  for (auto &x : c.comms)
    if (x && a.abort) a.abort(x), x = nullptr;
  MarkDead(c, why);
}

__global__ void sum_lanes_kernel(const int64_t *g, int nranks, int lanes, int64_t *out) {
  for (int j = threadIdx.x; j < lanes; j += blockDim.x) {
    int64_t s = 0;
    for (int r = 0; r < nranks; r++) s += g[(int64_t)r * lanes + j];
    out[j] = s;
  }
}

bool Collective(Comms &c, bool reduce, const std::vector<const int64_t *> &send, const std::vector<int64_t *> &recv,
                const std::vector<int64_t *> &scratch, const std::vector<hipStream_t> &streams, size_t count,
                std::string *err) {
  const int n = (int)c.devs.size();
  if (Knob("MBX_RCCL_TEST_FAIL")) {  // tests: a collective that reports an error before any rank's part runs
    *err = "injected collective failure (MBX_RCCL_TEST_FAIL)";
    return false;
  }
  if (c.loopback) {
    // the data movement of the collective as device copies after every
    // sender's pack: the all-gather lands every rank's block in every rank's
    // receive buffer; the reduce lands them in rank 0's scratch, summed there
    // by one small kernel
    std::vector<hipEvent_t> ev(n, nullptr);
    bool ok = true;
    for (int i = 0; i < n && ok; i++) {
      ok = hipSetDevice(c.devs[i]) == hipSuccess &&
           hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) == hipSuccess &&
           hipEventRecord(ev[i], streams[i]) == hipSuccess;
    }
    for (int j = 0; j < (reduce ? 1 : n) && ok; j++) {
      ok = hipSetDevice(c.devs[j]) == hipSuccess;
      int64_t *dst = reduce ? scratch[j] : recv[j];
      for (int i = 0; i < n && ok; i++)
        ok = hipStreamWaitEvent(streams[j], ev[i], 0) == hipSuccess &&
             hipMemcpyAsync(dst + (size_t)i * count, send[i], count * 8, hipMemcpyDeviceToDevice, streams[j]) ==
                 hipSuccess;
      if (ok && reduce) {
        hipLaunchKernelGGL(sum_lanes_kernel, dim3(1), dim3(64), 0, streams[j], (const int64_t *)dst, n, (int)count,
                           recv[j]);
        ok = hipGetLastError() == hipSuccess;
      }
    }
    for (int i = 0; i < n; i++)
      if (ev[i]) (void)hipEventDestroy(ev[i]);
    if (!ok) *err = "RCCL loopback: a HIP call failed";
    return ok;
  }
  // one thread drives every rank: the calls are fused into one group, so no
  // rank's collective waits for a call that is never made
  const Api &a = GetApi();
  ncclResult_t r = a.gstart();
  if (r != ncclSuccess) {
    *err = "ncclGroupStart: " + ErrText(a, r);
    return false;
  }
  ncclResult_t first = ncclSuccess;
  for (int i = 0; i < n; i++) {
    const ncclResult_t ri = reduce ? a.reduce(send[i], recv[i], count, ncclInt64, ncclSum, 0, c.comms[i], streams[i])
                                   : a.allgather(send[i], recv[i], count, ncclInt64, c.comms[i], streams[i]);
    if (ri != ncclSuccess && first == ncclSuccess) first = ri;
  }
  r = a.gend();
  if (first != ncclSuccess) {
    *err = std::string(reduce ? "ncclReduce: " : "ncclAllGather: ") + ErrText(a, first);
    return false;
  }
  if (r != ncclSuccess) {
    *err = "ncclGroupEnd: " + ErrText(a, r);
    return false;
  }
  return true;
}

std::string SelfTest(const std::vector<int> &devs, SelfTestInfo *info) {
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t i = 0; i < devs.size(); i++)
    for (size_t j = i + 1; j < devs.size(); j++)
      if (devs[i] == devs[j]) return "RCCL self-test: devices are not distinct (one rank per device)";
  if (devs.empty()) return "RCCL self-test: no device";
  // a fresh open on the helper thread, bounded as the combine's is; not shared
  // with connections and not remembered as a failure
  struct St {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    std::shared_ptr<Comms> c;
    std::string note;
  };
  auto st = std::make_shared<St>();
  std::thread([st, devs] {
    std::string note;
    auto c = OpenChecked(devs, &note);
    std::lock_guard<std::mutex> g(st->mu);
    st->c = c, st->note = note, st->done = true;
    st->cv.notify_all();
  }).detach();
  std::unique_lock<std::mutex> lk(st->mu);
  if (!st->cv.wait_for(lk, std::chrono::milliseconds(InitTimeoutMs()), [&] { return st->done; }))
    return "RCCL self-test: ncclCommInitAll + check did not complete within " + std::to_string(InitTimeoutMs()) +
           " ms";
  std::shared_ptr<Comms> c = st->c;
  const std::string note = st->note;
  st->c.reset();
  lk.unlock();
  if (!c) return note.empty() ? "RCCL unavailable" : note;
  if (info) {
    info->init_us = c->init_s * 1e6;
    info->check_us = c->check_us;
    info->count = c->count, info->user_rank = c->user_rank, info->cu_device = c->cu_device;
  }
  c.reset();  // ncclCommDestroy on every rank
  if (info) info->total_us = Since(t0);
  return "";
}

// element i of an integer column widened to int128 {lo, hi}
__device__ __forceinline__ void widen(uint8_t phys, const void *p, int64_t i, int64_t &lo, int64_t &hi) {
  bool unsigned_ = false;
  switch (phys) {
    case P_U8: lo = ((const uint8_t *)p)[i], unsigned_ = true; break;
    case P_I8: lo = ((const int8_t *)p)[i]; break;
    case P_I16: lo = ((const int16_t *)p)[i]; break;
    case P_U16: lo = ((const uint16_t *)p)[i], unsigned_ = true; break;
    case P_I32: lo = ((const int32_t *)p)[i]; break;
    case P_U32: lo = ((const uint32_t *)p)[i], unsigned_ = true; break;
    case P_U64: lo = ((const int64_t *)p)[i], unsigned_ = true; break;  // (zero-extended below)
    case P_I128:
      lo = ((const int64_t *)p)[2 * i], hi = ((const int64_t *)p)[2 * i + 1];
      return;
    default: lo = ((const int64_t *)p)[i]; break;
  }
  hi = unsigned_ ? 0 : (lo < 0 ? -1 : 0);
}

// one lane group per column: row 0's value widened to int128, its validity
__global__ void pack_lanes_kernel(PackDesc d, int64_t *dst) {
  const int j = threadIdx.x;
  if (j < d.ncols) {
    int64_t lo = 0, hi = 0;
    widen(d.phys[j], d.data[j], 0, lo, hi);
    const bool ok = !d.valid[j] || (d.valid[j][0] & 1);
    if (d.counts_only) {
      dst[j] = ok ? lo : 0;
    } else {
      dst[3 * j] = ok ? lo : 0;
      dst[3 * j + 1] = ok ? hi : 0;
      dst[3 * j + 2] = ok ? 1 : 0;
    }
  }
  if (j == 0) dst[d.counts_only ? d.ncols : 3 * d.ncols] = d.err ? *d.err : 0;
}

void Pack(const PackDesc &d, int64_t *dst, hipStream_t s) {
  hipLaunchKernelGGL(pack_lanes_kernel, dim3(1), dim3(64), 0, s, d, dst);
}

__global__ void combine_lanes_kernel(CombineDesc d, const int64_t *g, int64_t *out) {
  const int j = threadIdx.x;
  if (j < d.ncols) CombineColumn(g, d.nranks, LanesPerRank(d.ncols, false), j, d.kind[j], out + 3 * j);
}

void Combine(const CombineDesc &d, const int64_t *gathered, int64_t *out, hipStream_t s) {
  hipLaunchKernelGGL(combine_lanes_kernel, dim3(1), dim3(64), 0, s, d, gathered, out);
}

// one thread per partial GROUP BY row: its slot's presence lane and column
// lanes (the block was zeroed, so absent slots stay {0, 0, invalid})
__global__ void pack_rows_kernel(PackRowsDesc d, int64_t *dst) {
  const int64_t sl_lanes = SlotLanes(d.ncols);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < d.nrows; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t klo = 0, khi = 0;
    widen(d.key_phys, d.key, i, klo, khi);
    const bool knull = d.key_valid && !((d.key_valid[i >> 6] >> (i & 63)) & 1);
    const int64_t slot = knull ? d.nslot - 1 : klo - d.kmin;
    if (slot < 0 || slot >= d.nslot) continue;  // (the host derived kmin / nslot from these keys)
    int64_t *o = dst + slot * sl_lanes;
    o[0] = 1;
    for (int j = 0; j < d.ncols; j++) {
      int64_t lo = 0, hi = 0;
      widen(d.phys[j], d.data[j], i, lo, hi);
      const bool ok = !d.valid[j] || ((d.valid[j][i >> 6] >> (i & 63)) & 1);
      o[1 + 3 * j] = ok ? lo : 0;
      o[2 + 3 * j] = ok ? hi : 0;
      o[3 + 3 * j] = ok ? 1 : 0;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) dst[d.nslot * sl_lanes] = d.err ? *d.err : 0;
}

void PackRows(const PackRowsDesc &d, int64_t *dst, hipStream_t s) {
  const int64_t lanes = d.nslot * SlotLanes(d.ncols) + 1;
  (void)hipMemsetAsync(dst, 0, (size_t)lanes * 8, s);
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((d.nrows + 255) / 256, 1024));
  hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d, dst);
}

// one thread per slot: presence ORed over the ranks, every column combined as
// the global combine does; then every rank's error word after the slots
__global__ void combine_slots_kernel(CombineDesc d, int64_t nslot, const int64_t *g, int64_t *out) {
  const int64_t sl_lanes = SlotLanes(d.ncols), stride = nslot * sl_lanes + 1;
  for (int64_t sl = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; sl < nslot; sl += (int64_t)gridDim.x * blockDim.x) {
    int64_t present = 0;
    for (int r = 0; r < d.nranks; r++) present |= g[(int64_t)r * stride + sl * sl_lanes];
    int64_t *o = out + sl * sl_lanes;
    o[0] = present;
    for (int j = 0; j < d.ncols; j++)
      CombineColumn(g + sl * sl_lanes + 1, d.nranks, (int)stride, j, d.kind[j], o + 1 + 3 * j);
  }
  if (blockIdx.x == 0 && threadIdx.x < d.nranks)
    out[nslot * sl_lanes + threadIdx.x] = g[(int64_t)threadIdx.x * stride + stride - 1];
}

void CombineSlots(const CombineDesc &d, int64_t nslot, const int64_t *gathered, int64_t *out, hipStream_t s) {
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((nslot + 255) / 256, 64));
  hipLaunchKernelGGL(combine_slots_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d, nslot, gathered, out);
}

}  // namespace rc
}  // namespace mbx
