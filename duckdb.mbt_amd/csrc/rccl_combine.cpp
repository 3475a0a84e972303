// rccl_combine.cpp — RCCL communicators of a sharded connection and the pack /
// combine kernels around its collectives (see rccl_combine.h, combine.h).
#include "rccl_combine.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
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
    api.ok = api.init && api.destroy && api.allgather && api.reduce && api.errstr && api.gstart && api.gend;
    if (!api.ok) api.why = "librccl lacks an entry point";
  });
  return api;
}

std::string ErrText(const Api &a, ncclResult_t r) {
  return std::string("RCCL error: ") + (a.errstr ? a.errstr(r) : "?") + " (" + std::to_string((int)r) + ")";
}
}  // namespace

Comms::~Comms() {
  if (comms.empty()) return;
  const Api &a = GetApi();
  for (auto c : comms)
    if (c && a.destroy) a.destroy(c);
}

std::shared_ptr<Comms> Open(const std::vector<int> &devs, bool loopback, std::string *note) {
  auto c = std::make_shared<Comms>();
  c->devs = devs;
  if (loopback) {  // test stand-in: no communicator, the collectives become copies
    c->loopback = true;
    return c;
  }
  const Api &a = GetApi();
  if (!a.ok) {
    *note = a.why;
    return nullptr;
  }
  for (size_t i = 0; i < devs.size(); i++)
    for (size_t j = i + 1; j < devs.size(); j++)
      if (devs[i] == devs[j]) {
        *note = "shard devices are not distinct (RCCL takes one rank per device): host merge";
        return nullptr;
      }
  // the communicators are built on a helper thread, given a bounded time: an
  // init that never completes (a bootstrap that cannot reach itself, a link
  // down) leaves the host merge in charge instead of hanging the statement
  struct Init {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    ncclResult_t r = ncclInternalError;
    std::vector<ncclComm_t> comms;
  };
  auto st = std::make_shared<Init>();
  st->comms.assign(devs.size(), nullptr);
  std::thread([st, devs, &a] {
    const ncclResult_t r = a.init(st->comms.data(), (int)devs.size(), devs.data());
    std::lock_guard<std::mutex> g(st->mu);
    st->r = r;
    st->done = true;
    st->cv.notify_all();
  }).detach();
  static const int timeout_ms = [] {
    const char *v = Knob("MBX_RCCL_INIT_TIMEOUT_MS");
    return v ? std::max(1, atoi(v)) : 60000;
  }();
  std::unique_lock<std::mutex> lk(st->mu);
  if (!st->cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return st->done; })) {
    *note = "ncclCommInitAll did not complete within " + std::to_string(timeout_ms) + " ms: host merge";
    return nullptr;  // (the init thread keeps its communicators if it ever finishes)
  }
  if (st->r != ncclSuccess) {
    *note = "ncclCommInitAll: " + ErrText(a, st->r);
    return nullptr;
  }
  c->comms.assign(st->comms.begin(), st->comms.end());
  return c;
}

bool IsLoopback(const Comms &c) { return c.loopback; }

void Abort(Comms &c) {
  const Api &a = GetApi();
  for (auto &x : c.comms)
    if (x && a.abort) a.abort(x), x = nullptr;
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

std::string SelfTest(int device, double *us) {
  std::string note;
  const auto t0 = std::chrono::steady_clock::now();
  auto c = Open({device}, false, &note);
  if (!c) return note.empty() ? "RCCL unavailable" : note;
  int cur = 0;
  (void)hipGetDevice(&cur);
  std::string err;
  hipStream_t s = nullptr;
  int64_t *buf = nullptr;
  constexpr int kLanes = 97;  // an odd lane count: 3 columns x 32 + the error word
  int64_t host[3 * kLanes];
  for (int i = 0; i < kLanes; i++) host[i] = (int64_t)0x123456789abcdefLL * (i + 1) - (int64_t)i * i;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void **)&buf, sizeof(host)) != hipSuccess ||
      hipMemsetAsync(buf, 0xff, sizeof(host), s) != hipSuccess ||
      hipMemcpyAsync(buf, host, kLanes * 8, hipMemcpyHostToDevice, s) != hipSuccess) {
    err = "RCCL self-test: HIP setup failed";
  }
  // one rank: the reduce and the all-gather each return the send lanes
  if (err.empty() && !Collective(*c, true, {buf}, {buf + kLanes}, {nullptr}, {s}, kLanes, &err)) {
  } else if (err.empty() && !Collective(*c, false, {buf}, {buf + 2 * kLanes}, {nullptr}, {s}, kLanes, &err)) {
  }
  int64_t back[3 * kLanes];
  if (err.empty() && (hipMemcpyAsync(back, buf, sizeof(back), hipMemcpyDeviceToHost, s) != hipSuccess ||
                      hipStreamSynchronize(s) != hipSuccess))
    err = "RCCL self-test: HIP copy-back failed";
  if (err.empty())
    for (int i = 0; i < kLanes && err.empty(); i++)
      if (back[kLanes + i] != host[i] || back[2 * kLanes + i] != host[i])
        err = "RCCL self-test: lane " + std::to_string(i) + " differs after the collectives";
  if (s) (void)hipStreamSynchronize(s), (void)hipStreamDestroy(s);
  if (buf) (void)hipFree(buf);
  (void)hipSetDevice(cur);
  *us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  return err;
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
