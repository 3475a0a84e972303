// rccl_combine.cpp — RCCL communicators of a sharded connection and the pack /
// combine kernels around its collectives (see rccl_combine.h, combine.h).
#include "rccl_combine.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <mutex>

#include "phys.h"

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
  decltype(&ncclAllReduce) allreduce = nullptr;
  decltype(&ncclGetErrorString) errstr = nullptr;
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
    api.allreduce = (decltype(api.allreduce))dlsym(h, "ncclAllReduce");
    api.errstr = (decltype(api.errstr))dlsym(h, "ncclGetErrorString");
    api.ok = api.init && api.destroy && api.allgather && api.allreduce && api.errstr;
    if (!api.ok) api.why = "librccl lacks an entry point";
  });
  return api;
}

std::string ErrText(const Api &a, ncclResult_t r) {
  return std::string("RCCL error: ") + (a.errstr ? a.errstr(r) : "?") + " (" + std::to_string((int)r) + ")";
}
}  // namespace

struct Comms {
  std::vector<int> devs;
  std::vector<ncclComm_t> comms;
  ~Comms() {
    const Api &a = GetApi();
    for (auto c : comms)
      if (c && a.destroy) a.destroy(c);
  }
};

std::shared_ptr<Comms> Open(const std::vector<int> &devs, std::string *note) {
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
  int cur = 0;
  (void)hipGetDevice(&cur);
  auto c = std::make_shared<Comms>();
  c->devs = devs;
  c->comms.assign(devs.size(), nullptr);
  const ncclResult_t r = a.init(c->comms.data(), (int)devs.size(), devs.data());
  (void)hipSetDevice(cur);
  if (r != ncclSuccess) {
    c->comms.clear();
    *note = "ncclCommInitAll: " + ErrText(a, r);
    return nullptr;
  }
  return c;
}

bool AllGather(Comms &c, int rank, const int64_t *send, int64_t *recv, size_t count, hipStream_t s,
               std::string *err) {
  const Api &a = GetApi();
  const ncclResult_t r = a.allgather(send, recv, count, ncclInt64, c.comms[rank], s);
  if (r != ncclSuccess) *err = "ncclAllGather: " + ErrText(a, r);
  return r == ncclSuccess;
}

bool AllReduceSum(Comms &c, int rank, const int64_t *send, int64_t *recv, size_t count, hipStream_t s,
                  std::string *err) {
  const Api &a = GetApi();
  const ncclResult_t r = a.allreduce(send, recv, count, ncclInt64, ncclSum, c.comms[rank], s);
  if (r != ncclSuccess) *err = "ncclAllReduce: " + ErrText(a, r);
  return r == ncclSuccess;
}

// one lane group per column: row 0's value widened to int128, its validity
__global__ void pack_lanes_kernel(PackDesc d, int64_t *dst) {
  const int j = threadIdx.x;
  if (j < d.ncols) {
    const void *p = d.data[j];
    int64_t lo = 0, hi = 0;
    switch (d.phys[j]) {
      case P_U8: lo = *(const uint8_t *)p; break;
      case P_I8: lo = *(const int8_t *)p; break;
      case P_I16: lo = *(const int16_t *)p; break;
      case P_U16: lo = *(const uint16_t *)p; break;
      case P_I32: lo = *(const int32_t *)p; break;
      case P_U32: lo = *(const uint32_t *)p; break;
      case P_U64: lo = *(const int64_t *)p; break;  // (zero-extended below)
      case P_I128: lo = ((const int64_t *)p)[0], hi = ((const int64_t *)p)[1]; break;
      default: lo = *(const int64_t *)p; break;
    }
    if (d.phys[j] != P_I128 && d.phys[j] != P_U64 && d.phys[j] != P_U8 && d.phys[j] != P_U16 && d.phys[j] != P_U32)
      hi = lo < 0 ? -1 : 0;
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

}  // namespace rc
}  // namespace mbx
