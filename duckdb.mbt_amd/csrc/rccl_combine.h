// rccl_combine.h — RCCL communicators over a connection's shard devices and
// the two small kernels around the collective (mbx_combine=rccl).
//
// one process, ncclCommInitAll over the shard devices, COUNT
// as an ncclInt64 all-reduce, SUM int128 as an all-gather of 16-byte partials
// with a carry-correct combine on device 0.  librccl is opened with dlopen on
// first use, so the library loads (and the host merge runs) where it is
// absent.  Lane layout: combine.h.
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "combine.h"

namespace mbx {
namespace rc {

struct Comms;  // one ncclComm_t per shard device (rank i = devs[i])

// ncclCommInitAll over devs (distinct devices, one rank each); nullptr and a
// reason in *note when librccl is missing or the init fails.
std::shared_ptr<Comms> Open(const std::vector<int> &devs, std::string *note);

// rank's part of the collective on its device's stream (the caller keeps that
// device current); false and *err on an RCCL error
bool AllGather(Comms &c, int rank, const int64_t *send, int64_t *recv, size_t count, hipStream_t s, std::string *err);
bool AllReduceSum(Comms &c, int rank, const int64_t *send, int64_t *recv, size_t count, hipStream_t s,
                  std::string *err);

// the lanes of a one-row partial relation (row 0 of every column) and the
// device error word, written to dst by one small kernel
struct PackDesc {
  const void *data[kMaxCols];
  const uint64_t *valid[kMaxCols];
  uint8_t phys[kMaxCols];  // mbx::Phys of each column (integer classes only)
  int ncols;
  bool counts_only;
  const int32_t *err;
};
void Pack(const PackDesc &d, int64_t *dst, hipStream_t s);

// out[3 j ..] = CombineColumn over the nranks ranks' gathered lanes, on the device
struct CombineDesc {
  int8_t kind[kMaxCols];
  int ncols;
  int nranks;
};
void Combine(const CombineDesc &d, const int64_t *gathered, int64_t *out, hipStream_t s);

}  // namespace rc
}  // namespace mbx
