// rccl_combine.h — RCCL communicators over a connection's shard devices and
// the two small kernels around the collective (mbx_combine=rccl).
//
// one process, ncclCommInitAll over the shard devices, COUNT
// as an ncclInt64 reduce to device 0, SUM int128 as an all-gather of 16-byte partials
// with a carry-correct combine on device 0.  librccl is opened with dlopen on
// first use, so the library loads (and the host merge runs) where it is
// absent.  Lane layout: combine.h.
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "combine.h"

struct ncclComm;  // RCCL's communicator (ncclComm_t)

namespace mbx {
namespace rc {

// one communicator per shard device (rank i = devs[i]); none in loopback
struct Comms {
  std::vector<int> devs;
  std::vector<ncclComm *> comms;
  bool loopback = false;
  ~Comms();
};

// ncclCommInitAll over devs (distinct devices, one rank each); nullptr and a
// reason in *note when librccl is missing or the init fails.  loopback (tests
// only, MBX_EXPERIMENTS=1): no communicator; Collective moves the same lanes
// with device copies, so the pack / combine kernels and the host decode run on
// a box with one GPU (same-device shards).
std::shared_ptr<Comms> Open(const std::vector<int> &devs, bool loopback, std::string *note);
bool IsLoopback(const Comms &c);
// ncclCommAbort on every rank (a collective that never completed); the
// communicators are gone afterwards
void Abort(Comms &c);

// One collective over every rank, driven from the calling thread: rank i's
// count int64 lanes send[i] on streams[i] -> recv[i] (all-gather: n * count
// lanes in rank order on every rank; reduce: count lanes summed into rank 0's
// recv).  The RCCL calls are fused in one ncclGroupStart/End, so no rank can
// be left inside a collective that another rank never joined.  scratch[0]
// (n * count lanes) is used by the loopback reduce only.  false and *err on
// an RCCL / HIP error.
bool Collective(Comms &c, bool reduce, const std::vector<const int64_t *> &send, const std::vector<int64_t *> &recv,
                const std::vector<int64_t *> &scratch, const std::vector<hipStream_t> &streams, size_t count,
                std::string *err);

// Hardware check of the RCCL calls the combine makes, for a box with one GPU:
// a one-rank communicator on `device` (ncclCommInitAll on the helper thread),
// one grouped reduce and one grouped all-gather of 97 int64 lanes, the lanes
// checked.  Returns "" (and the wall time in *us) or what failed.
std::string SelfTest(int device, double *us);

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

// GROUP BY on one integer key: a rank's partial relation (nrows groups) packed
// into dense key slots -- slot = key - kmin, the NULL key in slot nslot - 1 --
// each SlotLanes(ncols) lanes {present, then {lo, hi, valid} per column}, the
// device error word after the last slot (nslot * SlotLanes + 1 lanes; PackRows
// zeroes the block first, so a group the rank lacks stays absent)
struct PackRowsDesc {
  const void *key;
  const uint64_t *key_valid;
  const void *data[kMaxCols];
  const uint64_t *valid[kMaxCols];
  uint8_t phys[kMaxCols];
  uint8_t key_phys;
  int ncols;
  int64_t nrows, kmin, nslot;
  const int32_t *err;
};
void PackRows(const PackRowsDesc &d, int64_t *dst, hipStream_t s);
// out[slot * SlotLanes ..] = the slot over the nranks gathered blocks (presence
// ORed, columns as CombineColumn), then every rank's error word
void CombineSlots(const CombineDesc &d, int64_t nslot, const int64_t *gathered, int64_t *out, hipStream_t s);

}  // namespace rc
}  // namespace mbx
