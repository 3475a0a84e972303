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

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "combine.h"

struct ncclComm;  // RCCL's communicator (ncclComm_t)

namespace mbx {
namespace rc {

// one communicator per shard device (rank i = devs[i]); none in loopback.
// Connections over the same device list share one set (Prepare), so a
// collective and its bounded wait run under `mu`.
struct Comms {
  std::vector<int> devs;
  std::vector<ncclComm *> comms;
  bool loopback = false;
  std::mutex mu;
  std::atomic<bool> dead{false};  // aborted or failed: never used again
  // what RCCL reports for each communicator (ncclCommCount / ncclCommUserRank /
  // ncclCommCuDevice; -1 where librccl lacks the query), and the open's cost
  std::vector<int> count, user_rank, cu_device;
  double init_s = 0;     // ncclCommInitAll
  double check_us = 0;   // the multi-rank check that gates the communicators
  ~Comms();
};

// One open of the communicators over a device list, run on a helper thread:
// ncclCommInitAll, then a check of every rank (one grouped ncclReduce and one
// ncclAllGather of known lanes, verified on every rank, and the rank count RCCL
// reports) -- the combine uses the communicators only when that check passed.
// A failed or timed-out open is remembered for the process, keyed by the
// device list, so later connections go straight to the host merge.
struct Init;
// Starts (or joins) the open for devs; never blocks.  Distinct devices only
// (the caller checks); a device list that failed before gets a finished Init
// carrying that failure.
std::shared_ptr<Init> Prepare(const std::vector<int> &devs);
// The communicators of an open, waiting for it up to MBX_RCCL_INIT_TIMEOUT_MS
// (default 30 s) from the open's start; nullptr and *note when unavailable.
// *waited_ms: how long this call blocked.
std::shared_ptr<Comms> Wait(const std::shared_ptr<Init> &in, std::string *note, double *waited_ms);
const char *InitState(const Init &in);  // "pending" / "ready" / "failed"
// the loopback stand-in (tests only, MBX_EXPERIMENTS=1): no communicator;
// Collective moves the same lanes with device copies, so the pack / combine
// kernels and the host decode run on a box with one GPU (same-device shards)
std::shared_ptr<Comms> OpenLoopback(const std::vector<int> &devs);
bool IsLoopback(const Comms &c);
// ncclCommAbort on every rank (a collective that never completed), then as
// MarkDead; the communicators are gone afterwards
void Abort(Comms &c, const std::string &why);
// the communicators failed (a collective error): every connection sharing them,
// and every later open of this device list in the process, takes the host merge
void MarkDead(Comms &c, const std::string &why);
// librccl has what the combine needs (ncclCommAbort included: a collective
// that cannot be aborted is never started); "" or why not
std::string ApiProblem();

// One collective over every rank, driven from the calling thread: rank i's
// count int64 lanes send[i] on streams[i] -> recv[i] (all-gather: n * count
// lanes in rank order on every rank; reduce: count lanes summed into rank 0's
// recv).  The RCCL calls are fused in one ncclGroupStart/End, so no rank can
// be left inside a collective that another rank never joined.  scratch[0]
// (n * count lanes) is used by the loopback reduce only.  false and *err on
// an RCCL / HIP error.  The caller holds c.mu until the streams have drained.
bool Collective(Comms &c, bool reduce, const std::vector<const int64_t *> &send, const std::vector<int64_t *> &recv,
                const std::vector<int64_t *> &scratch, const std::vector<hipStream_t> &streams, size_t count,
                std::string *err);

// Hardware check of the RCCL calls the combine makes, over `devs` (distinct
// devices; one device on a one-GPU box): a fresh ncclCommInitAll (on the
// helper thread, bounded) and the multi-rank check the combine is gated on.
// Returns "" or what failed; *info gets what RCCL reported.
struct SelfTestInfo {
  double init_us = 0, check_us = 0, total_us = 0;
  std::vector<int> count, user_rank, cu_device;
};
std::string SelfTest(const std::vector<int> &devs, SelfTestInfo *info);

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
