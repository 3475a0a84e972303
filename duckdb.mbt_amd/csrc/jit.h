// jit.h — run-time specialised expression kernels.
//
// The tile interpreter (vm_filter_kernel / vm_project_kernel in kernels.hip)
// reads every instruction at run time and keeps registers in LDS planes.  For
// a program seen before, jit.cpp emits HIP source in which every instruction
// is a vm_step(...) call with literal operands (vm_device.h), compiles it for
// gfx950 with hipRTC on a background thread and caches the code object by the
// program's shape (opcodes, registers, column types, outputs — not constant
// values, which stay kernel arguments).  Until the kernel is ready, and
// whenever compilation fails, the interpreter runs: results are identical.
//   MBX_JIT=0      never compile (interpreter only)
//   MBX_JIT=sync   compile on first use and wait (tests, benchmarks)
//   default        compile asynchronously, switch over when ready
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <string>

#include "vm.h"

namespace mbx {
namespace jit {

// true: launched the specialised filter (same outputs as dev::VmFilter)
bool VmFilter(const VmProgram &p, const dev::VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
              uint64_t *sel_bits, uint32_t *tile_counts, int32_t *err, hipStream_t s);
// true: launched the specialised projection (same outputs as dev::VmProject)
bool VmProject(const VmProgram &p, const dev::VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
               const uint64_t *sel_bits, const int64_t *tile_offsets, const dev::VmOuts &outs, int32_t *err,
               hipStream_t s);
// Fused scan -> filter -> project -> aggregate without GROUP BY: evaluates
// the predicate register p.pred_reg (255 = none) and, per aggregate j <
// p.n_out, the argument register p.out_reg[j] (255 = COUNT(*)) of class
// p.out_class[j] (VC_I64 / VC_I128 sums / VC_F64), and merges every wave's
// accumulators into states[j] (dev::AggState layout, pre-initialised) and the
// selected-row count into *count_star.  true: launched.
bool VmAggregate(const VmProgram &p, const dev::VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
                 void *states, unsigned long long *count_star, int32_t *err, hipStream_t s);
// Fused scan -> filter -> project -> GROUP BY over up to JIT_MAX_KEYS integer
// keys of small known range (column statistics): each selected row goes to
// slot sum_i digit_i * stride[i], digit_i = key_i - kmin[i], or radix[i] - 1
// for a NULL key when key_nullable[i].  The kernel keeps per-block LDS slot
// tables (R replicas, overflow-exact int64 sums) and merges them into
// count_star[slot] and states[j * nslots + slot] (dev::AggState layout,
// pre-initialised) for every aggregate j with p.out_reg[j] != 255 (class
// VC_I64 only; p.out_phys[j] = statistics needed, as for VmAggregate).
#define JIT_MAX_KEYS 4
struct GroupSpec {
  int32_t nkeys, nslots;
  uint8_t key_reg[JIT_MAX_KEYS], key_nullable[JIT_MAX_KEYS];
  int64_t kmin[JIT_MAX_KEYS], radix[JIT_MAX_KEYS], stride[JIT_MAX_KEYS];
};
// LDS bytes of one block's slot tables at R replicas.
size_t GroupLdsBytes(const VmProgram &p, int64_t nslots, int R);
bool VmGroupAggregate(const VmProgram &p, const dev::VmCols &cols, const GroupSpec &g, int64_t nrows,
                      int64_t range_start, int64_t range_step, void *states, unsigned long long *count_star,
                      int32_t *err, hipStream_t s);
std::string GroupSourceForTest(const VmProgram &p, const dev::VmCols &cols, const GroupSpec &g);
bool Enabled();
// Waits for every background compile.  Called on disconnect and from the
// Python binding's atexit: a compile still inside hipRTC while exit() runs
// the compiler's static destructors (registered after ours, so run first)
// can hang the process.
void JoinPending();

// The generated source for a program (exposed for tests and EXPLAIN).
std::string Source(const VmProgram &p, const dev::VmCols &cols, bool filter);
// Compiles source for gfx950 without loading it (no GPU needed); "" = ok,
// else the compiler log.
std::string CompileCheck(const std::string &src);
std::string AggSourceForTest(const VmProgram &p, const dev::VmCols &cols);

}  // namespace jit
}  // namespace mbx
