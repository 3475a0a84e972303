// kernels.hip — hand-written gfx950 (CDNA4) kernels of the columnar backend.
//
// All of this is HBM-bound integer/byte work: no MFMA.  Design rules applied
// (cdna_hip_programming.md §6 G2/G7/G11/G12/G13):
//   * 16-byte vector loads (global_load_dwordx4), several in flight per lane;
//   * wave64 ballot / mbcnt for predicate compaction and bit packing;
//   * per-thread -> per-wave (DPP/shuffle) -> per-block (LDS) reduction and
//     ONE global atomic per block and aggregate (128-bit sums as a carry-correct
//     pair of 64-bit atomics, exact in any order);
//   * GROUP BY on small key ranges in LDS-privatised replicated tables
//     (one replica per lane index -> no same-address conflicts inside a wave).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <limits>
#include <stdexcept>
#include <stdint.h>

#include "device.h"
#include "types.h"

// ---------------------------------------------------------------------------
// In-kernel clock stamps (diagnostic build only: make clockdiag compiles this
// file with MBX_CLOCK_STAMPS=1 into libduckdb_mb_amd_clk.so; in the product
// library no stamp instruction exists).  Thread 0 of each of the first
// kClkSlots workgroups of filter_agg_lds, group_direct_lds and the two-array
// ring read records the shader-clock counter (s_memtime) and the 100 MHz
// reference counter (s_memrealtime) once when its main loop starts and once
// when it has drained, with ordinary vector stores.  Clock of a workgroup =
// d(memtime) / d(realtime) x 100 MHz (MI355X_MICROARCH.md, DVFS item 6).
// ---------------------------------------------------------------------------
namespace mbx {
namespace dev {
constexpr int kClkSlots = 1024;
}
}  // namespace mbx
#if MBX_CLOCK_STAMPS
__device__ unsigned long long g_clk_stamps[mbx::dev::kClkSlots * 4];
__device__ __forceinline__ void clk_stamp(int part) {
  if (threadIdx.x == 0 && blockIdx.x < mbx::dev::kClkSlots) {
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    g_clk_stamps[blockIdx.x * 4 + part * 2] = c;
    g_clk_stamps[blockIdx.x * 4 + part * 2 + 1] = r;
  }
}
#define MBX_CLK(part) clk_stamp(part)
#else
#define MBX_CLK(part)
#endif
#include "vm.h"
#include "vm_device.h"
#include "knobs.h"

namespace mbx {
namespace dev {

static thread_local TempAllocFn g_talloc = nullptr;
static thread_local TempFreeFn g_tfree = nullptr;
static thread_local void *g_tctx = nullptr;
void SetTempAllocator(TempAllocFn a, TempFreeFn f, void *ctx) {
  g_talloc = a;
  g_tfree = f;
  g_tctx = ctx;
}
static void *TempAlloc(size_t bytes) {
  if (!g_talloc) throw std::runtime_error("device scratch allocator not set");
  void *p = g_talloc(bytes, g_tctx);
  if (!p) throw std::runtime_error("device scratch allocation failed");
  return p;
}
static void TempFree(void *p, size_t bytes) {
  if (p && g_tfree) g_tfree(p, bytes, g_tctx);
}

typedef __int128 i128;
typedef unsigned __int128 u128;

#define CHECK_LAUNCH() (void)hipGetLastError()

static int g_num_cus = 0;
int NumCUs() {
  if (!g_num_cus) {
    int d = 0;
    (void)hipGetDevice(&d);
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, d) == hipSuccess) g_num_cus = pr.multiProcessorCount;
    if (g_num_cus <= 0) g_num_cus = 256;
  }
  return g_num_cus;
}

static inline int GridFor(int64_t work_items, int per_block, int max_blocks) {
  int64_t b = (work_items + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > max_blocks) b = max_blocks;
  return (int)b;
}

// ---------------------------------------------------------------------------
// expression VM (tile interpreter)
// ---------------------------------------------------------------------------
// VM register planes [reg][row] in dynamic LDS sized to the program's
// register count (P.n_regs), not VM_MAX_REGS: short programs leave room for
// more resident workgroups, i.e. more row loads in flight per CU.
struct VmLds {
  int64_t *lo;
  int64_t *hi;
  uint8_t *nl;
};
__device__ __forceinline__ VmLds vm_regs(unsigned char *base, int n_regs) {
  VmLds R;
  R.lo = (int64_t *)base;
  R.hi = R.lo + (size_t)n_regs * VM_TILE;
  R.nl = (uint8_t *)(R.hi + (size_t)n_regs * VM_TILE);
  return R;
}
static size_t VmLdsBytes(int n_regs) { return (size_t)(n_regs < 1 ? 1 : n_regs) * VM_TILE * 17; }


// LDS-plane register file of the tile interpreter
struct LdsRF {
  const VmLds &R;
  int t;
  __device__ __forceinline__ int64_t &lo(int i) { return R.lo[i * VM_TILE + t]; }
  __device__ __forceinline__ int64_t &hi(int i) { return R.hi[i * VM_TILE + t]; }
  __device__ __forceinline__ uint8_t &nl(int i) { return R.nl[i * VM_TILE + t]; }
};

__device__ void vm_exec(const VmProgram &P, const VmCols &C, int64_t row, bool active, int64_t rs, int64_t rstep,
                        const VmLds &R, int t, int32_t *err) {
  LdsRF rf{R, t};
  for (int k = 0; k < P.n_ins; k++) {
    const VmIns I = P.ins[k];
    vm_step(P, C, I.op, I.dst, I.a, I.b, I.c, I.aux, row, active, rs, rstep, rf, err);
  }
}

__global__ __launch_bounds__(256) void vm_filter_kernel(VmProgram P, VmCols C, int64_t nrows, int64_t rs,
                                                        int64_t rstep, uint64_t *__restrict__ bits,
                                                        uint32_t *__restrict__ tile_counts, int32_t *err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char vm_lds[];
  VmLds R = vm_regs(vm_lds, P.n_regs);
  __shared__ uint32_t wcnt[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t ntiles = (nrows + VM_TILE - 1) / VM_TILE;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int64_t row = tile * VM_TILE + t;
    bool active = row < nrows;
    vm_exec(P, C, row, active, rs, rstep, R, t, err);
    const int pr = P.pred_reg;
    bool sel = active && !R.nl[(pr) * VM_TILE + t] && R.lo[(pr) * VM_TILE + t] != 0;
    uint64_t m = __ballot(sel);
    if (lane == 0) {
      bits[tile * 4 + w] = m;
      wcnt[w] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (t == 0) tile_counts[tile] = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void vm_project_kernel(VmProgram P, VmCols C, int64_t nrows, int64_t rs,
                                                         int64_t rstep, const uint64_t *__restrict__ bits,
                                                         const int64_t *__restrict__ tile_off, VmOuts O,
                                                         int32_t *err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char vm_lds[];
  VmLds R = vm_regs(vm_lds, P.n_regs);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t ntiles = (nrows + VM_TILE - 1) / VM_TILE;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int64_t row = tile * VM_TILE + t;
    bool sel;
    int64_t out_idx;
    if (bits) {
      const uint64_t *tb = bits + tile * 4;
      uint64_t b0 = tb[0], b1 = tb[1], b2 = tb[2], b3 = tb[3];
      if ((b0 | b1 | b2 | b3) == 0) continue;  // uniform across the block
      uint64_t mine = w == 0 ? b0 : w == 1 ? b1 : w == 2 ? b2 : b3;
      int before = (w > 0 ? __popcll(b0) : 0) + (w > 1 ? __popcll(b1) : 0) + (w > 2 ? __popcll(b2) : 0);
      sel = (mine >> lane) & 1ull;
      uint64_t lt = lane ? (mine & ((1ull << lane) - 1ull)) : 0ull;
      out_idx = tile_off[tile] + before + __popcll(lt);
    } else {
      sel = row < nrows;
      out_idx = row;
    }
    vm_exec(P, C, row, sel, rs, rstep, R, t, err);
    if (sel) {
      for (int o = 0; o < P.n_out; o++) {
        const int r = P.out_reg[o];
        store_phys(O.data[o], P.out_phys[o], out_idx, R.lo[(r) * VM_TILE + t], R.hi[(r) * VM_TILE + t]);
        if (R.nl[(r) * VM_TILE + t] && O.nullbits[o]) {
          atomicOr(&O.nullbits[o][out_idx >> 5], 1u << (out_idx & 31));
          if (O.anynull) O.anynull[o] = 1;
        }
      }
    }
  }
}

void VmFilter(const VmProgram &p, const VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
              uint64_t *sel_bits, uint32_t *tile_counts, int32_t *err, hipStream_t s) {
  if (nrows <= 0) return;
  int64_t ntiles = (nrows + VM_TILE - 1) / VM_TILE;
  int grid = GridFor(ntiles, 1, NumCUs() * 8);
  hipLaunchKernelGGL(vm_filter_kernel, dim3(grid), dim3(256), VmLdsBytes(p.n_regs), s, p, cols, nrows, range_start,
                     range_step, sel_bits,
                     tile_counts, err);
  CHECK_LAUNCH();
}

void VmProject(const VmProgram &p, const VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
               const uint64_t *sel_bits, const int64_t *tile_offsets, const VmOuts &outs, int32_t *err,
               hipStream_t s) {
  if (nrows <= 0) return;
  int64_t ntiles = (nrows + VM_TILE - 1) / VM_TILE;
  int grid = GridFor(ntiles, 1, NumCUs() * 8);
  hipLaunchKernelGGL(vm_project_kernel, dim3(grid), dim3(256), VmLdsBytes(p.n_regs), s, p, cols, nrows, range_start,
                     range_step,
                     sel_bits, tile_offsets, outs, err);
  CHECK_LAUNCH();
}

__global__ void invert_bits_kernel(uint64_t *bits, int64_t n) {
  const int64_t words = (n + 63) >> 6;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (int64_t)gridDim.x * blockDim.x) {
    uint64_t v = ~bits[w];
    if (w == words - 1 && (n & 63)) v &= (1ull << (n & 63)) - 1ull;
    bits[w] = v;
  }
}

void InvertNullBits(uint64_t *bits, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(invert_bits_kernel, dim3(GridFor((n + 63) >> 6, 256, NumCUs() * 4)), dim3(256), 0, s, bits, n);
  CHECK_LAUNCH();
}

__global__ void scan_total_kernel(const uint32_t *counts, const int64_t *offsets, int64_t n, int64_t *total) {
  *total = n ? offsets[n - 1] + (int64_t)counts[n - 1] : 0;
}

struct U32ToI64 {
  __host__ __device__ int64_t operator()(uint32_t x) const { return (int64_t)x; }
};

void ScanTileCounts(const uint32_t *counts, int64_t *offsets, int64_t n, int64_t *total, hipStream_t s) {
  if (n <= 0) {
    (void)hipMemsetAsync(total, 0, sizeof(int64_t), s);
    return;
  }
  hipcub::TransformInputIterator<int64_t, U32ToI64, const uint32_t *> it(counts, U32ToI64());
  size_t tmp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, offsets, (int)n, s);
  void *d_tmp = nullptr;
  d_tmp = TempAlloc(tmp);
  (void)hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp, it, offsets, (int)n, s);
  TempFree(d_tmp, tmp);
  hipLaunchKernelGGL(scan_total_kernel, dim3(1), dim3(1), 0, s, counts, offsets, n, total);
}

// selected rows of a 256-row step = popcount of its four ballot words
struct StepPopc {
  const unsigned long long *b;
  __host__ __device__ int64_t operator()(int64_t i) const {
    return (int64_t)(__popcll(b[4 * i]) + __popcll(b[4 * i + 1]) + __popcll(b[4 * i + 2]) + __popcll(b[4 * i + 3]));
  }
};

__global__ void scan_bits_total_kernel(const unsigned long long *bits, const int64_t *offsets, int64_t n,
                                       int64_t *total) {
  *total = n ? offsets[n - 1] + StepPopc{bits}(n - 1) : 0;
}

void ScanStepBits(const unsigned long long *bits, int64_t *offsets, int64_t steps, int64_t *total, hipStream_t s) {
  if (steps <= 0) {
    (void)hipMemsetAsync(total, 0, sizeof(int64_t), s);
    return;
  }
  hipcub::CountingInputIterator<int64_t> idx(0);
  hipcub::TransformInputIterator<int64_t, StepPopc, hipcub::CountingInputIterator<int64_t>> it(idx, StepPopc{bits});
  size_t tmp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, offsets, (int)steps, s);
  void *d_tmp = TempAlloc(tmp);
  (void)hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp, it, offsets, (int)steps, s);
  TempFree(d_tmp, tmp);
  hipLaunchKernelGGL(scan_bits_total_kernel, dim3(1), dim3(1), 0, s, bits, offsets, steps, total);
}

// ---------------------------------------------------------------------------
// fused scan -> filter -> aggregate (configs C2 and C5)
// ---------------------------------------------------------------------------
// Per-thread accumulators: count, int128 sum (lo/hi with carry), min, max.
struct Acc {
  uint64_t cnt;
  uint64_t slo;
  int64_t shi;
  int64_t mn, mx;
};

__device__ __forceinline__ void acc_add(Acc &A, bool ok, int64_t v) {
  A.cnt += ok;
  int64_t vv = ok ? v : 0;
  uint64_t nlo = A.slo + (uint64_t)vv;
  A.shi += (vv >> 63) + (nlo < A.slo ? 1 : 0);
  A.slo = nlo;
  A.mn = ok && v < A.mn ? v : A.mn;
  A.mx = ok && v > A.mx ? v : A.mx;
}

__device__ __forceinline__ void acc_merge(Acc &A, const Acc &B) {
  A.cnt += B.cnt;
  uint64_t nlo = A.slo + B.slo;
  A.shi += B.shi + (nlo < A.slo ? 1 : 0);
  A.slo = nlo;
  A.mn = B.mn < A.mn ? B.mn : A.mn;
  A.mx = B.mx > A.mx ? B.mx : A.mx;
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  return (uint64_t)__shfl_xor((long long)v, m, 64);
}

__device__ __forceinline__ void acc_wave_reduce(Acc &A) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    Acc B;
    B.cnt = shfl_xor_u64(A.cnt, m);
    B.slo = shfl_xor_u64(A.slo, m);
    B.shi = (int64_t)shfl_xor_u64((uint64_t)A.shi, m);
    B.mn = (int64_t)shfl_xor_u64((uint64_t)A.mn, m);
    B.mx = (int64_t)shfl_xor_u64((uint64_t)A.mx, m);
    acc_merge(A, B);
  }
}

__device__ __forceinline__ void agg_state_atomic(AggState *st, const Acc &A) {
  atomicAdd(&st->count, (unsigned long long)A.cnt);
  unsigned long long old = atomicAdd(&st->sum_lo, (unsigned long long)A.slo);
  unsigned long long carry = (old + (unsigned long long)A.slo) < old ? 1ull : 0ull;
  atomicAdd((unsigned long long *)&st->sum_hi, (unsigned long long)A.shi + carry);
  atomicMin(&st->min_i, (long long)A.mn);
  atomicMax(&st->max_i, (long long)A.mx);
}

// Block-level finish: wave shuffle reduction, LDS across the 4 waves, one
// set of atomics per block.
__device__ __forceinline__ void acc_block_commit(Acc &A, AggState *st, unsigned long long *cstar, bool count_is_star) {
  __shared__ Acc part[4];
  acc_wave_reduce(A);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) part[w] = A;
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc T = part[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); i++) acc_merge(T, part[i]);
    if (cstar) atomicAdd(cstar, (unsigned long long)T.cnt);
    if (st) agg_state_atomic(st, T);
  }
  (void)count_is_star;
}

typedef long long v2i64 __attribute__((ext_vector_type(2)));
typedef int v4i32 __attribute__((ext_vector_type(4)));
template <typename T, bool NT>
struct Vec4;  // 4 consecutive elements through 16-byte loads (global_load_dwordx4)
template <bool NT>
struct Vec4<int64_t, NT> {
  static __device__ __forceinline__ void load(const int64_t *__restrict__ p, int64_t g, int64_t v[4]) {
    const v2i64 *q = (const v2i64 *)p + 2 * g;
    v2i64 a, b;
    if (NT) {
      a = __builtin_nontemporal_load(q);
      b = __builtin_nontemporal_load(q + 1);
    } else {
      a = q[0];
      b = q[1];
    }
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
};
template <bool NT>
struct Vec4<int32_t, NT> {
  static __device__ __forceinline__ void load(const int32_t *__restrict__ p, int64_t g, int64_t v[4]) {
    v4i32 a = NT ? __builtin_nontemporal_load((const v4i32 *)p + g) : ((const v4i32 *)p)[g];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
};

// Row-pair loads: lane l of a wave reads rows {2l, 2l+1} of a 128-row wave
// step, so ONE load instruction covers a contiguous 1 KiB (int64) or 512 B
// (int32) with no holes — every cache line is requested once.  (Vec4 above
// makes each lane read 32 contiguous bytes as two 16-B loads: each load then
// spans 2 KiB with 16-B gaps and every line is requested twice.)
typedef int v2i32 __attribute__((ext_vector_type(2)));
template <typename T, bool NT>
struct Pair;
template <bool NT>
struct Pair<int64_t, NT> {
  static __device__ __forceinline__ void load(const int64_t *__restrict__ p, int64_t pi, int64_t &a, int64_t &b) {
    const v2i64 *q = (const v2i64 *)p + pi;
    v2i64 v = NT ? __builtin_nontemporal_load(q) : *q;
    a = v.x;
    b = v.y;
  }
};
template <bool NT>
struct Pair<int32_t, NT> {
  static __device__ __forceinline__ void load(const int32_t *__restrict__ p, int64_t pi, int64_t &a, int64_t &b) {
    const v2i32 *q = (const v2i32 *)p + pi;
    v2i32 v = NT ? __builtin_nontemporal_load(q) : *q;
    a = v.x;
    b = v.y;
  }
};

__device__ __forceinline__ void acc_count(Acc &A, bool ok) { A.cnt += ok; }

// MODE 0: aggregate over the predicate column; 1: over a second column;
// 2: COUNT only (no sum/min/max work in the loop).
// CHUNK: each workgroup streams one contiguous slice (vs a grid-stride sweep).
template <typename TP, typename TA, int MODE, int UNROLL, bool NT, bool CHUNK>
__global__ __launch_bounds__(256) void filter_agg_v4_kernel(const TP *__restrict__ p, const TA *__restrict__ a, int64_t n,
                                                         int64_t lo, uint64_t span, AggState *st,
                                                         unsigned long long *cstar) {
  Acc A;
  A.cnt = 0; A.slo = 0; A.shi = 0; A.mn = INT64_MAX; A.mx = INT64_MIN;
  const int64_t ngroups = n >> 2;  // groups of 4 elements
  int64_t g, gend, stride;
  if (CHUNK) {
    const int64_t per = (ngroups + gridDim.x - 1) / gridDim.x;
    g = (int64_t)blockIdx.x * per + threadIdx.x;
    gend = (int64_t)blockIdx.x * per + per;
    if (gend > ngroups) gend = ngroups;
    stride = blockDim.x;
  } else {
    g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    gend = ngroups;
    stride = (int64_t)gridDim.x * blockDim.x;
  }
  for (; g + (UNROLL - 1) * stride < gend; g += UNROLL * stride) {
    int64_t pv[UNROLL][4], av[UNROLL][4];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      Vec4<TP, NT>::load(p, g + u * stride, pv[u]);
      if (MODE == 1) Vec4<TA, NT>::load(a, g + u * stride, av[u]);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
#pragma unroll
      for (int e = 0; e < 4; e++) {
        int64_t x = pv[u][e];
        bool ok = (uint64_t)(x) - (uint64_t)(lo) <= span;
        if (MODE == 2) acc_count(A, ok);
        else if (MODE == 1) acc_add(A, ok, av[u][e]);
        else acc_add(A, ok, x);
      }
  }
  for (; g < gend; g += stride) {
    int64_t pv[4], av[4];
    Vec4<TP, NT>::load(p, g, pv);
    if (MODE == 1) Vec4<TA, NT>::load(a, g, av);
#pragma unroll
    for (int e = 0; e < 4; e++) {
      bool ok = (uint64_t)(pv[e]) - (uint64_t)(lo) <= span;
      if (MODE == 2) acc_count(A, ok);
      else acc_add(A, ok, MODE == 1 ? av[e] : pv[e]);
    }
  }
  // tail (n % 4 elements): handled by the first threads of block 0
  int64_t tail = (ngroups << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tail < n) {
    int64_t x = p[tail];
    bool ok = (uint64_t)(x) - (uint64_t)(lo) <= span;
    if (MODE == 2) acc_count(A, ok);
    else acc_add(A, ok, MODE == 1 ? (int64_t)a[tail] : x);
  }
  acc_block_commit(A, MODE == 2 ? nullptr : st, cstar, true);
}

// Row-pair version (default): U pair-loads in flight per lane.  Grid-stride
// over pairs, or one contiguous slice of pairs per workgroup (CHUNK).
template <typename TP, typename TA, int MODE, int UNROLL, bool NT, bool CHUNK>
__global__ __launch_bounds__(256) void filter_agg_kernel(const TP *__restrict__ p, const TA *__restrict__ a, int64_t n,
                                                         int64_t lo, uint64_t span, AggState *st,
                                                         unsigned long long *cstar) {
  Acc A;
  A.cnt = 0; A.slo = 0; A.shi = 0; A.mn = INT64_MAX; A.mx = INT64_MIN;
  const int64_t npairs = n >> 1;
  int64_t g, gend, stride;
  if (CHUNK) {
    const int64_t per = (npairs + gridDim.x - 1) / gridDim.x;
    g = (int64_t)blockIdx.x * per + threadIdx.x;
    gend = (int64_t)blockIdx.x * per + per;
    if (gend > npairs) gend = npairs;
    stride = blockDim.x;
  } else {
    g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    gend = npairs;
    stride = (int64_t)gridDim.x * blockDim.x;
  }
  for (; g + (UNROLL - 1) * stride < gend; g += UNROLL * stride) {
    int64_t p0[UNROLL], p1[UNROLL], a0[UNROLL], a1[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      Pair<TP, NT>::load(p, g + u * stride, p0[u], p1[u]);
      if (MODE == 1) Pair<TA, NT>::load(a, g + u * stride, a0[u], a1[u]);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      bool ok0 = (uint64_t)(p0[u]) - (uint64_t)(lo) <= span, ok1 = (uint64_t)(p1[u]) - (uint64_t)(lo) <= span;
      if (MODE == 2) {
        acc_count(A, ok0);
        acc_count(A, ok1);
      } else if (MODE == 1) {
        acc_add(A, ok0, a0[u]);
        acc_add(A, ok1, a1[u]);
      } else {
        acc_add(A, ok0, p0[u]);
        acc_add(A, ok1, p1[u]);
      }
    }
  }
  for (; g < gend; g += stride) {
    int64_t x0, x1, y0 = 0, y1 = 0;
    Pair<TP, NT>::load(p, g, x0, x1);
    if (MODE == 1) Pair<TA, NT>::load(a, g, y0, y1);
    bool ok0 = (uint64_t)(x0) - (uint64_t)(lo) <= span, ok1 = (uint64_t)(x1) - (uint64_t)(lo) <= span;
    if (MODE == 2) {
      acc_count(A, ok0);
      acc_count(A, ok1);
    } else {
      acc_add(A, ok0, MODE == 1 ? y0 : x0);
      acc_add(A, ok1, MODE == 1 ? y1 : x1);
    }
  }
  // odd last row: first thread of block 0
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    int64_t x = p[n - 1];
    bool ok = (uint64_t)(x) - (uint64_t)(lo) <= span;
    if (MODE == 2) acc_count(A, ok);
    else acc_add(A, ok, MODE == 1 ? (int64_t)a[n - 1] : x);
  }
  acc_block_commit(A, MODE == 2 ? nullptr : st, cstar, true);
}

// LDS-DMA streaming version: each wave owns a ring of DEPTH slots of 1 KiB
// (64 lanes x 16 B, global_load_lds_dwordx4) per column; waves walk the
// column's 1-KiB pieces grid-stride, so the whole chip streams through one
// contiguous window.  The oldest slot is consumed once at most DEPTH-1 newer
// pieces are pending (counted vmcnt, never 0 in the loop).  All LDS — ring
// and the final block reduction — lives in ONE __shared__ array (a second
// __shared__ object makes hipcc drain vmcnt before every ds_read).
// A piece is 128 int64 rows or 256 int32 rows; rows past the last whole
// piece are handled by wave 0 of block 0.  MODE 1 needs TP == TA here.
// MM: MIN/MAX requested.  NARROW: the host proved from the column's zone map
// that no lane's int64 partial sum can overflow, so the per-row int128 carry
// chain collapses to one int64 add (sign-extended once, before the reduce).
__device__ __forceinline__ void acc_row(Acc &A, bool ok, int64_t v, bool mm, bool narrow) {
  if (!narrow) {
    if (mm) {
      acc_add(A, ok, v);
    } else {
      A.cnt += ok;
      int64_t vv = ok ? v : 0;
      uint64_t nlo = A.slo + (uint64_t)vv;
      A.shi += (vv >> 63) + (nlo < A.slo ? 1 : 0);
      A.slo = nlo;
    }
    return;
  }
  A.cnt += ok;
  A.slo += (uint64_t)(ok ? v : 0);
  if (mm) {
    A.mn = ok && v < A.mn ? v : A.mn;
    A.mx = ok && v > A.mx ? v : A.mx;
  }
}

// MM: 0 no MIN/MAX, 1 int64 MIN/MAX, 2 int32 MIN/MAX (the zone map bounds |value|
// below 2^31: one v_min_i32 / v_max_i32 per row instead of 64-bit compare pairs)
template <typename T, int MODE, int DEPTH, int MM, bool NARROW>
__global__ __launch_bounds__(256) void filter_agg_lds_kernel(const T *__restrict__ p, const T *__restrict__ a, int64_t n,
                                                             int64_t lo, uint64_t span, AggState *st,
                                                             unsigned long long *cstar, AggPartial *partials) {
  constexpr int NS = MODE == 1 ? 2 : 1;
  constexpr int RPL = 16 / (int)sizeof(T);
  constexpr int64_t RP = 64 * RPL;
  __shared__ __attribute__((aligned(16))) v2i64 ring[4 * NS * DEPTH * 64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t npieces = n / RP;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t pc = (int64_t)blockIdx.x * 4 + w;
  v2i64 *slot0 = ring + w * NS * DEPTH * 64;
  const v2i64 *P = (const v2i64 *)p, *A2 = (const v2i64 *)a;
  Acc A;
  A.cnt = 0; A.slo = 0; A.shi = 0; A.mn = INT64_MAX; A.mx = INT64_MIN;
  int32_t mn32 = INT32_MAX, mx32 = INT32_MIN;
  auto row = [&](bool ok, int64_t v) {
    acc_row(A, ok, v, MM == 1, NARROW);
    if (MM == 2) {
      mn32 = min(mn32, ok ? (int32_t)v : INT32_MAX);
      mx32 = max(mx32, ok ? (int32_t)v : INT32_MIN);
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    int64_t q = pc + d * nw;
    q = q < npieces ? q : 0;  // keep the per-slot load count uniform (dummy piece 0)
    if (npieces > 0) {
      __builtin_amdgcn_global_load_lds((const void *)(P + q * 64 + lane), (void *)(slot0 + d * 64), 16, 0, 2);
      if (NS == 2)
        __builtin_amdgcn_global_load_lds((const void *)(A2 + q * 64 + lane), (void *)(slot0 + (DEPTH + d) * 64), 16, 0, 2);
    }
  }
  int k = 0;
  MBX_CLK(0);
  for (; pc < npieces; pc += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS * (DEPTH - 1)) : "memory");
    v2i64 x = slot0[k * 64 + lane];
    v2i64 y;
    if (NS == 2) y = slot0[(DEPTH + k) * 64 + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int64_t q = pc + DEPTH * nw;
    q = q < npieces ? q : pc;  // past the end: re-read the piece just consumed
    __builtin_amdgcn_global_load_lds((const void *)(P + q * 64 + lane), (void *)(slot0 + k * 64), 16, 0, 2);
    if (NS == 2)
      __builtin_amdgcn_global_load_lds((const void *)(A2 + q * 64 + lane), (void *)(slot0 + (DEPTH + k) * 64), 16, 0, 2);
    if (sizeof(T) == 8) {
      bool ok0 = (uint64_t)(x.x) - (uint64_t)(lo) <= span, ok1 = (uint64_t)(x.y) - (uint64_t)(lo) <= span;
      if (MODE == 2) {
        acc_count(A, ok0);
        acc_count(A, ok1);
      } else {
        row(ok0, MODE == 1 ? y.x : x.x);
        row(ok1, MODE == 1 ? y.y : x.y);
      }
    } else {
      const int *xi = (const int *)&x, *yi = (const int *)&y;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        bool ok = (uint64_t)((int64_t)xi[e]) - (uint64_t)(lo) <= span;
        if (MODE == 2) acc_count(A, ok);
        else row(ok, (int64_t)(MODE == 1 ? yi[e] : xi[e]));
      }
    }
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  MBX_CLK(1);
  if (blockIdx.x == 0 && w == 0) {
    for (int64_t i = npieces * RP + lane; i < n; i += 64) {
      int64_t xv = p[i];
      bool ok = (uint64_t)(xv) - (uint64_t)(lo) <= span;
      if (MODE == 2) acc_count(A, ok);
      else row(ok, MODE == 1 ? (int64_t)a[i] : xv);
    }
  }
  if (MM == 2) {  // no selected row leaves INT32_MAX / INT32_MIN: the emit reads a count of 0 as NULL
    A.mn = mn32;
    A.mx = mx32;
  }
  if (NARROW) A.shi = (int64_t)A.slo >> 63;
  // block reduction through the same LDS array
  acc_wave_reduce(A);
  __syncthreads();
  Acc *part = (Acc *)ring;
  if (lane == 0) part[w] = A;
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc T0 = part[0];
    for (int i = 1; i < 4; i++) acc_merge(T0, part[i]);
    if (partials) {
      partials[blockIdx.x] = AggPartial{T0.cnt, T0.slo, T0.shi, T0.mn, T0.mx};
    } else {
      if (cstar) atomicAdd(cstar, (unsigned long long)T0.cnt);
      if (MODE != 2 && st) agg_state_atomic(st, T0);
    }
  }
}

// Multi-column version of the LDS-DMA filter-aggregate.  A wave step covers
// 256 consecutive rows; each column's slice (1 KiB for int32, 2 KiB for
// int64) lands in the wave's ring slot through global_load_lds; each lane
// then owns 4 consecutive rows of every column.  A NULL-able column adds its
// step's 4 validity words (one exec-masked LDS-DMA instruction); a row counts
// only where every such column is non-NULL (the host admits a NULL-able
// aggregated column only where that is the SQL answer).  NI = LDS-DMA
// instructions per step (compile time: the counted vmcnt wait).
template <int NI, int DEPTH>
__global__ __launch_bounds__(256) void filter_multi_lds_kernel(FilterMultiDesc D, int64_t n, AggPartial *partials,
                                                               int slot_bytes) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fm_lds[];
  const int SB = slot_bytes;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = fm_lds + (size_t)w * DEPTH * SB;
  int off[FM_MAX], voff[FM_MAX];
  {
    int o = 0;
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      off[c] = o;
      if (c < D.ncol) o += D.col[c].phys == P_I64 ? 2048 : 1024;
    }
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      voff[c] = o;
      if (c < D.ncol && D.col[c].valid) o += 32;
    }
  }
  const int64_t nsteps = n >> 8;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t st = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t q, int d) {
    unsigned char *dst = ring + d * SB;
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      if (c >= D.ncol) break;
      const int B = D.col[c].phys == P_I64 ? 2048 : 1024;
      const unsigned char *src = (const unsigned char *)D.col[c].data + q * B;
      __builtin_amdgcn_global_load_lds((const void *)(src + lane * 16), (void *)(dst + off[c]), 16, 0, 2);
      if (B == 2048)
        __builtin_amdgcn_global_load_lds((const void *)(src + 1024 + lane * 16), (void *)(dst + off[c] + 1024), 16, 0, 2);
      if (D.col[c].valid && lane < 2)
        __builtin_amdgcn_global_load_lds((const void *)(D.col[c].valid + q * 4 + lane * 2), (void *)(dst + voff[c]), 16,
                                         0, 0);
    }
  };
  Acc A;
  A.cnt = 0; A.slo = 0; A.shi = 0; A.mn = INT64_MAX; A.mx = INT64_MIN;
  const bool mm32 = D.mm && D.mm32, mm = D.mm && !mm32, narrow = D.narrow;
  int32_t mn32 = INT32_MAX, mx32 = INT32_MIN;
  auto row = [&](bool ok, int64_t val) {
    acc_row(A, ok, val, mm, narrow);
    if (mm32) {
      mn32 = min(mn32, ok ? (int32_t)val : INT32_MAX);
      mx32 = max(mx32, ok ? (int32_t)val : INT32_MIN);
    }
  };
  if (nsteps > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      int64_t q = st + d * nw;
      issue(q < nsteps ? q : 0, d);
    }
  }
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * SB;
    int64_t v[FM_MAX][4];
    unsigned vm = 0xFu;  // rows 4 lane + e where every NULL-able column is valid
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      if (c >= D.ncol) break;
      if (D.col[c].phys == P_I64) {
        v2i64 x0 = *(const v2i64 *)(src + off[c] + lane * 32), x1 = *(const v2i64 *)(src + off[c] + lane * 32 + 16);
        v[c][0] = x0.x; v[c][1] = x0.y; v[c][2] = x1.x; v[c][3] = x1.y;
      } else {
        v4i32 x = *(const v4i32 *)(src + off[c] + lane * 16);
        v[c][0] = x.x; v[c][1] = x.y; v[c][2] = x.z; v[c][3] = x.w;
      }
      if (D.col[c].valid)
        vm &= (unsigned)(*(const uint64_t *)(src + voff[c] + (lane >> 4) * 8) >> (4 * (lane & 15))) & 0xFu;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int64_t q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
#pragma unroll
    for (int e = 0; e < 4; e++) {
      bool ok = (vm >> e) & 1u;
#pragma unroll
      for (int c = 0; c < FM_MAX; c++)
        if (c < D.ncol && D.col[c].is_pred) ok = ok && (uint64_t)(v[c][e]) - (uint64_t)(D.col[c].lo) <= D.col[c].span;
      int64_t val = 0;
#pragma unroll
      for (int c = 0; c < FM_MAX; c++)
        if (c == D.agg) val = v[c][e];
      if (D.agg < 0) acc_count(A, ok);
      else row(ok, val);
    }
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (blockIdx.x == 0 && w == 0) {
    for (int64_t i = (nsteps << 8) + lane; i < n; i += 64) {
      bool ok = true;
      int64_t val = 0;
      for (int c = 0; c < D.ncol; c++) {
        int64_t x = D.col[c].phys == P_I64 ? ((const int64_t *)D.col[c].data)[i] : (int64_t)((const int32_t *)D.col[c].data)[i];
        if (D.col[c].is_pred) ok = ok && (uint64_t)(x) - (uint64_t)(D.col[c].lo) <= D.col[c].span;
        if (D.col[c].valid) ok = ok && ((D.col[c].valid[i >> 6] >> (i & 63)) & 1);
        if (c == D.agg) val = x;
      }
      if (D.agg < 0) acc_count(A, ok);
      else row(ok, val);
    }
  }
  if (mm32) {  // a count of 0 makes the emit write NULL whatever these hold
    A.mn = mn32;
    A.mx = mx32;
  }
  if (narrow) A.shi = (int64_t)A.slo >> 63;
  acc_wave_reduce(A);
  __syncthreads();
  Acc *part = (Acc *)fm_lds;
  if (lane == 0) part[w] = A;
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc T0 = part[0];
    for (int i = 1; i < 4; i++) acc_merge(T0, part[i]);
    partials[blockIdx.x] = AggPartial{T0.cnt, T0.slo, T0.shi, T0.mn, T0.mx};
  }
}

// Compile-time layout of filter_multi_t: NC columns, bit c of WM = column c is
// 8 bytes wide (else 4); slices at fixed offsets, then the NULL-able columns'
// 32-B validity words (runtime: which columns, at the end of the slot).
template <int NC, int WM>
struct FmCols {
  static constexpr int w(int c) { return (WM >> c) & 1 ? 8 : 4; }
  static constexpr int off(int c) { return c == 0 ? 0 : off(c - 1) + w(c - 1) * 256; }
  static constexpr int ni() { return off(NC) / 1024; }
};
template <int N>
__device__ __forceinline__ void fm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// filter_multi_lds with the column layout as template parameters (the
// generic kernel above decides widths and predicate roles per column and row
// at run time: ≈865 instructions in its loop region, exec-mask branches for
// each short-circuit, SGPR spills).  Here every slice read has a fixed offset
// and width, predicates combine bitwise, and only the NULL-able columns
// (0..NC, their validity words one exec-masked LDS-DMA instruction each) stay
// run-time: a scalar switch picks the exact counted vmcnt for their number.
// The host puts the aggregated column first and gives every column that is
// not a predicate the always-true range [INT64_MIN, +2^64), so a row's test
// is the same branch-free compare for every column.  MODE: 0 COUNT only,
// 1 SUM (+COUNT) accumulated in int64 (no MIN/MAX; the grid bounds the sum),
// 3 the same plus MIN/MAX in int32 (the zone map bounds |value| < 2^31),
// 2 general (run-time MIN/MAX, int128 SUM, int32 MIN/MAX).
template <int NC, int WM, int DEPTH, int MODE>
__global__ __launch_bounds__(256) void filter_multi_t_kernel(FilterMultiDesc D, int64_t n, AggPartial *partials,
                                                             int slot_bytes) {
  typedef FmCols<NC, WM> L;
  extern __shared__ __attribute__((aligned(16))) unsigned char fmt_lds[];
  constexpr int NIC = L::ni();
  const int SB = slot_bytes;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = fmt_lds + (size_t)w * DEPTH * SB;
  int voff[NC];
  bool hv[NC];
  int64_t lo[NC];
  uint64_t span[NC];
  const unsigned char *colp[NC];
  int nvw = 0;
#pragma unroll
  for (int c = 0; c < NC; c++) {
    hv[c] = D.col[c].valid != nullptr;
    voff[c] = L::off(NC) + 32 * nvw;
    nvw += hv[c];
    lo[c] = D.col[c].lo;
    span[c] = D.col[c].span;
    colp[c] = (const unsigned char *)D.col[c].data + lane * 16;
  }
  const int64_t nsteps = n >> 8;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t st = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t q, int d) {
    unsigned char *dst = ring + d * SB;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      const unsigned char *src = colp[c] + q * (L::w(c) * 256);
      __builtin_amdgcn_global_load_lds((const void *)src, (void *)(dst + L::off(c)), 16, 0, 2);
      if (L::w(c) == 8)
        __builtin_amdgcn_global_load_lds((const void *)(src + 1024), (void *)(dst + L::off(c) + 1024), 16, 0, 2);
    }
#pragma unroll
    for (int c = 0; c < NC; c++)
      if (hv[c] && lane < 2)
        __builtin_amdgcn_global_load_lds((const void *)(D.col[c].valid + q * 4 + lane * 2), (void *)(dst + voff[c]), 16,
                                         0, 0);
  };
  Acc A;
  A.cnt = 0; A.slo = 0; A.shi = 0; A.mn = INT64_MAX; A.mx = INT64_MIN;
  const bool mm32 = D.mm && D.mm32, mm = D.mm && !mm32, narrow = D.narrow;
  int32_t mn32 = INT32_MAX, mx32 = INT32_MIN;
  if (nsteps > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      int64_t q = st + d * nw;
      issue(q < nsteps ? q : 0, d);
    }
  }
  int k = 0;
  for (; st < nsteps; st += nw) {
    switch (nvw) {  // wave-uniform: the exact count of the slots issued after this one
      case 0: fm_wait<NIC * (DEPTH - 1)>(); break;
      case 1: fm_wait<(NIC + 1) * (DEPTH - 1)>(); break;
      case 2: fm_wait<(NIC + 2) * (DEPTH - 1)>(); break;
      case 3: fm_wait<(NIC + 3) * (DEPTH - 1)>(); break;
      default: fm_wait<(NIC + 4) * (DEPTH - 1)>(); break;
    }
    const unsigned char *src = ring + k * SB;
    int64_t v[NC][4];
#pragma unroll
    for (int c = 0; c < NC; c++) {
      if (L::w(c) == 8) {
        v2i64 x0 = *(const v2i64 *)(src + L::off(c) + lane * 32), x1 = *(const v2i64 *)(src + L::off(c) + lane * 32 + 16);
        v[c][0] = x0.x; v[c][1] = x0.y; v[c][2] = x1.x; v[c][3] = x1.y;
      } else {
        v4i32 x = *(const v4i32 *)(src + L::off(c) + lane * 16);
        v[c][0] = x.x; v[c][1] = x.y; v[c][2] = x.z; v[c][3] = x.w;
      }
    }
    unsigned vm = 0xFu;  // rows 4 lane + e where every NULL-able column is valid
#pragma unroll
    for (int c = 0; c < NC; c++)
      if (hv[c]) vm &= (unsigned)(*(const uint64_t *)(src + voff[c] + (lane >> 4) * 8) >> (4 * (lane & 15))) & 0xFu;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int64_t q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
#pragma unroll
    for (int e = 0; e < 4; e++) {
      bool ok = (vm >> e) & 1u;
#pragma unroll
      for (int c = 0; c < NC; c++) ok = ok & ((uint64_t)(v[c][e]) - (uint64_t)(lo[c]) <= span[c]);
      const int64_t val = v[0][e];
      if constexpr (MODE == 0) {
        acc_count(A, ok);
      } else if constexpr (MODE == 1 || MODE == 3) {
        A.cnt += ok;
        A.slo += (uint64_t)(ok ? val : 0);
        if constexpr (MODE == 3) {
          mn32 = min(mn32, ok ? (int32_t)val : INT32_MAX);
          mx32 = max(mx32, ok ? (int32_t)val : INT32_MIN);
        }
      } else {
        acc_row(A, ok, val, mm, narrow);
        if (mm32) {
          mn32 = min(mn32, ok ? (int32_t)val : INT32_MAX);
          mx32 = max(mx32, ok ? (int32_t)val : INT32_MIN);
        }
      }
    }
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (blockIdx.x == 0 && w == 0) {
    for (int64_t i = (nsteps << 8) + lane; i < n; i += 64) {
      bool ok = true;
      int64_t val = 0;
      for (int c = 0; c < D.ncol; c++) {
        int64_t x = D.col[c].phys == P_I64 ? ((const int64_t *)D.col[c].data)[i] : (int64_t)((const int32_t *)D.col[c].data)[i];
        if (D.col[c].is_pred) ok = ok && (uint64_t)(x) - (uint64_t)(D.col[c].lo) <= D.col[c].span;
        if (D.col[c].valid) ok = ok && ((D.col[c].valid[i >> 6] >> (i & 63)) & 1);
        if (c == D.agg) val = x;
      }
      if (D.agg < 0) {
        acc_count(A, ok);
      } else {
        acc_row(A, ok, val, mm, narrow);
        if (mm32) {
          mn32 = min(mn32, ok ? (int32_t)val : INT32_MAX);
          mx32 = max(mx32, ok ? (int32_t)val : INT32_MIN);
        }
      }
    }
  }
  if (mm32) {  // a count of 0 makes the emit write NULL whatever these hold
    A.mn = mn32;
    A.mx = mx32;
  }
  if (narrow) A.shi = (int64_t)A.slo >> 63;
  acc_wave_reduce(A);
  __syncthreads();
  Acc *part = (Acc *)fmt_lds;
  if (lane == 0) part[w] = A;
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc T0 = part[0];
    for (int i = 1; i < 4; i++) acc_merge(T0, part[i]);
    partials[blockIdx.x] = AggPartial{T0.cnt, T0.slo, T0.shi, T0.mn, T0.mx};
  }
}

namespace {
template <int NC, int WM, int MODE>
void FmtLaunchM(const FilterMultiDesc &d, int64_t nrows, AggPartial *partials, int slot, int grid, int dp,
                hipStream_t s) {
  constexpr int ni = FmCols<NC, WM>::ni();
  if constexpr (ni <= 1) {
    hipLaunchKernelGGL((filter_multi_t_kernel<NC, WM, 6, MODE>), dim3(grid), dim3(256), (size_t)4 * 6 * slot, s, d,
                       nrows, partials, slot);
  } else if constexpr (ni == 2) {
    hipLaunchKernelGGL((filter_multi_t_kernel<NC, WM, 3, MODE>), dim3(grid), dim3(256), (size_t)4 * 3 * slot, s, d,
                       nrows, partials, slot);
  } else {
    if (dp == 3)
      hipLaunchKernelGGL((filter_multi_t_kernel<NC, WM, 3, MODE>), dim3(grid), dim3(256), (size_t)4 * 3 * slot, s, d,
                         nrows, partials, slot);
    else
      hipLaunchKernelGGL((filter_multi_t_kernel<NC, WM, 2, MODE>), dim3(grid), dim3(256), (size_t)4 * 2 * slot, s, d,
                         nrows, partials, slot);
  }
}
template <int NC, int WM>
void FmtLaunch(const FilterMultiDesc &d, int mode, int64_t nrows, AggPartial *partials, int slot, int grid, int dp,
               hipStream_t s) {
  if (mode == 0) FmtLaunchM<NC, WM, 0>(d, nrows, partials, slot, grid, dp, s);
  else if (mode == 1) FmtLaunchM<NC, WM, 1>(d, nrows, partials, slot, grid, dp, s);
  else if (mode == 3) FmtLaunchM<NC, WM, 3>(d, nrows, partials, slot, grid, dp, s);
  else FmtLaunchM<NC, WM, 2>(d, nrows, partials, slot, grid, dp, s);
}
template <int NC, int WM = 0>
void FmtDispatch(const FilterMultiDesc &d, int wm, int mode, int64_t nrows, AggPartial *partials, int slot, int grid,
                 int dp, hipStream_t s) {
  if constexpr (WM < (1 << NC)) {
    if (wm == WM) return FmtLaunch<NC, WM>(d, mode, nrows, partials, slot, grid, dp, s);
    FmtDispatch<NC, WM + 1>(d, wm, mode, nrows, partials, slot, grid, dp, s);
  }
}
}  // namespace

int FilterMultiPartials(const FilterMultiDesc &d_in, int64_t nrows, AggPartial *partials, hipStream_t s) {
  FilterMultiDesc d = d_in;
  int nld = 0, slot = 0;  // nld: LDS-DMA instructions per step (the executor keeps it <= 8)
  for (int c = 0; c < d.ncol; c++) {
    nld += d.col[c].phys == P_I64 ? 2 : 1;
    slot += d.col[c].phys == P_I64 ? 2048 : 1024;
    if (d.col[c].valid) {
      nld++;
      slot += 32;
    }
  }
  slot = (slot + 15) & ~15;
  // MBX_FM_DEPTH=<2..4>: ring depth for 3..5 loads per step (sweeps)
  int dp = 2;
  if (const char *ed = Knob("MBX_FM_DEPTH")) dp = atoi(ed) >= 2 && atoi(ed) <= 4 ? atoi(ed) : 2;
  const char *ev = Knob("MBX_FM_VARIANT");
  const bool templ = !(ev && strcmp(ev, "generic") == 0) && d.ncol >= 1 && d.ncol <= 4 && (dp == 2 || dp == 3);
  int grid = 0;
  auto plan = [&](int gpc) {
    grid = NumCUs() * gpc;
    int64_t need = (nrows >> 8) / 4 + 1;
    if (grid > need) grid = (int)need;
    if (grid > kMaxAggPartials) grid = kMaxAggPartials;
    // a lane sees at most (ceil(steps / waves) + 1) x 4 rows, tail included
    const int64_t waves = (int64_t)grid * 4, steps = nrows >> 8;
    const unsigned __int128 rows_per_lane = (unsigned __int128)(((steps + waves - 1) / waves + 1) * 4);
    d.narrow = d.maxabs <= (uint64_t)INT64_MAX &&
               (unsigned __int128)d.maxabs * rows_per_lane < ((unsigned __int128)1 << 63);
    const char *e32 = Knob("MBX_FA_MM32");
    d.mm32 = d.mm && d.narrow && d.maxabs < ((uint64_t)1 << 31) && !(e32 && e32[0] == '0');
  };
  auto mode_of = [&] { return d.agg < 0 ? 0 : (!d.mm && d.narrow) ? 1 : (d.mm32 && d.narrow) ? 3 : 2; };
  // Workgroups per CU: the generic kernel 3 (3.39 ms vs 3.79 at 2 for 1e9
  // rows of (x i64, k i32, v i64), profiles/r01_filter_multi_sweep.log); the
  // templated one 1 for its compile-time modes (COUNT, narrow SUM, narrow SUM
  // + int32 MIN/MAX) and 3 for the general mode and one-column SUMs
  // (profiles/r02_filter_multi_modes.log).
  const char *e = Knob("MBX_FM_BLOCKS_PER_CU");
  const int gpc_env = e && *e ? atoi(e) : 0;
  if (gpc_env > 0) {
    plan(gpc_env);
  } else if (!templ) {
    plan(3);
  } else {
    plan(1);
    const int m1 = mode_of();
    if (m1 == 2 || (m1 == 1 && d.ncol == 1)) plan(3);
  }
#define FM(L, DP)                                                                                            \
  hipLaunchKernelGGL((filter_multi_lds_kernel<L, DP>), dim3(grid), dim3(256), (size_t)4 * DP * slot, s, d, nrows, \
                     partials, slot)
  // the templated kernel (MBX_FM_VARIANT=generic keeps the one below)
  if (templ) {
    FilterMultiDesc t = d;  // aggregated column first; non-predicates always true
    if (t.agg > 0) {
      std::swap(t.col[0], t.col[t.agg]);
      t.agg = 0;
    }
    for (int c = 0; c < t.ncol; c++)
      if (!t.col[c].is_pred) {
        t.col[c].lo = INT64_MIN;
        t.col[c].span = ~0ull;
      }
    const int mode = mode_of();
    int wm = 0;
    for (int c = 0; c < t.ncol; c++)
      if (t.col[c].phys == P_I64) wm |= 1 << c;
    switch (t.ncol) {
      case 1: FmtDispatch<1>(t, wm, mode, nrows, partials, slot, grid, dp, s); break;
      case 2: FmtDispatch<2>(t, wm, mode, nrows, partials, slot, grid, dp, s); break;
      case 3: FmtDispatch<3>(t, wm, mode, nrows, partials, slot, grid, dp, s); break;
      default: FmtDispatch<4>(t, wm, mode, nrows, partials, slot, grid, dp, s); break;
    }
    CHECK_LAUNCH();
    return grid;
  }
#define FMD(L) \
  if (dp == 2) FM(L, 2); else if (dp == 3) FM(L, 3); else FM(L, 4);
  switch (nld) {
    case 1: FM(1, 6); break;
    case 2: FM(2, 3); break;
    case 3: FMD(3); break;
    case 4: FMD(4); break;
    case 5: FMD(5); break;
    case 6: FM(6, 2); break;
    case 7: FM(7, 2); break;
    default: FM(8, 2); break;
  }
#undef FMD
#undef FM
  CHECK_LAUNCH();
  return grid;
}

__global__ void init_agg_states_kernel(AggState *st, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    AggState z;
    z.count = 0; z.sum_lo = 0; z.sum_hi = 0;
    z.min_i = INT64_MAX; z.max_i = INT64_MIN;
    z.sum_f = 0; z.min_f = 0xFFFFFFFFFFFFFFFFull; z.max_f = 0;
    st[i] = z;
  }
}

__global__ void init_states_counts_kernel(AggState *st, int64_t n, unsigned long long *cs, int64_t nc) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n || i < nc; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n) {
      AggState z;
      z.count = 0; z.sum_lo = 0; z.sum_hi = 0;
      z.min_i = INT64_MAX; z.max_i = INT64_MIN;
      z.sum_f = 0; z.min_f = 0xFFFFFFFFFFFFFFFFull; z.max_f = 0;
      st[i] = z;
    }
    if (i < nc) cs[i] = 0;
  }
}

void InitAggStatesCounts(AggState *st, int64_t n, unsigned long long *cs, int64_t nc, hipStream_t s) {
  int64_t m = n > nc ? n : nc;
  if (m <= 0) return;
  hipLaunchKernelGGL(init_states_counts_kernel, dim3(GridFor(m, 256, 1024)), dim3(256), 0, s, st, n, cs, nc);
  CHECK_LAUNCH();
}

void InitAggStates(AggState *st, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(init_agg_states_kernel, dim3(GridFor(n, 256, 1024)), dim3(256), 0, s, st, n);
  CHECK_LAUNCH();
}

// Launch configuration of the fused filter-aggregate kernel.  The defaults
// were chosen by the A/B sweep recorded in profiles/ (tools/sweep_filter.py);
// MBX_FA_VARIANT="u<unroll>_<nt|pl>_<gs|ch>_g<blocks per CU>" overrides them
// for experiments.
struct FaVariant {
  int unroll = 8;
  bool nt = true;
  bool chunk = true;
  int blocks_per_cu = 1;
  bool pairs = true;  // row-pair layout (false: the older 32-B-per-lane Vec4 layout)
  int lds_depth = 6;  // >0: LDS-DMA ring of this depth per wave (blocks_per_cu then counts 256-thread blocks)
};

// Default: the LDS-DMA stream, 6 x 1 KiB slots per wave, one 256-thread
// workgroup per CU (one wave per SIMD) — 6.90 TB/s median on the 1e9-row
// COUNT vs 6.80 at depth 8 and 6.06 for the best register-load shape
// (profiles/r01_filter_sweep_lds.json, r01_filter_sweep_depth.json).
// MBX_FA_VARIANT overrides it: "d<depth>_g<blocks per CU>" (LDS-DMA) or
// "u<unroll>_<nt|pl>_<gs|ch>_g<blocks per CU>[_v4]" (register loads).
static FaVariant FaConfig(int mode) {
  FaVariant v;
  (void)mode;
  const char *e = Knob("MBX_FA_VARIANT");
  if (!e || !*e) return v;
  int u = 8, g = 4;
  char m1[8] = {0}, m2[8] = {0};
  if (sscanf(e, "d%d_g%d", &u, &g) == 2) {
    v.lds_depth = u;
    v.blocks_per_cu = g;
  } else if (sscanf(e, "u%d_%2s_%2s_g%d", &u, m1, m2, &g) == 4) {
    v.lds_depth = 0;
    v.unroll = u;
    v.nt = m1[0] == 'n';
    v.chunk = m2[0] == 'c';
    v.blocks_per_cu = g;
    v.pairs = strstr(e, "_v4") == nullptr;
  }
  return v;
}

static thread_local bool g_fa_pairs = true;
static thread_local bool g_fa_mm = true, g_fa_narrow = false, g_fa_mm32 = false;  // per launch, set by FilterAggStates
static thread_local AggPartial *g_fa_partials = nullptr;
template <typename TP, typename TA, int MODE, int U, bool NT, bool CH>
static void LaunchFA(const void *p, const void *a, int64_t n, int64_t lo, uint64_t span, AggState *st,
                     unsigned long long *cstar, int grid, hipStream_t s) {
  if (g_fa_pairs)
    hipLaunchKernelGGL((filter_agg_kernel<TP, TA, MODE, U, NT, CH>), dim3(grid), dim3(256), 0, s, (const TP *)p,
                       (const TA *)a, n, lo, span, st, cstar);
  else
    hipLaunchKernelGGL((filter_agg_v4_kernel<TP, TA, MODE, U, NT, CH>), dim3(grid), dim3(256), 0, s, (const TP *)p,
                       (const TA *)a, n, lo, span, st, cstar);
  CHECK_LAUNCH();
}

template <typename T, int MODE, int DEPTH>
static void LaunchFALds(const void *p, const void *a, int64_t n, int64_t lo, uint64_t span, AggState *st,
                        unsigned long long *cstar, int grid, hipStream_t s) {
#define FAL(MM, NW)                                                                                                   \
  hipLaunchKernelGGL((filter_agg_lds_kernel<T, MODE, DEPTH, MM, NW>), dim3(grid), dim3(256), 0, s, (const T *)p,   \
                     (const T *)a, n, lo, span, st, cstar, g_fa_partials)
  if (MODE == 2) FAL(0, false);
  else if (g_fa_mm) { if (g_fa_mm32) FAL(2, true); else if (g_fa_narrow) FAL(1, true); else FAL(1, false); }
  else { if (g_fa_narrow) FAL(0, true); else FAL(0, false); }
#undef FAL
  CHECK_LAUNCH();
}

// true when LaunchFilterAgg takes the LDS-DMA kernel for this shape
static bool FaUsesLds(const FaVariant &v, int mode, int pphys, int aphys) {
  return v.lds_depth > 0 && (mode != 1 || pphys == aphys);
}

template <typename TP, typename TA, int MODE>
static void LaunchFilterAgg(const FaVariant &v, const void *p, const void *a, int64_t n, int64_t lo, uint64_t span,
                            AggState *st, unsigned long long *cstar, int grid, hipStream_t s) {
  if constexpr (MODE != 1 || sizeof(TP) == sizeof(TA)) {
    if (v.lds_depth > 0) {
      switch (v.lds_depth) {
        case 1: case 2: case 3: case 4: LaunchFALds<TP, MODE, 4>(p, a, n, lo, span, st, cstar, grid, s); break;
        case 5: LaunchFALds<TP, MODE, 5>(p, a, n, lo, span, st, cstar, grid, s); break;
        case 6: LaunchFALds<TP, MODE, 6>(p, a, n, lo, span, st, cstar, grid, s); break;
        case 7: LaunchFALds<TP, MODE, 7>(p, a, n, lo, span, st, cstar, grid, s); break;
        case 8: LaunchFALds<TP, MODE, 8>(p, a, n, lo, span, st, cstar, grid, s); break;
        default: LaunchFALds<TP, MODE, 16>(p, a, n, lo, span, st, cstar, grid, s); break;
      }
      return;
    }
  }
#define FA(U, NT, CH) LaunchFA<TP, TA, MODE, U, NT, CH>(p, a, n, lo, span, st, cstar, grid, s)
#define FA_NTCH(U)                                          \
  if (v.nt) { if (v.chunk) FA(U, true, true); else FA(U, true, false); } \
  else { if (v.chunk) FA(U, false, true); else FA(U, false, false); }
  if (v.unroll <= 1) { FA_NTCH(1) }
  else if (v.unroll <= 2) { FA_NTCH(2) }
  else if (v.unroll <= 4) { FA_NTCH(4) }
  else { FA_NTCH(8) }
#undef FA_NTCH
#undef FA
}

int FilterAggStates(const void *pcol, int pphys, int64_t lo, int64_t hi, bool has_pred, const void *acol, int aphys,
                    int64_t nrows, AggState *st, unsigned long long *cstar, int grid_blocks, hipStream_t s,
                    bool need_minmax, uint64_t sum_maxabs, AggPartial *partials) {
  if (nrows <= 0) {
    InitAggStatesCounts(st, 1, cstar, 1, s);
    return 0;
  }
  uint64_t span = has_pred ? (uint64_t)hi - (uint64_t)lo : ~0ull;
  if (!has_pred) lo = INT64_MIN;
  int mode = acol == nullptr ? 2 : (acol == pcol ? 0 : 1);
  if (mode == 2) {
    const char *cs = Knob("MBX_FA_COUNT_AS_SUM");  // experiment: COUNT through the SUM-shaped loop
    if (cs && cs[0] == '1') {
      mode = 0;
      acol = pcol;
      aphys = pphys;
    }
  }
  FaVariant v = FaConfig(mode);
  g_fa_pairs = v.pairs;
  int grid = grid_blocks > 0 ? grid_blocks : NumCUs() * v.blocks_per_cu;
  int64_t groups = (nrows >> 2) + 1;
  if (grid > groups) grid = (int)groups;
  g_fa_mm = need_minmax;
  const bool use_partials = partials && FaUsesLds(v, mode, pphys, aphys) && grid <= kMaxAggPartials;
  g_fa_partials = use_partials ? partials : nullptr;
  if (!use_partials) InitAggStatesCounts(st, 1, cstar, 1, s);
  // LDS-DMA kernel: a lane sees at most (ceil(pieces / waves) + 1) pieces of
  // 16 B, i.e. that many times 2 (int64) or 4 (int32) rows, tail included.
  {
    const int asz = (mode == 1 ? aphys : pphys) == P_I64 ? 8 : 4;
    const int64_t rp = 64 * (16 / (pphys == P_I64 ? 8 : 4));
    const int64_t waves = (int64_t)grid * 4, pieces = nrows / rp;
    const int64_t rows_per_lane = ((pieces + waves - 1) / waves + 1) * (16 / (pphys == P_I64 ? 8 : 4));
    (void)asz;
    g_fa_narrow = sum_maxabs <= (uint64_t)INT64_MAX &&
                  (unsigned __int128)sum_maxabs * (unsigned __int128)rows_per_lane < ((unsigned __int128)1 << 63);
    // MIN/MAX in int32 when the zone map bounds |value| below 2^31 (MBX_FA_MM32=0 disables)
    const char *e32 = Knob("MBX_FA_MM32");
    g_fa_mm32 = g_fa_narrow && sum_maxabs < ((uint64_t)1 << 31) && !(e32 && e32[0] == '0');
  }
  if (pphys == P_I64) {
    if (mode == 0) LaunchFilterAgg<int64_t, int64_t, 0>(v, pcol, acol, nrows, lo, span, st, cstar, grid, s);
    else if (mode == 2) LaunchFilterAgg<int64_t, int64_t, 2>(v, pcol, acol, nrows, lo, span, st, cstar, grid, s);
    else if (aphys == P_I64) LaunchFilterAgg<int64_t, int64_t, 1>(v, pcol, acol, nrows, lo, span, st, cstar, grid, s);
    else LaunchFilterAgg<int64_t, int32_t, 1>(v, pcol, acol, nrows, lo, span, st, cstar, grid, s);
  } else {
    if (mode == 0) LaunchFilterAgg<int32_t, int32_t, 0>(v, pcol, acol, nrows, lo, span, st, cstar, grid, s);
    else if (mode == 2) LaunchFilterAgg<int32_t, int32_t, 2>(v, pcol, acol, nrows, lo, span, st, cstar, grid, s);
    else if (aphys == P_I64) LaunchFilterAgg<int32_t, int64_t, 1>(v, pcol, acol, nrows, lo, span, st, cstar, grid, s);
    else LaunchFilterAgg<int32_t, int32_t, 1>(v, pcol, acol, nrows, lo, span, st, cstar, grid, s);
  }
  g_fa_partials = nullptr;
  return use_partials ? grid : 0;
}

__global__ __launch_bounds__(256) void copy_kernel(const float4 *__restrict__ in, float4 *__restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

// ---------------------------------------------------------------------------
// HBM calibration: a float4 copy and an int64 read-reduce, timed with events
// ---------------------------------------------------------------------------
template <bool NT>
__global__ __launch_bounds__(256) void read_sum_kernel(const v2i64 *__restrict__ in, int64_t n, unsigned long long *out) {
  long long acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    v2i64 a, b, c, d;
    if (NT) {
      a = __builtin_nontemporal_load(in + i);
      b = __builtin_nontemporal_load(in + i + stride);
      c = __builtin_nontemporal_load(in + i + 2 * stride);
      d = __builtin_nontemporal_load(in + i + 3 * stride);
    } else {
      a = in[i]; b = in[i + stride]; c = in[i + 2 * stride]; d = in[i + 3 * stride];
    }
    acc += a.x ^ a.y ^ b.x ^ b.y ^ c.x ^ c.y ^ d.x ^ d.y;
  }
  for (; i < n; i += stride) acc += in[i].x ^ in[i].y;
  if (acc == 0x123456789) atomicAdd(out, 1ull);  // keeps the loads live
}

// the read shape of the hot kernels: one workgroup of 4 waves per CU, each
// wave an LDS-DMA ring of DEPTH x 1 KiB slots (16 B per lane, non-temporal)
template <int DEPTH>
__global__ __launch_bounds__(256) void ring_read_kernel(const unsigned char *__restrict__ in, int64_t nsteps,
                                                        unsigned long long *flag) {
  extern __shared__ __attribute__((aligned(16))) unsigned char rr_lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = rr_lds + w * DEPTH * 1024;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t st = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t q, int d) {
    __builtin_amdgcn_global_load_lds((const void *)(in + q * 1024 + lane * 16), (void *)(ring + d * 1024), 16, 0, 2);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) issue(st + d * nw < nsteps ? st + d * nw : 0, d);
  long long acc = 0;
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH - 1) : "memory");
    v2i64 x = *(const v2i64 *)(ring + k * 1024 + lane * 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int64_t q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    acc += x.x ^ x.y;
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x123456789) atomicAdd(flag, 1ull);
}

// the read shape of C3's group_direct_lds (d2_g1): one workgroup of 4 waves
// per CU; a wave step pulls 256 rows of a 4-byte column (1 KiB) and of an
// 8-byte column (2 KiB) into a DEPTH-deep ring of 3 KiB slots; no atomics
template <int DEPTH>
__global__ __launch_bounds__(256) void ring_read2_kernel(const unsigned char *__restrict__ k4,
                                                         const unsigned char *__restrict__ v8, int64_t nsteps,
                                                         unsigned long long *flag) {
  extern __shared__ __attribute__((aligned(16))) unsigned char r2_lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = r2_lds + w * DEPTH * 3072;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t st = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t q, int d) {
    unsigned char *dst = ring + d * 3072;
    __builtin_amdgcn_global_load_lds((const void *)(k4 + q * 1024 + lane * 16), (void *)dst, 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(v8 + q * 2048 + lane * 16), (void *)(dst + 1024), 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(v8 + q * 2048 + 1024 + lane * 16), (void *)(dst + 2048), 16, 0, 2);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) issue(st + d * nw < nsteps ? st + d * nw : 0, d);
  long long acc = 0;
  int k = 0;
  MBX_CLK(0);
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * 3072;
    v4i32 a = *(const v4i32 *)(src + lane * 16);
    v2i64 b = *(const v2i64 *)(src + 1024 + lane * 32), c = *(const v2i64 *)(src + 1024 + lane * 32 + 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int64_t q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    acc += (a.x ^ a.w) + (b.x ^ c.y);
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  MBX_CLK(1);
  if (acc == 0x123456789) atomicAdd(flag, 1ull);
}

// 16-B copy with 4 independent loads in flight per lane, non-temporal both ways
__global__ __launch_bounds__(256) void copy_nt4_kernel(const v4i32 *__restrict__ in, v4i32 *__restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    v4i32 a = __builtin_nontemporal_load(in + i), b = __builtin_nontemporal_load(in + i + stride);
    v4i32 c = __builtin_nontemporal_load(in + i + 2 * stride), d = __builtin_nontemporal_load(in + i + 3 * stride);
    __builtin_nontemporal_store(a, out + i);
    __builtin_nontemporal_store(b, out + i + stride);
    __builtin_nontemporal_store(c, out + i + 2 * stride);
    __builtin_nontemporal_store(d, out + i + 3 * stride);
  }
  for (; i < n; i += stride) out[i] = in[i];
}

// the same ring with every slot written back out (non-temporal 16-B stores):
// the copy shape of the materialising kernels.  Stores count in vmcnt too, so
// the wait allows the DEPTH-1 younger loads and as many stores.
// HALF: only lanes 0..31 store, packed (512 B per 1 KiB read): the 2:1
// read:write mix of a compaction at ~50 % selectivity
template <int DEPTH, bool HALF>
__global__ __launch_bounds__(256) void ring_copy_kernel(const unsigned char *__restrict__ in, unsigned char *__restrict__ out,
                                                        int64_t nsteps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char rc_lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = rc_lds + w * DEPTH * 1024;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t st = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t q, int d) {
    __builtin_amdgcn_global_load_lds((const void *)(in + q * 1024 + lane * 16), (void *)(ring + d * 1024), 16, 0, 2);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) issue(st + d * nw < nsteps ? st + d * nw : 0, d);
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (DEPTH - 1)) : "memory");
    v4i32 x = *(const v4i32 *)(ring + k * 1024 + lane * 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int64_t q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    if (!HALF) __builtin_nontemporal_store(x, (v4i32 *)(out + st * 1024 + lane * 16));
    else if (lane < 32) __builtin_nontemporal_store(x, (v4i32 *)(out + st * 512 + lane * 16));
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// out: [0] float4 copy, [1] non-temporal int64 read, [2] plain read, [3] the
// hot kernels' LDS-DMA ring read, [4] unrolled non-temporal 16-B copy, [5] the
// LDS-DMA ring copy, [6] the ring copy writing half of what it reads, [7] C3's
// two-array ring read (a 4-byte and an 8-byte column, 2-deep 3 KiB slots)
// (GB/s; a copy counts its read and its write)
void HbmCalibrate(void *buf_a, void *buf_b, int64_t bytes, int iters, double out[kCalibrateShapes], hipStream_t s) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  unsigned long long *flag = (unsigned long long *)buf_b;
  int64_t n16 = bytes / 16;
  int grid = NumCUs() * 8;
  const int64_t nsteps = bytes / 1024;
  const int64_t nsteps3 = bytes / 3072;  // [7]: 256-row steps of 4 + 8 bytes per row
  for (int k = 0; k < kCalibrateShapes; k++) {
    float best = 1e30f;
    for (int it = 0; it < iters + 1; it++) {
      (void)hipEventRecord(e0, s);
      if (k == 0) hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, s, (const float4 *)buf_a, (float4 *)buf_b, n16);
      else if (k == 1) hipLaunchKernelGGL(read_sum_kernel<true>, dim3(grid), dim3(256), 0, s, (const v2i64 *)buf_a, n16, flag);
      else if (k == 2) hipLaunchKernelGGL(read_sum_kernel<false>, dim3(grid), dim3(256), 0, s, (const v2i64 *)buf_a, n16, flag);
      else if (k == 3)
        hipLaunchKernelGGL(ring_read_kernel<6>, dim3(NumCUs()), dim3(256), 4 * 6 * 1024, s, (const unsigned char *)buf_a,
                           nsteps, flag);
      else if (k == 4)
        hipLaunchKernelGGL(copy_nt4_kernel, dim3(grid), dim3(256), 0, s, (const v4i32 *)buf_a, (v4i32 *)buf_b, n16);
      else if (k == 5)
        hipLaunchKernelGGL((ring_copy_kernel<6, false>), dim3(NumCUs()), dim3(256), 4 * 6 * 1024, s,
                           (const unsigned char *)buf_a, (unsigned char *)buf_b, nsteps);
      else if (k == 7)
        hipLaunchKernelGGL(ring_read2_kernel<2>, dim3(NumCUs()), dim3(256), 4 * 2 * 3072, s,
                           (const unsigned char *)buf_a, (const unsigned char *)buf_a + nsteps3 * 1024, nsteps3, flag);
      else
        hipLaunchKernelGGL((ring_copy_kernel<6, true>), dim3(NumCUs()), dim3(256), 4 * 6 * 1024, s,
                           (const unsigned char *)buf_a, (unsigned char *)buf_b, nsteps);
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (it > 0 && ms < best) best = ms;  // first launch is a warm-up
    }
    double moved = (k == 7 ? (double)nsteps3 * 3072 / (double)bytes : k == 6 ? 1.5 : k == 0 || (k >= 4 && k < 7) ? 2.0 : 1.0) *
                   (double)bytes;
    out[k] = moved / (best * 1e-3) / 1e9;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

// The clock stamps of the last stamped launch (diagnostic build): up to cap
// workgroups' {memtime start, realtime start, memtime end, realtime end};
// returns the count copied, 0 in the product library (no stamps compiled).
int ReadClockStamps(uint64_t *out, int cap, hipStream_t s) {
#if MBX_CLOCK_STAMPS
  const int n = std::min(cap, kClkSlots);
  if (n <= 0) return 0;
  if (hipStreamSynchronize(s) != hipSuccess) return 0;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk_stamps), (size_t)n * 4 * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return n;
#else
  (void)out, (void)cap, (void)s;
  return 0;
#endif
}

// ---------------------------------------------------------------------------
// fused GROUP BY on a small integer key range (config C3)
// ---------------------------------------------------------------------------
// LDS table with R replicas per key: replica = lane % R, so the 64 lanes of a
// wave never hit the same address in one ds_add.  Partial sums are int64
// (the host sizes seg_rows from the column statistics so they cannot
// overflow) and are folded into int128 global slots at every segment flush.
template <typename TK, typename TV, int NV, bool MM>
__global__ __launch_bounds__(256) void group_direct_kernel(const TK *__restrict__ keys, const TV *__restrict__ v0,
                                                           const TV *__restrict__ v1, int64_t n, int64_t kmin, int nk,
                                                           int R, int64_t chunk, int64_t seg_rows,
                                                           unsigned long long *cstar, AggState *st0, AggState *st1) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const int nslot = nk * R;
  unsigned int *cnt = (unsigned int *)lds_raw;
  long long *sum0 = (long long *)(lds_raw + ((nslot * 4 + 15) & ~15));
  long long *sum1 = sum0 + nslot;
  long long *mn0 = sum0 + (NV >= 2 ? 2 : 1) * nslot;
  long long *mx0 = mn0 + nslot;
  long long *mn1 = mx0 + nslot;
  long long *mx1 = mn1 + nslot;
  const int t = threadIdx.x, lane = t & 63;
  const int rep = lane % R;
  auto zero = [&]() {
    for (int i = t; i < nslot; i += blockDim.x) {
      cnt[i] = 0;
      if (NV >= 1) sum0[i] = 0;
      if (NV >= 2) sum1[i] = 0;
      if (MM) {
        mn0[i] = INT64_MAX; mx0[i] = INT64_MIN;
        if (NV >= 2) { mn1[i] = INT64_MAX; mx1[i] = INT64_MIN; }
      }
    }
  };
  auto flush = [&]() {
    __syncthreads();
    for (int k = t; k < nk; k += blockDim.x) {
      unsigned long long c = 0;
      i128 s0 = 0, s1 = 0;
      long long a0 = INT64_MAX, b0 = INT64_MIN, a1 = INT64_MAX, b1 = INT64_MIN;
      for (int r = 0; r < R; r++) {
        int sl = k * R + r;
        c += cnt[sl];
        if (NV >= 1) s0 += (i128)sum0[sl];
        if (NV >= 2) s1 += (i128)sum1[sl];
        if (MM) {
          a0 = mn0[sl] < a0 ? mn0[sl] : a0; b0 = mx0[sl] > b0 ? mx0[sl] : b0;
          if (NV >= 2) { a1 = mn1[sl] < a1 ? mn1[sl] : a1; b1 = mx1[sl] > b1 ? mx1[sl] : b1; }
        }
      }
      if (c) {
        atomicAdd(&cstar[k], c);
        Acc A;
        A.cnt = c;
        if (NV >= 1) {
          int64_t lo, hi;
          sp128(s0, lo, hi);
          A.slo = (uint64_t)lo; A.shi = hi; A.mn = MM ? a0 : INT64_MAX; A.mx = MM ? b0 : INT64_MIN;
          agg_state_atomic(&st0[k], A);
        }
        if (NV >= 2) {
          int64_t lo, hi;
          sp128(s1, lo, hi);
          A.slo = (uint64_t)lo; A.shi = hi; A.mn = MM ? a1 : INT64_MAX; A.mx = MM ? b1 : INT64_MIN;
          agg_state_atomic(&st1[k], A);
        }
      }
    }
    __syncthreads();
    zero();
    __syncthreads();
  };
  zero();
  __syncthreads();
  int64_t begin = (int64_t)blockIdx.x * chunk;
  int64_t end = begin + chunk < n ? begin + chunk : n;
  for (int64_t seg = begin; seg < end; seg += seg_rows) {
    int64_t seg_end = seg + seg_rows < end ? seg + seg_rows : end;
    // row-pair body (chunk/seg boundaries are multiples of 4): each load
    // instruction covers a contiguous 512 B (int32) / 1 KiB (int64) span;
    // GU pairs per lane are loaded before any LDS atomic is issued.
    constexpr int GU = 4;
    int64_t g0 = seg >> 1, g1 = seg_end >> 1;
    auto row = [&](int64_t k, int64_t a, int64_t b) {
      int sl = (int)(k - kmin) * R + rep;
      atomicAdd(&cnt[sl], 1u);
      if (NV >= 1) atomicAdd((unsigned long long *)&sum0[sl], (unsigned long long)a);
      if (NV >= 2) atomicAdd((unsigned long long *)&sum1[sl], (unsigned long long)b);
      if (MM) {
        atomicMin(&mn0[sl], (long long)a); atomicMax(&mx0[sl], (long long)a);
        if (NV >= 2) { atomicMin(&mn1[sl], (long long)b); atomicMax(&mx1[sl], (long long)b); }
      }
    };
    int64_t g = g0 + t;
    for (; g + (GU - 1) * (int64_t)blockDim.x < g1; g += GU * (int64_t)blockDim.x) {
      int64_t k0[GU], k1[GU], a0[GU], a1[GU], b0[GU], b1[GU];
#pragma unroll
      for (int u = 0; u < GU; u++) {
        int64_t gi = g + u * (int64_t)blockDim.x;
        Pair<TK, true>::load(keys, gi, k0[u], k1[u]);
        if (NV >= 1) Pair<TV, true>::load(v0, gi, a0[u], a1[u]);
        if (NV >= 2) Pair<TV, true>::load(v1, gi, b0[u], b1[u]);
      }
#pragma unroll
      for (int u = 0; u < GU; u++) {
        row(k0[u], NV >= 1 ? a0[u] : 0, NV >= 2 ? b0[u] : 0);
        row(k1[u], NV >= 1 ? a1[u] : 0, NV >= 2 ? b1[u] : 0);
      }
    }
    for (; g < g1; g += blockDim.x) {
      int64_t k0, k1, a0 = 0, a1 = 0, b0 = 0, b1 = 0;
      Pair<TK, true>::load(keys, g, k0, k1);
      if (NV >= 1) Pair<TV, true>::load(v0, g, a0, a1);
      if (NV >= 2) Pair<TV, true>::load(v1, g, b0, b1);
      row(k0, a0, b0);
      row(k1, a1, b1);
    }
    // odd last row (end is odd only at n)
    for (int64_t i = (g1 << 1) + t; i < seg_end; i += blockDim.x) {
      int sl = (int)((int64_t)keys[i] - kmin) * R + rep;
      atomicAdd(&cnt[sl], 1u);
      if (NV >= 1) atomicAdd((unsigned long long *)&sum0[sl], (unsigned long long)(int64_t)v0[i]);
      if (NV >= 2) atomicAdd((unsigned long long *)&sum1[sl], (unsigned long long)(int64_t)v1[i]);
      if (MM) {
        atomicMin(&mn0[sl], (long long)v0[i]); atomicMax(&mx0[sl], (long long)v0[i]);
        if (NV >= 2) { atomicMin(&mn1[sl], (long long)v1[i]); atomicMax(&mx1[sl], (long long)v1[i]); }
      }
    }
    flush();
  }
}

// LDS-DMA version of group_direct (the default when one flush at the end is
// overflow-safe).  A wave step covers 256 consecutive rows: the key slice and
// every value column's slice are pulled into the wave's ring slot with
// 16-B/lane global_load_lds (1 KiB per instruction, no VGPR staging); each
// lane then owns 4 consecutive rows.  Waves walk steps grid-stride.  The
// replicated LDS tables and the rings share ONE dynamic __shared__ array.
// Each row takes a ds_add_u32 for its COUNT and a ds_add_u64 for its SUM.  (A
// packed form -- the COUNT in the low bits of one ds_add_u64 per row, drained
// into registers every few thousand steps -- bounded this kernel while the
// compiler drained the ring before every LDS atomic; with the asm atomics
// below the plain form is faster: C3 1.684 vs 1.744 ms,
// profiles/r02_group_unpacked.log, so it was removed.)
// LDS atomics of the table as inline-asm ds_* ops that return nothing: the
// compiler puts an s_waitcnt vmcnt(0) in front of every atomic LDS access
// while LDS-DMA is in flight (it cannot prove the table and the ring do not
// alias), which drained the whole ring at every step.  The table is read only
// behind an explicit lgkmcnt(0) + barrier.
__device__ __forceinline__ uint32_t gd_lds(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ void gd_add_u32(unsigned int *p, unsigned int v) {
  asm volatile("ds_add_u32 %0, %1" ::"v"(gd_lds(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void gd_add_u64(long long *p, unsigned long long v) {
  asm volatile("ds_add_u64 %0, %1" ::"v"(gd_lds(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void gd_min_i64(long long *p, long long v) {
  asm volatile("ds_min_i64 %0, %1" ::"v"(gd_lds(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void gd_max_i64(long long *p, long long v) {
  asm volatile("ds_max_i64 %0, %1" ::"v"(gd_lds(p)), "v"(v) : "memory");
}

// VN: some of the key and value columns hold NULLs (gv says which; the
// choice is wave-uniform, so it costs scalar branches, not one kernel per
// mask).  Three 32-B steps of validity words (key, value 0, value 1: 256 rows
// each) ride the ring slot after the value slices, one exec-masked glds each;
// a column without NULLs re-reads a present column's words (an L2 hit, no HBM
// bytes), so every step issues the same count of loads for the counted wait.
// COUNT(*) takes one ds_add_u32 per row; a NULL-able value column's valid rows
// are counted in its own vcnt table, and its SUM / MIN / MAX see the valid rows
// only; a row whose key is NULL goes to the last key slot (nk - 1, the NULL
// group); a predicate on a NULL-able column fails on NULL.
template <typename TK, typename TV, int NV, bool MM, int DEPTH, bool VN = false>
__global__ __launch_bounds__(256) void group_direct_lds_kernel(const TK *__restrict__ keys, const TV *__restrict__ v0,
                                                               const TV *__restrict__ v1, int64_t n, int64_t kmin,
                                                               int nk, int R, size_t ring_off,
                                                               unsigned long long *cstar, AggState *st0,
                                                               AggState *st1, GroupPreds pr, GroupValidity gv,
                                                               unsigned long long *gpart) {
  const bool KN = VN && gv.key, V0N = VN && NV >= 1 && gv.v0, V1N = VN && NV >= 2 && gv.v1;
  constexpr int NVW = VN ? 3 : 0;  // validity steps per ring slot
  const uint64_t *const anyv = VN ? (gv.key ? gv.key : gv.v0 ? gv.v0 : gv.v1) : nullptr;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  constexpr int KB = 256 * (int)sizeof(TK), VB = 256 * (int)sizeof(TV);  // bytes per step
  constexpr int SBD = KB + NV * VB;                                        // key + value slices
  constexpr int OKV = SBD, OV0 = OKV + 32, OV1 = OV0 + 32;  // validity words
  constexpr int SB0 = SBD + 32 * NVW;
  // NLD counts the glds of a step without the optional predicate slice: with
  // one, the counted wait below is merely conservative (loads retire in order)
  constexpr int NLD = SBD / 1024 + NVW;
  // extra slices for predicate columns of their own, after the key/value slices
  int poff[GROUP_MAX_PRED];
  int PB = 0;
#pragma unroll
  for (int j = 0; j < GROUP_MAX_PRED; j++) {
    poff[j] = SB0 + PB;
    if (j < pr.n && pr.p[j].src == 1) PB += 256 * (pr.p[j].phys == P_I64 ? 8 : 4);
  }
  const int SB = SB0 + PB;
  const int nslot = nk * R;
  const int null_key = (nk - 1) * R;  // KN: the NULL group's slots
  unsigned int *cnt = (unsigned int *)lds_raw;
  unsigned long long *cnt64 = (unsigned long long *)lds_raw;  // VN: {COUNT(*), valid rows of value 0}
  long long *sum0 = (long long *)(lds_raw + ((nslot * (VN ? 8 : 4) + 15) & ~15));
  long long *sum1 = sum0 + nslot;
  long long *mn0 = sum0 + (NV >= 2 ? 2 : 1) * nslot;
  long long *mx0 = mn0 + nslot;
  long long *mn1 = mx0 + nslot;
  long long *mx1 = mn1 + nslot;
  // valid-row counts per slot of the NULL-able value columns, after the table
  // (GroupDirectLds sizes them)
  unsigned int *vcnt1 = (unsigned int *)(sum0 + (NV >= 2 ? 2 : 1) * nslot + (MM ? 2 * (NV >= 2 ? 2 : 1) * nslot : 0));
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int rep = lane % R;
  unsigned char *ring = lds_raw + ring_off + (size_t)w * DEPTH * SB;
  for (int i = t; i < nslot; i += blockDim.x) {
    if (VN) cnt64[i] = 0;
    else cnt[i] = 0;
    if (V1N) vcnt1[i] = 0;
    if (NV >= 1) sum0[i] = 0;
    if (NV >= 2) sum1[i] = 0;
    if (MM) {
      mn0[i] = INT64_MAX; mx0[i] = INT64_MIN;
      if (NV >= 2) { mn1[i] = INT64_MAX; mx1[i] = INT64_MIN; }
    }
  }
  __syncthreads();
  // one row: its key slot (the NULL group's when kv is false), COUNT(*), and
  // each value column's sum / min / max over its valid rows
  auto row = [&](int64_t k, int64_t a, int64_t b, bool kv, bool va, bool vb) {
    const int sl = (KN && !kv) ? null_key + rep : (int)(k - kmin) * R + rep;
    if (VN) {
      // branch-free: a NULL value adds 0 to its sum and the neutral element to
      // its min / max, so every lane issues the same LDS ops (no exec-mask
      // juggling per row)
      const bool a_ok = !V0N || va, b_ok = !V1N || vb;
      gd_add_u64((long long *)&cnt64[sl], 1ull + (a_ok ? (1ull << 32) : 0ull));
      if (NV >= 1) {
        gd_add_u64(&sum0[sl], a_ok ? (unsigned long long)a : 0ull);
        if (MM) { gd_min_i64(&mn0[sl], a_ok ? (long long)a : INT64_MAX); gd_max_i64(&mx0[sl], a_ok ? (long long)a : INT64_MIN); }
      }
      if (NV >= 2) {
        if (V1N) gd_add_u32(&vcnt1[sl], b_ok ? 1u : 0u);
        gd_add_u64(&sum1[sl], b_ok ? (unsigned long long)b : 0ull);
        if (MM) { gd_min_i64(&mn1[sl], b_ok ? (long long)b : INT64_MAX); gd_max_i64(&mx1[sl], b_ok ? (long long)b : INT64_MIN); }
      }
      return;
    }
    gd_add_u32(&cnt[sl], 1u);
    if (NV >= 1) {
      gd_add_u64(&sum0[sl], (unsigned long long)a);
      if (MM) { gd_min_i64(&mn0[sl], (long long)a); gd_max_i64(&mx0[sl], (long long)a); }
    }
    if (NV >= 2) {
      gd_add_u64(&sum1[sl], (unsigned long long)b);
      if (MM) { gd_min_i64(&mn1[sl], (long long)b); gd_max_i64(&mx1[sl], (long long)b); }
    }
  };
  const int64_t nsteps = n >> 8;
  const int64_t nw = (int64_t)gridDim.x * 4;
  // pr.xcd: blocks are dealt round-robin over the 8 XCDs, so block b's logical
  // index (b % 8) * (grid / 8) + b / 8 gives each XCD one contiguous eighth of
  // every grid-stride window instead of every eighth 1-KiB piece of it
  int64_t bl = blockIdx.x;
  if (pr.xcd && (gridDim.x & 7) == 0) bl = (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  int64_t st = bl * 4 + w;
  // issue one step's glds into slot d: key slice, each value slice, the validity words
  auto issue = [&](int64_t q, int d) {
    unsigned char *dst = ring + d * SB;
    const unsigned char *kp = (const unsigned char *)keys + q * KB;
#pragma unroll
    for (int j = 0; j < KB / 1024; j++)
      __builtin_amdgcn_global_load_lds((const void *)(kp + j * 1024 + lane * 16), (void *)(dst + j * 1024), 16, 0, 2);
    if (NV >= 1) {
      const unsigned char *vp = (const unsigned char *)v0 + q * VB;
#pragma unroll
      for (int j = 0; j < VB / 1024; j++)
        __builtin_amdgcn_global_load_lds((const void *)(vp + j * 1024 + lane * 16), (void *)(dst + KB + j * 1024), 16, 0, 2);
    }
    if (NV >= 2) {
      const unsigned char *vp = (const unsigned char *)v1 + q * VB;
#pragma unroll
      for (int j = 0; j < VB / 1024; j++)
        __builtin_amdgcn_global_load_lds((const void *)(vp + j * 1024 + lane * 16), (void *)(dst + KB + VB + j * 1024), 16,
                                         0, 2);
    }
    if (VN && lane < 2) {
      __builtin_amdgcn_global_load_lds((const void *)((KN ? gv.key : anyv) + q * 4 + lane * 2), (void *)(dst + OKV), 16,
                                       0, 2);
      __builtin_amdgcn_global_load_lds((const void *)((V0N ? gv.v0 : anyv) + q * 4 + lane * 2), (void *)(dst + OV0), 16,
                                       0, 2);
      __builtin_amdgcn_global_load_lds((const void *)((V1N ? gv.v1 : anyv) + q * 4 + lane * 2), (void *)(dst + OV1), 16,
                                       0, 2);
    }
#pragma unroll
    for (int j = 0; j < GROUP_MAX_PRED; j++) {
      if (j >= pr.n || pr.p[j].src != 1) continue;
      const int B = pr.p[j].phys == P_I64 ? 2048 : 1024;
      const unsigned char *pp = (const unsigned char *)pr.p[j].col + q * B;
      __builtin_amdgcn_global_load_lds((const void *)(pp + lane * 16), (void *)(dst + poff[j]), 16, 0, 2);
      if (B == 2048)
        __builtin_amdgcn_global_load_lds((const void *)(pp + 1024 + lane * 16), (void *)(dst + poff[j] + 1024), 16, 0,
                                         2);
    }
  };
  if (nsteps > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      int64_t q = st + d * nw;
      issue(q < nsteps ? q : 0, d);
    }
  }
  int k = 0;
  MBX_CLK(0);
  // this lane's 4 rows' bits of a step's validity words at byte offset o
  auto vbits = [&](const unsigned char *src, int o) {
    return (unsigned)(*(const uint64_t *)(src + o + (lane >> 4) * 8) >> (4 * (lane & 15))) & 0xFu;
  };
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLD * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * SB;
    int64_t kk[4], a[4], b[4];
    if (sizeof(TK) == 4) {
      v4i32 kv = *(const v4i32 *)(src + lane * 16);
      kk[0] = kv.x; kk[1] = kv.y; kk[2] = kv.z; kk[3] = kv.w;
    } else {
      v2i64 k0 = *(const v2i64 *)(src + lane * 32), k1 = *(const v2i64 *)(src + lane * 32 + 16);
      kk[0] = k0.x; kk[1] = k0.y; kk[2] = k1.x; kk[3] = k1.y;
    }
#pragma unroll
    for (int c = 0; c < NV; c++) {
      const unsigned char *vs = src + KB + c * VB;
      int64_t *o = c == 0 ? a : b;
      if (sizeof(TV) == 4) {
        v4i32 x = *(const v4i32 *)(vs + lane * 16);
        o[0] = x.x; o[1] = x.y; o[2] = x.z; o[3] = x.w;
      } else {
        v2i64 x0 = *(const v2i64 *)(vs + lane * 32), x1 = *(const v2i64 *)(vs + lane * 32 + 16);
        o[0] = x0.x; o[1] = x0.y; o[2] = x1.x; o[3] = x1.y;
      }
    }
    bool ok[4] = {true, true, true, true};
    const unsigned km = KN ? vbits(src, OKV) : 0xFu, am = V0N ? vbits(src, OV0) : 0xFu,
                   bm = V1N ? vbits(src, OV1) : 0xFu;
#pragma unroll
    for (int j = 0; j < GROUP_MAX_PRED; j++) {
      if (j >= pr.n) break;
      const GroupPred &g = pr.p[j];
      int64_t pv[4];
      if (g.src == 2) {
        pv[0] = kk[0]; pv[1] = kk[1]; pv[2] = kk[2]; pv[3] = kk[3];
      } else if (g.src == 3) {
        pv[0] = a[0]; pv[1] = a[1]; pv[2] = a[2]; pv[3] = a[3];
      } else if (g.phys != P_I64) {
        v4i32 x = *(const v4i32 *)(src + poff[j] + lane * 16);
        pv[0] = x.x; pv[1] = x.y; pv[2] = x.z; pv[3] = x.w;
      } else {
        v2i64 x0 = *(const v2i64 *)(src + poff[j] + lane * 32), x1 = *(const v2i64 *)(src + poff[j] + lane * 32 + 16);
        pv[0] = x0.x; pv[1] = x0.y; pv[2] = x1.x; pv[3] = x1.y;
      }
#pragma unroll
      for (int e = 0; e < 4; e++) ok[e] = ok[e] && (uint64_t)(pv[e]) - (uint64_t)(g.lo) <= g.span;
      // a predicate on a NULL-able key / value column fails on NULL
      const unsigned pm = g.src == 2 ? km : g.src == 3 ? am : 0xFu;
#pragma unroll
      for (int e = 0; e < 4; e++) ok[e] = ok[e] && ((pm >> e) & 1u);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int64_t q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
#pragma unroll
    for (int e = 0; e < 4; e++)
      if (ok[e])
        row(kk[e], NV >= 1 ? a[e] : 0, NV >= 2 ? b[e] : 0, ((km >> e) & 1u) != 0, ((am >> e) & 1u) != 0,
            ((bm >> e) & 1u) != 0);
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  MBX_CLK(1);
  if (blockIdx.x == 0) {
    auto bit = [](const uint64_t *v, int64_t i) { return ((v[i >> 6] >> (i & 63)) & 1) != 0; };
    for (int64_t i = (nsteps << 8) + t; i < n; i += blockDim.x) {
      int64_t kv = (int64_t)keys[i], av = NV >= 1 ? (int64_t)v0[i] : 0;
      const bool kr = !KN || bit(gv.key, i), ar = !V0N || bit(gv.v0, i), br = !V1N || bit(gv.v1, i);
      bool okr = true;
      for (int j = 0; j < pr.n; j++) {
        const GroupPred &g = pr.p[j];
        int64_t pv = g.src == 2 ? kv : g.src == 3 ? av
                   : (g.phys == P_I64 ? ((const int64_t *)g.col)[i] : (int64_t)((const int32_t *)g.col)[i]);
        okr = okr && (uint64_t)(pv) - (uint64_t)(g.lo) <= g.span && (g.src != 3 || ar) && (g.src != 2 || kr);
      }
      if (okr) row(kv, av, NV >= 2 ? (int64_t)v1[i] : 0, kr, ar, br);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this thread's table atomics (asm) have landed
  __syncthreads();
  for (int kq = t; kq < nk; kq += blockDim.x) {
    unsigned long long c = 0, vc0 = 0, vc1 = 0;
    i128 s0 = 0, s1 = 0;
    long long a0 = INT64_MAX, b0 = INT64_MIN, a1 = INT64_MAX, b1 = INT64_MIN;
    for (int r = 0; r < R; r++) {
      int sl = kq * R + r;
      if (VN) {
        c += cnt64[sl] & 0xFFFFFFFFull;
        vc0 += cnt64[sl] >> 32;
      } else {
        c += cnt[sl];
      }
      if (V1N) vc1 += vcnt1[sl];
      if (NV >= 1) s0 += (i128)sum0[sl];
      if (NV >= 2) s1 += (i128)sum1[sl];
      if (MM) {
        a0 = mn0[sl] < a0 ? mn0[sl] : a0; b0 = mx0[sl] > b0 ? mx0[sl] : b0;
        if (NV >= 2) { a1 = mn1[sl] < a1 ? mn1[sl] : a1; b1 = mx1[sl] > b1 ? mx1[sl] : b1; }
      }
    }
    if (!V0N) vc0 = c;
    if (!V1N) vc1 = c;
    if (gpart) {
      // this workgroup's record of key kq (key-major: group_partials_compact
      // reads one key's records contiguously); no global atomics
      unsigned long long *o = gpart + ((size_t)kq * gridDim.x + blockIdx.x) * GroupPartialWords(NV, MM);
      o[0] = c;
      int f = 1;
      if (NV >= 1) {
        int64_t lo, hi;
        sp128(s0, lo, hi);
        o[f++] = vc0;
        o[f++] = (unsigned long long)lo; o[f++] = (unsigned long long)hi;
        if (MM) { o[f++] = (unsigned long long)a0; o[f++] = (unsigned long long)b0; }
      }
      if (NV >= 2) {
        int64_t lo, hi;
        sp128(s1, lo, hi);
        o[f++] = vc1;
        o[f++] = (unsigned long long)lo; o[f++] = (unsigned long long)hi;
        if (MM) { o[f++] = (unsigned long long)a1; o[f++] = (unsigned long long)b1; }
      }
      continue;
    }
    if (c) atomicAdd(&cstar[kq], c);
    if (NV >= 1 && vc0) {
      Acc A;
      int64_t lo, hi;
      sp128(s0, lo, hi);
      A.cnt = vc0; A.slo = (uint64_t)lo; A.shi = hi; A.mn = MM ? a0 : INT64_MAX; A.mx = MM ? b0 : INT64_MIN;
      agg_state_atomic(&st0[kq], A);
    }
    if (NV >= 2 && vc1) {
      Acc A;
      int64_t lo, hi;
      sp128(s1, lo, hi);
      A.cnt = vc1; A.slo = (uint64_t)lo; A.shi = hi; A.mn = MM ? a1 : INT64_MAX; A.mx = MM ? b1 : INT64_MIN;
      agg_state_atomic(&st1[kq], A);
    }
  }
}

template <typename TK, typename TV, int NV, bool MM>
static void LaunchGroupDirect(const void *k, const void *v0, const void *v1, int64_t n, int64_t kmin, int nk, int R,
                              int64_t chunk, int64_t seg, unsigned long long *cstar, AggState *s0, AggState *s1,
                              int grid, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL((group_direct_kernel<TK, TV, NV, MM>), dim3(grid), dim3(256), lds, s, (const TK *)k,
                     (const TV *)v0, (const TV *)v1, n, kmin, nk, R, chunk, seg, cstar, s0, s1);
  CHECK_LAUNCH();
}

size_t GroupDirectLds(int nk, int R, int nv, bool mm, int vm) {
  size_t nslot = (size_t)nk * R;
  size_t b = (nslot * (vm ? 8 : 4) + 15) & ~(size_t)15;  // COUNT(*) (vm: + value 0's valid rows)
  b += nslot * 8 * (size_t)(nv >= 2 ? 2 : 1);
  if (mm) b += nslot * 8 * 2 * (size_t)(nv >= 2 ? 2 : 1);
  if (vm) b += 4 * ((nslot + 3) & ~(size_t)3);  // valid-row counts of value column 1
  return (b + 15) & ~(size_t)15;
}

bool GroupByDirectStates(const void *kcol, int kphys, int64_t kmin, int nk, const void *v0, const void *v1, int vphys,
                         int nv, bool mm, int64_t nrows, int64_t seg_rows, int R, unsigned long long *cstar,
                         AggState *st0, AggState *st1, int grid_blocks, hipStream_t s, const GroupPreds *pred,
                         uint64_t vmaxabs, const GroupValidity *gvp, GroupPartialsOut *po) {
  GroupValidity gv;
  memset(&gv, 0, sizeof(gv));
  if (gvp) gv = *gvp;
  const int vm = (gv.v0 ? 1 : 0) | (gv.v1 ? 2 : 0) | (gv.key ? 4 : 0);
  const bool vv = vm != 0;
  if ((gv.v0 && nv < 1) || (gv.v1 && nv < 2)) return false;
  if (po) po->used = false;
  // with po, the states are this call's to initialise: the atomic forms below
  // need them zeroed first, the partials form writes every one at the end
  auto init_states = [&] {
    if (po) InitAggStatesCounts(st0, po->state_slots, cstar, nk, s);
  };
  if (nrows <= 0) {
    init_states();
    return true;
  }
  GroupPreds pr;
  memset(&pr, 0, sizeof(pr));
  if (pred) pr = *pred;
  pr.xcd = 0;
  if (const char *ex = Knob("MBX_GD_XCD")) pr.xcd = atoi(ex) != 0;
  // LDS-DMA variant: one flush at the end, so a block's whole row share must
  // fit the overflow bound the host derived (seg_rows) — else the segmented
  // kernel below.  MBX_GD_VARIANT="d<depth>_g<blocks per CU>" / "seg".
  // Defaults from profiles/r02_group_sweep.log (after the table atomics stopped
  // draining the DMA ring): d2_g1 for value aggregates (C3 1.735-1.77 ms, 2-6 %
  // under d2_g3 on two boxes) and d2_g3 for COUNT-only tables (0.56 ms vs 0.62
  // on the segmented kernel).
  {
    // NULL-able columns (vv): three 2-deep workgroups per CU -- the validity
    // words' extra LDS reads and selects per step want more waves to hide
    // them (C3 with NULLs 1.90 ms at d2_g3 vs 2.13 at d2_g2 and 2.32 at d2_g1,
    // profiles/r06_gd_nulls/)
    int depth = 2, gpc = nv > 0 ? ((gvp && (gvp->key || gvp->v0 || gvp->v1)) ? 3 : 1) : 3;
    for (int j = 0; j < pr.n; j++)  // predicate slices of their own: a deeper ring (c3_where: d3 3.00 vs d2 3.32 ms)
      if (pr.p[j].src == 1) depth = 3;
    bool use = true;
    const char *e = Knob("MBX_GD_VARIANT");
    if (e && *e) use = sscanf(e, "d%d_g%d", &depth, &gpc) == 2 || pr.n != 0;
    if (vv && !use) return false;  // the segmented kernel below has no validity words
    // MBX_GD_R=<r>: fewer replicas (experiment; seg_rows scales with R)
    if (const char *er = Knob("MBX_GD_R")) {
      int r = atoi(er);
      while (use && r > 0 && R > r) {
        R >>= 1;
        if (seg_rows > 0) seg_rows >>= 1;
      }
    }
    if (use) {
      int grid = grid_blocks > 0 ? grid_blocks : NumCUs() * gpc;
      int64_t nsteps = nrows >> 8;
      int64_t waves = (int64_t)grid * 4;
      int64_t rows_per_block = ((nsteps + waves - 1) / waves) * 4 * 256 + 256;
      if (vv && depth > 3) depth = 3;  // the validity form is built for 2- and 3-deep rings
      size_t tab = GroupDirectLds(nk, R, nv, mm, vm);
      size_t ring_off = (tab + 15) & ~(size_t)15;
      size_t slot = 256 * (size_t)(kphys == P_I64 ? 8 : 4) + (size_t)nv * 256 * (vphys == P_I64 ? 8 : 4) +
                    (vv ? 3 * 32 : 0);
      for (int j = 0; j < pr.n; j++)
        if (pr.p[j].src == 1) slot += 256 * (size_t)(pr.p[j].phys == P_I64 ? 8 : 4);
      depth = depth <= 2 ? 2 : depth <= 3 ? 3 : depth <= 4 ? 4 : depth <= 6 ? 6 : 8;
      const size_t lds_cap = gpc <= 1 ? 150 * 1024 : gpc == 2 ? 76 * 1024 : 64 * 1024;
      size_t lds = ring_off + 4 * (size_t)depth * slot;
      // wide slots (predicate slices): trade table replicas for ring space;
      // seg_rows scales with R (rows per replica stay the same)
      while (lds > lds_cap && R > 1) {
        R >>= 1;
        if (seg_rows > 0) seg_rows >>= 1;
        tab = GroupDirectLds(nk, R, nv, mm, vm);
        ring_off = (tab + 15) & ~(size_t)15;
        lds = ring_off + 4 * (size_t)depth * slot;
      }
      // one flush at the end must be overflow-safe (else the segmented kernel)
      const bool one_flush = seg_rows <= 0 || seg_rows >= rows_per_block;
      // per-workgroup records reduced by group_partials_compact instead of the
      // flush's global atomics (every workgroup hitting the same nk states at
      // once): up to kGroupPartialKeys keys, when the caller gave room
      unsigned long long *gpart = nullptr;
      if (po && one_flush && lds <= lds_cap && nk <= kGroupPartialKeys &&
          (size_t)nk * grid * GroupPartialWords(nv, mm) * 8 <= po->bytes && !Knob("MBX_GD_ATOMIC_FLUSH")) {
        gpart = (unsigned long long *)po->buf;
        po->used = true;
        po->blocks = grid;
      }
      if (vv) {  // NULL-able columns: one flush only
        if (!one_flush || lds > lds_cap) return false;
        if (!gpart) init_states();
#define GLVV(TK, TV, NV, MM, D)                                                                                     \
  {                                                                                                                 \
    (void)hipFuncSetAttribute((const void *)group_direct_lds_kernel<TK, TV, NV, MM, D, true>,                      \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);                              \
    hipLaunchKernelGGL((group_direct_lds_kernel<TK, TV, NV, MM, D, true>), dim3(grid), dim3(256), lds, s,         \
                       (const TK *)kcol, (const TV *)v0, (const TV *)v1, nrows, kmin, nk, R, ring_off, cstar, st0,  \
                       st1, pr, gv, gpart);                                                                         \
  }
#define GLVN(TK, TV, MM, D)                                                                                       \
  if (nv == 0) { GLVV(TK, TV, 0, false, D) }                                                                        \
  else if (nv == 1) { GLVV(TK, TV, 1, MM, D) }                                                                      \
  else { GLVV(TK, TV, 2, MM, D) }
#define GLVVD(TK, TV)                                                                                             \
  if (mm) { if (depth == 2) { GLVN(TK, TV, true, 2) } else { GLVN(TK, TV, true, 3) } }                              \
  else { if (depth == 2) { GLVN(TK, TV, false, 2) } else { GLVN(TK, TV, false, 3) } }
        if (kphys == P_I32) {
          if (vphys == P_I64) { GLVVD(int32_t, int64_t) } else { GLVVD(int32_t, int32_t) }
        } else {
          if (vphys == P_I64) { GLVVD(int64_t, int64_t) } else { GLVVD(int64_t, int32_t) }
        }
#undef GLVVD
#undef GLVN
#undef GLVV
        CHECK_LAUNCH();
        return true;
      }
      if (one_flush && lds <= lds_cap) {
        if (!gpart) init_states();
#define GL(TK, TV, NV, MM, D)                                                                                      \
  if (lds > 64 * 1024) /* deep rings at one or two blocks per CU */                                               \
    (void)hipFuncSetAttribute((const void *)group_direct_lds_kernel<TK, TV, NV, MM, D, 0>,                         \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);                             \
  hipLaunchKernelGGL((group_direct_lds_kernel<TK, TV, NV, MM, D, 0>), dim3(grid), dim3(256), lds, s,               \
                     (const TK *)kcol, (const TV *)v0, (const TV *)v1, nrows, kmin, nk, R, ring_off, cstar, st0,   \
                     st1, pr, gv, gpart);
#define GLD(TK, TV, NV, MM)                                                                     \
  if (depth == 2) { GL(TK, TV, NV, MM, 2) } else if (depth == 3) { GL(TK, TV, NV, MM, 3) }      \
  else if (depth == 4) { GL(TK, TV, NV, MM, 4) } else if (depth == 6) { GL(TK, TV, NV, MM, 6) } \
  else { GL(TK, TV, NV, MM, 8) }
#define GLV(TK, TV)                                                                      \
  if (nv == 0) { GLD(TK, TV, 0, false) }                                                 \
  else if (nv == 1) { if (mm) { GLD(TK, TV, 1, true) } else { GLD(TK, TV, 1, false) } } \
  else { if (mm) { GLD(TK, TV, 2, true) } else { GLD(TK, TV, 2, false) } }
        if (kphys == P_I32) {
          if (vphys == P_I64) { GLV(int32_t, int64_t) } else { GLV(int32_t, int32_t) }
        } else {
          if (vphys == P_I64) { GLV(int64_t, int64_t) } else { GLV(int64_t, int32_t) }
        }
#undef GLV
#undef GLD
#undef GL
        CHECK_LAUNCH();
        return true;
      }
    }
  }
  if (pr.n) return false;  // a predicate needs the LDS-DMA kernel
  init_states();
  int grid = grid_blocks > 0 ? grid_blocks : NumCUs() * 4;
  int64_t chunk = (nrows + grid - 1) / grid;
  chunk = (chunk + 3) & ~(int64_t)3;
  grid = (int)((nrows + chunk - 1) / chunk);
  if (seg_rows <= 0 || seg_rows > chunk) seg_rows = chunk;
  seg_rows = (seg_rows + 3) & ~(int64_t)3;
  size_t lds = GroupDirectLds(nk, R, nv, mm);
#define GD(TK, TV, NV, MM) LaunchGroupDirect<TK, TV, NV, MM>(kcol, v0, v1, nrows, kmin, nk, R, chunk, seg_rows, cstar, st0, st1, grid, lds, s)
#define GDV(TK, TV)                         \
  if (nv == 0) GD(TK, TV, 0, false);        \
  else if (nv == 1) { if (mm) GD(TK, TV, 1, true); else GD(TK, TV, 1, false); } \
  else { if (mm) GD(TK, TV, 2, true); else GD(TK, TV, 2, false); }
  if (kphys == P_I32) {
    if (vphys == P_I64) { GDV(int32_t, int64_t) } else { GDV(int32_t, int32_t) }
  } else {
    if (vphys == P_I64) { GDV(int64_t, int64_t) } else { GDV(int64_t, int32_t) }
  }
#undef GDV
#undef GD
  return true;
}

// ---------------------------------------------------------------------------
// generic aggregation over compacted columns
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void reduce_column_kernel(const void *col, int phys, const uint64_t *valid, int64_t n,
                                                            AggState *st) {
  Acc A;
  A.cnt = 0; A.slo = 0; A.shi = 0; A.mn = INT64_MAX; A.mx = INT64_MIN;
  double sf = 0;
  uint64_t fmn = ~0ull, fmx = 0;
  const bool isf = phys == P_F64 || phys == P_F32;
  const bool is128 = phys == P_I128 || phys == P_U64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!bit_valid(valid, i)) continue;
    int64_t lo, hi;
    load_phys(col, phys, i, lo, hi);
    if (isf) {
      double d = __longlong_as_double(lo);
      A.cnt++;
      sf += d;
      uint64_t k = f64_order(d);
      fmn = k < fmn ? k : fmn;
      fmx = k > fmx ? k : fmx;
    } else if (is128) {
      A.cnt++;
      uint64_t nlo = A.slo + (uint64_t)lo;
      A.shi += hi + (nlo < A.slo ? 1 : 0);
      A.slo = nlo;
    } else {
      acc_add(A, true, lo);
    }
  }
  // floats: reduce separately
  __shared__ double sfs[4];
  __shared__ unsigned long long fmns[4], fmxs[4];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    sf += __shfl_xor(sf, m, 64);
    uint64_t o = shfl_xor_u64(fmn, m);
    fmn = o < fmn ? o : fmn;
    o = shfl_xor_u64(fmx, m);
    fmx = o > fmx ? o : fmx;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    sfs[w] = sf;
    fmns[w] = fmn;
    fmxs[w] = fmx;
  }
  acc_block_commit(A, st, nullptr, false);
  if (threadIdx.x == 0 && isf) {
    double s = 0;
    unsigned long long a = ~0ull, b = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) {
      s += sfs[i];
      a = fmns[i] < a ? fmns[i] : a;
      b = fmxs[i] > b ? fmxs[i] : b;
    }
    atomicAdd(&st->sum_f, s);
    atomicMin(&st->min_f, a);
    atomicMax(&st->max_f, b);
  }
}

void ReduceColumn(const void *col, int phys, const uint64_t *valid, int64_t n, AggState *out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(reduce_column_kernel, dim3(GridFor(n, 256 * 16, NumCUs() * 4)), dim3(256), 0, s, col, phys, valid,
                     n, out);
  CHECK_LAUNCH();
}

__global__ void key_range_kernel(const void *col, int phys, const uint64_t *valid, int64_t n, long long *out3) {
  long long mn = INT64_MAX, mx = INT64_MIN, c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!bit_valid(valid, i)) continue;
    int64_t lo, hi;
    load_phys(col, phys, i, lo, hi);
    mn = lo < mn ? lo : mn;
    mx = lo > mx ? lo : mx;
    c++;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    long long o = __shfl_xor(mn, m, 64);
    mn = o < mn ? o : mn;
    o = __shfl_xor(mx, m, 64);
    mx = o > mx ? o : mx;
    c += __shfl_xor(c, m, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&out3[0], mn);
    atomicMax(&out3[1], mx);
    atomicAdd((unsigned long long *)&out3[2], (unsigned long long)c);
  }
}

__global__ void init3_kernel(long long *o) {
  o[0] = INT64_MAX;
  o[1] = INT64_MIN;
  o[2] = 0;
}

// Zone map (min, max, non-NULL count) of an INT32 / INT64 column at HBM speed:
// the LDS-DMA ring of filter_agg_lds.  A wave step covers 256 rows: the
// step's values (1 KiB for int32, 2 KiB for int64) and, for a NULL-able
// column, its 4 validity words (one exec-masked LDS-DMA instruction) land in
// the wave's ring slot by global_load_lds, DEPTH steps in flight with a
// counted vmcnt (never 0 in the loop); each lane then owns 4 consecutive rows.
// Min / max stay in T's width.  Ring and reduction scratch share one
// __shared__ array; one atomic set per block.  Rows past the last whole step
// are done by wave 0 of block 0.  p is 16-B aligned; valid (if any) starts at
// row 0 of p.
template <typename T, bool VAL, int DEPTH>
__global__ __launch_bounds__(256) void zone_map_lds_kernel(const T *__restrict__ p, const uint64_t *__restrict__ valid,
                                                           int64_t n, long long *out3) {
  constexpr int VB = 256 * (int)sizeof(T);  // value bytes per step
  constexpr int SB = VB + (VAL ? 32 : 0);   // slot bytes
  constexpr int NI = (sizeof(T) == 8 ? 2 : 1) + (VAL ? 1 : 0);
  constexpr T TMAX = std::numeric_limits<T>::max();
  constexpr T TMIN = std::numeric_limits<T>::min();
  __shared__ __attribute__((aligned(16))) unsigned char ring[4 * DEPTH * SB];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *slot0 = ring + w * DEPTH * SB;
  const int64_t nsteps = n >> 8;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t st = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t q, int d) {
    unsigned char *dst = slot0 + d * SB;
    const unsigned char *src = (const unsigned char *)p + q * VB;
    __builtin_amdgcn_global_load_lds((const void *)(src + lane * 16), (void *)dst, 16, 0, 2);
    if (sizeof(T) == 8) __builtin_amdgcn_global_load_lds((const void *)(src + 1024 + lane * 16), (void *)(dst + 1024), 16, 0, 2);
    if (VAL && lane < 2) __builtin_amdgcn_global_load_lds((const void *)(valid + q * 4 + lane * 2), (void *)(dst + VB), 16, 0, 0);
  };
  T mn = TMAX, mx = TMIN;
  uint32_t c = 0;
  if (nsteps > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      const int64_t q = st + d * nw;
      issue(q < nsteps ? q : 0, d);  // keep the per-slot load count uniform (dummy step 0)
    }
  }
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (DEPTH - 1)) : "memory");
    const unsigned char *src = slot0 + k * SB;
    T v[4];
    if (sizeof(T) == 8) {
      const v2i64 a = ((const v2i64 *)src)[2 * lane], b = ((const v2i64 *)src)[2 * lane + 1];
      v[0] = (T)a.x; v[1] = (T)a.y; v[2] = (T)b.x; v[3] = (T)b.y;
    } else {
      const v4i32 a = ((const v4i32 *)src)[lane];
      v[0] = (T)a.x; v[1] = (T)a.y; v[2] = (T)a.z; v[3] = (T)a.w;
    }
    uint32_t vb = 0xFu;
    if (VAL) vb = (uint32_t)(((const uint64_t *)(src + VB))[lane >> 4] >> ((lane & 15) * 4)) & 0xFu;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int64_t q = st + DEPTH * nw;
    q = q < nsteps ? q : st;  // past the end: re-read the step just consumed
    issue(q, k);
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const bool ok = !VAL || ((vb >> e) & 1u);
      mn = ok && v[e] < mn ? v[e] : mn;
      mx = ok && v[e] > mx ? v[e] : mx;
      c += ok ? 1u : 0u;
    }
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (blockIdx.x == 0 && w == 0) {
    for (int64_t i = nsteps * 256 + lane; i < n; i += 64) {
      if (VAL && !((valid[i >> 6] >> (i & 63)) & 1ull)) continue;
      const T x = p[i];
      mn = x < mn ? x : mn;
      mx = x > mx ? x : mx;
      c++;
    }
  }
  long long lmn = (long long)mn, lmx = (long long)mx;
  unsigned long long lc = c;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    long long o = __shfl_xor(lmn, m, 64);
    lmn = o < lmn ? o : lmn;
    o = __shfl_xor(lmx, m, 64);
    lmx = o > lmx ? o : lmx;
    lc += __shfl_xor(lc, m, 64);
  }
  __syncthreads();  // every wave is done with its ring slots
  long long *part = (long long *)ring;
  if (lane == 0) {
    part[3 * w] = lmn;
    part[3 * w + 1] = lmx;
    part[3 * w + 2] = (long long)lc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long a = part[0], b = part[1], cc = part[2];
    for (int i = 1; i < 4; i++) {
      a = part[3 * i] < a ? part[3 * i] : a;
      b = part[3 * i + 1] > b ? part[3 * i + 1] : b;
      cc += part[3 * i + 2];
    }
    if (cc > 0) {
      atomicMin(&out3[0], a);
      atomicMax(&out3[1], b);
      atomicAdd((unsigned long long *)&out3[2], (unsigned long long)cc);
    }
  }
}

template <typename T, bool VAL>
static void LaunchZoneMap(const void *col, const uint64_t *valid, int64_t n, long long *out3, hipStream_t s) {
  const int64_t steps = n >> 8;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)NumCUs(), (steps + 3) / 4));
  hipLaunchKernelGGL((zone_map_lds_kernel<T, VAL, 6>), dim3(grid), dim3(256), 0, s, (const T *)col, valid, n, out3);
}

void KeyRange(const void *col, int phys, const uint64_t *valid, int64_t n, long long *out3, hipStream_t s) {
  hipLaunchKernelGGL(init3_kernel, dim3(1), dim3(1), 0, s, out3);
  if (n <= 0) {
    CHECK_LAUNCH();
    return;
  }
  const int sz = phys == P_I64 ? 8 : phys == P_I32 ? 4 : 0;
  const uintptr_t mis = (uintptr_t)col % 16;
  if (sz && n >= 1024 && (mis == 0 || (!valid && mis % sz == 0))) {
    // an appended range may start mid-vector: its first rows go through the
    // element-wise kernel, the 16-B aligned rest through the ring
    const int64_t head = mis ? (int64_t)((16 - mis) / sz) : 0;
    if (head)
      hipLaunchKernelGGL(key_range_kernel, dim3(1), dim3(64), 0, s, col, phys, (const uint64_t *)nullptr, head, out3);
    const void *body = (const char *)col + head * sz;
    if (sz == 8) {
      if (valid) LaunchZoneMap<int64_t, true>(body, valid, n - head, out3, s);
      else LaunchZoneMap<int64_t, false>(body, nullptr, n - head, out3, s);
    } else {
      if (valid) LaunchZoneMap<int32_t, true>(body, valid, n - head, out3, s);
      else LaunchZoneMap<int32_t, false>(body, nullptr, n - head, out3, s);
    }
    CHECK_LAUNCH();
    return;
  }
  hipLaunchKernelGGL(key_range_kernel, dim3(GridFor(n, 256 * 16, NumCUs() * 4)), dim3(256), 0, s, col, phys, valid,
                     n, out3);
  CHECK_LAUNCH();
}

void ColumnStats(const void *col, int phys, const uint64_t *valid, int64_t n, long long *out3, hipStream_t s) {
  KeyRange(col, phys, valid, n, out3, s);
}

__global__ void group_assign_kernel(const void *kcol, int kphys, const uint64_t *kvalid, int64_t kmin, int64_t nslots,
                                    int64_t n, int32_t *slot_of_row, unsigned long long *count_star) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t sl;
    if (!bit_valid(kvalid, i)) sl = (int32_t)(nslots - 1);
    else {
      int64_t lo, hi;
      load_phys(kcol, kphys, i, lo, hi);
      sl = (int32_t)(lo - kmin);
    }
    slot_of_row[i] = sl;
    atomicAdd(&count_star[sl], 1ull);
  }
}

void GroupAssign(const void *kcol, int kphys, const uint64_t *kvalid, int64_t kmin, int64_t nslots, int64_t n,
                 int32_t *slot_of_row, unsigned long long *count_star, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(group_assign_kernel, dim3(GridFor(n, 256 * 8, NumCUs() * 8)), dim3(256), 0, s, kcol, kphys,
                     kvalid, kmin, nslots, n, slot_of_row, count_star);
  CHECK_LAUNCH();
}

__global__ void group_reduce_kernel(const int32_t *slot_of_row, const void *col, int phys, const uint64_t *valid,
                                    int64_t n, AggState *states) {
  const bool isf = phys == P_F64 || phys == P_F32;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!bit_valid(valid, i)) continue;
    AggState *st = &states[slot_of_row[i]];
    int64_t lo, hi;
    load_phys(col, phys, i, lo, hi);
    atomicAdd(&st->count, 1ull);
    if (isf) {
      double d = __longlong_as_double(lo);
      atomicAdd(&st->sum_f, d);
      uint64_t k = f64_order(d);
      atomicMin(&st->min_f, (unsigned long long)k);
      atomicMax(&st->max_f, (unsigned long long)k);
    } else {
      unsigned long long old = atomicAdd(&st->sum_lo, (unsigned long long)lo);
      unsigned long long carry = (old + (unsigned long long)lo) < old ? 1ull : 0ull;
      atomicAdd((unsigned long long *)&st->sum_hi, (unsigned long long)hi + carry);
      if (phys != P_I128) {
        atomicMin(&st->min_i, (long long)lo);
        atomicMax(&st->max_i, (long long)lo);
      }
    }
  }
}

void GroupReduceColumn(const int32_t *slot_of_row, const void *col, int phys, const uint64_t *valid, int64_t n,
                       AggState *states, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(group_reduce_kernel, dim3(GridFor(n, 256 * 8, NumCUs() * 8)), dim3(256), 0, s, slot_of_row, col,
                     phys, valid, n, states);
  CHECK_LAUNCH();
}

__global__ __launch_bounds__(1024) void compact_slots_kernel(const unsigned long long *count_star, int64_t nslots,
                                                             int32_t *slot_list, int64_t *n_out) {
  __shared__ int wsum[16];
  __shared__ long long base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t off = 0; off < nslots; off += blockDim.x) {
    int64_t i = off + threadIdx.x;
    bool f = i < nslots && count_star[i] > 0;
    uint64_t m = __ballot(f);
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int before = 0;
    for (int k = 0; k < w; k++) before += wsum[k];
    int total = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); k++) total += wsum[k];
    uint64_t lt = lane ? (m & ((1ull << lane) - 1ull)) : 0ull;
    if (f) slot_list[base + before + __popcll(lt)] = (int32_t)i;
    __syncthreads();
    if (threadIdx.x == 0) base += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) *n_out = base;
}

__global__ void slot_flags_kernel(const unsigned long long *count_star, int64_t nslots, int32_t *flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = count_star[i] > 0;
}

__global__ void slot_scatter_kernel(const int32_t *flag, const int32_t *pos, int64_t nslots, int32_t *slot_list,
                                    int64_t *n_out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (int64_t)gridDim.x * blockDim.x) {
    if (flag[i]) slot_list[pos[i]] = (int32_t)i;
    if (i == nslots - 1) *n_out = (int64_t)pos[i] + flag[i];
  }
}

// Ordered list of the non-empty slots.  One workgroup for small tables; a
// device-wide scan (flags -> hipCUB exclusive sum -> scatter) for large ones.
// Writes the aggregate relation [key?, agg0, agg1, ...] from per-slot states,
// as workgroup `bid` of `nb` (emit_agg_kernel; the one workgroup of
// group_partials_compact_kernel).  Validity bitmaps are written as whole 64-bit
// words from a wave ballot (each wave owns 64 consecutive output rows), so the
// output bitmaps need no zeroing and no atomics.  part: LDS room for one Acc
// per wave (the partials reduction).
__device__ __forceinline__ void emit_agg_body(const EmitDesc &D, Acc *part, int64_t bid, int64_t nb) {
  if (D.npartials > 0) {
    // slot 0 from the filter-aggregate's per-workgroup partials (one workgroup)
    Acc A;
    A.cnt = 0; A.slo = 0; A.shi = 0; A.mn = INT64_MAX; A.mx = INT64_MIN;
    for (int i = threadIdx.x; i < D.npartials; i += blockDim.x) {
      const AggPartial &q = D.partials[i];
      Acc B;
      B.cnt = q.cnt; B.slo = q.slo; B.shi = q.shi; B.mn = q.mn; B.mx = q.mx;
      acc_merge(A, B);
    }
    acc_wave_reduce(A);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = A;
    __syncthreads();
    if (threadIdx.x == 0) {
      Acc T0 = part[0];
      for (int i = 1; i < (int)(blockDim.x >> 6); i++) acc_merge(T0, part[i]);
      unsigned long long *cs = (unsigned long long *)D.cstar;
      cs[0] = T0.cnt;
      for (int j = 0; j < D.nagg; j++) {
        AggState *S = D.a[j].states;
        if (!S) continue;
        S->count = T0.cnt;
        S->sum_lo = T0.slo;
        S->sum_hi = T0.shi;
        S->min_i = T0.mn;
        S->max_i = T0.mx;
      }
      __threadfence_block();
    }
    __syncthreads();
  }
  const int64_t n = D.slot_list ? *D.n_list : D.nslots;
  const int lane = threadIdx.x & 63;
  const int64_t stride = nb * blockDim.x;
  for (int64_t base = bid * blockDim.x + (threadIdx.x & ~63); base < n; base += stride) {
    const int64_t i = base + lane;
    const bool in = i < n;
    const int64_t sl = in ? (D.slot_list ? D.slot_list[i] : i) : 0;
    if (D.has_key) {
      bool kv = in && sl != D.null_slot;
      if (in) {
        int64_t k = D.key_msb ? (int64_t)(D.key_msb[sl] ^ 0x8000000000000000ull) : D.kmin + sl;
        if (kv) store_phys(D.key_out, D.key_phys, i, k, k >> 63);
        else store_phys(D.key_out, D.key_phys, i, 0, 0);
      }
      uint64_t m = __ballot(kv);
      if (lane == 0) {
        D.key_valid[base >> 5] = (uint32_t)m;
        if (base + 32 < n) D.key_valid[(base >> 5) + 1] = (uint32_t)(m >> 32);
      }
    }
    for (int q = 0; q < D.nkeys_c; q++) {
      const auto &K = D.kc[q];
      bool kv = in;
      if (in) {
        const int64_t dg = (sl / K.stride) % K.radix;
        kv = !(K.nullable && dg == K.radix - 1);
        const int64_t k = kv ? K.kmin + dg : 0;
        store_phys(K.out, K.phys, i, k, k >> 63);
      }
      uint64_t m = __ballot(kv);
      if (lane == 0) {
        K.valid[base >> 5] = (uint32_t)m;
        if (base + 32 < n) K.valid[(base >> 5) + 1] = (uint32_t)(m >> 32);
      }
    }
    for (int j = 0; j < D.nagg; j++) {
      const EmitAgg &A = D.a[j];
      bool valid = in;
      int64_t lo = 0, hi = 0;
      if (in) {
        if (A.kind == 0 /*COUNT_STAR*/) {
          lo = (int64_t)D.cstar[sl];
        } else {
          const AggState &S = A.states[sl];
          switch (A.kind) {
            case 1: /*COUNT*/ lo = (int64_t)S.count; break;
            case 2: /*SUM*/
              if (!S.count) { valid = false; break; }
              if (A.in_class == VC_F64) lo = __double_as_longlong(S.sum_f);
              else { lo = (int64_t)S.sum_lo; hi = S.sum_hi; }
              break;
            case 3: /*MIN*/
            case 4: /*MAX*/
              if (!S.count) { valid = false; break; }
              if (A.in_class == VC_F64) lo = __double_as_longlong(f64_unorder(A.kind == 3 ? S.min_f : S.max_f));
              else { lo = A.kind == 3 ? S.min_i : S.max_i; hi = lo >> 63; }
              break;
            default: /*AVG*/ {
              if (!S.count) { valid = false; break; }
              double v;
              if (A.in_class == VC_F64) v = S.sum_f / (double)S.count;
              else {
                double sum = i128_to_double(mk128((int64_t)S.sum_lo, S.sum_hi));
                double div = (double)S.count;
                for (int k = 0; k < A.avg_scale; k++) div *= 10.0;
                v = sum / div;
              }
              lo = __double_as_longlong(v);
              break;
            }
          }
        }
        if (valid) store_phys(A.out, A.out_phys, i, lo, hi);
        else store_phys(A.out, A.out_phys, i, 0, 0);
      }
      uint64_t m = __ballot(valid);
      if (lane == 0) {
        A.valid[base >> 5] = (uint32_t)m;
        if (base + 32 < n) A.valid[(base >> 5) + 1] = (uint32_t)(m >> 32);
      }
    }
  }
}

__global__ __launch_bounds__(256) void emit_agg_kernel(EmitDesc D) {
  __shared__ Acc part[4];
  emit_agg_body(D, part, blockIdx.x, gridDim.x);
}

// The group_direct_lds partials of nb workgroups reduced per key (one wave per
// key at a time, its lanes over the records, carry-correct int128 sums), every
// key's state and COUNT(*) slot written (empty keys as the initialisation
// leaves them), then the non-empty keys compacted in key order as
// compact_slots_kernel does, from the counts kept in LDS.
template <int NV, bool MM>
__global__ __launch_bounds__(1024) void group_partials_compact_kernel(const unsigned long long *gpart, int nb, int nk,
                                                                      unsigned long long *count_star, AggState *st0,
                                                                      AggState *st1, int32_t *slot_list,
                                                                      int64_t *n_out, EmitDesc D, int emit) {
  constexpr int W = GroupPartialWords(NV, MM);
  __shared__ unsigned long long kc[kGroupPartialKeys];
  __shared__ int wsum[16];
  __shared__ Acc part[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int kq = w; kq < nk; kq += nw) {
    unsigned long long c = 0;
    Acc A[NV > 0 ? NV : 1];
    for (int j = 0; j < (NV > 0 ? NV : 1); j++) {
      A[j].cnt = 0; A[j].slo = 0; A[j].shi = 0; A[j].mn = INT64_MAX; A[j].mx = INT64_MIN;
    }
#pragma unroll 4
    for (int b = lane; b < nb; b += 64) {  // (unrolled: a lane's records load together)
      const unsigned long long *o = gpart + ((size_t)kq * nb + b) * W;
      c += o[0];
      int f = 1;
#pragma unroll
      for (int j = 0; j < NV; j++) {
        Acc B;
        B.cnt = o[f]; B.slo = o[f + 1]; B.shi = (int64_t)o[f + 2];
        B.mn = MM ? (int64_t)o[f + 3] : INT64_MAX;
        B.mx = MM ? (int64_t)o[f + 4] : INT64_MIN;
        f += MM ? 5 : 3;
        acc_merge(A[j], B);
      }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) c += shfl_xor_u64(c, m);
#pragma unroll
    for (int j = 0; j < NV; j++) acc_wave_reduce(A[j]);
    if (lane == 0) {
      kc[kq] = c;
      count_star[kq] = c;
      for (int j = 0; j < 2; j++) {
        AggState z;
        z.count = 0; z.sum_lo = 0; z.sum_hi = 0;
        z.min_i = INT64_MAX; z.max_i = INT64_MIN;
        z.sum_f = 0; z.min_f = 0xFFFFFFFFFFFFFFFFull; z.max_f = 0;
        if (j < NV && A[j].cnt) {
          z.count = A[j].cnt; z.sum_lo = A[j].slo; z.sum_hi = A[j].shi;
          if (MM) { z.min_i = A[j].mn; z.max_i = A[j].mx; }
        }
        (j == 0 ? st0 : st1)[kq] = z;
      }
    }
  }
  __syncthreads();
  // compaction of the non-empty keys (one pass: nk <= blockDim.x)
  const int i = threadIdx.x;
  const bool f = i < nk && kc[i] > 0;
  const uint64_t m = __ballot(f);
  if (lane == 0) wsum[w] = __popcll(m);
  __syncthreads();
  int before = 0, total = 0;
  for (int k = 0; k < nw; k++) {
    before += k < w ? wsum[k] : 0;
    total += wsum[k];
  }
  const uint64_t lt = lane ? (m & ((1ull << lane) - 1ull)) : 0ull;
  if (f) slot_list[before + __popcll(lt)] = (int32_t)i;
  if (threadIdx.x == 0) *n_out = total;
  if (!emit) return;
  // the relation of the compacted keys (D reads the states, slot list and
  // count just written by this workgroup)
  __threadfence_block();
  __syncthreads();
  emit_agg_body(D, part, 0, 1);
}

void GroupPartialsCompact(const GroupPartialsOut &po, int nv, bool mm, int nk, unsigned long long *count_star,
                          AggState *st0, AggState *st1, int32_t *slot_list, int64_t *n_out, hipStream_t s,
                          const EmitDesc *emit) {
  EmitDesc D;
  if (emit) D = *emit;
  else memset(&D, 0, sizeof(D));
#define GPC(NV, MM)                                                                                               \
  hipLaunchKernelGGL((group_partials_compact_kernel<NV, MM>), dim3(1), dim3(1024), 0, s,                          \
                     (const unsigned long long *)po.buf, po.blocks, nk, count_star, st0, st1, slot_list, n_out, D, \
                     emit ? 1 : 0)
  if (nv == 0) GPC(0, false);
  else if (nv == 1) { if (mm) GPC(1, true); else GPC(1, false); }
  else { if (mm) GPC(2, true); else GPC(2, false); }
#undef GPC
  CHECK_LAUNCH();
}

void CompactSlots(const unsigned long long *count_star, int64_t nslots, int32_t *slot_list, int64_t *n_out,
                  hipStream_t s) {
  if (nslots <= (1 << 16)) {
    hipLaunchKernelGGL(compact_slots_kernel, dim3(1), dim3(1024), 0, s, count_star, nslots, slot_list, n_out);
    CHECK_LAUNCH();
    return;
  }
  int32_t *flag = (int32_t *)TempAlloc((size_t)nslots * 4);
  int32_t *pos = (int32_t *)TempAlloc((size_t)nslots * 4);
  const int grid = GridFor(nslots, 256 * 4, NumCUs() * 8);
  hipLaunchKernelGGL(slot_flags_kernel, dim3(grid), dim3(256), 0, s, count_star, nslots, flag);
  CHECK_LAUNCH();
  size_t tmp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, flag, pos, (int)nslots, s);
  void *d_tmp = TempAlloc(tmp ? tmp : 16);
  (void)hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp, flag, pos, (int)nslots, s);
  hipLaunchKernelGGL(slot_scatter_kernel, dim3(grid), dim3(256), 0, s, flag, pos, nslots, slot_list, n_out);
  CHECK_LAUNCH();
  TempFree(d_tmp, tmp ? tmp : 16);
  TempFree(pos, (size_t)nslots * 4);
  TempFree(flag, (size_t)nslots * 4);
}

// ---------------------------------------------------------------------------
// sort / gather
// ---------------------------------------------------------------------------
__global__ void sort_key_kernel(const void *col, int phys, const uint64_t *valid, int64_t n, const int64_t *perm,
                                bool desc, bool nulls_first, uint64_t *keys) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = perm ? perm[i] : i;
    uint64_t k;
    // NULL placement is a separate stable 1-bit pass (SortKeyNull), so the
    // full 64-bit value range stays distinct here
    if (!bit_valid(valid, r)) {
      k = 0ull;
    } else {
      int64_t lo, hi;
      load_phys(col, phys, r, lo, hi);
      if (phys == P_F64 || phys == P_F32) k = f64_order(__longlong_as_double(lo));
      else if (phys == P_U8 || phys == P_U16 || phys == P_U32 || phys == P_U64) k = (uint64_t)lo;
      else k = (uint64_t)lo ^ 0x8000000000000000ull;
      if (desc) k = ~k;
    }
    (void)nulls_first;
    keys[i] = k;
  }
}

void SortKeyU64(const void *col, int phys, const uint64_t *valid, int64_t n, const int64_t *perm, bool desc,
                bool nulls_first, uint64_t *keys, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sort_key_kernel, dim3(GridFor(n, 256 * 4, NumCUs() * 8)), dim3(256), 0, s, col, phys, valid, n,
                     perm, desc, nulls_first, keys);
  CHECK_LAUNCH();
}

void SortPairs(uint64_t *keys_in, int64_t *vals_in, uint64_t *keys_out, int64_t *vals_out, int64_t n, hipStream_t s,
               int end_bit) {
  if (n <= 0) return;
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, keys_in, keys_out, vals_in, vals_out, (int)n, 0, end_bit, s);
  void *d_tmp = nullptr;
  d_tmp = TempAlloc(tmp);
  (void)hipcub::DeviceRadixSort::SortPairs(d_tmp, tmp, keys_in, keys_out, vals_in, vals_out, (int)n, 0, end_bit, s);
  TempFree(d_tmp, tmp);
}

// 1-bit NULL-placement key: the last (most significant) pass of each ORDER BY key
__global__ void sort_key_null_kernel(const uint64_t *valid, int64_t n, const int64_t *perm, bool nulls_first,
                                     uint64_t *keys) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    bool isnull = !bit_valid(valid, perm ? perm[i] : i);
    keys[i] = (isnull != nulls_first) ? 1ull : 0ull;
  }
}

void SortKeyNull(const uint64_t *valid, int64_t n, const int64_t *perm, bool nulls_first, uint64_t *keys,
                 hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sort_key_null_kernel, dim3(GridFor(n, 256 * 4, NumCUs() * 8)), dim3(256), 0, s, valid, n, perm,
                     nulls_first, keys);
  CHECK_LAUNCH();
}

// VARCHAR ORDER BY: LSD over 8-byte chunks.  Chunk p of a string is its bytes
// [8p, 8p+8) big-endian, zero-padded (so a prefix sorts first); sorting the
// chunks from last to first with stable passes gives byte-wise (C collation)
// order.
__global__ void sort_key_str_kernel(const int64_t *offsets, const char *chars, const uint64_t *valid, int64_t n,
                                    const int64_t *perm, int64_t chunk, bool desc, uint64_t *keys) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = perm ? perm[i] : i;
    uint64_t k = 0;
    if (bit_valid(valid, r)) {
      int64_t b = offsets[r], e = offsets[r + 1];
      for (int j = 0; j < 8; j++) {
        int64_t at = b + chunk * 8 + j;
        k = (k << 8) | (at < e ? (uint8_t)chars[at] : 0u);
      }
      if (desc) k = ~k;
    }
    keys[i] = k;
  }
}

void SortKeyStr(const int64_t *offsets, const char *chars, const uint64_t *valid, int64_t n, const int64_t *perm,
                int64_t chunk, bool desc, uint64_t *keys, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sort_key_str_kernel, dim3(GridFor(n, 256 * 4, NumCUs() * 8)), dim3(256), 0, s, offsets, chars,
                     valid, n, perm, chunk, desc, keys);
  CHECK_LAUNCH();
}

__global__ void str_max_len_kernel(const int64_t *offsets, int64_t n, unsigned long long *out) {
  unsigned long long m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned long long l = (unsigned long long)(offsets[i + 1] - offsets[i]);
    m = l > m ? l : m;
  }
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long x = __shfl_xor(m, o);
    m = x > m ? x : m;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

void StrMaxLen(const int64_t *offsets, int64_t n, unsigned long long *out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, 8, s);
  if (n <= 0) return;
  hipLaunchKernelGGL(str_max_len_kernel, dim3(GridFor(n, 256 * 4, NumCUs() * 4)), dim3(256), 0, s, offsets, n, out);
  CHECK_LAUNCH();
}

__global__ void iota_kernel(int64_t *p, int64_t n, int64_t start) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = start + i;
}

void Iota(int64_t *p, int64_t n, int64_t start, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(iota_kernel, dim3(GridFor(n, 256 * 4, NumCUs() * 8)), dim3(256), 0, s, p, n, start);
  CHECK_LAUNCH();
}

__global__ void gather_fixed_kernel(const void *in, int phys, const uint64_t *in_valid, const int64_t *idx, int64_t n,
                                    void *out, uint32_t *out_valid) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = idx[i];
    int64_t lo, hi;
    load_phys(in, phys, r, lo, hi);
    if (phys == P_F32) {  // keep exact float bits
      ((float *)out)[i] = ((const float *)in)[r];
    } else if (phys == P_INTERVAL) {
      ((int64_t *)out)[2 * i] = ((const int64_t *)in)[2 * r];
      ((int64_t *)out)[2 * i + 1] = ((const int64_t *)in)[2 * r + 1];
    } else {
      store_phys(out, phys, i, lo, hi);
    }
    if (out_valid && bit_valid(in_valid, r)) atomicOr(&out_valid[i >> 5], 1u << (i & 31));
  }
}

void GatherFixed(const void *in, int phys, const uint64_t *in_valid, const int64_t *idx, int64_t n, void *out,
                 uint32_t *out_valid, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_fixed_kernel, dim3(GridFor(n, 256 * 4, NumCUs() * 8)), dim3(256), 0, s, in, phys, in_valid,
                     idx, n, out, out_valid);
  CHECK_LAUNCH();
}

__global__ void gather_slots_kernel(const unsigned char *in, int eb, const int32_t *idx, int64_t n, unsigned char *out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned char *src = in + (int64_t)idx[i] * eb;
    unsigned char *dst = out + i * eb;
    for (int k = 0; k < eb; k++) dst[k] = src[k];
  }
}

void GatherSlots(const void *in, int elem_bytes, const int32_t *idx, int64_t n, void *out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_slots_kernel, dim3(GridFor(n, 256, 1024)), dim3(256), 0, s, (const unsigned char *)in,
                     elem_bytes, idx, n, (unsigned char *)out);
  CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// strings
// ---------------------------------------------------------------------------
__global__ void str_len_kernel(const int64_t *codes, const uint64_t *valid, int64_t n, const int64_t *src_off,
                               const int64_t *pool_off, int64_t *lens) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t c = codes[i];
    int64_t L = 0;
    if (bit_valid(valid, i)) {
      if (c >= 0) L = src_off[c + 1] - src_off[c];
      else L = pool_off[-c] - pool_off[-c - 1];
    }
    lens[i] = L;
  }
}

void StringLengths(const int64_t *codes, const uint64_t *valid, int64_t n, const int64_t *src_off,
                   const int64_t *pool_off, int64_t *lens, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(str_len_kernel, dim3(GridFor(n, 256 * 4, NumCUs() * 8)), dim3(256), 0, s, codes, valid, n, src_off,
                     pool_off, lens);
  CHECK_LAUNCH();
}

void ScanLengths(const int64_t *lens, int64_t *offsets, int64_t n, hipStream_t s) {
  // offsets[0] = 0, offsets[i+1] = inclusive sum
  (void)hipMemsetAsync(offsets, 0, sizeof(int64_t), s);
  if (n <= 0) return;
  size_t tmp = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, tmp, lens, offsets + 1, (int)n, s);
  void *d_tmp = nullptr;
  d_tmp = TempAlloc(tmp);
  (void)hipcub::DeviceScan::InclusiveSum(d_tmp, tmp, lens, offsets + 1, (int)n, s);
  TempFree(d_tmp, tmp);
}

__global__ void str_copy_kernel(const int64_t *codes, const uint64_t *valid, int64_t n, const int64_t *src_off,
                                const char *src_chars, const int64_t *pool_off, const char *pool_chars,
                                const int64_t *out_off, char *out_chars) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!bit_valid(valid, i)) continue;
    int64_t c = codes[i];
    const char *src;
    int64_t L;
    if (c >= 0) {
      src = src_chars + src_off[c];
      L = src_off[c + 1] - src_off[c];
    } else {
      src = pool_chars + pool_off[-c - 1];
      L = pool_off[-c] - pool_off[-c - 1];
    }
    char *dst = out_chars + out_off[i];
    for (int64_t k = 0; k < L; k++) dst[k] = src[k];
  }
}

void StringCopy(const int64_t *codes, const uint64_t *valid, int64_t n, const int64_t *src_off, const char *src_chars,
                const int64_t *pool_off, const char *pool_chars, const int64_t *out_off, char *out_chars,
                hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(str_copy_kernel, dim3(GridFor(n, 256 * 4, NumCUs() * 8)), dim3(256), 0, s, codes, valid, n,
                     src_off, src_chars, pool_off, pool_chars, out_off, out_chars);
  CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// ingest helpers
// ---------------------------------------------------------------------------
template <typename T>
__global__ void synth_kernel(T *out, int64_t n, uint64_t seed, int64_t start, uint64_t m, int64_t add) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (T)((int64_t)(splitmix64(seed + (uint64_t)(start + i)) % m) + add);
}

void Synth(void *out, int phys, int64_t n, int64_t seed, int64_t start, int64_t m, int64_t add, hipStream_t s) {
  if (n <= 0) return;
  int grid = GridFor(n, 256 * 8, NumCUs() * 8);
  if (phys == P_I32)
    hipLaunchKernelGGL(synth_kernel<int32_t>, dim3(grid), dim3(256), 0, s, (int32_t *)out, n, (uint64_t)seed, start,
                       (uint64_t)m, add);
  else
    hipLaunchKernelGGL(synth_kernel<int64_t>, dim3(grid), dim3(256), 0, s, (int64_t *)out, n, (uint64_t)seed, start,
                       (uint64_t)m, add);
  CHECK_LAUNCH();
}

__global__ void bitmap_append_kernel(uint64_t *dst, int64_t dst_off, const uint64_t *src, int64_t n) {
  // one thread per destination word touched
  int64_t first = dst_off >> 6, last = (dst_off + n - 1) >> 6;
  for (int64_t wi = first + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; wi <= last;
       wi += (int64_t)gridDim.x * blockDim.x) {
    uint64_t word = 0;
    int64_t b0 = wi << 6;
    for (int k = 0; k < 64; k++) {
      int64_t db = b0 + k;
      if (db < dst_off || db >= dst_off + n) {
        word |= dst[wi] & (1ull << k);
        continue;
      }
      int64_t sb = db - dst_off;
      uint64_t bit = src ? ((src[sb >> 6] >> (sb & 63)) & 1ull) : 1ull;
      word |= bit << k;
    }
    dst[wi] = word;
  }
}

void BitmapAppend(uint64_t *dst, int64_t dst_off, const uint64_t *src, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  int64_t words = ((dst_off + n - 1) >> 6) - (dst_off >> 6) + 1;
  hipLaunchKernelGGL(bitmap_append_kernel, dim3(GridFor(words, 256, 4096)), dim3(256), 0, s, dst, dst_off, src, n);
  CHECK_LAUNCH();
}

void CopyKernel(const void *in, void *out, int64_t nbytes, hipStream_t s) {
  int64_t n = nbytes / 16;
  hipLaunchKernelGGL(copy_kernel, dim3(NumCUs() * 8), dim3(256), 0, s, (const float4 *)in, (float4 *)out, n);
  CHECK_LAUNCH();
}

}  // namespace dev
}  // namespace mbx

namespace mbx {
namespace dev {

void EmitAggRelation(const EmitDesc &d, hipStream_t s) {
  hipLaunchKernelGGL(emit_agg_kernel, dim3(d.npartials > 0 ? 1 : GridFor(d.nslots, 256, 1024)), dim3(256), 0, s, d);
  CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// hash GROUP BY
// ---------------------------------------------------------------------------
#define HT_EMPTY 0xFFFFFFFFFFFFFFFFull
#define HT_ROW_MASK ((1ull << 40) - 1)

__device__ __forceinline__ uint64_t hmix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// key value as (up to) 128 bits; floats normalised so -0.0 groups with 0.0
// and every NaN with every other NaN
__device__ __forceinline__ void key_bits(const HashKeyCol &c, int64_t r, uint64_t &w0, uint64_t &w1) {
  int64_t lo, hi;
  load_phys(c.data, c.phys, r, lo, hi);
  if (c.phys == P_F64 || c.phys == P_F32) {
    double d = __longlong_as_double(lo);
    if (d == 0.0) d = 0.0;
    if (d != d) d = __longlong_as_double(0x7FF8000000000000ll);
    lo = __double_as_longlong(d);
  }
  w0 = (uint64_t)lo;
  w1 = (uint64_t)hi;
}

__device__ uint64_t row_hash(const HashKeys &K, int64_t r) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int j = 0; j < K.nk; j++) {
    const HashKeyCol &c = K.k[j];
    if (!bit_valid(c.validity, r)) {
      h = hmix(h ^ 0x5BD1E9955BD1E995ull);
      continue;
    }
    if (c.phys == P_STR) {
      int64_t b = c.offsets[r], e = c.offsets[r + 1];
      uint64_t f = 0xCBF29CE484222325ull ^ (uint64_t)(e - b);
      for (int64_t i = b; i < e; i++) f = (f ^ (uint8_t)c.chars[i]) * 0x100000001B3ull;
      h = hmix(h ^ f);
    } else {
      uint64_t w0, w1;
      key_bits(c, r, w0, w1);
      h = hmix(h ^ w0);
      h = hmix(h ^ (w1 + 0x632BE59BD9B4E019ull));
    }
  }
  return h;
}

__device__ bool rows_equal(const HashKeys &K, int64_t a, int64_t b) {
  for (int j = 0; j < K.nk; j++) {
    const HashKeyCol &c = K.k[j];
    bool va = bit_valid(c.validity, a), vb = bit_valid(c.validity, b);
    if (va != vb) return false;
    if (!va) continue;
    if (c.phys == P_STR) {
      int64_t ab = c.offsets[a], ae = c.offsets[a + 1], bb = c.offsets[b], be = c.offsets[b + 1];
      if (ae - ab != be - bb) return false;
      for (int64_t i = 0; i < ae - ab; i++)
        if (c.chars[ab + i] != c.chars[bb + i]) return false;
    } else {
      uint64_t a0, a1, b0, b1;
      key_bits(c, a, a0, a1);
      key_bits(c, b, b0, b1);
      if (a0 != b0 || a1 != b1) return false;
    }
  }
  return true;
}

__global__ __launch_bounds__(256) void hash_insert_kernel(HashKeys K, int64_t n, unsigned long long *table,
                                                          uint64_t mask, int32_t *entry_of, int32_t *err) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = row_hash(K, r);
    const uint64_t tag = h >> 40;
    const unsigned long long mine = (tag << 40) | (uint64_t)r;
    uint64_t e = h & mask;
    int32_t got = -1;
    for (uint64_t probe = 0; probe <= mask; probe++) {
      unsigned long long cur = __hip_atomic_load(&table[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == HT_EMPTY) {
        unsigned long long prev = atomicCAS(&table[e], HT_EMPTY, mine);
        if (prev == HT_EMPTY) {
          got = (int32_t)e;
          break;
        }
        cur = prev;
      }
      if ((cur >> 40) == tag && rows_equal(K, (int64_t)(cur & HT_ROW_MASK), r)) {
        got = (int32_t)e;
        break;
      }
      e = (e + 1) & mask;
    }
    if (got < 0) atomicCAS(err, 0, E_HASH_FULL);  // cannot happen with cap >= 2n; never loops forever
    entry_of[r] = got < 0 ? 0 : got;
  }
}

__global__ void hash_occupancy_kernel(const unsigned long long *table, int64_t cap, int32_t *flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = table[i] != HT_EMPTY;
}

// pos = exclusive scan of the occupancy flags: entry e (occupied) -> group pos[e]
__global__ void hash_groups_kernel(const unsigned long long *table, const int32_t *flag, const int32_t *pos,
                                   int64_t cap, int32_t *gid_of_entry, int64_t *rep_row, int64_t *ngroups) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
    if (flag[i]) {
      gid_of_entry[i] = pos[i];
      rep_row[pos[i]] = (int64_t)(table[i] & HT_ROW_MASK);
    }
    if (i == cap - 1) *ngroups = (int64_t)pos[i] + flag[i];
  }
}

__global__ void hash_slots_kernel(int32_t *slot_of_row, const int32_t *gid_of_entry, int64_t n,
                                  unsigned long long *count_star) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    int32_t g = gid_of_entry[slot_of_row[r]];
    slot_of_row[r] = g;
    if (count_star) atomicAdd(&count_star[g], 1ull);
  }
}

__global__ void count_slots_kernel(const int32_t *slot_of_row, int64_t n, unsigned long long *count_star) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&count_star[slot_of_row[r]], 1ull);
}

void CountSlots(const int32_t *slot_of_row, int64_t n, unsigned long long *count_star, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(count_slots_kernel, dim3(GridFor(n, 256 * 4, NumCUs() * 8)), dim3(256), 0, s, slot_of_row, n,
                     count_star);
  CHECK_LAUNCH();
}

void HashGroupAssign(const HashKeys &k, int64_t n, unsigned long long *table, int64_t cap, int32_t *slot_of_row,
                     int32_t *gid_of_entry, int64_t *rep_row, unsigned long long *count_star, int64_t *ngroups,
                     int32_t *err, hipStream_t s) {
  // table must hold HT_EMPTY, count_star zeros (caller); gid_of_entry doubles as scan scratch
  if (n <= 0) {
    (void)hipMemsetAsync(ngroups, 0, 8, s);
    return;
  }
  const int grid = GridFor(n, 256 * 4, NumCUs() * 8);
  hipLaunchKernelGGL(hash_insert_kernel, dim3(grid), dim3(256), 0, s, k, n, table, (uint64_t)(cap - 1), slot_of_row,
                     err);
  CHECK_LAUNCH();
  int32_t *flag = nullptr, *pos = nullptr;
  flag = (int32_t *)TempAlloc((size_t)cap * 4);
  pos = (int32_t *)TempAlloc((size_t)cap * 4);
  const int cgrid = GridFor(cap, 256 * 4, NumCUs() * 8);
  hipLaunchKernelGGL(hash_occupancy_kernel, dim3(cgrid), dim3(256), 0, s, table, cap, flag);
  CHECK_LAUNCH();
  size_t tmp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, flag, pos, (int)cap, s);
  void *d_tmp = nullptr;
  d_tmp = TempAlloc(tmp ? tmp : 16);
  (void)hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp, flag, pos, (int)cap, s);
  hipLaunchKernelGGL(hash_groups_kernel, dim3(cgrid), dim3(256), 0, s, table, flag, pos, cap, gid_of_entry, rep_row,
                     ngroups);
  CHECK_LAUNCH();
  hipLaunchKernelGGL(hash_slots_kernel, dim3(grid), dim3(256), 0, s, slot_of_row, gid_of_entry, n, count_star);
  CHECK_LAUNCH();
  TempFree(d_tmp, tmp ? tmp : 16);
  TempFree(pos, (size_t)cap * 4);
  TempFree(flag, (size_t)cap * 4);
}

__global__ __launch_bounds__(256) void host_copy_kernel(HostCopyDesc D) {
  if ((int)blockIdx.x < D.nseg) {
    const HostCopySeg g = D.seg[blockIdx.x];
    const int64_t words = ((((uintptr_t)g.src | (uintptr_t)g.dst) & 7) == 0) ? g.bytes >> 3 : 0;
    const uint64_t *s8 = (const uint64_t *)g.src;
    uint64_t *d8 = (uint64_t *)g.dst;
    for (int64_t i = threadIdx.x; i < words; i += blockDim.x) d8[i] = s8[i];
    const uint8_t *s1 = (const uint8_t *)g.src;
    uint8_t *d1 = (uint8_t *)g.dst;
    for (int64_t i = (words << 3) + threadIdx.x; i < g.bytes; i += blockDim.x) d1[i] = s1[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *D.err_dst = *D.err_src;
  __threadfence_system();
}

void HostCopy(const HostCopyDesc &d, hipStream_t s) {
  hipLaunchKernelGGL(host_copy_kernel, dim3(d.nseg > 0 ? d.nseg : 1), dim3(256), 0, s, d);
  CHECK_LAUNCH();
}

// Arrow wire layout of one fixed-width column (reference duckdb_native.c
// :2572-2797, the *_nullable getters): values with NULL slots zeroed, then one
// validity byte per row (1 = valid).  Rows are independent; each thread does
// one row per grid-stride step, so loads and stores are coalesced.
template <typename T>
__global__ void arrow_wire_kernel(const T *__restrict__ src, const uint64_t *__restrict__ valid, int64_t n,
                                  T *__restrict__ vals, uint8_t *__restrict__ vbytes) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool ok = valid == nullptr || ((valid[i >> 6] >> (i & 63)) & 1);
    vals[i] = ok ? src[i] : (T)0;
    if (vbytes) vbytes[i] = ok ? 1 : 0;
  }
}

void ArrowWire(const void *src, const uint64_t *valid, int64_t n, int width, void *vals, uint8_t *vbytes,
               hipStream_t s) {
  if (n <= 0) return;
  const dim3 g(GridFor(n, 256 * 4, 4096)), b(256);
  switch (width) {
    case 1: hipLaunchKernelGGL(arrow_wire_kernel<uint8_t>, g, b, 0, s, (const uint8_t *)src, valid, n, (uint8_t *)vals, vbytes); break;
    case 4: hipLaunchKernelGGL(arrow_wire_kernel<uint32_t>, g, b, 0, s, (const uint32_t *)src, valid, n, (uint32_t *)vals, vbytes); break;
    case 8: hipLaunchKernelGGL(arrow_wire_kernel<uint64_t>, g, b, 0, s, (const uint64_t *)src, valid, n, (uint64_t *)vals, vbytes); break;
    default: return;
  }
  CHECK_LAUNCH();
}

__global__ void rebase_kernel(const int64_t *src, int64_t *dst, int64_t n, int64_t delta) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i] + delta;
}

void RebaseOffsets(const int64_t *src, int64_t *dst, int64_t n, int64_t delta, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(rebase_kernel, dim3(GridFor(n, 256 * 4, 4096)), dim3(256), 0, s, src, dst, n, delta);
  CHECK_LAUNCH();
}


// ---------------------------------------------------------------------------
// Filter -> compaction, two streaming passes (see device.h).  A one-pass form
// with a decoupled look-back over 2048/4096-row tiles measured slower on this
// chip (sel 4.1-9.8 ms vs 2-pass JIT 5.3 ms at 1e9 rows): a tile routinely
// finishes loading before its predecessor (4 predecessor polls per tile), so
// every workgroup waits out the slowest recent load while holding its slot.
// Both passes here stream with no inter-workgroup waits.
// ---------------------------------------------------------------------------

// pass 1: NI LDS-DMA instructions per wave step (1 per KiB of predicate
// slices, 1 per nullable column for its 4 validity words), DEPTH steps in flight
template <int NI, int DEPTH>
__global__ __launch_bounds__(256) void filter_bits_lds_kernel(FilterMultiDesc D, int64_t n, unsigned long long *bits,
                                                              int slot_bytes) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fb_lds[];
  const int SB = slot_bytes;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = fb_lds + (size_t)w * DEPTH * SB;
  int off[FM_MAX], voff[FM_MAX];
  {
    int o = 0;
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      off[c] = o;
      if (c < D.ncol) o += D.col[c].phys == P_I64 ? 2048 : 1024;
    }
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      voff[c] = o;
      if (c < D.ncol && D.col[c].valid) o += 32;
    }
  }
  const int64_t nsteps = n >> 8;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t st = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t q, int d) {
    unsigned char *dst = ring + d * SB;
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      if (c >= D.ncol) break;
      const int B = D.col[c].phys == P_I64 ? 2048 : 1024;
      const unsigned char *src = (const unsigned char *)D.col[c].data + q * B;
      __builtin_amdgcn_global_load_lds((const void *)(src + lane * 16), (void *)(dst + off[c]), 16, 0, 2);
      if (B == 2048)
        __builtin_amdgcn_global_load_lds((const void *)(src + 1024 + lane * 16), (void *)(dst + off[c] + 1024), 16, 0, 2);
      // the step's 4 validity words: lanes 0-1, 16 B each (exec-masked, still one vmcnt)
      if (D.col[c].valid && lane < 2)
        __builtin_amdgcn_global_load_lds((const void *)(D.col[c].valid + q * 4 + lane * 2), (void *)(dst + voff[c]), 16,
                                         0, 0);
    }
  };
  // one step's 4 ballot words: lanes 0..3 store a word each (32 contiguous bytes)
  auto emit = [&](int64_t step, const bool ok[4]) {
    unsigned long long b[4];
#pragma unroll
    for (int e = 0; e < 4; e++) b[e] = __ballot(ok[e]);
    const unsigned long long mine = lane == 0 ? b[0] : lane == 1 ? b[1] : lane == 2 ? b[2] : b[3];
    if (lane < 4) __builtin_nontemporal_store(mine, bits + step * 4 + lane);
  };
  if (nsteps > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      int64_t q = st + d * nw;
      issue(q < nsteps ? q : 0, d);
    }
  }
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * SB;
    int64_t v[FM_MAX][4];
    unsigned vm = 0xFu;  // rows 4 lane + e whose predicate columns are all non-NULL
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      if (c >= D.ncol) break;
      if (D.col[c].phys == P_I64) {
        v2i64 x0 = *(const v2i64 *)(src + off[c] + lane * 32), x1 = *(const v2i64 *)(src + off[c] + lane * 32 + 16);
        v[c][0] = x0.x; v[c][1] = x0.y; v[c][2] = x1.x; v[c][3] = x1.y;
      } else {
        v4i32 x = *(const v4i32 *)(src + off[c] + lane * 16);
        v[c][0] = x.x; v[c][1] = x.y; v[c][2] = x.z; v[c][3] = x.w;
      }
      if (D.col[c].valid)
        vm &= (unsigned)(*(const uint64_t *)(src + voff[c] + (lane >> 4) * 8) >> (4 * (lane & 15))) & 0xFu;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int64_t q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    bool ok[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      ok[e] = (vm >> e) & 1u;
#pragma unroll
      for (int c = 0; c < FM_MAX; c++)
        if (c < D.ncol) ok[e] = ok[e] && (uint64_t)(v[c][e]) - (uint64_t)(D.col[c].lo) <= D.col[c].span;
    }
    emit(st, ok);
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the partial last step (n % 256 rows): block 0, wave 0, scalar loads
  if (blockIdx.x == 0 && w == 0 && (n & 255)) {
    bool ok[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int64_t i = (nsteps << 8) + 4 * lane + e;
      ok[e] = i < n;
      for (int c = 0; c < D.ncol && ok[e]; c++) {
        const int64_t x = D.col[c].phys == P_I64 ? ((const int64_t *)D.col[c].data)[i]
                                                 : (int64_t)((const int32_t *)D.col[c].data)[i];
        ok[e] = (uint64_t)(x) - (uint64_t)(D.col[c].lo) <= D.col[c].span &&
                (!D.col[c].valid || ((D.col[c].valid[i >> 6] >> (i & 63)) & 1));
      }
    }
    emit(nsteps, ok);
  }
}

void FilterBits(const FilterMultiDesc &d, int64_t nrows, unsigned long long *bits, hipStream_t s) {
  if (nrows <= 0) return;
  int ni = 0, slot = 0;
  for (int c = 0; c < d.ncol; c++) {
    ni += d.col[c].phys == P_I64 ? 2 : 1;
    slot += d.col[c].phys == P_I64 ? 2048 : 1024;
    if (d.col[c].valid) {
      ni++;
      slot += 32;
    }
  }
  slot = (slot + 15) & ~15;
  int gpc = 3;
  if (const char *e = Knob("MBX_FB_BLOCKS_PER_CU")) gpc = atoi(e) > 0 ? atoi(e) : 3;
  int grid = NumCUs() * gpc;
  const int64_t need = (nrows >> 8) / 4 + 1;
  if (grid > need) grid = (int)need;
  int dp = 0;  // MBX_FB_DEPTH: ring depth override (sweeps)
  if (const char *e = Knob("MBX_FB_DEPTH")) dp = atoi(e);
#define FB(L, DP)                                                                                           \
  hipLaunchKernelGGL((filter_bits_lds_kernel<L, DP>), dim3(grid), dim3(256), (size_t)4 * DP * slot, s, d, \
                     nrows, bits, slot)
#define FBD(L, DEF) \
  if ((dp ? dp : DEF) <= 2) FB(L, 2); else if ((dp ? dp : DEF) <= 3) FB(L, 3); else if ((dp ? dp : DEF) <= 4) FB(L, 4); else FB(L, 6);
  switch (ni) {  // the executor keeps ni <= 8
    case 1: FBD(1, 6); break;
    case 2: FBD(2, 3); break;
    case 3: FBD(3, 2); break;
    case 4: FBD(4, 2); break;
    case 5: FB(5, 2); break;
    case 6: FB(6, 2); break;
    case 7: FB(7, 2); break;
    default: FB(8, 2); break;
  }
#undef FBD
#undef FB
  CHECK_LAUNCH();
}

// Validity of the compacted rows.  A wave owns a chunk of CV_CHUNK (8) consecutive
// 256-row steps and prefetches the chunk's ballot words, validity words and
// step offsets with one load each per lane.  Per step, each lane writes the
// validity bytes of its selected rows (rows 4 lane + e) at their rank into the
// wave's 256-byte LDS staging row; four ballots over the staged bytes give the
// step's 256-bit run of output validity (run word q = ballot of bytes 64 q + lane).
// The run lands at bit offset[step] of the output through a carry word kept
// across the chunk's steps, so output words are written once with plain
// stores; only a chunk's first word (when a previous chunk may share it) and
// its final carry are ORed atomically: device-scope atomics leave the XCD's L2
// and are slow, so they are kept to about two per chunk.
#define CV_CHUNK 8
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
  return (uint64_t)hi << 32 | lo;
}

__global__ __launch_bounds__(256) void compact_validity_kernel(const unsigned long long *bits, const int64_t *offs,
                                                               int64_t n, const uint64_t *vin, uint64_t *vout) {
  __shared__ __attribute__((aligned(16))) uint8_t stage_lds[4][256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t *stage = stage_lds[w];
  const uint64_t lt = (1ull << lane) - 1;
  const int64_t steps = (n + 255) >> 8, nwords = (n + 63) >> 6;
  const int64_t nchunks = (steps + CV_CHUNK - 1) / CV_CHUNK;
  for (int64_t ch = (int64_t)blockIdx.x * 4 + w; ch < nchunks; ch += (int64_t)gridDim.x * 4) {
    const int64_t s0 = ch * CV_CHUNK;
    // the chunk's 4 x 32 ballot words and validity words: 2 of each per lane
    const int64_t bw = 4 * s0 + 2 * lane;
    const bool in0 = bw < 4 * steps, in1 = bw + 1 < 4 * steps;
    const uint64_t pb0 = in0 ? bits[bw] : 0, pb1 = in1 ? bits[bw + 1] : 0;
    const uint64_t pv0 = bw < nwords ? vin[bw] : 0, pv1 = bw + 1 < nwords ? vin[bw + 1] : 0;
    const int64_t po = lane < CV_CHUNK && s0 + lane < steps ? offs[s0 + lane] : 0;
    int64_t carry_idx = -1, first_word = -1;
    uint64_t carry_val = 0;
    bool first_shared = false;
    auto put = [&](int64_t W, uint64_t val) {  // one complete (or final) output word
      if (W == first_word && first_shared) {
        if (val) atomicOr((unsigned long long *)&vout[W], (unsigned long long)val);
      } else {
        vout[W] = val;
      }
    };
    for (int j = 0; j < CV_CHUNK && s0 + j < steps; j++) {
      const uint64_t b0 = readlane64(pb0, 2 * j), b1 = readlane64(pb1, 2 * j);
      const uint64_t b2 = readlane64(pb0, 2 * j + 1), b3 = readlane64(pb1, 2 * j + 1);
      const int cnt = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
      if (cnt == 0) continue;  // wave-uniform
      const int64_t o = readlane64((uint64_t)po, j);
      // this lane's validity word: chunk word 4 j + (lane >> 4), held by lane (4 j + (lane >> 4)) / 2
      const int src = (4 * j + (lane >> 4)) >> 1;
      const uint64_t v0 = __shfl(pv0, src), v1 = __shfl(pv1, src);
      const uint64_t vword = ((lane >> 4) & 1) ? v1 : v0;
      const unsigned m = (unsigned)((b0 >> lane) & 1) | (unsigned)((b1 >> lane) & 1) << 1 |
                         (unsigned)((b2 >> lane) & 1) << 2 | (unsigned)((b3 >> lane) & 1) << 3;
      const int r0 = __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
      const unsigned vb = (unsigned)(vword >> (4 * (lane & 15))) & 0xFu;
      int r = r0;
#pragma unroll
      for (int e = 0; e < 4; e++)
        if ((m >> e) & 1u) stage[r++] = (uint8_t)((vb >> e) & 1u);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      uint64_t R[4];  // run word q, bit i = staged byte 64 q + i
#pragma unroll
      for (int qw = 0; qw < 4; qw++) R[qw] = __ballot(64 * qw + lane < cnt && stage[64 * qw + lane]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging reads done before the next step's writes
      const int64_t w0 = o >> 6, w1 = (o + cnt - 1) >> 6;
      if (first_word < 0) {
        first_word = w0;
        first_shared = (o & 63) != 0;
      }
      if (carry_idx >= 0 && carry_idx != w0) {  // the carry word is complete
        if (lane == 0) put(carry_idx, carry_val);
        carry_idx = -1;
      }
      const int64_t W = w0 + lane;
      uint64_t val = 0;
      if (lane <= 4 && W <= w1) {
        const int64_t sh = 64 * W - o;  // run bit at output bit 64 W; in [-63, 256)
        if (sh < 0) {
          val = R[0] << (-sh);
        } else {
          const int qw = (int)(sh >> 6), rb = (int)(sh & 63);
          const uint64_t a0 = qw == 0 ? R[0] : qw == 1 ? R[1] : qw == 2 ? R[2] : R[3];
          const uint64_t a1 = qw == 0 ? R[1] : qw == 1 ? R[2] : qw == 2 ? R[3] : 0;
          val = rb ? (a0 >> rb) | (a1 << (64 - rb)) : a0;
        }
        if (W == carry_idx) val |= carry_val;
        if (W < w1) put(W, val);
      }
      carry_val = readlane64(val, (int)(w1 - w0));
      carry_idx = w1;
    }
    if (carry_idx >= 0 && lane == 0 && carry_val)  // the next chunk may share it
      atomicOr((unsigned long long *)&vout[carry_idx], (unsigned long long)carry_val);
  }
}

void CompactValidity(const unsigned long long *bits, const int64_t *step_offsets, int64_t nrows,
                     const uint64_t *valid_in, uint64_t *valid_out, hipStream_t s) {
  if (nrows <= 0) return;
  const int64_t chunks = ((nrows + 255) >> 8) / CV_CHUNK + 1;
  hipLaunchKernelGGL(compact_validity_kernel, dim3(GridFor(chunks, 4, NumCUs() * 32)), dim3(256), 0, s, bits,
                     step_offsets, nrows, valid_in, valid_out);
  CHECK_LAUNCH();
}

// pass 2: NLD KiB of output slices per wave step
template <int NLD, int DEPTH>
__global__ __launch_bounds__(256) void compact_lds_kernel(CompactDesc D, int64_t n, const unsigned long long *bits,
                                                          const int64_t *offs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char cp_lds[];
  constexpr int SB = NLD * 1024 + 64;  // output slices + the step's metadata (4 ballot words, offset pair)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = cp_lds + (size_t)w * DEPTH * SB;
  unsigned char *stage = cp_lds + (size_t)4 * DEPTH * SB + (size_t)w * 2048;  // 256 rows x 8 B per wave
  int off[FC_MAX_OUT];
  {
    int o = 0;
#pragma unroll
    for (int c = 0; c < FC_MAX_OUT; c++) {
      off[c] = o;
      if (c < D.nout) o += D.ow[c] * 256;
    }
  }
  const uint64_t lt = (1ull << lane) - 1;
  const int64_t nsteps = n >> 8;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t st = (int64_t)blockIdx.x * 4 + w;
  // one step into slot d: every output slice, then the metadata in one
  // exec-masked LDS-DMA (lanes 0-1: the 32 B of ballot words, lane 2: the
  // 16-B aligned offset pair holding offs[q]) — NLD + 1 loads per step
  auto issue = [&](int64_t q, int d) {
    unsigned char *dst = ring + d * SB;
#pragma unroll
    for (int c = 0; c < FC_MAX_OUT; c++) {
      if (c >= D.nout) break;
      const int B = D.ow[c] * 256;
      const unsigned char *src = (const unsigned char *)D.src[c] + q * B;
      __builtin_amdgcn_global_load_lds((const void *)(src + lane * 16), (void *)(dst + off[c]), 16, 0, 2);
      if (B == 2048)
        __builtin_amdgcn_global_load_lds((const void *)(src + 1024 + lane * 16), (void *)(dst + off[c] + 1024), 16, 0, 2);
    }
    const unsigned char *msrc = lane < 2 ? (const unsigned char *)(bits + q * 4) + lane * 16
                                         : (const unsigned char *)(offs + (q & ~(int64_t)1));
    if (lane < 3) __builtin_amdgcn_global_load_lds((const void *)msrc, (void *)(dst + NLD * 1024), 16, 0, 0);
  };
  if (nsteps > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      int64_t q = st + d * nw;
      issue(q < nsteps ? q : 0, d);
    }
  }
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NLD + 1) * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * SB;
    const unsigned long long *meta = (const unsigned long long *)(src + NLD * 1024);
    const unsigned long long b0 = meta[0], b1 = meta[1], b2 = meta[2], b3 = meta[3];
    const int64_t o0 = (int64_t)meta[4 + (st & 1)];
    int64_t v[FC_MAX_OUT][4];
#pragma unroll
    for (int c = 0; c < FC_MAX_OUT; c++) {
      if (c >= D.nout) break;
      if (D.ow[c] == 8) {
        v2i64 x0 = *(const v2i64 *)(src + off[c] + lane * 32), x1 = *(const v2i64 *)(src + off[c] + lane * 32 + 16);
        v[c][0] = x0.x; v[c][1] = x0.y; v[c][2] = x1.x; v[c][3] = x1.y;
      } else {
        v4i32 x = *(const v4i32 *)(src + off[c] + lane * 16);
        v[c][0] = x.x; v[c][1] = x.y; v[c][2] = x.z; v[c][3] = x.w;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int64_t q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    const unsigned m = (unsigned)((b0 >> lane) & 1) | (unsigned)((b1 >> lane) & 1) << 1 |
                       (unsigned)((b2 >> lane) & 1) << 2 | (unsigned)((b3 >> lane) & 1) << 3;
    // rank of this lane's first selected row inside the step; step total
    const int r0 = __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
    const int cnt = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
    // each column: selected values -> the wave's staging area at their rank,
    // then consecutive lanes store consecutive rows
#pragma unroll
    for (int c = 0; c < FC_MAX_OUT; c++) {
      if (c >= D.nout) break;
      int r = r0;
      if (D.ow[c] == 8) {
#pragma unroll
        for (int e = 0; e < 4; e++)
          if ((m >> e) & 1u) ((int64_t *)stage)[r++] = v[c][e];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int i = lane; i < cnt; i += 64) ((int64_t *)D.dst[c])[o0 + i] = ((const int64_t *)stage)[i];
      } else {
#pragma unroll
        for (int e = 0; e < 4; e++)
          if ((m >> e) & 1u) ((int32_t *)stage)[r++] = (int32_t)v[c][e];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int i = lane; i < cnt; i += 64) ((int32_t *)D.dst[c])[o0 + i] = ((const int32_t *)stage)[i];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next column overwrites
    }
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the partial last step: block 0, wave 0, scalar loads
  if (blockIdx.x == 0 && w == 0 && (n & 255)) {
    const unsigned long long b0 = bits[nsteps * 4], b1 = bits[nsteps * 4 + 1], b2 = bits[nsteps * 4 + 2],
                             b3 = bits[nsteps * 4 + 3];
    const unsigned m = (unsigned)((b0 >> lane) & 1) | (unsigned)((b1 >> lane) & 1) << 1 |
                       (unsigned)((b2 >> lane) & 1) << 2 | (unsigned)((b3 >> lane) & 1) << 3;
    int64_t pos = offs[nsteps] + __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
    for (int e = 0; e < 4; e++) {
      const int64_t i = (nsteps << 8) + 4 * lane + e;
      if (!((m >> e) & 1u)) continue;  // rows past n are never selected
      for (int c = 0; c < D.nout; c++) {
        if (D.ow[c] == 8) ((int64_t *)D.dst[c])[pos] = ((const int64_t *)D.src[c])[i];
        else ((int32_t *)D.dst[c])[pos] = ((const int32_t *)D.src[c])[i];
      }
      pos++;
    }
  }
}

// copies row `row` of a w-byte column to position `pos` of another
__device__ __forceinline__ void fc_copy_row(const void *src, void *dst, int w, int64_t row, int64_t pos) {
  switch (w) {
    case 1: ((uint8_t *)dst)[pos] = ((const uint8_t *)src)[row]; break;
    case 2: ((uint16_t *)dst)[pos] = ((const uint16_t *)src)[row]; break;
    case 4: ((uint32_t *)dst)[pos] = ((const uint32_t *)src)[row]; break;
    case 8: ((uint64_t *)dst)[pos] = ((const uint64_t *)src)[row]; break;
    default: ((v4i32 *)dst)[pos] = ((const v4i32 *)src)[row]; break;
  }
}

// pass 2 for any mix of 1/2/4/8/16-byte outputs: every column's slice of a
// step (256 x w bytes, 1-4 LDS-DMA instructions; 1- and 2-byte slices use 16
// and 32 lanes) lands in the ring; each column's selected rows are copied
// slot -> per-wave staging area (LDS to LDS, at their rank) and stored out with
// consecutive lanes on consecutive rows; the slot is refilled after the last
// column.  NI = LDS-DMA instructions per step (compile time: the counted wait).
template <int NI, int DEPTH>
__global__ __launch_bounds__(256) void compact_any_lds_kernel(CompactDesc D, int64_t n, const unsigned long long *bits,
                                                              const int64_t *offs, int slot_bytes) {
  extern __shared__ __attribute__((aligned(16))) unsigned char ca_lds[];
  const int SB = slot_bytes;  // Σ 256 w + 64 (metadata), a multiple of 16
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = ca_lds + (size_t)w * DEPTH * SB;
  unsigned char *stage = ca_lds + (size_t)4 * DEPTH * SB + (size_t)w * 4096;  // 256 rows x 16 B per wave
  int off[FC_MAX_OUT];
  int meta_off = 0;
  {
    int o = 0;
#pragma unroll
    for (int c = 0; c < FC_MAX_OUT; c++) {
      off[c] = o;
      if (c < D.nout) o += D.ow[c] * 256;
    }
    meta_off = o;
  }
  const uint64_t lt = (1ull << lane) - 1;
  const int64_t nsteps = n >> 8;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t st = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t q, int d) {
    unsigned char *dst = ring + d * SB;
#pragma unroll
    for (int c = 0; c < FC_MAX_OUT; c++) {
      if (c >= D.nout) break;
      const int B = D.ow[c] * 256;
      const unsigned char *src = (const unsigned char *)D.src[c] + q * B;
      for (int j = 0; j < B; j += 1024)
        if (j + lane * 16 < B)
          __builtin_amdgcn_global_load_lds((const void *)(src + j + lane * 16), (void *)(dst + off[c] + j), 16, 0, 2);
    }
    const unsigned char *msrc = lane < 2 ? (const unsigned char *)(bits + q * 4) + lane * 16
                                         : (const unsigned char *)(offs + (q & ~(int64_t)1));
    if (lane < 3) __builtin_amdgcn_global_load_lds((const void *)msrc, (void *)(dst + meta_off), 16, 0, 0);
  };
  if (nsteps > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      int64_t q = st + d * nw;
      issue(q < nsteps ? q : 0, d);
    }
  }
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * SB;
    const unsigned long long *meta = (const unsigned long long *)(src + meta_off);
    const unsigned long long b0 = meta[0], b1 = meta[1], b2 = meta[2], b3 = meta[3];
    const int64_t o0 = (int64_t)meta[4 + (st & 1)];
    const unsigned m = (unsigned)((b0 >> lane) & 1) | (unsigned)((b1 >> lane) & 1) << 1 |
                       (unsigned)((b2 >> lane) & 1) << 2 | (unsigned)((b3 >> lane) & 1) << 3;
    const int r0 = __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
    const int cnt = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
#pragma unroll 1
    for (int c = 0; c < D.nout; c++) {
      const int ow = D.ow[c];
      const unsigned char *cs = src + off[c];
      int r = r0;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        if (!((m >> e) & 1u)) continue;
        const int row = 4 * lane + e;
        switch (ow) {
          case 1: stage[r] = cs[row]; break;
          case 2: ((uint16_t *)stage)[r] = ((const uint16_t *)cs)[row]; break;
          case 4: ((uint32_t *)stage)[r] = ((const uint32_t *)cs)[row]; break;
          case 8: ((uint64_t *)stage)[r] = ((const uint64_t *)cs)[row]; break;
          default: ((v4i32 *)stage)[r] = ((const v4i32 *)cs)[row]; break;
        }
        r++;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      unsigned char *dst = (unsigned char *)D.dst[c];
      switch (ow) {
        case 1: for (int i = lane; i < cnt; i += 64) dst[o0 + i] = stage[i]; break;
        case 2: for (int i = lane; i < cnt; i += 64) ((uint16_t *)dst)[o0 + i] = ((const uint16_t *)stage)[i]; break;
        case 4: for (int i = lane; i < cnt; i += 64) ((uint32_t *)dst)[o0 + i] = ((const uint32_t *)stage)[i]; break;
        case 8: for (int i = lane; i < cnt; i += 64) ((uint64_t *)dst)[o0 + i] = ((const uint64_t *)stage)[i]; break;
        default: for (int i = lane; i < cnt; i += 64) ((v4i32 *)dst)[o0 + i] = ((const v4i32 *)stage)[i]; break;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging reads done before the next column
    }
    int64_t q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (blockIdx.x == 0 && w == 0 && (n & 255)) {  // the partial last step
    const unsigned long long b0 = bits[nsteps * 4], b1 = bits[nsteps * 4 + 1], b2 = bits[nsteps * 4 + 2],
                             b3 = bits[nsteps * 4 + 3];
    const unsigned m = (unsigned)((b0 >> lane) & 1) | (unsigned)((b1 >> lane) & 1) << 1 |
                       (unsigned)((b2 >> lane) & 1) << 2 | (unsigned)((b3 >> lane) & 1) << 3;
    int64_t pos = offs[nsteps] + __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
    for (int e = 0; e < 4; e++) {
      const int64_t i = (nsteps << 8) + 4 * lane + e;
      if (!((m >> e) & 1u)) continue;
      for (int c = 0; c < D.nout; c++) fc_copy_row(D.src[c], D.dst[c], D.ow[c], i, pos);
      pos++;
    }
  }
}

static void CompactAny(const CompactDesc &d, int64_t nrows, const unsigned long long *bits, const int64_t *step_offsets,
                       int grid, hipStream_t s) {
  int ni = 1, sb = 64;
  for (int c = 0; c < d.nout; c++) {
    ni += (d.ow[c] * 256 + 1023) / 1024;
    sb += d.ow[c] * 256;
  }
  const size_t lds = (size_t)4 * 2 * sb + 4 * 4096;
#define CA(N)                                                                                               \
  hipLaunchKernelGGL((compact_any_lds_kernel<N, 2>), dim3(grid), dim3(256), lds, s, d, nrows, bits, step_offsets, sb)
  switch (ni) {
    case 2: CA(2); break;
    case 3: CA(3); break;
    case 4: CA(4); break;
    case 5: CA(5); break;
    case 6: CA(6); break;
    case 7: CA(7); break;
    case 8: CA(8); break;
    default: CA(9); break;
  }
#undef CA
  CHECK_LAUNCH();
}

void CompactColumns(const CompactDesc &d, int64_t nrows, const unsigned long long *bits, const int64_t *step_offsets,
                    hipStream_t s) {
  if (nrows <= 0 || d.nout <= 0) return;
  bool any = false;
  for (int c = 0; c < d.nout; c++) any |= d.ow[c] != 4 && d.ow[c] != 8;
  if (any) {
    int gpc = 3;
    if (const char *e = Knob("MBX_CP_BLOCKS_PER_CU")) gpc = atoi(e) > 0 ? atoi(e) : 3;
    int grid = NumCUs() * gpc;
    const int64_t need = (nrows >> 8) / 4 + 1;
    if (grid > need) grid = (int)need;
    CompactAny(d, nrows, bits, step_offsets, grid, s);
    return;
  }
  int nld = 0;
  for (int c = 0; c < d.nout; c++) nld += d.ow[c] / 4;
  if (nld > 8) throw std::runtime_error("CompactColumns: more than 8 KiB of outputs per step");
  int gpc = 3;
  if (const char *e = Knob("MBX_CP_BLOCKS_PER_CU")) gpc = atoi(e) > 0 ? atoi(e) : 3;
  int grid = NumCUs() * gpc;
  const int64_t need = (nrows >> 8) / 4 + 1;
  if (grid > need) grid = (int)need;
  int dp = 0;  // MBX_CP_DEPTH: ring depth override (sweeps)
  if (const char *e = Knob("MBX_CP_DEPTH")) dp = atoi(e);
#define CP(L, DP)                                                                                              \
  hipLaunchKernelGGL((compact_lds_kernel<L, DP>), dim3(grid), dim3(256), (size_t)4 * DP * (L * 1024 + 64) + 4 * 2048, s, d, \
                     nrows, bits, step_offsets)
#define CPD(L, DEF) \
  if ((dp ? dp : DEF) <= 2) CP(L, 2); else if ((dp ? dp : DEF) <= 3) CP(L, 3); else if ((dp ? dp : DEF) <= 4) CP(L, 4); else CP(L, 6);
  switch (nld) {
    case 1: CPD(1, 6); break;
    case 2: CPD(2, 3); break;
    case 3: CPD(3, 2); break;
    case 4: CPD(4, 2); break;
    case 5: CP(5, 2); break;
    case 6: CP(6, 2); break;
    case 7: CP(7, 2); break;
    default: CP(8, 2); break;
  }
#undef CPD
#undef CP
  CHECK_LAUNCH();
}

}  // namespace dev
}  // namespace mbx
