// c3_probe.hip — research microbenchmark (not part of the product): what
// bounds the C3 GROUP BY kernel's read pattern?  Streams a 4-B key column and
// an 8-B value column (1e9 rows) through a per-wave LDS-DMA ring, the shape
// group_direct_lds uses (one 256-row step = 1 KiB key + 2 KiB value), with
//   work 0: no compute (pure two-array stream),
//   work 1: + the LDS table atomics (u32 count + u64 sum per row, R = 64),
//   work 2: + the packed atomic only (u64 per row),
// and a single-array stream of the same bytes for comparison.
//   hipcc --offload-arch=gfx950 -O3 -o c3_probe tools/c3_probe.hip && ./c3_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef int v4i32 __attribute__((ext_vector_type(4)));
typedef long long v2i64 __attribute__((ext_vector_type(2)));

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <int DEPTH, int WORK>
__global__ __launch_bounds__(256) void two_stream(const int *__restrict__ keys, const long long *__restrict__ vals,
                                                  long long nsteps, unsigned long long *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr int SB = 3072, R = 64, NK = 32;
  unsigned int *cnt = (unsigned int *)lds;                      // NK*R*4 = 8 KiB
  unsigned long long *sum = (unsigned long long *)(lds + 8192);  // NK*R*8 = 16 KiB
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  unsigned char *ring = lds + 24576 + w * DEPTH * SB;
  for (int i = t; i < NK * R; i += 256) { cnt[i] = 0; sum[i] = 0; }
  __syncthreads();
  const long long nw = (long long)gridDim.x * 4;
  long long st = (long long)blockIdx.x * 4 + w;
  auto issue = [&](long long q, int d) {
    unsigned char *dst = ring + d * SB;
    const unsigned char *kp = (const unsigned char *)keys + q * 1024;
    const unsigned char *vp = (const unsigned char *)vals + q * 2048;
    __builtin_amdgcn_global_load_lds((const void *)(kp + lane * 16), (void *)dst, 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(vp + lane * 16), (void *)(dst + 1024), 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(vp + 1024 + lane * 16), (void *)(dst + 2048), 16, 0, 2);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    long long q = st + d * nw;
    issue(q < nsteps ? q : 0, d);
  }
  long long acc = 0;
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * SB;
    v4i32 kv = *(const v4i32 *)(src + lane * 16);
    v2i64 a0 = *(const v2i64 *)(src + 1024 + lane * 32), a1 = *(const v2i64 *)(src + 1024 + lane * 32 + 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    int kk[4] = {kv.x & 31, kv.y & 31, kv.z & 31, kv.w & 31};
    long long a[4] = {a0.x, a0.y, a1.x, a1.y};
    if (WORK == 0) {
      acc += kk[0] + kk[1] + kk[2] + kk[3] + a[0] + a[1] + a[2] + a[3];
    } else {
#pragma unroll
      for (int e = 0; e < 4; e++) {
        int sl = kk[e] * R + lane;
        if (WORK == 1) {
          atomicAdd(&cnt[sl], 1u);
          atomicAdd(&sum[sl], (unsigned long long)a[e]);
        } else {
          atomicAdd(&sum[sl], ((unsigned long long)a[e] << 12) + 1ull);
        }
      }
    }
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (WORK) acc += cnt[t] + sum[t];
  if (acc == 0x5a5a5a5a5a5aLL) atomicAdd(out, 1ull);
}

// pure two-array stream with WAVES waves per block and cache policy AUX on the
// LDS-DMA loads (2 = nt, 0 = default); round 2: is there a faster stream shape?
template <int DEPTH, int WAVES, int AUX>
__global__ __launch_bounds__(WAVES * 64) void two_stream_w(const int *__restrict__ keys, const long long *__restrict__ vals,
                                                          long long nsteps, unsigned long long *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr int SB = 3072;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  unsigned char *ring = lds + w * DEPTH * SB;
  const long long nw = (long long)gridDim.x * WAVES;
  long long st = (long long)blockIdx.x * WAVES + w;
  auto issue = [&](long long q, int d) {
    unsigned char *dst = ring + d * SB;
    const unsigned char *kp = (const unsigned char *)keys + q * 1024;
    const unsigned char *vp = (const unsigned char *)vals + q * 2048;
    __builtin_amdgcn_global_load_lds((const void *)(kp + lane * 16), (void *)dst, 16, 0, AUX);
    __builtin_amdgcn_global_load_lds((const void *)(vp + lane * 16), (void *)(dst + 1024), 16, 0, AUX);
    __builtin_amdgcn_global_load_lds((const void *)(vp + 1024 + lane * 16), (void *)(dst + 2048), 16, 0, AUX);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    long long q = st + d * nw;
    issue(q < nsteps ? q : 0, d);
  }
  long long acc = 0;
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * SB;
    v4i32 kv = *(const v4i32 *)(src + lane * 16);
    v2i64 a0 = *(const v2i64 *)(src + 1024 + lane * 32);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    acc += kv.x + a0.x;
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x5a5a5a5a5a5aLL) atomicAdd(out, 1ull);
}

// pure three-array stream of filter_multi's shape (x int64 2 KiB + k int32 1 KiB
// + v int64 2 KiB per 256-row step): the ceiling for that kernel
template <int DEPTH, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void three_stream_w(const long long *__restrict__ xs, const int *__restrict__ keys,
                                                            const long long *__restrict__ vals, long long nsteps,
                                                            unsigned long long *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr int SB = 5120;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  unsigned char *ring = lds + w * DEPTH * SB;
  const long long nw = (long long)gridDim.x * WAVES;
  long long st = (long long)blockIdx.x * WAVES + w;
  auto issue = [&](long long q, int d) {
    unsigned char *dst = ring + d * SB;
    const unsigned char *xp = (const unsigned char *)xs + q * 2048;
    const unsigned char *kp = (const unsigned char *)keys + q * 1024;
    const unsigned char *vp = (const unsigned char *)vals + q * 2048;
    __builtin_amdgcn_global_load_lds((const void *)(xp + lane * 16), (void *)dst, 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(xp + 1024 + lane * 16), (void *)(dst + 1024), 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(kp + lane * 16), (void *)(dst + 2048), 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(vp + lane * 16), (void *)(dst + 3072), 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(vp + 1024 + lane * 16), (void *)(dst + 4096), 16, 0, 2);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    long long q = st + d * nw;
    issue(q < nsteps ? q : 0, d);
  }
  long long acc = 0;
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * SB;
    v2i64 a0 = *(const v2i64 *)(src + lane * 32);
    v4i32 kv = *(const v4i32 *)(src + 2048 + lane * 16);
    v2i64 b0 = *(const v2i64 *)(src + 3072 + lane * 32);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    acc += a0.x + kv.x + b0.x;
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x5a5a5a5a5a5aLL) atomicAdd(out, 1ull);
}

// the same bytes as ONE array: 3 KiB contiguous per step
template <int DEPTH>
__global__ __launch_bounds__(256) void one_stream(const unsigned char *__restrict__ in, long long nsteps,
                                                  unsigned long long *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr int SB = 3072;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  unsigned char *ring = lds + w * DEPTH * SB;
  const long long nw = (long long)gridDim.x * 4;
  long long st = (long long)blockIdx.x * 4 + w;
  auto issue = [&](long long q, int d) {
    unsigned char *dst = ring + d * SB;
    const unsigned char *p = in + q * 3072;
#pragma unroll
    for (int j = 0; j < 3; j++)
      __builtin_amdgcn_global_load_lds((const void *)(p + j * 1024 + lane * 16), (void *)(dst + j * 1024), 16, 0, 2);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    long long q = st + d * nw;
    issue(q < nsteps ? q : 0, d);
  }
  long long acc = 0;
  int k = 0;
  for (; st < nsteps; st += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
    const unsigned char *src = ring + k * SB;
    v4i32 x = *(const v4i32 *)(src + lane * 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long q = st + DEPTH * nw;
    issue(q < nsteps ? q : st, k);
    acc += x.x + x.y;
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x5a5a5a5a5a5aLL) atomicAdd(out, 1ull);
}

// software-pipelined form: the next slot's ds_reads are issued BEFORE this
// step's table atomics, so the counted lgkmcnt wait before the refill waits
// for the reads only (LDS ops retire in order), never for the atomics.
template <int DEPTH, bool PACKED>
__global__ __launch_bounds__(256) void two_stream_pipe(const int *__restrict__ keys, const long long *__restrict__ vals,
                                                       long long nsteps, unsigned long long *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr int SB = 3072, R = 64, NK = 32;
  constexpr int NAT = PACKED ? 4 : 8;
  unsigned int *cnt = (unsigned int *)lds;
  unsigned long long *sum = (unsigned long long *)(lds + 8192);
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  unsigned char *ring = lds + 24576 + w * DEPTH * SB;
  for (int i = t; i < NK * R; i += 256) { cnt[i] = 0; sum[i] = 0; }
  __syncthreads();
  const long long nw = (long long)gridDim.x * 4;
  long long st = (long long)blockIdx.x * 4 + w;
  auto issue = [&](long long q, int d) {
    unsigned char *dst = ring + d * SB;
    const unsigned char *kp = (const unsigned char *)keys + q * 1024;
    const unsigned char *vp = (const unsigned char *)vals + q * 2048;
    __builtin_amdgcn_global_load_lds((const void *)(kp + lane * 16), (void *)dst, 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(vp + lane * 16), (void *)(dst + 1024), 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(vp + 1024 + lane * 16), (void *)(dst + 2048), 16, 0, 2);
  };
  if (st >= nsteps) return;
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    long long q = st + d * nw;
    issue(q < nsteps ? q : 0, d);
  }
  v4i32 kv;
  v2i64 a0, a1;
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
  kv = *(const v4i32 *)(ring + lane * 16);
  a0 = *(const v2i64 *)(ring + 1024 + lane * 32);
  a1 = *(const v2i64 *)(ring + 1024 + lane * 32 + 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  issue(st + DEPTH * nw < nsteps ? st + DEPTH * nw : st, 0);
  int k = 0;
  for (;;) {
    const long long nx = st + nw;
    const int k1 = k + 1 == DEPTH ? 0 : k + 1;
    v4i32 nkv;
    v2i64 na0, na1;
    if (nx < nsteps) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
      const unsigned char *src = ring + k1 * SB;
      nkv = *(const v4i32 *)(src + lane * 16);
      na0 = *(const v2i64 *)(src + 1024 + lane * 32);
      na1 = *(const v2i64 *)(src + 1024 + lane * 32 + 16);
    }
    int kk[4] = {kv.x & 31, kv.y & 31, kv.z & 31, kv.w & 31};
    long long a[4] = {a0.x, a0.y, a1.x, a1.y};
#pragma unroll
    for (int e = 0; e < 4; e++) {
      int sl = kk[e] * R + lane;
      if (PACKED) {
        atomicAdd(&sum[sl], ((unsigned long long)a[e] << 12) + 1ull);
      } else {
        atomicAdd(&cnt[sl], 1u);
        atomicAdd(&sum[sl], (unsigned long long)a[e]);
      }
    }
    if (nx >= nsteps) break;
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NAT) : "memory");
    const long long q = nx + DEPTH * nw;
    issue(q < nsteps ? q : nx, k1);
    kv = nkv; a0 = na0; a1 = na1;
    st = nx;
    k = k1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  long long acc = cnt[t] + sum[t];
  if (acc == 0x5a5a5a5a5a5aLL) atomicAdd(out, 1ull);
}

// loader/consumer split: 4 loader waves stream (the fast 4-wave shape) into
// per-loader rings; NC consumer waves (NC/4 per loader, alternating steps) do
// the table atomics.  LDS flags: full[w][d] = step+1 once landed, done[w][d] =
// step+1 once consumed.  Every spin is bounded (a broken handshake ends, wrong,
// instead of hanging).
template <int DEPTH, int NC>
__global__ __launch_bounds__(256 + 64 * NC) void two_stream_lc(const int *__restrict__ keys,
                                                               const long long *__restrict__ vals, long long nsteps,
                                                               unsigned long long *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr int SB = 3072, R = 64, NK = 32, CPL = NC / 4;
  unsigned int *cnt = (unsigned int *)lds;
  unsigned long long *sum = (unsigned long long *)(lds + 8192);
  volatile int *full = (volatile int *)(lds + 24576);        // [4][DEPTH]
  volatile int *done = (volatile int *)(lds + 24576 + 256);  // [4][DEPTH]
  unsigned char *rings = lds + 24576 + 512;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  for (int i = t; i < NK * R; i += blockDim.x) { cnt[i] = 0; sum[i] = 0; }
  if (t < 4 * DEPTH) { full[t] = 0; done[t] = 0; }
  __syncthreads();
  const long long nw = (long long)gridDim.x * 4;
  int bad = 0;
  if (wave < 4) {  // loader
    const int w = wave;
    unsigned char *ring = rings + w * DEPTH * SB;
    auto issue = [&](long long q, int d) {
      unsigned char *dst = ring + d * SB;
      const unsigned char *kp = (const unsigned char *)keys + q * 1024;
      const unsigned char *vp = (const unsigned char *)vals + q * 2048;
      __builtin_amdgcn_global_load_lds((const void *)(kp + lane * 16), (void *)dst, 16, 0, 2);
      __builtin_amdgcn_global_load_lds((const void *)(vp + lane * 16), (void *)(dst + 1024), 16, 0, 2);
      __builtin_amdgcn_global_load_lds((const void *)(vp + 1024 + lane * 16), (void *)(dst + 2048), 16, 0, 2);
    };
    long long nmine = 0;
    for (long long st = (long long)blockIdx.x * 4 + w; st < nsteps; st += nw) nmine++;
    for (long long j = 0; j < nmine + DEPTH - 1; j++) {
      if (j < nmine) {
        const int d = (int)(j % DEPTH);
        if (j >= DEPTH) {  // the slot's previous step must be consumed
          int sp = 0;
          while (done[w * DEPTH + d] < (int)(j - DEPTH + 1)) {
            __builtin_amdgcn_s_sleep(1);
            if (++sp > (1 << 22)) { bad = 1; break; }
          }
        }
        issue((long long)blockIdx.x * 4 + w + j * nw, d);
      }
      // publish the oldest in-flight step once it has landed
      const long long pj = j - (DEPTH - 1);
      if (pj >= 0) {
        if (j < nmine) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) full[w * DEPTH + (int)(pj % DEPTH)] = (int)(pj + 1);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {  // consumer
    const int c = wave - 4, w = c % 4, phase = c / 4;
    const unsigned char *ring = rings + w * DEPTH * SB;
    long long nmine = 0;
    for (long long st = (long long)blockIdx.x * 4 + w; st < nsteps; st += nw) nmine++;
    for (long long j = phase; j < nmine; j += CPL) {
      const int d = (int)(j % DEPTH);
      int sp = 0;
      while (full[w * DEPTH + d] < (int)(j + 1)) {
        __builtin_amdgcn_s_sleep(1);
        if (++sp > (1 << 22)) { bad = 1; break; }
      }
      const unsigned char *src = ring + d * SB;
      v4i32 kv = *(const v4i32 *)(src + lane * 16);
      v2i64 a0 = *(const v2i64 *)(src + 1024 + lane * 32), a1 = *(const v2i64 *)(src + 1024 + lane * 32 + 16);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) done[w * DEPTH + d] = (int)(j + 1);
      int kk[4] = {kv.x & 31, kv.y & 31, kv.z & 31, kv.w & 31};
      long long a[4] = {a0.x, a0.y, a1.x, a1.y};
#pragma unroll
      for (int e = 0; e < 4; e++) {
        int sl = kk[e] * R + lane;
        atomicAdd(&sum[sl], ((unsigned long long)a[e] << 12) + 1ull);
      }
    }
  }
  __syncthreads();
  long long acc = cnt[t % 2048] + sum[t % 2048] + bad;
  if (acc == 0x5a5a5a5a5a5aLL || bad) atomicAdd(out, 1ull);
}

__global__ void fill_keys(int *k, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned long long z = (unsigned long long)i + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    k[i] = (int)((z ^ (z >> 31)) & 31);
  }
}

template <typename F>
static float TimeIt(F f, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int i = 0; i < iters; i++) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
  const long long n = argc > 1 ? atoll(argv[1]) : 1000000000LL;
  const long long nsteps = n / 256;
  int *k;
  long long *v;
  unsigned char *one;
  unsigned long long *out;
  CK(hipMalloc(&k, nsteps * 1024));
  CK(hipMalloc(&v, nsteps * 2048));
  CK(hipMalloc(&one, nsteps * 3072));
  CK(hipMalloc(&out, 8));
  hipLaunchKernelGGL(fill_keys, dim3(4096), dim3(256), 0, 0, k, nsteps * 256);
  CK(hipMemset(v, 2, nsteps * 2048));
  CK(hipMemset(one, 3, nsteps * 3072));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double bytes = (double)nsteps * 3072;
  auto report = [&](const char *name, int d, int g, float ms) {
    printf("%-12s d%d g%d  %.4f ms  %.0f GB/s\n", name, d, g, ms, bytes / ms / 1e6);
    fflush(stdout);
  };
#define RUN2(D, W, G)                                                                                         \
  {                                                                                                           \
    size_t lds = 24576 + 4 * (D) * 3072;                                                                      \
    CK(hipFuncSetAttribute((const void *)two_stream<D, W>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    float ms = TimeIt([&] { hipLaunchKernelGGL((two_stream<D, W>), dim3(cus * (G)), dim3(256), lds, 0, k, v, nsteps, out); }, 15); \
    report(W == 0 ? "two/none" : W == 1 ? "two/atom2" : "two/packed", D, G, ms);                              \
  }
#define RUN1(D, G)                                                                                            \
  {                                                                                                           \
    size_t lds = 4 * (D) * 3072;                                                                              \
    CK(hipFuncSetAttribute((const void *)one_stream<D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    float ms = TimeIt([&] { hipLaunchKernelGGL((one_stream<D>), dim3(cus * (G)), dim3(256), lds, 0, one, nsteps, out); }, 15); \
    report("one/none", D, G, ms);                                                                             \
  }
#define RUNP(D, P, G)                                                                                         \
  {                                                                                                           \
    size_t lds = 24576 + 4 * (D) * 3072;                                                                      \
    CK(hipFuncSetAttribute((const void *)two_stream_pipe<D, P>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    float ms = TimeIt([&] { hipLaunchKernelGGL((two_stream_pipe<D, P>), dim3(cus * (G)), dim3(256), lds, 0, k, v, nsteps, out); }, 15); \
    report(P ? "pipe/packed" : "pipe/atom2", D, G, ms);                                                      \
  }
#define RUNLC(D, NC)                                                                                          \
  {                                                                                                           \
    size_t lds = 24576 + 512 + 4 * (D) * 3072;                                                                \
    CK(hipFuncSetAttribute((const void *)two_stream_lc<D, NC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    CK(hipMemset(out, 0, 8));                                                                                 \
    float ms = TimeIt([&] { hipLaunchKernelGGL((two_stream_lc<D, NC>), dim3(cus), dim3(256 + 64 * (NC)), lds, 0, k, v, nsteps, out); }, 15); \
    unsigned long long flag = 0;                                                                              \
    CK(hipMemcpy(&flag, out, 8, hipMemcpyDeviceToHost));                                                      \
    printf("lc NC=%d ", NC);                                                                                  \
    report(flag ? "lc/BAD" : "lc/packed", D, 1, ms);                                                          \
  }
#define RUNW(D, W, A, G)                                                                                      \
  {                                                                                                           \
    size_t lds = (W) * (D) * 3072;                                                                            \
    CK(hipFuncSetAttribute((const void *)two_stream_w<D, W, A>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    float ms = TimeIt([&] { hipLaunchKernelGGL((two_stream_w<D, W, A>), dim3(cus * (G)), dim3((W) * 64), lds, 0, k, v, nsteps, out); }, 15); \
    printf("w%d aux%d ", W, A);                                                                               \
    report("two/none", D, G, ms);                                                                             \
  }
#define RUN3(D, W, G)                                                                                         \
  {                                                                                                           \
    size_t lds = (W) * (D) * 5120;                                                                            \
    CK(hipFuncSetAttribute((const void *)three_stream_w<D, W>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    float ms = TimeIt([&] { hipLaunchKernelGGL((three_stream_w<D, W>), dim3(cus * (G)), dim3((W) * 64), lds, 0, x3, k, v, nsteps, out); }, 15); \
    printf("three w%d d%d g%d  %.4f ms  %.0f GB/s\n", W, D, G, ms, 20e9 * ((double)nsteps * 256 / 1e9) / (ms * 1e6)); \
  }
  if (argc > 2 && argv[2][0] == '3') {  // round 2: the filter_multi shape (x i64, k i32, v i64)
    long long *x3;
    CK(hipMalloc((void **)&x3, (size_t)nsteps * 2048));
    CK(hipMemset(x3, 1, (size_t)nsteps * 2048));
    RUN3(2, 4, 1) RUN3(3, 4, 1) RUN3(4, 4, 1) RUN3(2, 4, 2) RUN3(3, 4, 2) RUN3(2, 4, 3) RUN3(3, 4, 3)
    RUN3(2, 8, 1) RUN3(3, 8, 1) RUN3(2, 4, 1) RUN3(2, 4, 3)
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'w') {  // round 2: waves per block and cache policy of the pure stream
    RUNW(2, 4, 2, 1) RUNW(2, 4, 0, 1) RUNW(3, 4, 2, 1) RUNW(2, 8, 2, 1) RUNW(2, 8, 0, 1) RUNW(3, 8, 2, 1)
    RUNW(4, 8, 2, 1) RUNW(2, 16, 2, 1) RUNW(2, 12, 2, 1) RUNW(2, 8, 2, 2) RUNW(2, 4, 2, 2) RUNW(2, 4, 2, 3)
    RUNW(2, 4, 2, 1) RUNW(2, 8, 2, 1)
    RUN1(2, 1) RUN1(6, 1)
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'o') {  // round 3: the value array's offset from the key array in one allocation
    unsigned char *big;
    const size_t kb = (size_t)nsteps * 1024, vb = (size_t)nsteps * 2048;
    CK(hipMalloc((void **)&big, kb + vb + ((size_t)64 << 20)));
    hipLaunchKernelGGL(fill_keys, dim3(4096), dim3(256), 0, 0, (int *)big, nsteps * 256);
    const size_t deltas[] = {0, 4096, 65536, 262144, 524288, 1 << 20, 1536 << 10, (2 << 20) + 65536, 3 << 20,
                             5 << 20, 17 << 20, 33 << 20, 0};
    for (size_t dv : deltas) {
      long long *vv = (long long *)(big + kb + dv);
      CK(hipMemset(vv, 2, vb));
      size_t lds = 24576 + 4 * 2 * 3072;
      CK(hipFuncSetAttribute((const void *)two_stream<2, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      float ms = TimeIt([&] { hipLaunchKernelGGL((two_stream<2, 0>), dim3(cus), dim3(256), lds, 0, (int *)big, vv, nsteps, out); }, 15);
      printf("delta %9zu  ", dv);
      report("two/none", 2, 1, ms);
    }
    // separate allocations, as the engine makes them
    RUN2(2, 0, 1)
    return 0;
  }
  if (argc > 2 && (argv[2][0] == 'c' || argv[2][0] == 'g')) {
    // round 5: GB-scale offsets of the value array from the key array inside
    // ONE allocation -- physically contiguous ('c', hipDeviceMallocContiguous)
    // or a plain hipMalloc ('g') -- each delta timed twice, interleaved
    unsigned char *big;
    const size_t kb = (size_t)nsteps * 1024, vb = (size_t)nsteps * 2048, slack = (size_t)4 << 30;
    if (argv[2][0] == 'c') CK(hipExtMallocWithFlags((void **)&big, kb + vb + slack, hipDeviceMallocContiguous));
    else CK(hipMalloc((void **)&big, kb + vb + slack));
    hipLaunchKernelGGL(fill_keys, dim3(4096), dim3(256), 0, 0, (int *)big, nsteps * 256);
    const size_t M = 1 << 20;
    const size_t deltas[] = {0, 4096, 64 << 10, 1 * M, 2 * M, 6 * M, 64 * M, 96 * M, 256 * M, 512 * M + 4 * M,
                             1024 * M, 1536 * M, 2048 * M, 3072 * M + 2 * M, 4095 * M};
    size_t lds = 24576 + 4 * 2 * 3072;
    CK(hipFuncSetAttribute((const void *)two_stream<2, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void *)two_stream<2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int rep = 0; rep < 2; rep++)
      for (size_t dv : deltas) {
        long long *vv = (long long *)(big + kb + dv);
        CK(hipMemset(vv, 2, vb));
        float ms = TimeIt([&] { hipLaunchKernelGGL((two_stream<2, 0>), dim3(cus), dim3(256), lds, 0, (int *)big, vv, nsteps, out); }, 9);
        float ma = TimeIt([&] { hipLaunchKernelGGL((two_stream<2, 1>), dim3(cus), dim3(256), lds, 0, (int *)big, vv, nsteps, out); }, 9);
        printf("%s rep %d delta_MiB %9.3f  stream %.4f ms  with_atomics %.4f ms  %.0f GB/s\n", argv[2][0] == 'c' ? "contig" : "malloc",
               rep, dv / (double)M, ms, ma, bytes / ms / 1e6);
        fflush(stdout);
      }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'r') {
    // round 5: separate allocations as the engine makes them, re-made 8 times
    // with a filler of varying size allocated first (placement varies)
    size_t lds = 24576 + 4 * 2 * 3072;
    CK(hipFuncSetAttribute((const void *)two_stream<2, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFree(k));
    CK(hipFree(v));
    CK(hipFree(one));
    for (int rep = 0; rep < 8; rep++) {
      void *fill = nullptr;
      const size_t fb = ((size_t)(rep * 3 % 8) << 30) + ((size_t)rep << 21);
      if (fb) CK(hipMalloc(&fill, fb));
      int *k2;
      long long *v2;
      if (rep & 1) {
        CK(hipMalloc(&v2, nsteps * 2048));
        CK(hipMalloc(&k2, nsteps * 1024));
      } else {
        CK(hipMalloc(&k2, nsteps * 1024));
        CK(hipMalloc(&v2, nsteps * 2048));
      }
      hipLaunchKernelGGL(fill_keys, dim3(4096), dim3(256), 0, 0, k2, nsteps * 256);
      CK(hipMemset(v2, 2, nsteps * 2048));
      float ms = TimeIt([&] { hipLaunchKernelGGL((two_stream<2, 0>), dim3(cus), dim3(256), lds, 0, k2, v2, nsteps, out); }, 9);
      printf("separate rep %d filler_GiB %.3f order %s  k %p v %p  stream %.4f ms  %.0f GB/s\n", rep, fb / 1073741824.0,
             rep & 1 ? "v,k" : "k,v", (void *)k2, (void *)v2, ms, bytes / ms / 1e6);
      fflush(stdout);
      CK(hipFree(k2));
      CK(hipFree(v2));
      if (fill) CK(hipFree(fill));
    }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'l') {
    RUNLC(4, 4) RUNLC(6, 4) RUNLC(4, 8) RUNLC(6, 8) RUNLC(8, 8) RUNLC(6, 12)
    RUN2(2, 0, 1) RUN2(2, 2, 3)
    return 0;
  }
  RUNP(3, false, 1) RUNP(4, false, 1) RUNP(6, false, 1) RUNP(3, true, 1) RUNP(4, true, 1) RUNP(6, true, 1)
  RUNP(3, false, 2) RUNP(3, true, 2) RUNP(2, false, 3) RUNP(2, true, 3)
  RUN2(2, 0, 1) RUN2(2, 1, 3) RUN2(2, 2, 3)
  RUN1(2, 1) RUN1(2, 2) RUN1(2, 3) RUN1(4, 1) RUN1(4, 2) RUN1(6, 1)
  RUN2(2, 0, 1) RUN2(2, 0, 2) RUN2(2, 0, 3) RUN2(4, 0, 1) RUN2(4, 0, 2) RUN2(6, 0, 1)
  RUN2(2, 1, 2) RUN2(2, 1, 3) RUN2(4, 1, 1) RUN2(4, 1, 2) RUN2(6, 1, 1)
  RUN2(2, 2, 2) RUN2(2, 2, 3) RUN2(4, 2, 1) RUN2(4, 2, 2) RUN2(6, 2, 1)
  return 0;
}
