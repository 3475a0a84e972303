// hbm_probe.hip — research microbenchmark (not part of the product): read
// bandwidth of several streaming strategies on one MI355X, best of N.
//   hipcc --offload-arch=gfx950 -O3 -o hbm_probe tools/hbm_probe.hip && ./hbm_probe [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef long long v2i64 __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void reg_read(const v2i64 *__restrict__ in, long long n, unsigned long long *out) {
  long long acc = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    v2i64 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(in + i + u * stride) : in[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; u++) acc += v[u].x ^ v[u].y;
  }
  for (; i < n; i += stride) acc += in[i].x;
  if (acc == 0x5a5a5a5a5a5aLL) atomicAdd(out, 1ull);
}

// contiguous slice per workgroup, U loads in flight per lane
template <int U, bool NT>
__global__ __launch_bounds__(256) void reg_read_chunk(const v2i64 *__restrict__ in, long long n, unsigned long long *out) {
  long long acc = 0;
  long long per = (n + gridDim.x - 1) / gridDim.x;
  long long b = (long long)blockIdx.x * per, e = b + per < n ? b + per : n;
  long long i = b + threadIdx.x;
  for (; i + (U - 1) * 256 < e; i += U * 256) {
    v2i64 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(in + i + u * 256) : in[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; u++) acc += v[u].x ^ v[u].y;
  }
  for (; i < e; i += 256) acc += in[i].x;
  if (acc == 0x5a5a5a5a5a5aLL) atomicAdd(out, 1ull);
}

// LDS-DMA stream: each wave owns DEPTH 1-KiB slots; a piece = 64 lanes x 16 B.
template <int DEPTH, int AUX>
__global__ __launch_bounds__(256) void lds_dma_read(const v2i64 *__restrict__ in, long long npieces,
                                                    unsigned long long *out) {
  __shared__ __attribute__((aligned(16))) v2i64 lds[4 * DEPTH * 64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * 4;
  long long p = (long long)blockIdx.x * 4 + w;  // this wave's first piece; stride nw
  v2i64 *slot0 = lds + w * DEPTH * 64;
  long long acc = 0;
  int issued = 0;
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    long long q = p + d * nw;
    if (q < npieces) {
      __builtin_amdgcn_global_load_lds((const void *)(in + q * 64 + lane), (void *)(slot0 + d * 64), 16, 0, AUX);
      issued++;
    }
  }
  int k = 0;
  for (; p < npieces; p += nw) {
    // oldest piece (slot k) has landed once at most DEPTH-1 newer ones are pending
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH - 1) : "memory");
    v2i64 v = slot0[k * 64 + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long q = p + DEPTH * nw;
    if (q < npieces) {
      __builtin_amdgcn_global_load_lds((const void *)(in + q * 64 + lane), (void *)(slot0 + k * 64), 16, 0, AUX);
    } else {
      // keep the counted wait valid: an empty slot of the ring issues a dummy load of piece p (already read)
      __builtin_amdgcn_global_load_lds((const void *)(in + p * 64 + lane), (void *)(slot0 + k * 64), 16, 0, AUX);
    }
    acc += v.x ^ v.y;
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x5a5a5a5a5a5aLL) atomicAdd(out, 1ull);
}

// Like lds_dma_read, but each ring step of a wave covers PPS contiguous pieces.
template <int DEPTH, int PPS>
__global__ __launch_bounds__(256) void lds_dma_read_pps(const v2i64 *__restrict__ in, long long npieces,
                                                        unsigned long long *out) {
  __shared__ __attribute__((aligned(16))) v2i64 lds[4 * DEPTH * PPS * 64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long nsteps = npieces / PPS;
  const long long nw = (long long)gridDim.x * 4;
  long long p = (long long)blockIdx.x * 4 + w;
  v2i64 *slot0 = lds + w * DEPTH * PPS * 64;
  long long acc = 0;
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    long long q = p + d * nw;
    q = q < nsteps ? q : 0;
#pragma unroll
    for (int j = 0; j < PPS; j++)
      __builtin_amdgcn_global_load_lds((const void *)(in + (q * PPS + j) * 64 + lane), (void *)(slot0 + (d * PPS + j) * 64), 16, 0, 2);
  }
  int k = 0;
  for (; p < nsteps; p += nw) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DEPTH - 1) * PPS) : "memory");
    v2i64 v[PPS];
#pragma unroll
    for (int j = 0; j < PPS; j++) v[j] = slot0[(k * PPS + j) * 64 + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long q = p + DEPTH * nw;
    q = q < nsteps ? q : p;
#pragma unroll
    for (int j = 0; j < PPS; j++)
      __builtin_amdgcn_global_load_lds((const void *)(in + (q * PPS + j) * 64 + lane), (void *)(slot0 + (k * PPS + j) * 64), 16, 0, 2);
#pragma unroll
    for (int j = 0; j < PPS; j++) acc += v[j].x ^ v[j].y;
    k = k + 1 == DEPTH ? 0 : k + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x5a5a5a5a5a5aLL) atomicAdd(out, 1ull);
}

#define CHK(x) do { hipError_t e_ = (x); if (e_) { printf("HIP error %s at %s\n", hipGetErrorString(e_), #x); exit(1); } } while (0)

__global__ void fill_random(long long *p, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned long long z = (unsigned long long)i * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    p[i] = (long long)((z ^ (z >> 31)) % 50 + 1);
  }
}

int main(int argc, char **argv) {
  double gib = argc > 1 ? atof(argv[1]) : 8.0;
  int mode = argc > 2 ? atoi(argv[2]) : 0;  // bit0: random fill, bit1: hipMallocAsync, bit2: quick set only
  size_t alloc_bytes = (size_t)(gib * (1ull << 30)) & ~(size_t)1023;
  // optional 3rd arg: bytes actually read (default: the whole allocation)
  size_t bytes = argc > 3 ? ((size_t)atof(argv[3]) & ~(size_t)1023) : alloc_bytes;
  long long n16 = bytes / 16, npieces = bytes / 1024;
  void *buf;
  unsigned long long *flag;
  if (mode & 2) {
    CHK(hipMallocAsync(&buf, alloc_bytes, 0));
    CHK(hipStreamSynchronize(0));
  } else {
    CHK(hipMalloc(&buf, alloc_bytes));
  }
  CHK(hipMalloc(&flag, 8));
  if (mode & 1)
    hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (long long *)buf, (long long)(alloc_bytes / 8));
  else
    CHK(hipMemset(buf, 1, alloc_bytes));
  CHK(hipDeviceSynchronize());
  printf("== alloc %.2f GiB read %zu B mode %d\n", gib, bytes, mode);
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  auto run = [&](const char *name, auto launch) {
    float best = 1e30f, sum = 0;
    int iters = 20;
    std::vector<float> all;
    for (int it = 0; it < iters + 2; it++) {
      CHK(hipEventRecord(a));
      launch();
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (it >= 2) {
        all.push_back(ms);
        best = ms < best ? ms : best;
        sum += ms;
      }
    }
    std::sort(all.begin(), all.end());
    float med = all[all.size() / 2];
    printf("%-28s best %7.3f ms %7.1f GB/s   mean %7.1f GB/s  median %7.1f GB/s\n", name, best,
           bytes / (best * 1e-3) / 1e9, bytes / (sum / iters * 1e-3) / 1e9, bytes / (med * 1e-3) / 1e9);
    fflush(stdout);
  };
  const v2i64 *in = (const v2i64 *)buf;
  if (mode & 8) {
#define PPSRUN(D, P, G)                                                                                     \
  run("ldsdma d" #D " pps" #P " g" #G, [&] {                                                                \
    hipLaunchKernelGGL((lds_dma_read_pps<D, P>), dim3(cus * G), dim3(256), 0, 0, in, npieces, flag);       \
  })
    PPSRUN(8, 1, 1); PPSRUN(4, 2, 1); PPSRUN(8, 2, 1); PPSRUN(4, 4, 1); PPSRUN(2, 4, 1); PPSRUN(16, 1, 1);
    PPSRUN(2, 8, 1); PPSRUN(6, 1, 1); PPSRUN(12, 1, 1); PPSRUN(3, 2, 2); PPSRUN(4, 1, 2);
    PPSRUN(8, 1, 1);
    return 0;
  }
  if (mode & 4) {
    for (int g : {4, 8}) {
      char nm[64];
      snprintf(nm, 64, "reg u8 nt ch g%d", g);
      run(nm, [&] { hipLaunchKernelGGL((reg_read_chunk<8, true>), dim3(cus * g), dim3(256), 0, 0, in, n16, flag); });
      snprintf(nm, 64, "reg u4 nt gs g%d", g);
      run(nm, [&] { hipLaunchKernelGGL((reg_read<4, true>), dim3(cus * g), dim3(256), 0, 0, in, n16, flag); });
      snprintf(nm, 64, "ldsdma d8 nt g%d", g / 4);
      run(nm, [&] { hipLaunchKernelGGL((lds_dma_read<8, 2>), dim3(cus * g / 4), dim3(256), 0, 0, in, npieces, flag); });
    }
    return 0;
  }
  for (int g : {4, 8, 16}) {
    char nm[64];
    snprintf(nm, 64, "reg u4 nt gs g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((reg_read<4, true>), dim3(cus * g), dim3(256), 0, 0, in, n16, flag); });
    snprintf(nm, 64, "reg u8 nt gs g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((reg_read<8, true>), dim3(cus * g), dim3(256), 0, 0, in, n16, flag); });
    snprintf(nm, 64, "reg u4 pl gs g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((reg_read<4, false>), dim3(cus * g), dim3(256), 0, 0, in, n16, flag); });
    snprintf(nm, 64, "reg u8 pl ch g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((reg_read_chunk<8, false>), dim3(cus * g), dim3(256), 0, 0, in, n16, flag); });
    snprintf(nm, 64, "reg u8 nt ch g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((reg_read_chunk<8, true>), dim3(cus * g), dim3(256), 0, 0, in, n16, flag); });
    snprintf(nm, 64, "reg u16 pl ch g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((reg_read_chunk<16, false>), dim3(cus * g), dim3(256), 0, 0, in, n16, flag); });
  }
  for (int g : {1, 2, 4, 8}) {
    char nm[64];
    snprintf(nm, 64, "ldsdma d8 default g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((lds_dma_read<8, 0>), dim3(cus * g), dim3(256), 0, 0, in, npieces, flag); });
    snprintf(nm, 64, "ldsdma d8 nt g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((lds_dma_read<8, 2>), dim3(cus * g), dim3(256), 0, 0, in, npieces, flag); });
    snprintf(nm, 64, "ldsdma d16 nt g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((lds_dma_read<16, 2>), dim3(cus * g), dim3(256), 0, 0, in, npieces, flag); });
    snprintf(nm, 64, "ldsdma d4 nt g%d", g);
    run(nm, [&] { hipLaunchKernelGGL((lds_dma_read<4, 2>), dim3(cus * g), dim3(256), 0, 0, in, npieces, flag); });
  }
  return 0;
}
