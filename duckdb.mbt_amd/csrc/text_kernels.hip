// text_kernels.hip — result values as text on the device, in the reference
// shim's string wire layout ([s0 \0 s1 \0 ...], a NULL is an empty string;
// /root/reference/src/duckdb_native.c:2456-2514 and :2687-2797), for the
// Arrow string getters of integer / BOOLEAN / DECIMAL / HUGEINT columns
// (the reference maps DECIMAL and HUGEINT to "string": :2336-2338).
//
// Two passes over the column: each row's text length (+1 for the NUL) -> an
// exclusive scan gives every row's offset -> each row writes its text there.
// The spelling is HostColumn::FormatInto's (format.cpp): [-]digits for
// integers, [-]int.frac with the fraction zero-padded to the scale for
// DECIMAL, true/false for BOOLEAN.  Magnitudes below 2^64 use a two-digit
// table; above, the value is split by 10^19 with a 128/64 long division.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device.h"
#include "vm_device.h"

namespace mbx {
namespace dev {

namespace {

__constant__ char kDigits2[201] =
    "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
    "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
    "8081828384858687888990919293949596979899";

// digits of u written backwards ending at `end`; returns the count (>= 1)
__device__ __forceinline__ int u64_back(uint64_t u, char *end) {
  char *p = end;
  while (u >= 100) {
    const uint64_t q = u / 100;
    const int r = (int)(u - q * 100);
    *--p = kDigits2[2 * r + 1];
    *--p = kDigits2[2 * r];
    u = q;
  }
  if (u >= 10) {
    *--p = kDigits2[2 * u + 1];
    *--p = kDigits2[2 * u];
  } else {
    *--p = (char)('0' + u);
  }
  return (int)(end - p);
}

// u / d for a u128 u and a 64-bit d, remainder in *rem (shift-subtract; only
// reached for |values| >= 2^64)
__device__ u128 divmod_u128(u128 u, uint64_t d, uint64_t *rem) {
  u128 q = 0, r = 0;
  for (int b = 127; b >= 0; b--) {
    r = (r << 1) | (uint64_t)((u >> b) & 1);
    if (r >= d) {
      r -= d;
      q |= (u128)1 << b;
    }
  }
  *rem = (uint64_t)r;
  return q;
}

// the text of row `row` into out (>= 48 bytes); its length (0 for NULL)
__device__ int format_row(const TextCol &C, int64_t row, char *out) {
  if (!bit_valid(C.valid, row)) return 0;
  int64_t lo, hi;
  load_phys(C.data, C.phys, row, lo, hi);
  if (C.kind == TEXT_BOOL) {
    if (lo) {
      out[0] = 't'; out[1] = 'r'; out[2] = 'u'; out[3] = 'e';
      return 4;
    }
    out[0] = 'f'; out[1] = 'a'; out[2] = 'l'; out[3] = 's'; out[4] = 'e';
    return 5;
  }
  const i128 x = (i128)(((u128)(uint64_t)hi << 64) | (uint64_t)lo);
  const bool neg = x < 0;
  u128 u = neg ? (u128)0 - (u128)x : (u128)x;
  char dig[48];
  char *end = dig + sizeof(dig), *p = end;
  while (u >> 64) {
    uint64_t r;
    u = divmod_u128(u, 10000000000000000000ull, &r);
    int k = u64_back(r, p);
    p -= k;
    for (; k < 19; k++) *--p = '0';
  }
  p -= u64_back((uint64_t)u, p);
  const int nd = (int)(end - p);
  int o = 0;
  if (neg) out[o++] = '-';
  const int scale = C.kind == TEXT_DECIMAL ? C.scale : 0;
  if (scale == 0) {
    for (int i = 0; i < nd; i++) out[o++] = p[i];
  } else if (nd <= scale) {
    out[o++] = '0';
    out[o++] = '.';
    for (int i = nd; i < scale; i++) out[o++] = '0';
    for (int i = 0; i < nd; i++) out[o++] = p[i];
  } else {
    for (int i = 0; i < nd - scale; i++) out[o++] = p[i];
    out[o++] = '.';
    for (int i = nd - scale; i < nd; i++) out[o++] = p[i];
  }
  return o;
}

__global__ __launch_bounds__(256) void text_lengths_kernel(TextCol C, int64_t n, uint32_t *lens) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    char buf[48];
    lens[i] = (uint32_t)format_row(C, i, buf) + 1;
  }
}

__global__ __launch_bounds__(256) void text_write_kernel(TextCol C, int64_t n, const int64_t *offs, char *chars,
                                                         uint8_t *vbytes) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    char buf[48];
    const int k = format_row(C, i, buf);
    char *dst = chars + offs[i];
    for (int j = 0; j < k; j++) dst[j] = buf[j];
    dst[k] = '\0';
    if (vbytes) vbytes[i] = (uint8_t)bit_valid(C.valid, i);
  }
}

// a text column's int64 offsets (the exclusive scan, n + 1 entries) as the
// host's 32-bit ones (the caller checked the total fits)
__global__ __launch_bounds__(256) void offsets_u32_kernel(const int64_t *__restrict__ o, uint32_t *__restrict__ out,
                                                         int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)o[i];
}

}  // namespace

void OffsetsU32(const int64_t *offsets, uint32_t *out, int64_t m, hipStream_t s) {
  if (m <= 0) return;
  int64_t blocks = (m + 255) / 256;
  if (blocks > (int64_t)NumCUs() * 16) blocks = (int64_t)NumCUs() * 16;
  hipLaunchKernelGGL(offsets_u32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, offsets, out, m);
  (void)hipGetLastError();
}

void TextLengths(const TextCol &c, int64_t n, uint32_t *lens, hipStream_t s) {
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > (int64_t)NumCUs() * 16) blocks = (int64_t)NumCUs() * 16;
  hipLaunchKernelGGL(text_lengths_kernel, dim3((unsigned)blocks), dim3(256), 0, s, c, n, lens);
  (void)hipGetLastError();
}

void TextWrite(const TextCol &c, int64_t n, const int64_t *offsets, char *chars, uint8_t *vbytes, hipStream_t s) {
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > (int64_t)NumCUs() * 16) blocks = (int64_t)NumCUs() * 16;
  hipLaunchKernelGGL(text_write_kernel, dim3((unsigned)blocks), dim3(256), 0, s, c, n, offsets, chars, vbytes);
  (void)hipGetLastError();
}

}  // namespace dev
}  // namespace mbx
