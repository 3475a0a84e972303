// vm_device.h — device side of the expression VM: value helpers and the
// semantics of every VM instruction (vm_step).  Compiled twice: into
// kernels.hip, where the tile interpreter calls vm_step with the instruction
// read at run time and registers in LDS planes, and — as source text — into
// the run-time compiled expression kernels (jit.cpp), where every call has
// literal operands so the switch folds away and the registers live in VGPRs.
#pragma once
#include <stdint.h>

#include "phys.h"
#include "vm.h"

namespace mbx {
namespace dev {

typedef __int128 i128;
typedef unsigned __int128 u128;

__device__ __forceinline__ bool bit_valid(const uint64_t *v, int64_t row) {
  return v == nullptr || ((v[row >> 6] >> (row & 63)) & 1ull);
}

__device__ __forceinline__ void load_phys(const void *data, int phys, int64_t row, int64_t &lo, int64_t &hi) {
  switch (phys) {
    case P_U8: lo = ((const uint8_t *)data)[row]; hi = 0; break;
    case P_I8: lo = ((const int8_t *)data)[row]; hi = lo >> 63; break;
    case P_I16: lo = ((const int16_t *)data)[row]; hi = lo >> 63; break;
    case P_U16: lo = ((const uint16_t *)data)[row]; hi = 0; break;
    case P_I32: lo = ((const int32_t *)data)[row]; hi = lo >> 63; break;
    case P_U32: lo = ((const uint32_t *)data)[row]; hi = 0; break;
    case P_I64: lo = ((const int64_t *)data)[row]; hi = lo >> 63; break;
    case P_U64: lo = (int64_t)((const uint64_t *)data)[row]; hi = 0; break;
    case P_I128: {
      const int64_t *p = (const int64_t *)data + 2 * row;
      lo = p[0];
      hi = p[1];
      break;
    }
    case P_F32: {
      double d = ((const float *)data)[row];
      lo = __double_as_longlong(d);
      hi = 0;
      break;
    }
    case P_F64: lo = ((const int64_t *)data)[row]; hi = 0; break;
    default: lo = row; hi = 0; break;  // P_STR: the row index is the string code
  }
}

__device__ __forceinline__ void store_phys(void *data, int phys, int64_t row, int64_t lo, int64_t hi) {
  switch (phys) {
    case P_U8: ((uint8_t *)data)[row] = (uint8_t)lo; break;
    case P_I8: ((int8_t *)data)[row] = (int8_t)lo; break;
    case P_I16: ((int16_t *)data)[row] = (int16_t)lo; break;
    case P_U16: ((uint16_t *)data)[row] = (uint16_t)lo; break;
    case P_I32: ((int32_t *)data)[row] = (int32_t)lo; break;
    case P_U32: ((uint32_t *)data)[row] = (uint32_t)lo; break;
    case P_I64: case P_U64: case P_F64: case P_STR: ((int64_t *)data)[row] = lo; break;
    case P_I128: {
      int64_t *p = (int64_t *)data + 2 * row;
      p[0] = lo;
      p[1] = hi;
      break;
    }
    case P_F32: ((float *)data)[row] = (float)__longlong_as_double(lo); break;
    default: break;
  }
}

__device__ __forceinline__ i128 mk128(int64_t lo, int64_t hi) { return (i128)(((u128)(uint64_t)hi << 64) | (uint64_t)lo); }
__device__ __forceinline__ void sp128(i128 v, int64_t &lo, int64_t &hi) {
  lo = (int64_t)(uint64_t)(u128)v;
  hi = (int64_t)(uint64_t)((u128)v >> 64);
}

__device__ __forceinline__ bool add_ovf128(i128 a, i128 b, i128 &r) {
  r = (i128)((u128)a + (u128)b);
  return ((a ^ r) & (b ^ r)) < 0;
}
__device__ __forceinline__ bool sub_ovf128(i128 a, i128 b, i128 &r) {
  r = (i128)((u128)a - (u128)b);
  return ((a ^ b) & (a ^ r)) < 0;
}
__device__ __forceinline__ bool mul_ovf128(i128 a, i128 b, i128 &r) {
  bool neg = (a < 0) != (b < 0);
  u128 ua = a < 0 ? (u128)0 - (u128)a : (u128)a;
  u128 ub = b < 0 ? (u128)0 - (u128)b : (u128)b;
  uint64_t ah = (uint64_t)(ua >> 64), al = (uint64_t)ua, bh = (uint64_t)(ub >> 64), bl = (uint64_t)ub;
  if (ah && bh) return true;
  u128 lo = (u128)al * bl;
  u128 mid = (u128)ah * bl + (u128)al * bh;
  if (mid >> 64) return true;
  u128 res = lo + (mid << 64);
  if (res < lo) return true;
  u128 lim = neg ? ((u128)1 << 127) : (((u128)1 << 127) - 1);
  if (res > lim) return true;
  r = neg ? (i128)((u128)0 - res) : (i128)res;
  return false;
}
__device__ __forceinline__ u128 udiv128(u128 n, u128 d) {
  // shift-subtract division (rare path: HUGEINT / DECIMAL(>18) division)
  if (d == 0) return 0;
  if ((n >> 64) == 0 && (d >> 64) == 0) return (u128)((uint64_t)n / (uint64_t)d);
  u128 q = 0, r = 0;
  for (int i = 127; i >= 0; i--) {
    r = (r << 1) | ((n >> i) & 1);
    if (r >= d) {
      r -= d;
      q |= (u128)1 << i;
    }
  }
  return q;
}
__device__ __forceinline__ i128 sdiv128(i128 a, i128 b) {
  bool neg = (a < 0) != (b < 0);
  u128 ua = a < 0 ? (u128)0 - (u128)a : (u128)a;
  u128 ub = b < 0 ? (u128)0 - (u128)b : (u128)b;
  u128 q = udiv128(ua, ub);
  return neg ? (i128)((u128)0 - q) : (i128)q;
}
__device__ __forceinline__ i128 smod128(i128 a, i128 b) { return a - sdiv128(a, b) * b; }

__device__ __forceinline__ i128 pow10_128(int k) {
  i128 r = 1;
  for (int i = 0; i < k; i++) r *= 10;
  return r;
}
__device__ __forceinline__ int64_t pow10_64(int k) {
  int64_t r = 1;
  for (int i = 0; i < k; i++) r *= 10;
  return r;
}

// int128 -> double through the magnitude (no cancellation between the
// halves); exact rounding whenever |v| < 2^64.
__device__ __forceinline__ double u128_to_double(u128 m) {
  uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
  if (hi == 0) return (double)lo;
  return (double)hi * 18446744073709551616.0 + (double)lo;
}
__device__ __forceinline__ double i128_to_double(i128 v) {
  if (v < 0) return -u128_to_double((u128)0 - (u128)v);
  return u128_to_double((u128)v);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ void raise_err(int32_t *err, int32_t code) {
  if (err) atomicCAS(err, 0, code);
}

__device__ __forceinline__ uint64_t f64_order(double d) {
  uint64_t u = (uint64_t)__double_as_longlong(d);
  if (d != d) return 0xFFFFFFFFFFFFFFFFull;  // NaN sorts last
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double f64_unorder(uint64_t k) {
  uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)u);
}

__device__ __forceinline__ bool cmp_res(int c, int k) {
  // c = -1/0/1 comparison, k = cmp kind
  switch (k) {
    case 0: return c == 0;
    case 1: return c != 0;
    case 2: return c < 0;
    case 3: return c <= 0;
    case 4: return c > 0;
    default: return c >= 0;
  }
}

// One VM instruction for the calling thread's row.  RF is the register file:
// lo(i) / hi(i) / nl(i) return references to register i of this row.
// UNCOND (run-time compiled kernels): `row` is always a valid row index, so
// column loads are issued unconditionally (no branch between a row's loads)
// and `active` only masks validity and error reporting.
template <class RF, bool UNCOND = false>
__device__ __forceinline__ void vm_step(const VmProgram &P, const VmCols &C, int op, int d, int a, int b, int c,
                                        int aux, int64_t row, bool active, int64_t rs, int64_t rstep, RF &R,
                                        int32_t *err) {
    int64_t lo = 0, hi = 0;
    uint8_t nl = 0;
    switch (op) {
      case V_LOADCOL: {
        const VmCol &col = C.c[a];
        if (UNCOND) {
          nl = (active && bit_valid(col.validity, row)) ? 0 : 1;
          load_phys(col.data, col.phys, row, lo, hi);
        } else if (active) {
          nl = bit_valid(col.validity, row) ? 0 : 1;
          load_phys(col.data, col.phys, row, lo, hi);
        } else {
          nl = 1;
        }
        break;
      }
      case V_LOADRANGE: lo = rs + row * rstep; hi = lo >> 63; break;
      case V_CONST: lo = P.consts[a].lo; hi = P.consts[a].hi; nl = (uint8_t)P.consts[a].isnull; break;
      case V_MOV: lo = R.lo(a); hi = R.hi(a); nl = R.nl(a); break;
      case V_SELECT: {
        bool cond = !R.nl(a) && R.lo(a) != 0;
        lo = cond ? R.lo(b) : R.lo(c);
        hi = cond ? R.hi(b) : R.hi(c);
        nl = cond ? R.nl(b) : R.nl(c);
        break;
      }
      case V_COALESCE: {
        bool an = R.nl(a);
        lo = an ? R.lo(b) : R.lo(a);
        hi = an ? R.hi(b) : R.hi(a);
        nl = an ? R.nl(b) : R.nl(a);
        break;
      }
      case V_AND: {
        bool an = R.nl(a), bn = R.nl(b);
        bool av = R.lo(a) != 0, bv = R.lo(b) != 0;
        if ((!an && !av) || (!bn && !bv)) { lo = 0; nl = 0; }
        else if (an || bn) { nl = 1; }
        else { lo = 1; }
        break;
      }
      case V_OR: {
        bool an = R.nl(a), bn = R.nl(b);
        bool av = R.lo(a) != 0, bv = R.lo(b) != 0;
        if ((!an && av) || (!bn && bv)) { lo = 1; nl = 0; }
        else if (an || bn) { nl = 1; }
        else { lo = 0; }
        break;
      }
      case V_ISNULL: lo = R.nl(a) ? 1 : 0; break;
      case V_ISNOTNULL: lo = R.nl(a) ? 0 : 1; break;
      case V_DISTINCT_I: case V_DISTINCT_L: case V_DISTINCT_F: {
        bool an = R.nl(a), bn = R.nl(b);
        bool same;
        if (an || bn) same = an && bn;
        else if (op == V_DISTINCT_F) {
          double x = __longlong_as_double(R.lo(a)), y = __longlong_as_double(R.lo(b));
          same = (x == y) || (x != x && y != y);
        } else same = R.lo(a) == R.lo(b) && R.hi(a) == R.hi(b);
        lo = aux ? same : !same;
        break;
      }
      case V_SYNTH: {
        nl = R.nl(a) | R.nl(b) | R.nl(c);
        uint64_t m = (uint64_t)R.lo(c);
        if (!nl && m) {
          lo = (int64_t)(splitmix64((uint64_t)R.lo(a) + (uint64_t)R.lo(b)) % m);
        } else {
          nl = 1;
        }
        break;
      }
      default: {
        // null-propagating unary/binary ops
        nl = R.nl(a);
        if (op >= V_ADD_I && op != V_NOT && op != V_I2L && op != V_U2L && op != V_L2I && op != V_I2F &&
            op != V_L2F && op != V_F2I && op != V_F2L && op != V_CHECK_I && op != V_CHECK_L &&
            op != V_SCALEUP_I && op != V_SCALEUP_L && op != V_SCALEDN_I && op != V_SCALEDN_L &&
            op != V_DEC2F_I && op != V_DEC2F_L && op != V_F2DEC_I && op != V_F2DEC_L &&
            op != V_TOBOOL_I && op != V_TOBOOL_F && op != V_NEG_I && op != V_NEG_L && op != V_NEG_F &&
            op != V_ABS_I && op != V_ABS_L && op != V_ABS_F)
          nl |= R.nl(b);
        const int64_t xa = R.lo(a), xah = R.hi(a);
        const int64_t xb = R.lo(b), xbh = R.hi(b);
        bool ok = active && !nl;
        switch (op) {
          case V_ADD_I: if (__builtin_add_overflow(xa, xb, &lo) && ok) raise_err(err, E_OVF_ADD); break;
          case V_SUB_I: if (__builtin_sub_overflow(xa, xb, &lo) && ok) raise_err(err, E_OVF_SUB); break;
          case V_MUL_I: if (__builtin_mul_overflow(xa, xb, &lo) && ok) raise_err(err, E_OVF_MUL); break;
          case V_DIV_I:
            if (xb == 0) nl = 1;
            else if (xa == INT64_MIN && xb == -1) { if (ok) raise_err(err, E_OVF_MUL); }
            else lo = xa / xb;
            break;
          case V_MOD_I:
            if (xb == 0) nl = 1;
            else if (xb == -1) lo = 0;
            else lo = xa % xb;
            break;
          case V_NEG_I: if (__builtin_sub_overflow((int64_t)0, xa, &lo) && ok) raise_err(err, E_OVF_NEG); break;
          case V_ABS_I:
            if (xa == INT64_MIN && ok) raise_err(err, E_OVF_NEG);
            lo = xa < 0 ? -xa : xa;
            break;
          case V_ADD_L: case V_SUB_L: case V_MUL_L: {
            i128 r, x = mk128(xa, xah), y = mk128(xb, xbh);
            bool o = op == V_ADD_L ? add_ovf128(x, y, r) : op == V_SUB_L ? sub_ovf128(x, y, r) : mul_ovf128(x, y, r);
            if (o && ok) raise_err(err, op == V_ADD_L ? E_OVF_ADD : op == V_SUB_L ? E_OVF_SUB : E_OVF_MUL);
            sp128(r, lo, hi);
            break;
          }
          case V_DIV_L: case V_MOD_L: {
            i128 x = mk128(xa, xah), y = mk128(xb, xbh);
            if (y == 0) { nl = 1; break; }
            i128 r = op == V_DIV_L ? sdiv128(x, y) : smod128(x, y);
            sp128(r, lo, hi);
            break;
          }
          case V_NEG_L: {
            i128 r;
            if (sub_ovf128((i128)0, mk128(xa, xah), r) && ok) raise_err(err, E_OVF_NEG);
            sp128(r, lo, hi);
            break;
          }
          case V_ABS_L: {
            i128 x = mk128(xa, xah);
            sp128(x < 0 ? -x : x, lo, hi);
            break;
          }
          case V_ADD_F: case V_SUB_F: case V_MUL_F: case V_DIV_F: case V_MOD_F: case V_IDIV_F: {
            double x = __longlong_as_double(xa), y = __longlong_as_double(xb), r = 0;
            switch (op) {
              case V_ADD_F: r = x + y; break;
              case V_SUB_F: r = x - y; break;
              case V_MUL_F: r = x * y; break;
              case V_DIV_F: if (y == 0) nl = 1; else r = x / y; break;
              case V_MOD_F: if (y == 0) nl = 1; else r = fmod(x, y); break;
              default: if (y == 0) nl = 1; else r = trunc(x / y); break;
            }
            if (aux == 1) r = (double)(float)r;  // FLOAT result
            lo = __double_as_longlong(r);
            break;
          }
          case V_NEG_F: lo = __double_as_longlong(-__longlong_as_double(xa)); break;
          case V_ABS_F: lo = __double_as_longlong(fabs(__longlong_as_double(xa))); break;
          case V_CMP_I: lo = cmp_res(xa < xb ? -1 : xa > xb ? 1 : 0, aux); break;
          case V_CMP_L: {
            i128 x = mk128(xa, xah), y = mk128(xb, xbh);
            lo = cmp_res(x < y ? -1 : x > y ? 1 : 0, aux);
            break;
          }
          case V_CMP_F: {
            double x = __longlong_as_double(xa), y = __longlong_as_double(xb);
            bool nx = x != x, ny = y != y;
            int cc = (nx || ny) ? (nx == ny ? 0 : (nx ? 1 : -1)) : (x < y ? -1 : x > y ? 1 : 0);
            lo = cmp_res(cc, aux);
            break;
          }
          case V_NOT: lo = xa == 0; break;
          case V_TOBOOL_I: lo = (xa != 0 || xah != 0); break;
          case V_TOBOOL_F: lo = __longlong_as_double(xa) != 0.0; break;
          case V_I2L: lo = xa; hi = xa >> 63; break;
          case V_U2L: lo = xa; hi = 0; break;
          case V_L2I: {
            i128 x = mk128(xa, xah);
            i128 mn = b == 255 ? (i128)INT64_MIN : mk128(P.consts[b].lo, P.consts[b].hi);
            i128 mx = c == 255 ? (i128)INT64_MAX : mk128(P.consts[c].lo, P.consts[c].hi);
            if ((x < mn || x > mx) && ok) raise_err(err, E_CAST_RANGE);
            lo = xa;
            break;
          }
          case V_CHECK_I: {
            if ((xa < P.consts[b].lo || xa > P.consts[c].lo) && ok) raise_err(err, E_CAST_RANGE);
            lo = xa;
            break;
          }
          case V_CHECK_L: {
            i128 x = mk128(xa, xah);
            if ((x < mk128(P.consts[b].lo, P.consts[b].hi) || x > mk128(P.consts[c].lo, P.consts[c].hi)) && ok)
              raise_err(err, E_CAST_RANGE);
            lo = xa;
            hi = xah;
            break;
          }
          case V_I2F: lo = __double_as_longlong((double)xa); break;
          case V_L2F: lo = __double_as_longlong(i128_to_double(mk128(xa, xah))); break;
          case V_F2I: case V_F2L: {
            double x = rint(__longlong_as_double(xa));
            bool bad = !(x >= -1.7014118346046923e38 && x < 1.7014118346046923e38);
            i128 v = bad ? 0 : (i128)x;
            i128 mn = mk128(P.consts[b].lo, P.consts[b].hi), mx = mk128(P.consts[c].lo, P.consts[c].hi);
            if ((bad || v < mn || v > mx) && ok) raise_err(err, E_CAST_RANGE);
            sp128(v, lo, hi);
            break;
          }
          case V_SCALEUP_I: if (__builtin_mul_overflow(xa, pow10_64(aux), &lo) && ok) raise_err(err, E_DEC_OVF); break;
          case V_SCALEUP_L: {
            i128 r;
            if (mul_ovf128(mk128(xa, xah), pow10_128(aux), r) && ok) raise_err(err, E_DEC_OVF);
            sp128(r, lo, hi);
            break;
          }
          case V_SCALEDN_I: {
            int64_t p = pow10_64(aux), q = xa / p, r = xa % p;
            int64_t ar = r < 0 ? -r : r;
            if (2 * ar >= p) q += xa < 0 ? -1 : 1;
            lo = q;
            break;
          }
          case V_SCALEDN_L: {
            i128 x = mk128(xa, xah), p = pow10_128(aux);
            i128 q = sdiv128(x, p), r = x - q * p;
            i128 ar = r < 0 ? -r : r;
            if (2 * ar >= p) q += x < 0 ? -1 : 1;
            sp128(q, lo, hi);
            break;
          }
          case V_DEC2F_I: lo = __double_as_longlong((double)xa / (double)pow10_64(aux)); break;
          case V_DEC2F_L: lo = __double_as_longlong(i128_to_double(mk128(xa, xah)) / (double)pow10_128(aux)); break;
          case V_F2DEC_I: case V_F2DEC_L: {
            double x = rint(__longlong_as_double(xa) * (double)pow10_128(aux));
            bool bad = !(x >= -1.7014118346046923e38 && x < 1.7014118346046923e38);
            i128 v = bad ? 0 : (i128)x;
            i128 mn = mk128(P.consts[b].lo, P.consts[b].hi), mx = mk128(P.consts[c].lo, P.consts[c].hi);
            if ((bad || v < mn || v > mx) && ok) raise_err(err, E_CAST_RANGE);
            sp128(v, lo, hi);
            break;
          }
          default: break;
        }
        break;
      }
    }
    R.lo(d) = lo;
    R.hi(d) = hi;
    R.nl(d) = nl;
}

}  // namespace dev
}  // namespace mbx
