// vm.h — the device expression program (shared by the host compiler in
// executor.cpp and the tile interpreter in kernels.hip).
//
// A program evaluates scalar expressions for a tile of 256 rows at a time.
// Registers live in LDS as [reg][row] planes (lo 64 bits, hi 64 bits, null
// byte), so operand indices are wave-uniform LDS offsets rather than
// runtime-indexed private arrays (which hipcc would spill to scratch).
#pragma once
#include <stdint.h>

namespace mbx {

#define VM_MAX_INS 80
#define VM_MAX_REGS 12
#define VM_MAX_CONST 24
#define VM_MAX_COLS 12
#define VM_MAX_OUT 12
#define VM_TILE 256

enum VmOpc : uint8_t {
  V_LOADCOL = 0,  // r[dst] <- col[a]                         (aux = phys)
  V_LOADRANGE,    // r[dst] <- range_start + row * range_step
  V_CONST,        // r[dst] <- const[a]
  V_MOV,          // r[dst] <- r[a]
  // integer arithmetic in 64 bits with overflow -> error
  V_ADD_I, V_SUB_I, V_MUL_I, V_DIV_I, V_MOD_I, V_NEG_I, V_ABS_I,
  // 128-bit
  V_ADD_L, V_SUB_L, V_MUL_L, V_DIV_L, V_MOD_L, V_NEG_L, V_ABS_L,
  // double
  V_ADD_F, V_SUB_F, V_MUL_F, V_DIV_F, V_MOD_F, V_NEG_F, V_ABS_F, V_IDIV_F,
  // comparisons (aux = 0 EQ,1 NE,2 LT,3 LE,4 GT,5 GE) -> boolean in lo
  V_CMP_I, V_CMP_L, V_CMP_F,
  // three-valued logic
  V_AND, V_OR, V_NOT, V_ISNULL, V_ISNOTNULL,
  V_DISTINCT_I, V_DISTINCT_L, V_DISTINCT_F,  // aux=1 -> NOT DISTINCT
  // conversions
  V_I2L,          // sign-extend 64 -> 128
  V_U2L,          // zero-extend 64 -> 128 (UBIGINT storage)
  V_L2I,          // 128 -> 64 (range check; b/c = const ids of lo/hi bound, 255 = int64 range)
  V_I2F, V_L2F,   // -> double
  V_F2I, V_F2L,   // double -> integer (round to nearest even, range check via b/c)
  V_CHECK_I,      // range check r[a] within [const[b], const[c]] (64 bit), then copy
  V_CHECK_L,      // same for 128-bit registers
  V_SCALEUP_I, V_SCALEUP_L,  // r = r * 10^aux (overflow -> error)
  V_SCALEDN_I, V_SCALEDN_L,  // r = round_half_away(r / 10^aux)
  V_DEC2F_I, V_DEC2F_L,      // double(r) / 10^aux
  V_F2DEC_I, V_F2DEC_L,      // round(r * 10^aux) with range check const[b], const[c]
  V_TOBOOL_I, V_TOBOOL_F,    // r != 0
  V_SELECT,       // r[dst] <- (r[a] valid && r[a] != 0) ? r[b] : r[c]
  V_COALESCE,     // r[dst] <- r[a] valid ? r[a] : r[b]
  V_SYNTH,        // r[dst] <- splitmix64(r[a] + r[b]) mod r[c]
  V_NOP,
};

struct VmIns {
  uint8_t op, dst, a, b, c, pad;
  uint16_t aux;
};

struct VmConst {
  int64_t lo, hi;
  int32_t isnull, pad;
};

struct VmCol {
  const void *data;
  const uint64_t *validity;  // null: all valid
  int32_t phys;
  int32_t pad;
};

struct VmProgram {
  VmIns ins[VM_MAX_INS];
  VmConst consts[VM_MAX_CONST];
  int32_t n_ins, n_const, n_regs;
  int32_t n_out;
  uint8_t out_reg[VM_MAX_OUT];
  uint8_t out_phys[VM_MAX_OUT];   // store format of each output
  uint8_t out_class[VM_MAX_OUT];
  uint8_t pred_reg;               // predicate register (filter programs)
  uint8_t pad[3];
};

// Error codes written by kernels to the device error word.
enum VmErr : int32_t {
  E_NONE = 0,
  E_OVF_ADD = 1,
  E_OVF_SUB = 2,
  E_OVF_MUL = 3,
  E_OVF_NEG = 4,
  E_CAST_RANGE = 5,
  E_DEC_OVF = 6,
  E_HASH_FULL = 7,
  E_KEY_RANGE = 8,  // a GROUP BY key outside the zone map its slot table was sized from
};

namespace dev {
struct VmCols {
  VmCol c[VM_MAX_COLS];
  int32_t n;
};

struct VmOuts {
  void *data[VM_MAX_OUT];
  // 32-bit-word view of a zeroed NULL bitmap (bit = 1: row is NULL), or null.
  // Only NULL rows touch it (rare), so the common all-valid output costs no
  // bitmap traffic; InvertNullBits turns it into a validity bitmap when
  // anynull says one is needed.
  uint32_t *nullbits[VM_MAX_OUT];
  int32_t *anynull;  // per output: set to 1 if a NULL was written
};
}  // namespace dev

}  // namespace mbx
