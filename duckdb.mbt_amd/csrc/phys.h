// phys.h — physical storage classes of device column values (shared by the
// host code, the kernels and the run-time compiled expression kernels).
#pragma once
#include <stdint.h>

namespace mbx {

// Physical storage of one value in a device column chunk.
enum Phys : uint8_t {
  P_U8 = 0,   // BOOLEAN, UTINYINT
  P_I8,       // TINYINT
  P_I16,      // SMALLINT, DECIMAL(w<=4)
  P_U16,      // USMALLINT
  P_I32,      // INTEGER, DATE, DECIMAL(w<=9)
  P_U32,      // UINTEGER
  P_I64,      // BIGINT, TIME, TIMESTAMP, DECIMAL(w<=18)
  P_U64,      // UBIGINT
  P_I128,     // HUGEINT, DECIMAL(w<=38)
  P_F32,      // FLOAT
  P_F64,      // DOUBLE
  P_STR,      // VARCHAR / BLOB: int64 offsets[n+1] + chars
  P_INTERVAL, // 16 B {int32 months, int32 days, int64 micros}
};

}  // namespace mbx
