// knobs.h — the MBX_* tuning and experiment switches.
//
// They are read from the environment only when MBX_EXPERIMENTS=1 is set as
// well, so a stray variable in a caller's process (a MoonBit program linking
// the library) cannot change kernel shapes, force the slow VM / two-pass
// paths or inject test faults: without the opt-in every switch reads as unset
// and the measured defaults run.  The tests and tools/ set the opt-in.
#pragma once
#include <stdlib.h>

namespace mbx {

inline const char *Knob(const char *name) {
  static const bool on = [] {
    const char *e = getenv("MBX_EXPERIMENTS");
    return e && e[0] == '1';
  }();
  return on ? getenv(name) : nullptr;
}

}  // namespace mbx
