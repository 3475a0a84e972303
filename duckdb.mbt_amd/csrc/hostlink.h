// Host link (C4 read-back): device -> pageable host copies at PCIe rate.
#pragma once
#include <cstddef>
#include <string>

namespace mbx {

// Copies n bytes from device memory `src` (on `device`, already produced:
// the caller has synchronised the producing stream) into pageable host
// memory `dst`, and returns when the bytes are there.  Large copies run on a
// per-device pool of host threads, each with its own stream and pinned
// double buffer, after advising huge pages for `dst` (see hostlink.cpp).
// Returns "" or the HIP error text.
std::string LinkD2H(int device, void *dst, const void *src, size_t n);

}  // namespace mbx
