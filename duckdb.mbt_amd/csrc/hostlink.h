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

// The mid-size (2-32 MiB) copy method for every device from now on: -1 the
// measured choice (default), 0 the runtime's copy, 1 a registered
// destination, 2 the pinned bounce (duckdb_mbx_set_link_mode; A/B legs).
void SetLinkMode(int mode);
// Per device and size class: each method's trial medians (GB/s), the method
// kept, and the calls served -- JSON text.
std::string LinkStatsJson();

}  // namespace mbx
