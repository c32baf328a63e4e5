// Page-locked host allocations made by this library, with their device-visible
// addresses (tfs_crc32_host_malloc_pinned, tfs_crc_group_host_malloc, and each
// context's own staging / result buffers).  The close path's zero-copy post asks
// whether a base is page-locked and for its device address once per batch; the HIP
// runtime answers both (hipPointerGetAttributes, hipHostGetDevicePointer) under its
// process-wide memory-object lock, and the post held ctx->mu meanwhile.  For
// allocations the library made itself the registry answers without a HIP call;
// anything else (memory the caller registered or allocated through HIP itself)
// still goes to the runtime.
#pragma once

#include <cstddef>
#include <cstdint>

namespace tfscrc {

// Record [host, host + bytes) with device-visible address dev (re-registering a
// base replaces its entry).
void pin_register(void* host, size_t bytes, void* dev);
// Forget the allocation starting at host (before it is freed).
void pin_unregister(void* host);
// true when p lies inside a registered allocation; *dev = p's device-visible address.
bool pin_lookup(const void* p, void** dev);

}  // namespace tfscrc
