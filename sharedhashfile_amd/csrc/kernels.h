// Internal launcher interface between the C-ABI layer (shf_hash_batch.hip) and
// the kernels (kernels.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace shfhb {

enum OutMode { kOutHash = 0, kOutUid = 1 };
enum KernelChoice { kKernelAuto = 0, kKernelFixed16 = 1, kKernelTiled = 2, kKernelGeneric = 3, kKernelSpan = 4 };

// keys: device pointer to n * key_len bytes; out: n x 16 B (hash) or n x 8 B (uid).
hipError_t launch_fixed(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, void* out, int out_mode,
                        hipStream_t st, int kernel);

// Key i = bytes[offsets[i] - off_base, offsets[i+1] - off_base); offsets on device.
hipError_t launch_var(const void* bytes, const uint64_t* offsets, uint64_t off_base, uint64_t n, uint32_t seed,
                      void* out, int out_mode, hipStream_t st, int kernel = kKernelAuto);

}  // namespace shfhb
