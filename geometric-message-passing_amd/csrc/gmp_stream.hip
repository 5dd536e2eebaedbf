// CU-partitioned streams for the side-stream weight gradients (DESIGN.md §3 "EGNN step").
//
// The weight-gradient outer sums of a layer's backward are leaves of the autograd graph and run
// on a side stream beside the critical path's node-level kernels (LayerNorm backward, the small
// node GEMMs, the sender-side segmented sums).  Launched on an ordinary stream, a split-K outer
// sum occupies every CU it can get (512-thread workgroups at ~250 VGPRs: one per SIMD set) and
// the main stream's kernels queue behind its waves.  A stream created with a CU mask only ever
// dispatches onto the masked CUs, so the rest of the chip stays free for the critical path --
// a hardware partition instead of a grid-size cap (which the split-K reduction pays for in
// fewer, longer workgroups).
//
// The mask selects `cus` of the device's CUs spread evenly over the CU index space (ROCm maps
// consecutive mask bits round-robin over the shader engines / XCDs, so an even spread keeps
// every XCD's L2 in use).

#include <cstdint>
#include <vector>

#include "gmp_common.h"

using namespace gmp;

extern "C" {

// Creates a stream restricted to `cus` CUs of the current device (0 < cus <= the CU count; a
// value >= the CU count gives an unmasked stream).  *stream receives the hipStream_t.
int gmp_stream_create_cu_share(int cus, void** stream) {
  GMP_CHECK_ARG(stream && cus > 0);
  const int total = device_cu_count();
  hipStream_t s = nullptr;
  if (cus >= total) {
    const int rc = hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (rc) return rc;
    *stream = s;
    return GMP_OK;
  }
  std::vector<uint32_t> mask((total + 31) / 32, 0u);
  for (int i = 0; i < cus; ++i) {
    const int cu = (int)((int64_t)i * total / cus);
    mask[cu >> 5] |= 1u << (cu & 31);
  }
  const int rc = hip_check(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  if (rc) return rc;
  *stream = s;
  return GMP_OK;
}

int gmp_stream_destroy(void* stream) {
  return hip_check(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)));
}

}  // extern "C"
