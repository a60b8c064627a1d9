// Shared host-side plumbing for libslam355.so: thread-local error string,
// argument checks and HIP launch checks.  Device code is written directly for
// gfx950 (wave64, 160 KiB LDS); there is no other target.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <type_traits>

#include "../../include/slam355.h"

namespace slam {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace slam

#define SLAM_REQUIRE(cond, ...)                 \
  do {                                          \
    if (!(cond)) {                              \
      ::slam::set_error(__VA_ARGS__);           \
      return SLAM_ERR_ARG;                      \
    }                                           \
  } while (0)

#define SLAM_HIP(call)                                                        \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess) {                                                   \
      ::slam::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                  \
      return SLAM_ERR_HIP;                                                    \
    }                                                                         \
  } while (0)

// Check the launch that was just issued (launch-configuration errors only;
// faults surface at the next synchronising call).
#define SLAM_LAUNCHED(name) SLAM_HIP(hipGetLastError())

constexpr int kWave = 64;  // gfx950 wavefront

// Compile-time loop: f(std::integral_constant<int, i>) for i in [B, E).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Lane m of each 16-lane row, broadcast to the whole row (DPP row_newbcast,
// gfx90a+; on f64 it lowers to v_mov_b64_dpp or folds into the consumer).
template <int M>
__device__ __forceinline__ double bcast16(double v) {
  static_assert(M >= 0 && M < 16, "row lane");
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + M, 0xf, 0xf, true);
}
