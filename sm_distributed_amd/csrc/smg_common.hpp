// Shared helpers of libsmg: error reporting, launch checks, block reductions (wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "../../include/smg.h"

namespace smg {

void set_error(const char* fmt, ...);

#define SMG_CHECK_ARG(cond, ...)          \
  do {                                    \
    if (!(cond)) {                        \
      ::smg::set_error(__VA_ARGS__);      \
      return SMG_ERR_INVALID;             \
    }                                     \
  } while (0)

#define SMG_HIP(call)                                                                  \
  do {                                                                                 \
    hipError_t _e = (call);                                                            \
    if (_e != hipSuccess) {                                                            \
      ::smg::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(_e), __FILE__, \
                       __LINE__);                                                      \
      return SMG_ERR_HIP;                                                              \
    }                                                                                  \
  } while (0)

#define SMG_LAUNCH_CHECK()                                                                   \
  do {                                                                                       \
    hipError_t _e = hipGetLastError();                                                       \
    if (_e != hipSuccess) {                                                                  \
      ::smg::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, \
                       __LINE__);                                                            \
      return SMG_ERR_HIP;                                                                    \
    }                                                                                        \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int WAVE = 64;

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

// Block-wide sum of NV doubles; `scratch` holds NV * (BLOCK/64) doubles of LDS.  Result broadcast.
template <int BLOCK, int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* scratch) {
  constexpr int NW = BLOCK / WAVE;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = wave_sum(v[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) scratch[j * NW + wid] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += scratch[j * NW + w];
    v[j] = s;
  }
  __syncthreads();
}

}  // namespace smg
