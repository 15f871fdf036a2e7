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

// ---- DPP cross-lane primitives (VALU latency instead of ds_bpermute round trips).  They require the
// whole wave to be active (uniform control flow); results of the reductions are wave-uniform.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp_i<CTRL>((int)b), hi = dpp_i<CTRL>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
enum : int { DPP_QP_1032 = 0xB1, DPP_QP_2301 = 0x4E, DPP_ROR4 = 0x124, DPP_ROR8 = 0x128, DPP_SHR1 = 0x111,
             DPP_SHR2 = 0x112, DPP_SHR4 = 0x114, DPP_SHR8 = 0x118, DPP_BCAST15 = 0x142, DPP_BCAST31 = 0x143 };

// sum over the 64 lanes, combined in a fixed order (row sums, then rows 0..3): deterministic
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_d<DPP_QP_1032>(v);
  v += dpp_d<DPP_QP_2301>(v);
  v += dpp_d<DPP_ROR4>(v);
  v += dpp_d<DPP_ROR8>(v);
  return ((readlane_d(v, 0) + readlane_d(v, 16)) + readlane_d(v, 32)) + readlane_d(v, 48);
}
__device__ __forceinline__ double wave_max_dpp(double v) {
  v = fmax(v, dpp_d<DPP_QP_1032>(v));
  v = fmax(v, dpp_d<DPP_QP_2301>(v));
  v = fmax(v, dpp_d<DPP_ROR4>(v));
  v = fmax(v, dpp_d<DPP_ROR8>(v));
  return fmax(fmax(readlane_d(v, 0), readlane_d(v, 16)), fmax(readlane_d(v, 32), readlane_d(v, 48)));
}
// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ int wave_incl_scan_dpp(int x) {
  x += dpp_i<DPP_SHR1>(x);
  x += dpp_i<DPP_SHR2>(x);
  x += dpp_i<DPP_SHR4>(x);
  x += dpp_i<DPP_SHR8>(x);
  x += dpp_i<DPP_BCAST15, 0xA>(x);
  x += dpp_i<DPP_BCAST31, 0xC>(x);
  return x;
}

// Double-double (hi + lo) prefix sums of (v, v^2): smg_hit_prefix_sums writes one DD4 per 64-point block.  A
// window sum is then a difference of two nearby prefixes, exact to ~1 ulp of the window's own sum plus
// ~eps^2 of the total mass before it, instead of ~eps of that mass (a faint window far into a bright dataset).
// TwoSum needs unfused, unreassociated f64 arithmetic: the library is built with -ffp-contract=off.
struct DD4 {
  double xh, xl, yh, yl;
};
__host__ __device__ __forceinline__ void dd_add(double ah, double al, double bh, double bl, double& h, double& l) {
  const double s = ah + bh;
  const double v = s - ah;
  double e = (ah - (s - v)) + (bh - v);  // TwoSum error of ah + bh
  e += al + bl;
  h = s + e;
  l = e - (h - s);
}
struct DD4Add {
  __host__ __device__ DD4 operator()(const DD4& a, const DD4& b) const {
    DD4 r;
    dd_add(a.xh, a.xl, b.xh, b.xl, r.xh, r.xl);
    dd_add(a.yh, a.yl, b.yh, b.yl, r.yh, r.yl);
    return r;
  }
};
// (prefix at b) - (prefix at a) of one component, rounded to f64
__device__ __forceinline__ double dd_diff(double bh, double bl, double ah, double al) { return (bh - ah) + (bl - al); }

// Block-wide sum of NV doubles; `scratch` holds NV * (BLOCK/64) doubles of LDS.  Result broadcast.
template <int BLOCK, int NV, bool DPP = false>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* scratch) {
  constexpr int NW = BLOCK / WAVE;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = DPP ? wave_sum_dpp(v[j]) : wave_sum(v[j]);
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

#ifndef SMG_XCDS
#define SMG_XCDS 8  // XCDs of the device (gfx950: 8); diagnostic 1 = no XCD locality (one range, no hwreg read)
#endif
constexpr int XCDS = SMG_XCDS;

// The XCD this workgroup runs on (HW_REG_XCC_ID, 0-7).  Blocks are observed to be dealt round-robin over the XCDs,
// but which XCD a block lands on is not fixed, and with other work resident (a copy kernel on another stream) the
// deal can skip an XCD, so blockIdx % 8 no longer groups the blocks of one XCD; the register is exact.  Speed only:
// any range may be scored by any workgroup (the ion passes' ranges, the sort's tiles).
__device__ __forceinline__ int home_xcd() {
  if constexpr (XCDS == 1) {
    return 0;
  } else {
    int x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x % XCDS;
  }
}

}  // namespace smg
