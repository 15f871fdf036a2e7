// Peak-list preparation on gfx950: hit packing, global m/z sort, ppm-window search, legacy sampler.
//
// Reference behaviour (frulo/SM_distributed):
//   formula_imager_segm.py:60-63  _sp_df_gen   (sp_id -> pixel join)
//   formula_imager_segm.py:73-74  sort_values('mz') per segment/chunk
//   formula_imager_segm.py:79-82  f64 ppm bounds + searchsorted('l' / 'r')
//   formula_imager.py:9-38        legacy prefix-sum sampler
#include <cstring>
#include <stdarg.h>

#include <rocprim/device/device_scan.hpp>

#include "smg_common.hpp"

namespace smg {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

// ---------------------------------------------------------------------------------------------
// pack: one thread per spectrum-chunk.  Each block handles one spectrum at a time (grid-stride),
// streaming its intensities with coalesced loads and writing 8-byte hits.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) pack_hits_kernel(const int64_t* __restrict__ sp_off,
                                                        const int32_t* __restrict__ pixel_map,
                                                        int64_t n_spectra,
                                                        const float* __restrict__ ints,
                                                        uint64_t* __restrict__ hits) {
  for (int64_t s = blockIdx.x; s < n_spectra; s += gridDim.x) {
    const int64_t a = sp_off[s], b = sp_off[s + 1];
    const uint64_t pix = (uint32_t)pixel_map[s];
    for (int64_t i = a + threadIdx.x; i < b; i += blockDim.x) {
      hits[i] = pix | ((uint64_t)__float_as_uint(ints[i]) << 32);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// window search.  Bounds are computed exactly as the reference lambda evaluates them
// (`mz - mz*ppm*1e-6`: ((mz*ppm)*1e-6) then subtract; the library is built with
// -ffp-contract=off so no FMA changes the rounding), compared in f64 against the f32 keys.
// ---------------------------------------------------------------------------------------------
// Both bounds of a window in one branch-free loop: the trip count (ceil(log2 n)) does not depend on the data, so
// the two searches advance together with their loads in flight side by side (half the dependent-load chain of
// two binary searches run one after the other).  Invariant: the answer lies in [b, b + len]; at len == 1 it is
// b + (a[b] < x) (lower) / b + (a[b] <= x) (upper).  Same results as searchsorted 'left' / 'right'.
__global__ void __launch_bounds__(256) window_bounds_kernel(const double* __restrict__ peak_mz,
                                                            const int64_t* __restrict__ order,
                                                            int64_t n_windows, double ppm,
                                                            const float* __restrict__ mz_sorted,
                                                            int64_t n_points, int64_t* __restrict__ lo,
                                                            int64_t* __restrict__ hi) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_windows) return;
  const int64_t w = order ? order[t] : t;
  const double mz = peak_mz[w];
  const double d = mz * ppm * 1e-6;
  const double lower = mz - d;
  const double upper = mz + d;
  if (n_points <= 0) {
    lo[w] = hi[w] = 0;
    return;
  }
  int64_t bl = 0, bu = 0, len = n_points;
  while (len > 1) {
    const int64_t half = len >> 1;
    const double vl = (double)mz_sorted[bl + half - 1];
    const double vu = (double)mz_sorted[bu + half - 1];
    bl += (vl < lower) ? half : 0;
    bu += (vu <= upper) ? half : 0;
    len -= half;
  }
  lo[w] = bl + (((double)mz_sorted[bl] < lower) ? 1 : 0);
  hi[w] = bu + (((double)mz_sorted[bu] <= upper) ? 1 : 0);
}

// ---------------------------------------------------------------------------------------------
// legacy sampler: one wave per (spectrum, window-chunk); each lane one window.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t lb_d(const double* a, int64_t n, double x) {
  int64_t lo = 0, len = n;
  while (len > 0) {
    int64_t half = len >> 1, mid = lo + half;
    if (a[mid] < x) { lo = mid + 1; len -= half + 1; } else { len = half; }
  }
  return lo;
}
__device__ __forceinline__ int64_t ub_d(const double* a, int64_t n, double x) {
  int64_t lo = 0, len = n;
  while (len > 0) {
    int64_t half = len >> 1, mid = lo + half;
    if (a[mid] <= x) { lo = mid + 1; len -= half + 1; } else { len = half; }
  }
  return lo;
}

__global__ void __launch_bounds__(256) sample_spectra_kernel(
    const int64_t* __restrict__ sp_off, const double* __restrict__ mzs, const double* __restrict__ cum,
    int64_t n_spectra, const double* __restrict__ lower, const double* __restrict__ upper,
    int64_t n_windows, int64_t* __restrict__ ow, int64_t* __restrict__ os, double* __restrict__ ov,
    int64_t capacity, unsigned long long* __restrict__ count) {
  const int64_t s = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_spectra || j >= n_windows) return;
  const int64_t a = sp_off[s], n = sp_off[s + 1] - a;
  const double* m = mzs + a;
  const double* c = cum + a + s;  // n+1 cumulative values
  const double v = c[ub_d(m, n, upper[j])] - c[lb_d(m, n, lower[j])];
  if (v > 0.001) {
    const unsigned long long k = atomicAdd(count, 1ull);
    if ((int64_t)k < capacity) {
      ow[k] = j;
      os[k] = s;
      ov[k] = v;
    }
  }
}

// duplicate-candidate flags: one workgroup per spectrum (grid-stride).  A spectrum of <= FLAG_TILE points is
// staged in LDS by one coalesced read, so the sortedness check and the neighbour tests read LDS.  With `state`
// (one byte per point: the flag the hit currently carries), a hit is read and written only when its flag
// changes, so a repeated pass reads 5 B per point instead of 12; without it every hit is read.
constexpr int FLAG_TILE = 4096;
constexpr int FLAG_THREADS = 256;
constexpr int FLAG_U = FLAG_TILE / FLAG_THREADS;  // points per thread of a tile, loads in flight together

// m/z of spectrum positions [l0, l0 + n) into smz[0, n), n <= FLAG_TILE: all of a thread's loads issued at once
__device__ __forceinline__ void flag_load_tile(const float* __restrict__ mz, int64_t l0, int n, float* smz) {
  float r[FLAG_U];
#pragma unroll
  for (int u = 0; u < FLAG_U; ++u) {
    const int i = threadIdx.x + u * FLAG_THREADS;
    r[u] = i < n ? mz[l0 + i] : 0.0f;
  }
#pragma unroll
  for (int u = 0; u < FLAG_U; ++u) {
    const int i = threadIdx.x + u * FLAG_THREADS;
    if (i < n) smz[i] = r[u];
  }
}

__device__ __forceinline__ int flag_tile_unsorted(const float* smz, int n) {
  int un = 0;
  for (int i = threadIdx.x + 1; i < n; i += FLAG_THREADS) un |= (smz[i] < smz[i - 1]);
  return un;
}

// Flags of tile entries [j0, j1) (spectrum position l0 + j).  The tile holds a point's spectrum neighbours
// whenever they exist (one halo point each side), so "has a previous / next point" is j > 0 / j + 1 < n.
// The state bytes are loaded together up front; a hit is read and written only when its flag changes.
__device__ __forceinline__ void flag_tile_store(const float* smz, int n, int j0, int j1, int64_t l0, bool all,
                                                double slack, uint64_t* __restrict__ hits,
                                                uint8_t* __restrict__ state) {
  uint8_t st[FLAG_U];
#pragma unroll
  for (int u = 0; u < FLAG_U; ++u) {
    const int j = j0 + threadIdx.x + u * FLAG_THREADS;
    st[u] = (state && j < j1) ? state[l0 + j] : (uint8_t)0;
  }
#pragma unroll
  for (int u = 0; u < FLAG_U; ++u) {
    const int j = j0 + threadIdx.x + u * FLAG_THREADS;
    if (j >= j1) continue;
    bool f = all;
    if (!f) {
      const double m = (double)smz[j];
      if (j > 0) f = f || (m - (double)smz[j - 1] <= slack * m);
      if (j + 1 < n) {
        const double m2 = (double)smz[j + 1];
        f = f || (m2 - m <= slack * m2);
      }
    }
    const int64_t i = l0 + j;
    if (state) {
      if (st[u] != (uint8_t)f) {
        state[i] = (uint8_t)f;
        const uint64_t h = hits[i];
        hits[i] = f ? (h | 0x80000000ull) : (h & ~0x80000000ull);
      }
    } else {
      const uint64_t h = hits[i];
      const uint64_t nh = f ? (h | 0x80000000ull) : (h & ~0x80000000ull);
      if (nh != h) hits[i] = nh;
    }
  }
}

__global__ void __launch_bounds__(FLAG_THREADS) flag_duplicates_kernel(const int64_t* __restrict__ sp_off,
                                                                       int64_t n_spectra,
                                                                       const float* __restrict__ mz,
                                                                       uint64_t* __restrict__ hits, double ppm,
                                                                       const uint8_t* __restrict__ force,
                                                                       uint8_t* __restrict__ state) {
  __shared__ float smz[FLAG_TILE];
  const double slack = 2.0 * ppm * 1e-6 / (1.0 - ppm * 1e-6) * (1.0 + 1e-9);
  constexpr int CORE = FLAG_TILE - 2;  // points flagged per tile of a long spectrum (plus one halo point a side)
  for (int64_t s = blockIdx.x; s < n_spectra; s += gridDim.x) {
    const int64_t a = sp_off[s], b = sp_off[s + 1];
    if (b - a <= FLAG_TILE) {
      const int n = (int)(b - a);
      flag_load_tile(mz, a, n, smz);
      __syncthreads();
      const bool all = __syncthreads_or(flag_tile_unsorted(smz, n)) || (force && force[s]);
      flag_tile_store(smz, n, 0, n, a, all, slack, hits, state);
      __syncthreads();  // smz is reused by the next spectrum
    } else {
      // longer spectra (config 5: Poisson(5000)): tiles of CORE points with their halo; a sortedness pass over
      // every tile first (an unsorted spectrum flags all of its points), then the flags tile by tile
      int un = 0;
      for (int64_t c0 = a; c0 < b; c0 += CORE) {
        const int64_t c1 = c0 + CORE < b ? c0 + CORE : b;
        const int64_t l0 = c0 > a ? c0 - 1 : a, l1 = c1 < b ? c1 + 1 : b;
        flag_load_tile(mz, l0, (int)(l1 - l0), smz);
        __syncthreads();
        un |= flag_tile_unsorted(smz, (int)(l1 - l0));
        __syncthreads();
      }
      const bool all = __syncthreads_or(un) || (force && force[s]);
      for (int64_t c0 = a; c0 < b; c0 += CORE) {
        const int64_t c1 = c0 + CORE < b ? c0 + CORE : b;
        const int64_t l0 = c0 > a ? c0 - 1 : a, l1 = c1 < b ? c1 + 1 : b;
        flag_load_tile(mz, l0, (int)(l1 - l0), smz);
        __syncthreads();
        flag_tile_store(smz, (int)(l1 - l0), (int)(c0 - l0), (int)(c1 - l0), l0, all, slack, hits, state);
        __syncthreads();
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// m/z slice of the resident dataset (the points one rank's windows can touch, multi-GPU strong scaling):
// every point with lo <= mz <= hi (compared in f64, as the window search compares), in dataset order, with
// the duplicate-candidate flag of smg_flag_duplicates computed on the way.  Spectra must be m/z-sorted (a
// centroided imzML spectrum is), so each spectrum's slice is one contiguous run found by two binary searches.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) slice_count_kernel(const int64_t* __restrict__ sp_off, int64_t n_spectra,
                                                          const float* __restrict__ mz, double lo, double hi,
                                                          int64_t* __restrict__ first, int64_t* __restrict__ count) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_spectra) return;
  const int64_t a = sp_off[s], b = sp_off[s + 1];
  int64_t l = a, len = b - a;  // first point with mz >= lo
  while (len > 0) {
    const int64_t h = len >> 1;
    if ((double)mz[l + h] < lo) {
      l += h + 1;
      len -= h + 1;
    } else {
      len = h;
    }
  }
  int64_t u = l;  // first point with mz > hi
  len = b - l;
  while (len > 0) {
    const int64_t h = len >> 1;
    if ((double)mz[u + h] <= hi) {
      u += h + 1;
      len -= h + 1;
    } else {
      len = h;
    }
  }
  first[s] = l;
  count[s] = u - l;
}

// one wave per spectrum (four per workgroup, grid-stride; a spectrum's run is a few hundred points): copies its
// run [first, first + n) to out at out_off[s], flagging a point when its spectrum neighbour (inside or outside the
// slice) lies within one window width, or when the spectrum's pixel is shared (force)
__global__ void __launch_bounds__(256) slice_copy_kernel(const int64_t* __restrict__ sp_off, int64_t n_spectra,
                                                         const float* __restrict__ mz,
                                                         const uint64_t* __restrict__ hits,
                                                         const int64_t* __restrict__ first,
                                                         const int64_t* __restrict__ out_off, double ppm,
                                                         const uint8_t* __restrict__ force,
                                                         float* __restrict__ out_mz, uint64_t* __restrict__ out_hits) {
  const double slack = 2.0 * ppm * 1e-6 / (1.0 - ppm * 1e-6) * (1.0 + 1e-9);
  constexpr int WPB = 4;  // waves per workgroup
  const int lane = threadIdx.x & 63;
  for (int64_t s = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6); s < n_spectra; s += (int64_t)gridDim.x * WPB) {
    const int64_t a = sp_off[s], b = sp_off[s + 1];
    const int64_t f = first[s], o = out_off[s], n = out_off[s + 1] - o;
    const bool all = force && force[s];
    for (int64_t j = lane; j < n; j += 64) {
      const int64_t i = f + j;
      const double m = (double)mz[i];
      bool fl = all;
      if (i > a) fl = fl || (m - (double)mz[i - 1] <= slack * m);
      if (i + 1 < b) {
        const double m2 = (double)mz[i + 1];
        fl = fl || (m2 - m <= slack * m2);
      }
      const uint64_t h = hits[i];
      out_mz[o + j] = mz[i];
      out_hits[o + j] = fl ? (h | 0x80000000ull) : (h & ~0x80000000ull);
    }
  }
}

// calibration stream: every lane reads 8-byte words, grid-stride, coalesced (the access width of the ion
// kernel's hit loads); XOR-folded per block so nothing is elided
__global__ void stream_read_kernel(const uint64_t* __restrict__ p, int64_t n, uint64_t* __restrict__ out) {
  uint64_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  acc = wave_sum(acc);  // any fold will do
  if ((threadIdx.x & 63) == 0) atomicXor(reinterpret_cast<unsigned long long*>(out + blockIdx.x),
                                          (unsigned long long)acc);
}

// Prefix sums of (v, v^2) over the m/z-sorted hits at 64-point granularity: cum64[b] = sums over points
// [0, 64*b) (exclusive, cum64[0] = 0) as double-double pairs (DD4, smg_common.hpp).  A window sum is the
// difference of two block prefixes plus the partial sums of at most 63 points at either end (ion_desc_kernel),
// accurate to the window's own magnitude however much intensity precedes it in m/z order.  Squares only for
// points without the duplicate-candidate flag: a flagged point may share its pixel with another point of the
// window and is squared after the per-pixel sum (ion kernel).  One wave per block: a coalesced 512-B read, a
// fixed-order DPP reduction (plain f64: its error is relative to the block's own 64 points).
// Each wave takes BS_PER_WAVE consecutive 64-point blocks and has all their loads in flight at once
// (chunk_sums_kernel below).
constexpr int BS_PER_WAVE = 8;


// Prefix sums of the block sums without a library scan (reduce, then scan): the 64-point blocks in chunks of
// PS_CHUNK; chunk_sums_kernel writes every block's sums (one wave per block, as described above) and each chunk's
// double-double total, chunk_base_kernel scans the chunk totals, chunk_scan_kernel scans each chunk from its
// base.  Every sum is formed in one fixed order: the result does not depend on scheduling.
constexpr int PS_CHUNK = 2048;            // 64-point blocks per chunk
constexpr int PS_T = 256;                 // threads per chunk workgroup
constexpr int PS_BPT = PS_CHUNK / PS_T;   // blocks per thread in the scan
static_assert(PS_CHUNK % (4 * BS_PER_WAVE) == 0, "waves take whole groups of blocks");

__device__ __forceinline__ DD4 dd4_add(const DD4& a, const DD4& b) { return DD4Add()(a, b); }
__device__ __forceinline__ DD4 dd4_shfl_up(const DD4& v, int o) {
  return DD4{__shfl_up(v.xh, o, 64), __shfl_up(v.xl, o, 64), __shfl_up(v.yh, o, 64), __shfl_up(v.yl, o, 64)};
}

// packed hits: each lane loads four consecutive points (two 16-byte loads), so a 64-point block is one 16-lane row
// and one row-sum pass of the wave gives four blocks' sums; each iteration's 16 blocks land in lanes 0-15, which
// store them with one instruction and add them into per-lane double-double accumulators (one dd4_add for all
// sixteen), summed in lane order at the end.  The order of every sum is fixed (a block: the lane's four points
// pairwise, then the row; the chunk total by lane, then by wave).
constexpr int BS_QUADS = 4;  // four-block groups per wave and iteration
static_assert(PS_CHUNK % (4 * 4 * BS_QUADS) == 0, "waves take whole iterations of blocks");
__device__ __forceinline__ double rows16_sum(double v) {  // every lane: the sum of its 16-lane row
  v += dpp_d<DPP_QP_1032>(v);
  v += dpp_d<DPP_QP_2301>(v);
  v += dpp_d<DPP_ROR4>(v);
  v += dpp_d<DPP_ROR8>(v);
  return v;
}
__global__ void __launch_bounds__(PS_T) chunk_sums_packed_kernel(const uint64_t* __restrict__ hits, int64_t n,
                                                                 double2* __restrict__ bs, DD4* __restrict__ ctot) {
  __shared__ DD4 wt[PS_T / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nblk = (n + 63) >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * PS_CHUNK;
  const bool al16 = (reinterpret_cast<uintptr_t>(hits) & 15) == 0;
  DD4 acc{0.0, 0.0, 0.0, 0.0};  // lane j < 16: blocks j, j + 16, ... of this wave
  constexpr int PER_WAVE = PS_CHUNK / (PS_T / 64);
  constexpr int BPI = 4 * BS_QUADS;  // blocks per iteration
  const int row = lane >> 4, rl = lane & 15;
  for (int g = 0; g < PER_WAVE; g += BPI) {
    const int64_t blk0 = c0 + (int64_t)w * PER_WAVE + g;
    if (blk0 >= nblk) break;  // wave-uniform
    uint64_t h[BS_QUADS][4];
#pragma unroll
    for (int j = 0; j < BS_QUADS; ++j) {
      const int64_t i = (blk0 + 4 * j + row) * 64 + 4 * rl;  // this lane's four points
#pragma unroll
      for (int u = 0; u < 4; ++u) h[j][u] = 0ull;
      if (i + 3 < n && al16) {
        const ulonglong2 q0 = reinterpret_cast<const ulonglong2*>(hits + i)[0];
        const ulonglong2 q1 = reinterpret_cast<const ulonglong2*>(hits + i)[1];
        h[j][0] = q0.x;
        h[j][1] = q0.y;
        h[j][2] = q1.x;
        h[j][3] = q1.y;
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (i + u < n) h[j][u] = hits[i + u];
      }
    }
    double ma = 0.0, mb = 0.0;  // lane k < 16: block k of the iteration
#pragma unroll
    for (int j = 0; j < BS_QUADS; ++j) {
      double v[4], q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = (double)__uint_as_float((uint32_t)(h[j][u] >> 32));
        q[u] = ((uint32_t)h[j][u] >> 31) != 0u ? 0.0 : v[u] * v[u];
      }
      const double s = rows16_sum((v[0] + v[1]) + (v[2] + v[3]));
      const double t = rows16_sum((q[0] + q[1]) + (q[2] + q[3]));
      const double a0 = readlane_d(s, 0), a1 = readlane_d(s, 16), a2 = readlane_d(s, 32), a3 = readlane_d(s, 48);
      const double b0 = readlane_d(t, 0), b1 = readlane_d(t, 16), b2 = readlane_d(t, 32), b3 = readlane_d(t, 48);
      if ((lane >> 2) == j) {
        const int r = lane & 3;
        ma = r == 0 ? a0 : r == 1 ? a1 : r == 2 ? a2 : a3;
        mb = r == 0 ? b0 : r == 1 ? b1 : r == 2 ? b2 : b3;
      }
    }
    if (lane < BPI && blk0 + lane < nblk) {
      const DD4 d{ma, 0.0, mb, 0.0};
      bs[blk0 + lane] = make_double2(ma, mb);
      acc = dd4_add(acc, d);
    }
  }
  DD4 t = acc;  // lane 0 gathers lanes 1..15 in order
#pragma unroll
  for (int j = 1; j < BPI; ++j) {
    const DD4 o{__shfl(acc.xh, j, 64), __shfl(acc.xl, j, 64), __shfl(acc.yh, j, 64), __shfl(acc.yl, j, 64)};
    t = dd4_add(t, o);
  }
  if (lane == 0) wt[w] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    DD4 c = wt[0];
#pragma unroll
    for (int i = 1; i < PS_T / 64; ++i) c = dd4_add(c, wt[i]);
    ctot[blockIdx.x] = c;
  }
}

template <int FMT>
__global__ void __launch_bounds__(PS_T) chunk_sums_kernel(const void* __restrict__ hits,
                                                          const double* __restrict__ hit_vals, int64_t n,
                                                          double2* __restrict__ bs, DD4* __restrict__ ctot) {
  __shared__ DD4 wt[PS_T / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nblk = (n + 63) >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * PS_CHUNK;
  DD4 acc{0.0, 0.0, 0.0, 0.0};  // lane 0: this wave's blocks, in order
  constexpr int PER_WAVE = PS_CHUNK / (PS_T / 64);
  for (int g = 0; g < PER_WAVE; g += BS_PER_WAVE) {
    const int64_t blk0 = c0 + (int64_t)w * PER_WAVE + g;
    if (blk0 >= nblk) break;  // wave-uniform
    double v[BS_PER_WAVE];
    bool dup[BS_PER_WAVE];
#pragma unroll
    for (int j = 0; j < BS_PER_WAVE; ++j) {
      const int64_t i = (blk0 + j) * 64 + lane;
      v[j] = 0.0;
      dup[j] = false;
      if (i < n) {
        if constexpr (FMT == SMG_HITS_PACKED_F32) {
          const uint64_t h = reinterpret_cast<const uint64_t*>(hits)[i];
          v[j] = (double)__uint_as_float((uint32_t)(h >> 32));
          dup[j] = ((uint32_t)h >> 31) != 0u;
        } else {
          v[j] = hit_vals[i];
          dup[j] = (reinterpret_cast<const uint32_t*>(hits)[i] >> 31) != 0u;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < BS_PER_WAVE; ++j) {
      const double a = wave_sum_dpp(v[j]), b = wave_sum_dpp(dup[j] ? 0.0 : v[j] * v[j]);
      if (lane == 0 && blk0 + j < nblk) {
        const DD4 d{a, 0.0, b, 0.0};
        bs[blk0 + j] = make_double2(a, b);
        acc = dd4_add(acc, d);
      }
    }
  }
  if (lane == 0) wt[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    DD4 t = wt[0];
#pragma unroll
    for (int i = 1; i < PS_T / 64; ++i) t = dd4_add(t, wt[i]);
    ctot[blockIdx.x] = t;
  }
}

// exclusive scan of the chunk totals in one workgroup: each thread a run of chunks, the thread totals scanned in
// each wave (shuffles, fixed order) and across the waves (the 16 wave totals in order, in LDS)
constexpr int PSB_T = 1024;
__global__ void __launch_bounds__(PSB_T) chunk_base_kernel(const DD4* __restrict__ ctot, int64_t nch,
                                                           DD4* __restrict__ cbase) {
  __shared__ DD4 wt[PSB_T / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t per = (nch + PSB_T - 1) / PSB_T;
  const int64_t a = t * per, b = a + per < nch ? a + per : nch;
  DD4 s{0.0, 0.0, 0.0, 0.0};
  for (int64_t i = a; i < b; ++i) s = dd4_add(s, ctot[i]);
  DD4 incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const DD4 y = dd4_shfl_up(incl, o);
    if (lane >= o) incl = dd4_add(y, incl);
  }
  if (lane == 63) wt[w] = incl;
  __syncthreads();
  DD4 run{0.0, 0.0, 0.0, 0.0};
  for (int i = 0; i < w; ++i) run = dd4_add(run, wt[i]);
  const DD4 ex = dd4_shfl_up(incl, 1);
  if (lane > 0) run = dd4_add(run, ex);
  for (int64_t i = a; i < b; ++i) {
    cbase[i] = run;
    run = dd4_add(run, ctot[i]);
  }
}

// each chunk's inclusive prefixes from its base: a thread scans PS_BPT consecutive blocks, the thread totals are
// combined in order through the waves and the LDS; out[b] = sums over blocks [0, b]
__global__ void __launch_bounds__(PS_T) chunk_scan_kernel(const double2* __restrict__ bs, const DD4* __restrict__ cbase,
                                                          int64_t nblk, DD4* __restrict__ out) {
  __shared__ DD4 wt[PS_T / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * PS_CHUNK + (int64_t)threadIdx.x * PS_BPT;
  DD4 loc[PS_BPT];
  DD4 s{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 0; j < PS_BPT; ++j) {
    const double2 q = b0 + j < nblk ? bs[b0 + j] : make_double2(0.0, 0.0);
    const DD4 x{q.x, 0.0, q.y, 0.0};
    s = dd4_add(s, x);
    loc[j] = s;
  }
  // exclusive prefix of the thread totals within the wave (in lane order), then across the waves
  DD4 incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const DD4 y = dd4_shfl_up(incl, o);
    if (lane >= o) incl = dd4_add(y, incl);
  }
  if (lane == 63) wt[w] = incl;
  __syncthreads();
  DD4 base = cbase[blockIdx.x];
  for (int i = 0; i < w; ++i) base = dd4_add(base, wt[i]);
  DD4 ex = dd4_shfl_up(incl, 1);
  if (lane > 0) base = dd4_add(base, ex);
#pragma unroll
  for (int j = 0; j < PS_BPT; ++j)
    if (b0 + j < nblk) out[b0 + j] = dd4_add(base, loc[j]);
}

}  // namespace smg

using namespace smg;

extern "C" {

#ifndef SMG_GIT_REV
#define SMG_GIT_REV "unknown"
#endif
const char* smg_version(void) { return "smg 0.2.0 (gfx950) git " SMG_GIT_REV; }

const char* smg_last_error(void) { return g_last_error.c_str(); }

int smg_pack_hits(const int64_t* sp_off, const int32_t* pixel_map, int64_t n_spectra, const float* ints,
                  int64_t n_points, uint64_t* hits, void* stream) {
  SMG_CHECK_ARG(n_spectra >= 0 && n_points >= 0, "negative sizes");
  if (n_spectra == 0 || n_points == 0) return SMG_OK;
  SMG_CHECK_ARG(sp_off && pixel_map && ints && hits, "null pointer");
  const int64_t grid = n_spectra < (1 << 20) ? n_spectra : (1 << 20);
  hipLaunchKernelGGL(pack_hits_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), sp_off,
                     pixel_map, n_spectra, ints, hits);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_flag_duplicates(const int64_t* sp_off, int64_t n_spectra, const float* mz, uint64_t* hits,
                        int64_t n_points, double ppm, const uint8_t* force, uint8_t* flag_state, void* stream) {
  SMG_CHECK_ARG(n_spectra >= 0 && n_points >= 0 && ppm >= 0 && ppm < 1e6, "bad arguments");
  if (n_spectra == 0 || n_points == 0) return SMG_OK;
  SMG_CHECK_ARG(sp_off && mz && hits, "null pointer");
  const int64_t grid = n_spectra < (1 << 20) ? n_spectra : (1 << 20);
  hipLaunchKernelGGL(flag_duplicates_kernel, dim3((unsigned)grid), dim3(FLAG_THREADS), 0, as_stream(stream), sp_off,
                     n_spectra, mz, hits, ppm, force, flag_state);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

// smg_sort_points / smg_sort_points_flag: smg_sort.hip

int smg_window_bounds(const double* peak_mz, const int64_t* order, int64_t n_windows, double ppm,
                      const float* mz_sorted, int64_t n_points, int64_t* lo, int64_t* hi, void* stream) {
  SMG_CHECK_ARG(n_windows >= 0 && n_points >= 0, "negative sizes");
  if (n_windows == 0) return SMG_OK;
  SMG_CHECK_ARG(peak_mz && lo && hi && (mz_sorted || n_points == 0), "null pointer");
  const int64_t grid = (n_windows + 255) / 256;
  hipLaunchKernelGGL(window_bounds_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), peak_mz,
                     order, n_windows, ppm, mz_sorted, n_points, lo, hi);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

// one thread per ion: its scored windows' runs (layout window or empty) and its table-row flag
__global__ void align_windows_kernel(const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
                                     const int64_t* __restrict__ win_off, const int64_t* __restrict__ kt_off,
                                     const uint8_t* __restrict__ sel, int64_t n_ions, int64_t* __restrict__ lo2,
                                     int64_t* __restrict__ hi2, uint8_t* __restrict__ keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ions) return;
  const int64_t w0 = win_off[i], nw = win_off[i + 1] - w0;
  const int64_t t0 = kt_off[i], nt = kt_off[i + 1] - t0;
  bool has = false, hit = false;
  for (int64_t k = 0; k < nw; ++k) {
    const int64_t a = lo[w0 + k], b = hi[w0 + k];
    has |= b > a;
    if (k < nt) {
      lo2[t0 + k] = a;
      hi2[t0 + k] = b;
      hit |= (k < 32) && (b > a);
    }
  }
  for (int64_t k = nw; k < nt; ++k) lo2[t0 + k] = hi2[t0 + k] = 0;
  keep[i] = (has && hit && (!sel || sel[i])) ? 1 : 0;
}

int smg_align_windows(const int64_t* lo, const int64_t* hi, const int64_t* win_off, const int64_t* kt_off,
                      const uint8_t* sel, int64_t n_ions, int64_t* lo2, int64_t* hi2, uint8_t* keep, void* stream) {
  SMG_CHECK_ARG(n_ions >= 0, "negative size");
  if (n_ions == 0) return SMG_OK;
  SMG_CHECK_ARG(lo && hi && win_off && kt_off && lo2 && hi2 && keep, "null pointer");
  hipLaunchKernelGGL(align_windows_kernel, dim3((unsigned)((n_ions + 255) / 256)), dim3(256), 0, as_stream(stream),
                     lo, hi, win_off, kt_off, sel, n_ions, lo2, hi2, keep);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_sample_spectra(const int64_t* sp_off, const double* mzs, const double* cum_ints, int64_t n_spectra,
                       const double* lower, const double* upper, int64_t n_windows, int64_t* out_window,
                       int64_t* out_spectrum, double* out_value, int64_t capacity, int64_t* count,
                       void* stream) {
  SMG_CHECK_ARG(n_spectra >= 0 && n_windows >= 0 && capacity >= 0, "negative sizes");
  SMG_CHECK_ARG(count != nullptr, "null count");
  SMG_HIP(hipMemsetAsync(count, 0, sizeof(int64_t), as_stream(stream)));
  if (n_spectra == 0 || n_windows == 0) return SMG_OK;
  SMG_CHECK_ARG(n_spectra < 65536, "n_spectra too large for the legacy sampler grid");
  dim3 grid((unsigned)((n_windows + 255) / 256), (unsigned)n_spectra);
  hipLaunchKernelGGL(sample_spectra_kernel, grid, dim3(256), 0, as_stream(stream), sp_off, mzs, cum_ints,
                     n_spectra, lower, upper, n_windows, out_window, out_spectrum, out_value, capacity,
                     reinterpret_cast<unsigned long long*>(count));
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

static hipError_t slice_scan(void* tmp, size_t& bytes, const int64_t* in, int64_t* out, int64_t n, hipStream_t st) {
  return rocprim::exclusive_scan(tmp, bytes, in, out, (int64_t)0, (size_t)n, rocprim::plus<int64_t>(), st, false);
}

int smg_slice_mz_workspace_size(int64_t n_spectra, size_t* bytes) {
  SMG_CHECK_ARG(bytes != nullptr && n_spectra >= 0, "bad arguments");
  size_t b0 = 0;
  hipError_t e = slice_scan(nullptr, b0, nullptr, nullptr, n_spectra + 1, 0);
  if (e != hipSuccess) {
    set_error("rocprim scan workspace query failed: %s", hipGetErrorString(e));
    return SMG_ERR_HIP;
  }
  *bytes = 256 + 2 * (((size_t)(n_spectra + 1) * 8 + 255) / 256 * 256) + b0;
  return SMG_OK;
}

int smg_slice_mz_count(const int64_t* sp_off, int64_t n_spectra, const float* mz, double lo, double hi,
                       int64_t* out_sp_off, void* workspace, size_t workspace_bytes, void* stream) {
  SMG_CHECK_ARG(n_spectra >= 0 && sp_off && out_sp_off, "bad arguments");
  hipStream_t st = as_stream(stream);
  if (n_spectra == 0) {
    SMG_HIP(hipMemsetAsync(out_sp_off, 0, sizeof(int64_t), st));
    return SMG_OK;
  }
  SMG_CHECK_ARG(mz && workspace, "null pointer");
  size_t need = 0;
  int rc = smg_slice_mz_workspace_size(n_spectra, &need);
  if (rc) return rc;
  if (workspace_bytes < need) {
    set_error("slice workspace too small: %zu < %zu", workspace_bytes, need);
    return SMG_ERR_WORKSPACE;
  }
  unsigned char* w = reinterpret_cast<unsigned char*>(workspace) + 256;
  const size_t arr = ((size_t)(n_spectra + 1) * 8 + 255) / 256 * 256;
  int64_t* first = reinterpret_cast<int64_t*>(w);
  int64_t* count = reinterpret_cast<int64_t*>(w + arr);
  unsigned char* tmp = w + 2 * arr;
  size_t tb = need - 256 - 2 * arr;
  SMG_HIP(hipMemsetAsync(count + n_spectra, 0, sizeof(int64_t), st));
  hipLaunchKernelGGL(slice_count_kernel, dim3((unsigned)((n_spectra + 255) / 256)), dim3(256), 0, st, sp_off,
                     n_spectra, mz, lo, hi, first, count);
  SMG_LAUNCH_CHECK();
  SMG_HIP(slice_scan(tmp, tb, count, out_sp_off, n_spectra + 1, st));
  return SMG_OK;
}

int smg_slice_mz_copy(const int64_t* sp_off, int64_t n_spectra, const float* mz, const uint64_t* hits,
                      const int64_t* out_sp_off, double ppm, const uint8_t* force, float* out_mz,
                      uint64_t* out_hits, const void* workspace, void* stream) {
  SMG_CHECK_ARG(n_spectra >= 0 && ppm >= 0 && ppm < 1e6, "bad arguments");
  if (n_spectra == 0) return SMG_OK;
  SMG_CHECK_ARG(sp_off && mz && hits && out_sp_off && out_mz && out_hits && workspace, "null pointer");
  const int64_t* first = reinterpret_cast<const int64_t*>(reinterpret_cast<const unsigned char*>(workspace) + 256);
  const int64_t nwg = (n_spectra + 3) / 4;
  const int64_t grid = nwg < (1 << 20) ? nwg : (1 << 20);
  hipLaunchKernelGGL(slice_copy_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), sp_off, n_spectra,
                     mz, hits, first, out_sp_off, ppm, force, out_mz, out_hits);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_debug_stream_read(const uint64_t* data, int64_t n_words, uint64_t* out, int32_t n_blocks, void* stream) {
  SMG_CHECK_ARG(data && out && n_words >= 0 && n_blocks > 0, "bad arguments");
  hipStream_t st = as_stream(stream);
  SMG_HIP(hipMemsetAsync(out, 0, (size_t)n_blocks * 8, st));
  hipLaunchKernelGGL(stream_read_kernel, dim3((unsigned)n_blocks), dim3(256), 0, st, data, n_words, out);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int smg_hit_prefix_sums_workspace_size(int64_t n_points, size_t* bytes) {
  SMG_CHECK_ARG(bytes != nullptr && n_points >= 0, "bad arguments");
  const int64_t nblk = (n_points + 63) / 64 > 0 ? (n_points + 63) / 64 : 1;
  const int64_t nch = (nblk + PS_CHUNK - 1) / PS_CHUNK;
  *bytes = 256 + ((size_t)nblk * sizeof(DD4) + 255) / 256 * 256 + 2 * (((size_t)nch * sizeof(DD4) + 255) / 256 * 256);
  return SMG_OK;
}

int smg_hit_prefix_sums(int32_t hit_format, const void* hits, const double* hit_vals, int64_t n_points,
                        double* cum64, void* workspace, size_t workspace_bytes, void* stream) {
  SMG_CHECK_ARG(n_points >= 0, "negative n_points");
  SMG_CHECK_ARG(hit_format == SMG_HITS_PACKED_F32 || hit_format == SMG_HITS_SPLIT_F64, "bad hit_format");
  SMG_CHECK_ARG(cum64 != nullptr, "null pointer");
  hipStream_t st = as_stream(stream);
  SMG_HIP(hipMemsetAsync(cum64, 0, sizeof(DD4), st));
  if (n_points == 0) return SMG_OK;
  SMG_CHECK_ARG(hits && workspace && (hit_format == SMG_HITS_PACKED_F32 || hit_vals), "null pointer");
  size_t need = 0;
  int rc = smg_hit_prefix_sums_workspace_size(n_points, &need);
  if (rc) return rc;
  if (workspace_bytes < need) {
    set_error("prefix-sum workspace too small: %zu < %zu", workspace_bytes, need);
    return SMG_ERR_WORKSPACE;
  }
  const int64_t nblk = (n_points + 63) / 64;
  const int64_t nch = (nblk + PS_CHUNK - 1) / PS_CHUNK;
  if (nch > 0x7FFFFFFF) {
    set_error("too many points for one prefix sum: %lld", (long long)n_points);
    return SMG_ERR_UNSUPPORTED;
  }
  unsigned char* p = reinterpret_cast<unsigned char*>(workspace) + 256;
  double2* bs = reinterpret_cast<double2*>(p);  // a block's two plain f64 sums (its DD4 with zero low parts)
  p += ((size_t)nblk * sizeof(DD4) + 255) / 256 * 256;
  DD4* ctot = reinterpret_cast<DD4*>(p);
  p += ((size_t)nch * sizeof(DD4) + 255) / 256 * 256;
  DD4* cbase = reinterpret_cast<DD4*>(p);
  if (hit_format == SMG_HITS_PACKED_F32)
    hipLaunchKernelGGL(chunk_sums_packed_kernel, dim3((unsigned)nch), dim3(PS_T), 0, st,
                       static_cast<const uint64_t*>(hits), n_points, bs, ctot);
  else
    hipLaunchKernelGGL(chunk_sums_kernel<SMG_HITS_SPLIT_F64>, dim3((unsigned)nch), dim3(PS_T), 0, st, hits,
                       hit_vals, n_points, bs, ctot);
  SMG_LAUNCH_CHECK();
  hipLaunchKernelGGL(chunk_base_kernel, dim3(1), dim3(PSB_T), 0, st, ctot, nch, cbase);
  SMG_LAUNCH_CHECK();
  hipLaunchKernelGGL(chunk_scan_kernel, dim3((unsigned)nch), dim3(PS_T), 0, st, bs, cbase, nblk,
                     reinterpret_cast<DD4*>(cum64) + 1);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
