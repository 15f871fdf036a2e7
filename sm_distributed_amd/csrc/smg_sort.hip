// Global m/z sort of the resident peak list on gfx950: a hand-written stable LSD radix sort of the f32 m/z bit
// patterns carrying the packed 8-byte hits, with the duplicate-candidate flags fused into its first pass.
//
// Reference behaviour (frulo/SM_distributed):
//   formula_imager_segm.py:73-74  sp_df.sort_values('mz') -- the segment's peaks in m/z order (pandas' sort is
//                                 stable for equal m/z only by accident of its algorithm; the windows are sums,
//                                 so only the set of points per window matters; this sort is stable anyway)
//
// Design (DESIGN.md "The m/z sort"):
//   * keys: positive f32 m/z, whose bit patterns order like the values; only the low key_bits bits vary across a
//     dataset (27 for m/z in [100, 1000)), sorted in ceil(key_bits / 9) passes of <= 9-bit digits;
//   * one histogram pass reads the keys once for every pass's digit counts, one tiny scan turns them into bin bases;
//   * each sort pass is a single kernel (a tile of 8192 points per 512-thread workgroup, tiles claimed in order
//     from a ticket counter): wave-private digit ranking by ballot matching, the tile's digit counts published at
//     once and the tile's global bin offsets resolved by a look-back over the earlier tiles' published counts
//     (a tile only waits on tiles with smaller tickets, all of which are resident), then the tile is reordered by
//     digit in LDS so that the stores come out as contiguous runs per digit;
//   * 78 KB of LDS per workgroup (one 64 KB exchange buffer, which holds the wave histograms while ranking, the
//     keys, then the values): two tiles per CU, so one tile's loads overlap the other's ranking and stores;
//   * the duplicate-candidate flags (smg_flag_duplicates) are computed by the histogram pass, which reads the keys
//     in dataset order anyway: a bit per position marks the spectrum starts (from sp_off, one small kernel), so a
//     point's spectrum neighbours are its dataset neighbours across no start (spectra must be m/z-sorted and no
//     pixel shared: the host takes the separate flag pass otherwise); no pixel is read.  The first sort pass sets
//     bit 31 of each hit from one flag bit per position.
// Traffic per pass: 12 B read + 12 B written per point plus 2-8 B of look-back status per 1 KB of tile.
#include <rocprim/device/device_radix_sort.hpp>

#include "smg_common.hpp"

namespace smg {

#ifndef SMG_SRT_IPT
#define SMG_SRT_IPT 16
#endif
#ifndef SMG_SRT_VLOAD  // where the values are loaded: 0 after the keys' stores, 1 before them, 2 after the ranking
#define SMG_SRT_VLOAD 0
#endif
#ifndef SMG_SRT_WPE
#define SMG_SRT_WPE 4
#endif
#ifndef SMG_SRT_LB  // look-back words per round trip
#define SMG_SRT_LB 4
#endif
constexpr int SRT_T = 512;                  // threads per tile
constexpr int SRT_IPT = SMG_SRT_IPT;        // points per thread
constexpr int SRT_TILE = SRT_T * SRT_IPT;   // 8192 points per tile
constexpr int SRT_WAVES = SRT_T / 64;
constexpr int SRT_BINS = 512;               // digits of at most 9 bits
constexpr int SRT_MAXP = 4;                 // passes (31 key bits: 4 x 8)
constexpr int HST_T = 256;

// look-back status word: flag in the top two bits (1 = this tile's count, 2 = inclusive prefix over tiles <= it),
// the value below; 32-bit words while every prefix fits in 30 bits
template <typename S>
struct StatusBits;
template <>
struct StatusBits<uint32_t> {
  static constexpr int SH = 30;
};
template <>
struct StatusBits<unsigned long long> {
  static constexpr int SH = 62;
};

template <typename S>
__device__ __forceinline__ void status_store(S* p, S v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename S>
__device__ __forceinline__ S status_load(const S* p) {
  return __hip_atomic_load(const_cast<S*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exclusive prefix over the 512 threads of a workgroup (red: SRT_WAVES entries of LDS)
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) red[w] = x;
  __syncthreads();
  T off = 0;
#pragma unroll
  for (int i = 0; i < SRT_WAVES; ++i) off += i < w ? red[i] : (T)0;
  return off + x - v;
}

// The duplicate-candidate flag of the point at position i (the flag pass's rule, smg_prep.hip flag_tile_store):
// its spectrum's previous or next point lies within one window width, compared in f64.  m: its m/z, mp / mn: the
// m/z at positions i - 1 / i + 1, st0 / st1: spectrum starts at i / i + 1.
__device__ __forceinline__ bool dup_flag(int64_t i, int64_t n, uint32_t k, uint32_t kp, uint32_t kn, bool st0, bool st1,
                                         double slack) {
  const double m = (double)__uint_as_float(k), mp = (double)__uint_as_float(kp), mn = (double)__uint_as_float(kn);
  const bool fp = i > 0 && !st0 && m - mp <= slack * m;
  const bool fn = i + 1 < n && !st1 && mn - m <= slack * mn;
  return fp || fn;
}

// digit histograms of every pass in one read of the keys: per-workgroup LDS counts, then one global add per bin.
// With flags != nullptr it also writes the duplicate-candidate flag of every point (one bit per position, dataset
// order; spectrum starts in starts[]) for the first sort pass, which then only reads them.
__global__ void __launch_bounds__(HST_T) sort_hist_kernel(const uint32_t* __restrict__ keys, int64_t n, int passes,
                                                          int dbits, unsigned long long* __restrict__ hist,
                                                          const uint32_t* __restrict__ starts,
                                                          uint32_t* __restrict__ flags, double slack) {
  __shared__ uint32_t h[SRT_MAXP * SRT_BINS];
  for (int i = threadIdx.x; i < SRT_MAXP * SRT_BINS; i += HST_T) h[i] = 0;
  __syncthreads();
  const uint32_t mask = (1u << dbits) - 1u;
  auto add = [&](uint32_t k) {
#pragma unroll
    for (int p = 0; p < SRT_MAXP; ++p)
      if (p < passes) atomicAdd(&h[p * SRT_BINS + ((k >> (p * dbits)) & mask)], 1u);
  };
  // the top digit of consecutive points of an m/z-sorted spectrum repeats: for it, a lane's four keys and then
  // a run of lanes with one digit are added at once (LDS atomics on one address serialise)
  const int lane = threadIdx.x & 63;
  const int top = passes - 1;
  auto add4 = [&](const uint4 q) {  // wave-uniform
#pragma unroll
    for (int p = 0; p < SRT_MAXP - 1; ++p) {
      if (p < top) {
        atomicAdd(&h[p * SRT_BINS + ((q.x >> (p * dbits)) & mask)], 1u);
        atomicAdd(&h[p * SRT_BINS + ((q.y >> (p * dbits)) & mask)], 1u);
        atomicAdd(&h[p * SRT_BINS + ((q.z >> (p * dbits)) & mask)], 1u);
        atomicAdd(&h[p * SRT_BINS + ((q.w >> (p * dbits)) & mask)], 1u);
      }
    }
    const int sh = top * dbits;
    const int d0 = (q.x >> sh) & mask, d1 = (q.y >> sh) & mask, d2 = (q.z >> sh) & mask, d3 = (q.w >> sh) & mask;
    const bool same = d0 == d1 && d1 == d2 && d2 == d3;
    if (!same) {
      atomicAdd(&h[top * SRT_BINS + d0], 1u);
      atomicAdd(&h[top * SRT_BINS + d1], 1u);
      atomicAdd(&h[top * SRT_BINS + d2], 1u);
      atomicAdd(&h[top * SRT_BINS + d3], 1u);
    }
    const int sd = same ? d0 : -1;
    const int prev = __shfl_up(sd, 1, 64);
    const bool bound = lane == 0 || prev != sd;
    const uint64_t heads = __ballot(bound);
    const uint64_t later = lane == 63 ? 0ull : heads & ~((2ull << lane) - 1ull);
    const int next = later ? __ffsll((unsigned long long)later) - 1 : 64;
    if (same && bound) atomicAdd(&h[top * SRT_BINS + sd], 4u * (uint32_t)(next - lane));
  };
  const int64_t stride = (int64_t)gridDim.x * HST_T;
  // 16-byte loads where the keys are 16-byte aligned (a torch allocation is; a view may not be)
  const int64_t head = (int64_t)((16 - (reinterpret_cast<uintptr_t>(keys) & 15)) & 15) / 4;
  const int64_t h0 = head < n ? head : n;
  const int64_t n4 = (n - h0) >> 2;
  const uint4* k4 = reinterpret_cast<const uint4*>(keys + h0);
  auto start = [&](int64_t i) -> bool { return i < n && ((starts[i >> 5] >> (i & 31)) & 1u); };
  // flags of one point (positions outside the whole-chunk range: the head, the tail); atomicOr into its word
  auto flag1 = [&](int64_t i) {
    const uint32_t k = keys[i], kp = i > 0 ? keys[i - 1] : 0u, kn = i + 1 < n ? keys[i + 1] : 0u;
    if (dup_flag(i, n, k, kp, kn, start(i), start(i + 1), slack)) atomicOr(&flags[i >> 5], 1u << (i & 31));
  };
  // flags of a chunk's quad: the neighbours come from the adjacent lanes, the chunk's two outer ones from memory;
  // with the chunk 32-point aligned (h0 == 0), eight lanes' nibbles make one flag word, stored by the first of them
  auto flag4 = [&](int64_t ch, const uint4 q) {  // wave-uniform
    const int64_t i = h0 + (ch * 64 + lane) * 4;
    uint32_t kp = __shfl_up(q.w, 1, 64), kn = __shfl_down(q.x, 1, 64);
    if (lane == 0) kp = i > 0 ? keys[i - 1] : 0u;
    if (lane == 63) kn = i + 4 < n ? keys[i + 4] : 0u;
    const uint32_t sw0 = starts[i >> 5], sw1 = starts[(i + 4) >> 5];
    auto st = [&](int j) { const int64_t p = i + j; return ((((p >> 5) == (i >> 5)) ? sw0 : sw1) >> (p & 31)) & 1u; };
    uint32_t nib = (uint32_t)dup_flag(i, n, q.x, kp, q.y, st(0), st(1), slack) |
                   ((uint32_t)dup_flag(i + 1, n, q.y, q.x, q.z, st(1), st(2), slack) << 1) |
                   ((uint32_t)dup_flag(i + 2, n, q.z, q.y, q.w, st(2), st(3), slack) << 2) |
                   ((uint32_t)dup_flag(i + 3, n, q.w, q.z, kn, st(3), i + 4 < n ? st(4) : 0u, slack) << 3);
    if (h0 == 0) {
      uint32_t word = nib;
#pragma unroll
      for (int j = 1; j < 8; ++j) word |= __shfl_down(nib, j, 8) << (4 * j);
      if ((lane & 7) == 0) flags[i >> 5] = word;
    } else if (nib) {
      atomicOr(&flags[i >> 5], nib << (i & 31));
      if ((i & 31) > 28) atomicOr(&flags[(i >> 5) + 1], nib >> (32 - (i & 31)));
    }
  };
  // whole waves over chunks of 64 quads (wave-uniform loop bounds), four chunks' loads in flight per round
  const int64_t nw = stride >> 6, nchunk = n4 >> 6;
  int64_t c = ((int64_t)blockIdx.x * HST_T + threadIdx.x) >> 6;
  for (; c + 3 * nw < nchunk; c += 4 * nw) {
    uint4 q[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) q[r] = k4[(c + r * nw) * 64 + lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      add4(q[r]);
      if (flags) flag4(c + r * nw, q[r]);
    }
  }
  for (; c < nchunk; c += nw) {
    const uint4 q = k4[c * 64 + lane];
    add4(q);
    if (flags) flag4(c, q);
  }
  const int64_t t = (int64_t)blockIdx.x * HST_T + threadIdx.x;
  if (t < h0) {
    add(keys[t]);
    if (flags) flag1(t);
  }
  for (int64_t i = h0 + nchunk * 256 + t; i < n; i += stride) {
    add(keys[i]);
    if (flags) flag1(i);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < passes * SRT_BINS; i += HST_T)
    if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

// bin bases: exclusive prefix of each pass's digit counts (one workgroup per pass)
__global__ void __launch_bounds__(SRT_BINS) sort_scan_kernel(const unsigned long long* __restrict__ hist,
                                                             int64_t* __restrict__ binbase) {
  __shared__ int64_t red[SRT_WAVES];
  const int p = blockIdx.x, d = threadIdx.x;
  binbase[p * SRT_BINS + d] = block_excl_scan<int64_t>((int64_t)hist[p * SRT_BINS + d], red);
}

// the digits' bases of one pass from their totals (reduce-then-scan: no histogram pass)
__global__ void __launch_bounds__(SRT_BINS) sort_digit_base_kernel(const int64_t* __restrict__ total,
                                                                   int64_t* __restrict__ binbase) {
  __shared__ int64_t red[SRT_WAVES];
  const int d = threadIdx.x;
  binbase[d] = block_excl_scan<int64_t>(total[d], red);
}

// FLAG pass: one bit per point position marking the first point of a spectrum (sp_off; an empty spectrum marks
// its successor's start, which that one marks anyway)
__global__ void __launch_bounds__(256) sort_mark_starts_kernel(const int64_t* __restrict__ sp_off, int64_t n_spectra,
                                                               int64_t n, uint32_t* __restrict__ bits) {
  for (int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x; s < n_spectra; s += (int64_t)gridDim.x * 256) {
    const int64_t o = sp_off[s];
    if (o < n) atomicOr(&bits[o >> 5], 1u << (o & 31));
  }
}

// Reduce-then-scan offsets of one pass (no look-back chain: each tile's global offsets are known before its
// scatter).  sort_count_kernel: every tile's digit counts, tile-major (counts[t][d], coalesced); sort_chunk_sum_kernel:
// per chunk of SRT_CT tiles, each digit's total; sort_chunk_scan_kernel: per digit, the exclusive prefix over the chunks
// from the digit's base; sort_tile_offsets_kernel: per chunk, each tile's offsets (in place of its counts).  The
// scan reads ~2 x 4 B per tile and digit; the count pass re-reads the keys (4 B per point).
constexpr int SRT_CT = 64;  // tiles per chunk of the offsets scan
// With flags != nullptr (the first pass of flag_and_sort) it also writes the duplicate-candidate flag of every point
// of the tile (one bit per dataset position; spectrum starts in starts[]), the rule of dup_flag: the keys are read
// in dataset order here, a quad per lane, the neighbours of a quad's ends from the adjacent lanes (or memory).
template <typename S>
__global__ void __launch_bounds__(SRT_T) sort_count_kernel(const uint32_t* __restrict__ kin, int64_t n, int shift,
                                                           int dbits, S* __restrict__ counts,
                                                           const uint32_t* __restrict__ starts,
                                                           uint32_t* __restrict__ flags, double slack) {
  static_assert(SRT_T == SRT_BINS && SRT_IPT % 4 == 0, "a thread per digit; keys in 16-byte loads");
  __shared__ uint32_t h[SRT_BINS];
  const int tid = threadIdx.x, lane = tid & 63;
  h[tid] = 0u;
  __syncthreads();
  const int64_t t = blockIdx.x, base = t * SRT_TILE;
  const uint32_t mask = (1u << dbits) - 1u;
  auto start = [&](int64_t i) -> uint32_t { return i < n ? (starts[i >> 5] >> (i & 31)) & 1u : 0u; };
  if (base + SRT_TILE <= n && (reinterpret_cast<uintptr_t>(kin) & 15) == 0) {
    const uint4* k4 = reinterpret_cast<const uint4*>(kin + base);
    uint4 q[SRT_IPT / 4];
#pragma unroll
    for (int u = 0; u < SRT_IPT / 4; ++u) q[u] = k4[u * SRT_T + tid];
#pragma unroll
    for (int u = 0; u < SRT_IPT / 4; ++u) {
      atomicAdd(&h[(q[u].x >> shift) & mask], 1u);
      atomicAdd(&h[(q[u].y >> shift) & mask], 1u);
      atomicAdd(&h[(q[u].z >> shift) & mask], 1u);
      atomicAdd(&h[(q[u].w >> shift) & mask], 1u);
    }
    if (flags != nullptr) {
#pragma unroll
      for (int u = 0; u < SRT_IPT / 4; ++u) {
        const int64_t i = base + (int64_t)(u * SRT_T + tid) * 4;  // 32-point aligned per 8 lanes (base % 32 == 0)
        uint32_t kp = __shfl_up(q[u].w, 1, 64), kn = __shfl_down(q[u].x, 1, 64);
        if (lane == 0) kp = i > 0 ? kin[i - 1] : 0u;
        if (lane == 63) kn = i + 4 < n ? kin[i + 4] : 0u;
        const uint32_t sw = starts[i >> 5];
        auto st = [&](int j) { return (sw >> ((i + j) & 31)) & 1u; };  // j < 4: the quad's word
        const uint32_t st4 = ((i + 4) & 31) ? st(4) : start(i + 4);
        const uint32_t nib = (uint32_t)dup_flag(i, n, q[u].x, kp, q[u].y, st(0), st(1), slack) |
                             ((uint32_t)dup_flag(i + 1, n, q[u].y, q[u].x, q[u].z, st(1), st(2), slack) << 1) |
                             ((uint32_t)dup_flag(i + 2, n, q[u].z, q[u].y, q[u].w, st(2), st(3), slack) << 2) |
                             ((uint32_t)dup_flag(i + 3, n, q[u].w, q[u].z, kn, st(3), st4, slack) << 3);
        uint32_t word = nib;
#pragma unroll
        for (int j = 1; j < 8; ++j) word |= __shfl_down(nib, j, 8) << (4 * j);
        if ((lane & 7) == 0) flags[i >> 5] = word;
      }
    }
  } else {
    for (int64_t i = base + tid; i < n && i < base + SRT_TILE; i += SRT_T) {
      const uint32_t k = kin[i];
      atomicAdd(&h[(k >> shift) & mask], 1u);
      if (flags != nullptr) {
        const uint32_t kp = i > 0 ? kin[i - 1] : 0u, kn = i + 1 < n ? kin[i + 1] : 0u;
        if (dup_flag(i, n, k, kp, kn, start(i), start(i + 1), slack)) atomicOr(&flags[i >> 5], 1u << (i & 31));
      }
    }
  }
  __syncthreads();
  counts[t * SRT_BINS + tid] = (S)h[tid];
}
template <typename S>
__global__ void __launch_bounds__(SRT_BINS) sort_chunk_sum_kernel(const S* __restrict__ counts, int64_t ntiles,
                                                                  S* __restrict__ ctot) {
  const int d = threadIdx.x;
  const int64_t c = blockIdx.x, t0 = c * SRT_CT, t1 = t0 + SRT_CT < ntiles ? t0 + SRT_CT : ntiles;
  S s = 0;
  for (int64_t t = t0; t < t1; ++t) s += counts[t * SRT_BINS + d];
  ctot[c * SRT_BINS + d] = s;
}
// one workgroup per digit: the exclusive prefix of its chunk totals (1024 chunks per round, a carried base)
constexpr int SRT_SCAN_T = 1024;
// (binbase == nullptr: the prefixes start at 0 and the digit's total goes to total[d]; the bases are added when the
// tiles' offsets are formed, sort_tile_offsets_kernel)
template <typename S>
__global__ void __launch_bounds__(SRT_SCAN_T) sort_chunk_scan_kernel(S* __restrict__ ctot, int64_t nchunks,
                                                                     const int64_t* __restrict__ binbase,
                                                                     int64_t* __restrict__ total) {
  __shared__ S wsum[SRT_SCAN_T / 64];
  const int d = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  S run = binbase != nullptr ? (S)binbase[d] : (S)0;
  for (int64_t c0 = 0; c0 < nchunks; c0 += SRT_SCAN_T) {
    const int64_t c = c0 + tid;
    const S x = c < nchunks ? ctot[c * SRT_BINS + d] : (S)0;
    S inc = x;  // inclusive prefix within the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const S y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    S before = run, all = 0;
#pragma unroll
    for (int i = 0; i < SRT_SCAN_T / 64; ++i) {
      const S t = wsum[i];
      before += i < w ? t : (S)0;
      all += t;
    }
    if (c < nchunks) ctot[c * SRT_BINS + d] = before + inc - x;
    run += all;
    __syncthreads();
  }
  if (total != nullptr && tid == 0) total[d] = (int64_t)run;
}
template <typename S>
__global__ void __launch_bounds__(SRT_BINS) sort_tile_offsets_kernel(S* __restrict__ counts, int64_t ntiles,
                                                                     const S* __restrict__ ctot,
                                                                     const int64_t* __restrict__ binbase) {
  const int d = threadIdx.x;
  const int64_t c = blockIdx.x, t0 = c * SRT_CT, t1 = t0 + SRT_CT < ntiles ? t0 + SRT_CT : ntiles;
  S run = ctot[c * SRT_BINS + d] + (binbase != nullptr ? (S)binbase[d] : (S)0);
  for (int64_t t = t0; t < t1; ++t) {
    const S x = counts[t * SRT_BINS + d];
    counts[t * SRT_BINS + d] = run;
    run += x;
  }
}

// One LSD pass over digit bits [shift, shift + dbits).  FLAG: the first pass, which also sets the duplicate-
// candidate flag (bit 31 of the hit) from the dataset-order neighbours.
// Values go through LDS whole (8-byte words) when a tile's values fit the 64 KB exchange buffer, else as two
// rounds of 4-byte halves (SPLIT; the second round's loads hit the lines the first one brought into L2).
template <typename S, bool FLAG>
__global__ void __launch_bounds__(SRT_T, SMG_SRT_WPE) sort_pass_kernel(const uint32_t* __restrict__ kin,
                                                                    const uint64_t* __restrict__ vin,
                                                                    uint32_t* __restrict__ kout,
                                                                    uint64_t* __restrict__ vout, int64_t n, int shift,
                                                                    int dbits, const int64_t* __restrict__ binbase,
                                                                    S* __restrict__ status,
                                                                    unsigned* __restrict__ ticket,
                                                                    const uint32_t* __restrict__ flagbits,
                                                                    const S* __restrict__ offsets) {
  constexpr bool SPLIT = SRT_TILE * 8 > 65536;
  constexpr int XWORDS = 65536 / 8;
  // exchange buffer: the wave histograms (u16 [SRT_WAVES][SRT_BINS]) while ranking, then the tile's keys in digit
  // order, then its values (or value halves)
  __shared__ __attribute__((aligned(16))) uint64_t xbuf[XWORDS];
  __shared__ int64_t s_gbase[SRT_BINS];   // global position of the tile's first point of each digit, minus its
  __shared__ uint32_t s_lstart[SRT_BINS]; // local start (so that position = s_gbase[d] + local index)
  __shared__ int64_t s_red[SRT_WAVES];
  __shared__ unsigned s_tile;
  static_assert(SRT_TILE * 4 <= 65536, "the keys of a tile must fit the exchange buffer");
  static_assert(SRT_TILE <= 65536, "wave ranks are packed in 16 bits");
  constexpr int SH = StatusBits<S>::SH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint16_t* wh = reinterpret_cast<uint16_t*>(xbuf);
  uint32_t* xk = reinterpret_cast<uint32_t*>(xbuf);
  reinterpret_cast<uint4*>(xbuf)[tid] = make_uint4(0u, 0u, 0u, 0u);  // 512 x 16 B: the 8 KB of wave histograms
  // Look-back: tiles in ticket order.  Reduce-then-scan (offsets given): XCD x takes tiles from its own contiguous
  // eighth of the input (ticket[x]; HW_REG_XCC_ID says which XCD this is), then steals from the next ones when its
  // eighth is done; its scattered runs into each digit's range then abut in its own L2 (consecutive tiles' pieces of
  // one line merge there instead of reaching HBM as partial lines from two XCDs).  Each block takes one tile, so
  // every tile is taken exactly once.
  if (tid == 0) {
    if (offsets == nullptr) {
      s_tile = atomicAdd(ticket, 1u);
    } else {
      const int home = home_xcd();
      const int64_t nt = gridDim.x, q = nt / XCDS, r = nt % XCDS;
      for (int i = 0; i < XCDS; ++i) {
        const int64_t x = (home + i) % XCDS, a = x * q + (x < r ? x : r), len = q + (x < r ? 1 : 0);
        const unsigned k = atomicAdd(ticket + x, 1u);
        if ((int64_t)k < len) {
          s_tile = (unsigned)(a + k);
          break;
        }
      }
    }
  }
  __syncthreads();
  const int64_t t = s_tile;
  const int64_t base = t * SRT_TILE;
  const int64_t wbase = base + (int64_t)w * (64 * SRT_IPT);  // a wave's points: SRT_IPT rows of 64 consecutive
  const uint32_t mask = (1u << dbits) - 1u;
  const int nb = 1 << dbits;
  const bool full = base + SRT_TILE <= n;

  // keys first; the values are loaded after the ranking (held through it with the keys, they would spill).  Past
  // the end: the last digit, after every real point of the tile (never stored).
  uint32_t k[SRT_IPT];
  if (full) {
#pragma unroll
    for (int u = 0; u < SRT_IPT; ++u) k[u] = kin[wbase + u * 64 + lane];
  } else {
#pragma unroll
    for (int u = 0; u < SRT_IPT; ++u) {
      const int64_t i = wbase + u * 64 + lane;
      k[u] = i < n ? kin[i] : 0xFFFFFFFFu;
    }
  }

  // ranking: each wave counts its rows in order (row u, lane) -- the stable order of its points -- into its own
  // u16 histogram; the lanes of one digit find each other with one ballot per digit bit
  uint32_t rk[SRT_IPT];
  uint16_t* myh = wh + w * SRT_BINS;
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int u = 0; u < SRT_IPT; ++u) {
    const uint32_t d = (k[u] >> shift) & mask;
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 9; ++b) {  // bits at and above dbits are 0 in every lane: those ballots change nothing
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      peers &= bit ? bal : ~bal;
    }
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    const uint32_t old = myh[d];
    if (below == 0) myh[d] = (uint16_t)(old + (uint32_t)__popcll(peers));
    rk[u] = (old + below) | (d << 16);  // the digit rides along (one register per point, not two)
  }
  __syncthreads();

  // per digit (one thread each): wave prefixes, the tile's count, published at once for later tiles' look-back
  const int d = tid;
  uint32_t cnt = 0;
  if (d < nb) {
#pragma unroll
    for (int ww = 0; ww < SRT_WAVES; ++ww) {
      const uint32_t c = wh[ww * SRT_BINS + d];
      wh[ww * SRT_BINS + d] = (uint16_t)cnt;
      cnt += c;
    }
    if (offsets == nullptr) status_store(status + t * SRT_BINS + d, (S)((t == 0 ? (S)2 : (S)1) << SH) | (S)cnt);
  }
  const uint32_t lstart = (uint32_t)block_excl_scan<int64_t>((int64_t)cnt, s_red);
  if (d < nb) {
    int64_t excl = 0;
#ifndef SMG_SRT_NOLB
#define SMG_SRT_NOLB 0  // diagnostic (timing only, wrong order): no look-back; every tile writes from its bin's start
#endif
    if (offsets != nullptr) {
      excl = (int64_t)offsets[t * SRT_BINS + d] - binbase[d];  // (the offsets include the bin base)
    } else if (t > 0 && !SMG_SRT_NOLB) {
      // SMG_SRT_LB earlier tiles' words loaded together per round trip, consumed newest first until an inclusive
      // prefix; a word not yet published ends the round (the ones before it are kept, the walk resumes there)
      for (int64_t j = t - 1;;) {
        S sw[SMG_SRT_LB];
#pragma unroll
        for (int q = 0; q < SMG_SRT_LB; ++q)
          sw[q] = j - q >= 0 ? status_load(status + (j - q) * SRT_BINS + d) : (S)((S)2 << SH);
        int used = SMG_SRT_LB;
        bool done = false;
#pragma unroll
        for (int q = 0; q < SMG_SRT_LB; ++q) {
          if (done || used < SMG_SRT_LB) continue;
          const uint32_t fl = (uint32_t)(sw[q] >> SH);
          if (fl == 0) {
            used = q;
            continue;
          }
          excl += (int64_t)(sw[q] & (((S)1 << SH) - 1));
          if (fl == 2) done = true;
        }
        if (done) break;
        j -= used;
        if (used < SMG_SRT_LB) __builtin_amdgcn_s_sleep(1);
      }
      status_store(status + t * SRT_BINS + d, (S)((S)2 << SH) | (S)(excl + cnt));
    }
    s_gbase[d] = binbase[d] + excl - (int64_t)lstart;
    s_lstart[d] = lstart;
  }
  __syncthreads();

  // local index of each point in digit order, then the keys through LDS
#pragma unroll
  for (int u = 0; u < SRT_IPT; ++u) {
    const uint32_t dd = rk[u] >> 16;
    rk[u] = (rk[u] & 0xFFFFu) + s_lstart[dd] + wh[w * SRT_BINS + dd];
  }
  __syncthreads();  // the wave histograms are overwritten below
#pragma unroll
  for (int u = 0; u < SRT_IPT; ++u) xk[rk[u]] = k[u];
  __syncthreads();
  const int64_t left = n - base;
  const int nvalid = left < SRT_TILE ? (int)left : SRT_TILE;
  uint32_t dj[(SRT_IPT + 1) / 2];  // the digit of each slot this thread stores, two per word
#pragma unroll
  for (int u = 0; u < SRT_IPT; ++u) {
    const int j = u * SRT_T + tid;
    const uint32_t kk = xk[j];
    const uint32_t dd = (kk >> shift) & mask;
    if (u & 1)
      dj[u >> 1] |= dd << 16;
    else
      dj[u >> 1] = dd;
    if (j < nvalid) kout[s_gbase[dd] + j] = kk;
  }
  auto slot_digit = [&](int u) { return (dj[u >> 1] >> ((u & 1) * 16)) & 0xFFFFu; };
  // FLAG: the duplicate-candidate flags were computed by the histogram pass (one bit per dataset position, in
  // flagbits).  The wave's SRT_IPT rows of 64 points are 2 * SRT_IPT consecutive flag words: one load (a word per
  // lane) beside the values', then row u's word comes from lane 2u + (lane >> 5).  Read here, after the keys are
  // out of registers (held from the start, they spilled), and as one memory instruction instead of one per row
  // (bits past n are never stored)
  static_assert(SRT_IPT <= 32 && 2 * SRT_IPT <= 64, "a flag word per lane");
  uint32_t fw = 0u;
  if constexpr (FLAG) {
    const int64_t fw0 = wbase >> 5, nfw = (n + 31) >> 5;
    fw = (lane < 2 * SRT_IPT && fw0 + lane < nfw) ? flagbits[fw0 + lane] : 0u;
  }
  auto flag_of = [&](int u) -> bool {
    const uint32_t word = (uint32_t)__shfl((int)fw, 2 * u + (lane >> 5), 64);
    return ((word >> (lane & 31)) & 1u) != 0u;
  };

  if constexpr (!SPLIT) {
    // the values (not loaded before: with the keys they would spill)
    uint64_t v[SRT_IPT];
    if (full) {
#pragma unroll
      for (int u = 0; u < SRT_IPT; ++u) v[u] = vin[wbase + u * 64 + lane];
    } else {
#pragma unroll
      for (int u = 0; u < SRT_IPT; ++u) {
        const int64_t i = wbase + u * 64 + lane;
        v[u] = i < n ? vin[i] : 0ull;
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SRT_IPT; ++u) {
      uint64_t x = v[u];
      if constexpr (FLAG) x = flag_of(u) ? (x | 0x80000000ull) : (x & ~0x80000000ull);
      xbuf[rk[u]] = x;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SRT_IPT; ++u) {
      const int j = u * SRT_T + tid;
      if (j < nvalid) vout[s_gbase[slot_digit(u)] + j] = xbuf[j];
    }
  } else {
    const uint32_t* vw = reinterpret_cast<const uint32_t*>(vin);
    uint32_t* ow = reinterpret_cast<uint32_t*>(vout);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      uint32_t v[SRT_IPT];
      if (full) {
#pragma unroll
        for (int u = 0; u < SRT_IPT; ++u) v[u] = vw[2 * (wbase + u * 64 + lane) + half];
      } else {
#pragma unroll
        for (int u = 0; u < SRT_IPT; ++u) {
          const int64_t i = wbase + u * 64 + lane;
          v[u] = i < n ? vw[2 * i + half] : 0u;
        }
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < SRT_IPT; ++u) {
        uint32_t x = v[u];
        if (FLAG && half == 0) x = flag_of(u) ? (x | 0x80000000u) : (x & ~0x80000000u);
        xk[rk[u]] = x;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < SRT_IPT; ++u) {
        const int j = u * SRT_T + tid;
        if (j < nvalid) ow[2 * (s_gbase[slot_digit(u)] + j) + half] = xk[j];
      }
    }
  }
}

// ---- host side ---------------------------------------------------------------------------------------------
struct SortPlan {
  int passes, dbits;
  int64_t ntiles, nchunks;
  bool wide;  // 64-bit look-back words
  size_t off_hist, off_base, off_status, status_bytes, off_s0, start_bytes, off_fl, off_tk, off_tv, total;
};

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

static SortPlan sort_plan(int64_t n, int key_bits) {
  SortPlan p;
  p.passes = (key_bits + 8) / 9;
  if (p.passes < 1) p.passes = 1;
  p.dbits = (key_bits + p.passes - 1) / p.passes;
  if (p.dbits < 1) p.dbits = 1;
  p.ntiles = (n + SRT_TILE - 1) / SRT_TILE;
  p.wide = n >= (int64_t(1) << 30);
  const size_t sw = p.wide ? 8 : 4;
  p.off_hist = 256;  // [0, 256): the passes' ticket counters
  p.off_base = p.off_hist + SRT_MAXP * SRT_BINS * 8;
  p.off_status = p.off_base + SRT_MAXP * SRT_BINS * 8;
  // two look-back regions, used by alternate passes: the region of pass p >= 2 is zeroed again after pass p - 2
  // (the workspace does not grow with the number of passes: ~2 B per point at 64-bit words)
  p.status_bytes = (size_t)(p.passes < 2 ? p.passes : 2) * (size_t)p.ntiles * SRT_BINS * sw;
  // reduce-then-scan (the default): the tiles' counts / offsets and the chunk totals in the same space
  p.nchunks = (p.ntiles + SRT_CT - 1) / SRT_CT;
  const size_t rts = (size_t)(p.ntiles + p.nchunks) * SRT_BINS * sw;
  if (p.status_bytes < rts) p.status_bytes = rts;
  p.off_s0 = align_up(p.off_status + p.status_bytes, 256);  // FLAG pass: spectrum-start bits
  p.start_bytes = (size_t)((n + 31) / 32 + 2) * 4;
  p.off_fl = align_up(p.off_s0 + p.start_bytes, 256);  // FLAG pass: the flag bits (the same size)
  p.off_tk = align_up(p.off_fl + p.start_bytes, 256);
  p.off_tv = align_up(p.off_tk + (size_t)n * 4, 256);
  p.total = p.off_tv + (size_t)n * 8;
  return p;
}

// 0 = rocPRIM onesweep (A/B reference), 1 = the hand-written sort with reduce-then-scan tile offsets and XCD-contiguous
// tiles (default; 9.85 ms at config 3), 2 = the same with decoupled look-back in ticket order (round 3; 11.15 ms,
// profiles/round4/r4sort3_*)
static int g_sort_impl = 1;

#ifndef SMG_SORT_RADIX_BITS
#define SMG_SORT_RADIX_BITS 9
#endif
#ifndef SMG_SORT_BLOCK
#define SMG_SORT_BLOCK 512
#endif
#ifndef SMG_SORT_IPT
#define SMG_SORT_IPT 16
#endif
#ifndef SMG_HIST_BLOCK
#define SMG_HIST_BLOCK 512
#endif
#ifndef SMG_HIST_IPT
#define SMG_HIST_IPT 64
#endif
// the library sort kept for A/B timing (smg_debug_sort_impl(0)): onesweep, three 9-bit passes, 512 x 16 tiles
// (its best configuration on MI355X, scripts/sort_ab.sh)
using RocSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<SMG_HIST_BLOCK, SMG_HIST_IPT>,
                                        rocprim::kernel_config<SMG_SORT_BLOCK, SMG_SORT_IPT>, SMG_SORT_RADIX_BITS,
                                        rocprim::block_radix_rank_algorithm::match>>;

static int roc_workspace(int64_t n, size_t* bytes) {
  size_t tb = 0;
  const uint32_t* kin = nullptr;
  uint32_t* kout = nullptr;
  const uint64_t* vin = nullptr;
  uint64_t* vout = nullptr;
  hipError_t e = rocprim::radix_sort_pairs<RocSortConfig>(nullptr, tb, kin, kout, vin, vout, (size_t)n, 0, 31,
                                                          (hipStream_t)0, false);
  if (e != hipSuccess) {
    set_error("rocprim workspace query failed: %s", hipGetErrorString(e));
    return SMG_ERR_HIP;
  }
  *bytes = tb;
  return SMG_OK;
}

template <typename S>
static int run_passes(const SortPlan& P, const uint32_t* mz, const uint64_t* hits, int64_t n, uint32_t* ko,
                      uint64_t* vo, unsigned char* ws, bool flag, double slack, hipStream_t st) {
  const size_t region = (size_t)P.ntiles * SRT_BINS;  // look-back words per pass
  const uint32_t* flagbits = reinterpret_cast<const uint32_t*>(ws + P.off_fl);
  unsigned* tickets = reinterpret_cast<unsigned*>(ws);
  const int64_t* binbase = reinterpret_cast<const int64_t*>(ws + P.off_base);
  S* status = reinterpret_cast<S*>(ws + P.off_status);
  uint32_t* tk = reinterpret_cast<uint32_t*>(ws + P.off_tk);
  uint64_t* tv = reinterpret_cast<uint64_t*>(ws + P.off_tv);
  const uint32_t* ki = mz;
  const uint64_t* vi = hits;
  const bool rts = g_sort_impl != 2;
  S* counts = status;                                   // reduce-then-scan: [ntiles][bins] counts, then offsets
  S* ctot = status + (size_t)P.ntiles * SRT_BINS;       // [nchunks][bins] chunk totals, then chunk offsets
  for (int p = 0; p < P.passes; ++p) {
    // the last pass writes the caller's arrays, the ones before alternate with the workspace copy
    const bool to_out = ((P.passes - 1 - p) & 1) == 0;
    uint32_t* kdst = to_out ? ko : tk;
    uint64_t* vdst = to_out ? vo : tv;
    S* sp = status + (size_t)(p & 1) * region;
    const S* offs = nullptr;
    if (rts) {
      // counts (with the duplicate flags in the first pass of flag_and_sort), chunk totals, the digits' totals and
      // bases (no histogram pass), the tiles' offsets
      int64_t* bb = const_cast<int64_t*>(binbase) + p * SRT_BINS;
      int64_t* totals = reinterpret_cast<int64_t*>(ws + P.off_hist);
      const bool fl0 = flag && p == 0;
      hipLaunchKernelGGL(sort_count_kernel<S>, dim3((unsigned)P.ntiles), dim3(SRT_T), 0, st, ki, n, p * P.dbits,
                         P.dbits, counts, fl0 ? reinterpret_cast<const uint32_t*>(ws + P.off_s0) : nullptr,
                         fl0 ? const_cast<uint32_t*>(flagbits) : nullptr, slack);
      hipLaunchKernelGGL(sort_chunk_sum_kernel<S>, dim3((unsigned)P.nchunks), dim3(SRT_BINS), 0, st, counts,
                         P.ntiles, ctot);
      hipLaunchKernelGGL(sort_chunk_scan_kernel<S>, dim3(SRT_BINS), dim3(SRT_SCAN_T), 0, st, ctot, P.nchunks,
                         (const int64_t*)nullptr, totals);
      hipLaunchKernelGGL(sort_digit_base_kernel, dim3(1), dim3(SRT_BINS), 0, st, totals, bb);
      hipLaunchKernelGGL(sort_tile_offsets_kernel<S>, dim3((unsigned)P.nchunks), dim3(SRT_BINS), 0, st, counts,
                         P.ntiles, ctot, bb);
      SMG_LAUNCH_CHECK();
      offs = counts;
    } else if (p >= 2) {
      SMG_HIP(hipMemsetAsync(sp, 0, region * sizeof(S), st));  // pass p - 2's look-back words
    }
    unsigned* tk_p = rts ? tickets + XCDS * p : tickets + p;  // (reduce-then-scan: one counter per XCD and pass)
    if (flag && p == 0)
      hipLaunchKernelGGL((sort_pass_kernel<S, true>), dim3((unsigned)P.ntiles), dim3(SRT_T), 0, st, ki, vi, kdst,
                         vdst, n, p * P.dbits, P.dbits, binbase + p * SRT_BINS, sp, tk_p, flagbits, offs);
    else
      hipLaunchKernelGGL((sort_pass_kernel<S, false>), dim3((unsigned)P.ntiles), dim3(SRT_T), 0, st, ki, vi, kdst,
                         vdst, n, p * P.dbits, P.dbits, binbase + p * SRT_BINS, sp, tk_p, nullptr, offs);
    SMG_LAUNCH_CHECK();
    ki = kdst;
    vi = vdst;
  }
  return SMG_OK;
}

static int native_sort(const float* mz, const uint64_t* hits, int64_t n, int key_bits, float* mz_sorted,
                       uint64_t* hits_sorted, void* workspace, size_t workspace_bytes, bool flag, double ppm,
                       const int64_t* sp_off, int64_t n_spectra, hipStream_t st) {
  const SortPlan P = sort_plan(n, key_bits);
  if (workspace_bytes < P.total) {
    set_error("sort workspace too small: %zu < %zu", workspace_bytes, P.total);
    return SMG_ERR_WORKSPACE;
  }
  if (P.ntiles > 0x7FFFFFFF) {
    set_error("too many points for one sort: %lld", (long long)n);
    return SMG_ERR_UNSUPPORTED;
  }
  unsigned char* ws = reinterpret_cast<unsigned char*>(workspace);
  const bool rts = g_sort_impl != 2;  // reduce-then-scan: no histogram pass, no look-back words
  // tickets, histograms and the first two passes' look-back words start at zero
  SMG_HIP(hipMemsetAsync(ws, 0, rts ? P.off_status : P.off_status + P.status_bytes, st));
  const uint32_t* keys = reinterpret_cast<const uint32_t*>(mz);
  if (flag) {  // spectrum starts first: the histogram pass computes the flags from them
    SMG_HIP(hipMemsetAsync(ws + P.off_s0, 0, P.off_fl + P.start_bytes - P.off_s0, st));  // start and flag bits
    int64_t g = (n_spectra + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(sort_mark_starts_kernel, dim3((unsigned)g), dim3(256), 0, st, sp_off, n_spectra, n,
                       reinterpret_cast<uint32_t*>(ws + P.off_s0));
    SMG_LAUNCH_CHECK();
  }
  const double slack = 2.0 * ppm * 1e-6 / (1.0 - ppm * 1e-6) * (1.0 + 1e-9);
  if (!rts) {  // look-back form: every pass's digit bases (and the flags) from one read of the keys first
    int64_t hb = (n + (int64_t)HST_T * 16 - 1) / ((int64_t)HST_T * 16);
    if (hb > 2048) hb = 2048;
    hipLaunchKernelGGL(sort_hist_kernel, dim3((unsigned)hb), dim3(HST_T), 0, st, keys, n, P.passes, P.dbits,
                       reinterpret_cast<unsigned long long*>(ws + P.off_hist),
                       flag ? reinterpret_cast<const uint32_t*>(ws + P.off_s0) : nullptr,
                       flag ? reinterpret_cast<uint32_t*>(ws + P.off_fl) : nullptr, slack);
    SMG_LAUNCH_CHECK();
    hipLaunchKernelGGL(sort_scan_kernel, dim3((unsigned)P.passes), dim3(SRT_BINS), 0, st,
                       reinterpret_cast<const unsigned long long*>(ws + P.off_hist),
                       reinterpret_cast<int64_t*>(ws + P.off_base));
    SMG_LAUNCH_CHECK();
  }
  uint32_t* ko = reinterpret_cast<uint32_t*>(mz_sorted);
  return P.wide ? run_passes<unsigned long long>(P, keys, hits, n, ko, hits_sorted, ws, flag, slack, st)
                : run_passes<uint32_t>(P, keys, hits, n, ko, hits_sorted, ws, flag, slack, st);
}

}  // namespace smg

using namespace smg;

extern "C" {

int smg_sort_points_workspace_size(int64_t n_points, size_t* bytes) {
  SMG_CHECK_ARG(bytes != nullptr && n_points >= 0, "bad arguments");
  size_t roc = 0;
  int rc = roc_workspace(n_points, &roc);
  if (rc) return rc;
  const size_t mine = sort_plan(n_points, 31).total;  // the most passes any key width takes
  *bytes = (roc > mine ? roc : mine) + 256;
  return SMG_OK;
}

static int sort_args(const float* mz, const uint64_t* hits, int64_t n_points, int32_t* key_bits, float* mz_sorted,
                     uint64_t* hits_sorted, void* workspace, size_t workspace_bytes, size_t* need) {
  SMG_CHECK_ARG(n_points >= 0, "negative n_points");
  SMG_CHECK_ARG(*key_bits >= 0 && *key_bits <= 31, "key_bits must be in [0, 31] (0 = all 31)");
  if (*key_bits == 0) *key_bits = 31;
  if (n_points == 0) return SMG_OK;
  SMG_CHECK_ARG(mz && hits && mz_sorted && hits_sorted && workspace, "null pointer");
  SMG_CHECK_ARG((const void*)mz != (const void*)mz_sorted && (const void*)hits != (const void*)hits_sorted,
                "the sort is not in place");
  int rc = smg_sort_points_workspace_size(n_points, need);
  if (rc) return rc;
  if (workspace_bytes < *need) {
    set_error("sort workspace too small: %zu < %zu", workspace_bytes, *need);
    return SMG_ERR_WORKSPACE;
  }
  return SMG_OK;
}

int smg_sort_points(const float* mz, const uint64_t* hits, int64_t n_points, int32_t key_bits, float* mz_sorted,
                    uint64_t* hits_sorted, void* workspace, size_t workspace_bytes, void* stream) {
  size_t need = 0;
  int rc = sort_args(mz, hits, n_points, &key_bits, mz_sorted, hits_sorted, workspace, workspace_bytes, &need);
  if (rc || n_points == 0) return rc;
  if (g_sort_impl == 0) {
    size_t tb = need - 256;
    // positive float32 keys order like their bit patterns; bit 31 (sign) is always 0
    SMG_HIP(rocprim::radix_sort_pairs<RocSortConfig>(workspace, tb, reinterpret_cast<const uint32_t*>(mz),
                                                     reinterpret_cast<uint32_t*>(mz_sorted), hits, hits_sorted,
                                                     (size_t)n_points, 0, (unsigned)key_bits, as_stream(stream),
                                                     false));
    return SMG_OK;
  }
  return native_sort(mz, hits, n_points, key_bits, mz_sorted, hits_sorted, workspace, workspace_bytes, false, 0.0,
                     nullptr, 0, as_stream(stream));
}

int smg_sort_points_flag(const int64_t* sp_off, int64_t n_spectra, const float* mz, const uint64_t* hits,
                         int64_t n_points, int32_t key_bits, double ppm, float* mz_sorted, uint64_t* hits_sorted,
                         void* workspace, size_t workspace_bytes, void* stream) {
  SMG_CHECK_ARG(ppm >= 0 && ppm < 1e6, "bad ppm");
  SMG_CHECK_ARG(n_spectra >= 1 || n_points == 0, "a dataset with points has spectra");
  SMG_CHECK_ARG(sp_off != nullptr || n_points == 0, "null sp_off");
  size_t need = 0;
  int rc = sort_args(mz, hits, n_points, &key_bits, mz_sorted, hits_sorted, workspace, workspace_bytes, &need);
  if (rc || n_points == 0) return rc;
  return native_sort(mz, hits, n_points, key_bits, mz_sorted, hits_sorted, workspace, workspace_bytes, true, ppm,
                     sp_off, n_spectra, as_stream(stream));
}

int smg_debug_sort_impl(int32_t which) {
  SMG_CHECK_ARG(which >= 0 && which <= 2, "which: 0 = rocPRIM, 1 = hand-written (reduce-then-scan), 2 = hand-written (look-back)");
  g_sort_impl = which;
  return SMG_OK;
}

}  // extern "C"
