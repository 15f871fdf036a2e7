// Fused ion imaging + MSM scoring on gfx950.
//
// One ion = K theoretical isotope windows.  Window w's image is the run [lo[w], hi[w]) of the
// m/z-sorted hit array (pixel, intensity); duplicate pixels are summed (coo.toarray()).
// Replaces, in frulo/SM_distributed:
//   formula_imager_segm.py:84-92   per-window COO construction   (_gen_iso_images)
//   formula_imager_segm.py:95-109  per-ion image list             (_img_pairs_to_list)
//   formula_img_validator.py:72-84 compute(): spectral / spatial / chaos
//   pyImagingMSpec 0.1.1 isotope_pattern_match / isotope_image_correlation,
//   cpyImagingMSpec 0.0.4 measure_of_chaos   (restated, see oracle/msm_oracle.py)
//
// Three passes (launch_metrics):
//  * main LDS pass (ion_pipe_kernel<512>): persistent, software-pipelined; two 512-thread workgroups per CU,
//    one ion at a time per workgroup with the principal image in LDS (pixel bitmap + rank prefix + f64 values),
//    the other isotope windows streamed once and joined against it, measure_of_chaos by the threshold
//    decomposition of flat morphology (Kruskal over eL with an LDS union-find).  See the kernel's comment.
//  * big-ion LDS pass (ion_pipe_kernel<1024>): the same code with one 1024-thread workgroup per CU and the
//    whole LDS, over the main pass's rejects (principal window > 2560 points, duplicate-list overflow).
//  * dense path (ion_dense_kernel): persistent workgroups with a global-memory scratch slot of N_px-sized
//    images, for what the LDS passes cannot take (K > 8, principal window > 8192 points, images > 2^18 px).
#include <stdarg.h>

#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "smg_common.hpp"
#include "smg_ion.hpp"

namespace smg {

constexpr int BLOCK = 256;           // dense (global-scratch) kernel
constexpr int NW = BLOCK / WAVE;

// Diagnostic build only (-DSMG_STAMPS): per-phase wall cycles of the LDS kernel, summed over workgroups
// into a buffer of their own (read back by smg_debug_stamps); the shipped build executes no stamp.
#ifdef SMG_STAMPS
__device__ unsigned long long g_stamps[16];
// thread 0 of each workgroup accumulates its phase cycles in LDS and adds them to g_stamps once at exit
#define STAMP_DECL()                                               \
  __shared__ unsigned long long _sacc[16];                         \
  unsigned long long _st0 = 0, _st1 = 0;                           \
  if (threadIdx.x == 0) {                                          \
    for (int _i = 0; _i < 16; ++_i) _sacc[_i] = 0;                 \
    _st0 = __builtin_amdgcn_s_memtime();                           \
  }
#define STAMP_INIT()
#define STAMP(i)                                                   \
  do {                                                             \
    if (threadIdx.x == 0) {                                        \
      _st1 = __builtin_amdgcn_s_memtime();                         \
      _sacc[i] += _st1 - _st0;                                     \
      _st0 = _st1;                                                 \
    }                                                              \
  } while (0)
#define STAMP_FLUSH()                                              \
  do {                                                             \
    if (threadIdx.x == 0)                                          \
      for (int _i = 0; _i < 16; ++_i) atomicAdd(&g_stamps[_i], _sacc[_i]); \
  } while (0)
#else
#define STAMP_DECL()
#define STAMP_INIT()
#define STAMP(i)
#define STAMP_FLUSH()
#endif



// formula_img_validator.py:78-84 + the restated pyImagingMSpec functions; writes the outputs.
__device__ void finalize_ion(int K, const double* __restrict__ t, const double* s, double sx, double sxx,
                             const double* sy, const double* syy, const double* sxy, double npx,
                             double chaos_raw, int64_t ion, uint32_t flags, double* oc, double* osp,
                             double* osc, double* omsm, uint32_t* oflags) {
  // isotope_pattern_match
  double tt = 0.0, ss = 0.0;
  for (int k = 0; k < K; ++k) {
    tt += t[k] * t[k];
    ss += s[k] * s[k];
  }
  const double nt = sqrt(tt), ns = sqrt(ss);
  double acc = 0.0;
  for (int k = 0; k < K; ++k) acc += fabs(t[k] / nt - s[k] / ns);
  double spectral = 1.0 - acc / (double)K;
  if (spectral == 1.0) spectral = 0.0;

  // isotope_image_correlation: np.corrcoef rows, weights = theor[1:]
  double spatial = 0.0;
  if (K >= 2) {
    const double n1 = npx - 1.0;
    const double sxx_c = (sxx - sx * sx / npx) / n1;
    const double sd0 = sqrt(sxx_c);
    double num = 0.0, den = 0.0;
    for (int k = 1; k < K; ++k) {
      const double syy_c = (syy[k] - sy[k] * sy[k] / npx) / n1;
      const double sxy_c = (sxy[k] - sx * sy[k] / npx) / n1;
      double r = sxy_c / sqrt(syy_c) / sd0;
      if (!isnan(r)) r = r > 1.0 ? 1.0 : (r < -1.0 ? -1.0 : r);
      if (isinf(r)) r = 0.0;
      num += r * t[k];
      den += t[k];
    }
    spatial = num / den;
  }

  double chaos = chaos_raw;
  if (!isnan(chaos) && fabs(chaos - 1.0) <= 1e-8 + 1e-5) chaos = 0.0;  // np.isclose(moc, 1.0)

  chaos = clean(chaos);
  spatial = clean(spatial);
  spectral = clean(spectral);
  oc[ion] = chaos;
  osp[ion] = spatial;
  osc[ion] = spectral;
  omsm[ion] = chaos * spatial * spectral;
  oflags[ion] = flags;
}

template <int NW_ = NW>
__device__ __forceinline__ double block_max(double v, double* scratch) {
  constexpr int NW = NW_;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_max(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  double m = scratch[0];
  for (int w = 1; w < NW; ++w) m = scratch[w] > m ? scratch[w] : m;
  __syncthreads();
  return m;
}

// ---------------------------------------------------------------------------------------------
// LDS bitmap + rank helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool bm_test(const uint32_t* bm, int p) { return (bm[p >> 5] >> (p & 31)) & 1u; }

__device__ __forceinline__ int bm_rank(const uint32_t* bm, const uint16_t* pf, int p) {
  const uint64_t w = reinterpret_cast<const uint64_t*>(bm)[p >> 6];
  const uint64_t m = (p & 63) ? (w & ((1ull << (p & 63)) - 1ull)) : 0ull;
  return (int)pf[p >> 6] + __popcll(m);
}

// exclusive popcount prefix over the first n <= CAP 64-bit words w: thread t scans WPT consecutive words
// serially, thread totals are scanned across the wave (DPP) and the waves.  Returns the total.
template <int NW_, int CAP>
__device__ int prefix_words(const uint64_t* w, uint16_t* pf, int n, int* wscratch) {
  constexpr int NW = NW_;
  constexpr int WPT = (CAP + NW * WAVE - 1) / (NW * WAVE);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int a = tid * WPT;
  int c[WPT];
  int tot = 0;
#pragma unroll
  for (int i = 0; i < WPT; ++i) {
    c[i] = (a + i < n) ? __popcll(w[a + i]) : 0;
    tot += c[i];
  }
  const int inc = wave_incl_scan_dpp(tot);
  if (lane == 63) wscratch[wid] = inc;
  __syncthreads();
  int off = inc - tot, all = 0;
#pragma unroll
  for (int v = 0; v < NW; ++v) {
    const int x = wscratch[v];
    off += (v < wid) ? x : 0;
    all += x;
  }
#pragma unroll
  for (int i = 0; i < WPT; ++i) {
    if (a + i < n) pf[a + i] = (uint16_t)off;
    off += c[i];
  }
  __syncthreads();
  return all;
}

// the same over the pixel bitmap (n64 <= NPX_LDS_MAX/64 words)
template <int NW_>
__device__ int bm_build_prefix(const uint32_t* bm, uint16_t* pf, int n64, int* wscratch) {
  static_assert((NPX_LDS_MAX / 64) % WAVE == 0, "prefix geometry");
  return prefix_words<NW_, NPX_LDS_MAX / 64>(reinterpret_cast<const uint64_t*>(bm), pf, n64, wscratch);
}

// bits of image row `row`, columns c0..c0+6 (bit j <-> column c0+j), masked by the valid-column mask cv;
// 0 outside the image.  c0 >= -3: the bitmap has a zero guard word in front (Lay::o_guard).
__device__ __forceinline__ uint32_t bits7(const uint32_t* bm, int row, int c0, uint32_t cv, const Params& P) {
  const bool rv = (unsigned)row < (unsigned)P.nrows;
  const int st = (rv ? row : 0) * P.ncols + c0;
  const int w = st >> 5;
  const uint32_t v = __builtin_amdgcn_alignbit(bm[w + 1], bm[w], (uint32_t)(st & 31)) & cv;
  return rv ? v : 0u;
}


// LDS carve of the persistent kernel.  Everything but the pixel bitmap and its rank prefix has a
// compile-time offset (immediate ds_* offsets, no offset SGPRs); the bitmap (npx bits, a zero guard word in
// front) and the prefix (one u16 per 64-bit word) come last and are sized at run time (Params::w32, o_pf).
static inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }
static constexpr uint32_t cal16(uint32_t x) { return (x + 15u) & ~15u; }
constexpr int DSEG = 64;   // deferred duplicate-candidate tail points per wave and ion (NW * DSEG = block)
constexpr int DTBL = 512;  // their (pixel, window)-keyed sum table
template <int NW, int CAPC>
struct Lay {
  static constexpr uint32_t o_vals = 0;                                // principal f64 values, rank order
  static constexpr uint32_t o_L = cal16(o_vals + (uint32_t)CAPC * 8);  // level index, rank order
  static constexpr uint32_t o_filt = cal16(o_L + CAPC);  // tail duplicate lists, later the chaos E arrays
  static constexpr uint32_t o_dkey = o_filt;                             // [NW][DSEG] (pixel << 3 | window)
  static constexpr uint32_t o_dval = cal16(o_dkey + NW * DSEG * 4);      // [NW][DSEG] values
  static constexpr uint32_t o_dcnt = cal16(o_dval + NW * DSEG * 8);      // [NW] entries per wave
  static constexpr uint32_t o_tkey = cal16(o_dcnt + NW * 4);              // (pixel, window)-keyed f64 sums
  static constexpr uint32_t o_tval = cal16(o_tkey + DTBL * 4);
  static constexpr uint32_t filt_bytes = (o_tval + DTBL * 8 - o_filt) > 5u * CAPC ? (o_tval + DTBL * 8 - o_filt)
                                                                                 : 5u * CAPC;
  static constexpr uint32_t o_part = cal16(o_filt + filt_bytes);  // [MAXK][NW][4] per-wave window partials
  static constexpr uint32_t o_red = cal16(o_part + MAXK * NW * 4 * 8);
  static constexpr uint32_t o_ctr = cal16(o_red + 8 * NW * 8);
  static constexpr uint32_t o_wsc = cal16(o_ctr + C_NCTR * 4);
  static constexpr uint32_t o_desc = cal16(o_wsc + NW * 4);  // two ion descriptors (current, next)
  static constexpr uint32_t o_guard = cal16(o_desc + 2 * 384);
  static constexpr uint32_t o_bm = o_guard + 16;
  static int w32(int npx) { return (((npx + 31) / 32 + 2) + 3) & ~3; }
  static uint32_t o_pf(int npx) { return cal16(o_bm + (uint32_t)w32(npx) * 4); }
  static size_t bytes(int npx) { return cal16(o_pf(npx) + (uint32_t)(w32(npx) / 2) * 2); }
};

// Two-level carve for images above NPX_LDS_MAX pixels (ion_pipe_kernel<..., TWO = true>): the principal
// pixel set is kept as its non-empty 64-pixel words only, compacted in word order (W[r] at o_bm, their rank
// prefix B[r] at o_B), behind a top-level bitmap of words (T at o_T, one bit per 64-pixel word, two zero guard
// words at the end) with its own rank prefix (TP at Params::o_pf).  W holds up to CAPC words (a word per
// principal point at worst), so LDS no longer scales with the image: 1000x1000 px needs 2 KB of T.
template <int NW, int CAPC>
struct Lay2 : Lay<NW, CAPC> {
  using Base = Lay<NW, CAPC>;
  static constexpr uint32_t o_B = cal16(Base::o_desc + 2 * 384);
  static constexpr uint32_t o_guard = cal16(o_B + (uint32_t)CAPC * 2);
  static constexpr uint32_t o_bm = o_guard + 16;
  static constexpr uint32_t o_T = o_bm + (uint32_t)CAPC * 8;
  __host__ __device__ static int nT(int npx) { return ((((npx + 63) / 64) / 64 + 2) + 1) & ~1; }  // even: uint4 zeroing
  // u32 words of W and T together (zeroed as one range, like the direct bitmap)
  static int w32(int npx) { return (int)((CAPC * 8 + nT(npx) * 8) / 4); }
  static uint32_t o_pf(int npx) { return o_T + (uint32_t)nT(npx) * 8; }
  static size_t bytes(int npx) { return cal16(o_pf(npx) + (uint32_t)nT(npx) * 2); }
  static_assert(CAPC % 2 == 0, "W zeroed in uint4s");
};
constexpr int NPX_TWO_MAX = 1 << 23;  // two-level pass: top-level prefix over <= 2^23/4096 + 2 words
constexpr int TOPCAP = NPX_TWO_MAX / 4096 + 2;

// The digit of an MSD radix-select pass: over the 256 bin counts (16-B aligned), the bin d whose cumulative count
// first exceeds k (four bins per lane, one DPP scan, one ballot), computed by every wave for itself (no broadcast):
// returns d, sets k to k minus the count below d and cnt to the count of d (wave-uniform).
__device__ __forceinline__ int hist_find(const uint32_t* hist, int& k, int& cnt) {
  const int lane = threadIdx.x & 63;
  const uint4 c = reinterpret_cast<const uint4*>(hist)[lane];
  const int s4 = (int)(c.x + c.y + c.z + c.w);
  const int incl = wave_incl_scan_dpp(s4);
  const uint64_t over = __ballot(incl > k);
  const int L = over ? __ffsll((unsigned long long)over) - 1 : WAVE - 1;
  const int b0 = incl - s4, b1 = b0 + (int)c.x, b2 = b1 + (int)c.y, b3 = b2 + (int)c.z;
  const int j = b1 > k ? 0 : b2 > k ? 1 : b3 > k ? 2 : 3;  // (no indexed array: it would live in scratch)
  const int base = j == 0 ? b0 : j == 1 ? b1 : j == 2 ? b2 : b3;
  const int cj = (int)(j == 0 ? c.x : j == 1 ? c.y : j == 2 ? c.z : c.w);
  const int d = __shfl(4 * lane + j, L, WAVE);
  const int kb = __shfl(k - base, L, WAVE);
  cnt = __shfl(cj, L, WAVE);
  k = kb;
  return d;
}

// The i0-th smallest (0-based) of a set of positive doubles and, with pair, the (i0 + 1)-th (i0 + 1 < n): an MSD
// radix select over the f64 bit patterns (positive values: ordered like the values), one 8-bit LDS histogram per
// byte (two buffers in turn: a pass clears the next one while every wave reads the current one, so a pass takes two
// barriers), that stops as soon as the selected byte prefix holds a single element (it is then fetched whole),
// usually after three or four of the eight bytes.  The next order statistic is then the smallest element above the
// prefix, found in the same fetch pass; after a select down to the last byte (the element repeats) it is the same
// value when more elements than needed equal it, else the smallest value above it (one more pass).  visit(f) calls
// f(bits) for each element this thread owns (any partition of the set over the NT threads of the block; called once
// per pass, so it must enumerate the same set every time).  hist: 2 x 256 u32 (16-B aligned), sh: 1 int, dsh: 2 u64
// of LDS.
// lo, hi: the bit patterns of the set's smallest and largest elements when known (else 0, ~0): the passes start at
// the first byte where they differ (the bytes above it are common to every element), and none runs when they agree.
template <int NT, class Visit>
__device__ void select_pair(Visit&& visit, int i0, bool pair, uint32_t* hist, int* sh, unsigned long long* dsh,
                            double& a, double& b, uint64_t lo = 0ull, uint64_t hi = ~0ull) {
  const int tid = threadIdx.x;
  const uint64_t diff = lo ^ hi;
  if (diff == 0ull) {  // every element is the same value
    a = b = __longlong_as_double((long long)lo);
    return;
  }
  const int top = (63 - __clzll((long long)diff)) & ~7;  // shift of the highest differing byte
  uint64_t mask = top == 56 ? 0ull : ~((1ull << (top + 8)) - 1ull);
  uint64_t prefix = lo & mask;
  int k = i0;
  for (int i = tid; i < 256; i += NT) hist[i] = 0u;
  if (tid == 0) dsh[0] = dsh[1] = ~0ull;
  __syncthreads();
  int cur = 0;
  bool fetched = false;
  for (int shift = top; shift >= 0; shift -= 8) {
    uint32_t* h = hist + 256 * cur;
    visit([&](uint64_t bits) {
      if ((bits & mask) == prefix) atomicAdd(&h[(bits >> shift) & 255u], 1u);
    });
    __syncthreads();
    int cnt;
    const int d = hist_find(h, k, cnt);
    for (int i = tid; i < 256; i += NT) hist[256 * (cur ^ 1) + i] = 0u;  // the next pass's buffer
    cur ^= 1;
    prefix |= (uint64_t)d << shift;
    mask |= 255ull << shift;
    if (cnt == 1 && shift > 0) {  // a single element carries the prefix: it is the one, the next is above the prefix
      uint64_t abv = ~0ull;
      visit([&](uint64_t bits) {
        const uint64_t mb = bits & mask;
        if (mb == prefix) dsh[0] = bits;
        else if (mb > prefix) abv = bits < abv ? bits : abv;
      });
      if (pair && abv != ~0ull) atomicMin(&dsh[1], (unsigned long long)abv);
      __syncthreads();
      prefix = dsh[0];
      fetched = true;
      break;
    }
    __syncthreads();  // the next buffer is clear before the next pass's adds
  }
  a = __longlong_as_double((long long)prefix);
  b = a;
  if (!pair || fetched) {
    if (pair) b = __longlong_as_double((long long)dsh[1]);  // i0 + 1 < n: an element lies above
    __syncthreads();  // (dsh is read above before any later use of the scratch)
    return;
  }
  __syncthreads();
  if (tid == 0) {
    sh[0] = 0;
    *dsh = ~0ull;
  }
  __syncthreads();
  int le = 0;
  uint64_t above = ~0ull;
  visit([&](uint64_t bits) {
    if (bits <= prefix) ++le;
    else above = bits < above ? bits : above;
  });
  if (le) atomicAdd(&sh[0], le);
  if (above != ~0ull) atomicMin(dsh, (unsigned long long)above);
  __syncthreads();
  if (sh[0] < i0 + 2) b = __longlong_as_double((long long)*dsh);  // fewer than i0 + 2 elements <= a
  __syncthreads();
}

// np.percentile(positive values, q) ('linear' method: numpy's _compute_virtual_index with alpha = beta = 1,
// _get_indexes, _get_gamma, _lerp) of the n > 0 positive values visit enumerates (select_pair's contract)
template <int NT, class Visit>
__device__ double percentile_of(Visit&& visit, int n, double q, uint32_t* hist, int* sh, unsigned long long* dsh,
                                uint64_t lo = 0ull, uint64_t hi = ~0ull) {
  const double qq = q / 100.0;
  const double vi = (double)n * qq + (1.0 + qq * (1.0 - 1.0 - 1.0)) - 1.0;
  int i0, i1;
  double gamma;
  if (vi >= (double)(n - 1)) {
    i0 = i1 = n - 1;
    gamma = 0.0;
  } else if (vi < 0.0) {
    i0 = i1 = 0;
    gamma = 0.0;
  } else {
    i0 = (int)floor(vi);
    i1 = i0 + 1;
    gamma = vi - floor(vi);
  }
  double a, b;
  select_pair<NT>(visit, i0, i1 != i0, hist, sh, dsh, a, b, lo, hi);
  const double d = b - a;
  return gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
}

// The q-th percentiles of several sets at once (the hot-spot clip's tail images): one MSD radix select per set (the
// scheme of select_pair, percentile_of's index arithmetic), all sets of a batch of SB advancing together so that
// each round reads the elements once for every set in it (the tail windows' points come from HBM / L2: one latency
// per round instead of one per set and pass).  State per set in LDS; wave j finishes the round of the batch's set j
// (its 256-bin histogram: the digit, then the bins cleared for the next round).  visit(f) calls f(set, bits) for
// every element this thread owns (the same partition every round); n[set]: the set's size (0: no clip, thr +inf).
struct SelSet {
  unsigned long long prefix, mask, dsh;  // selected prefix and its mask; FETCH, FPAIR: the element; PAIR: min above
  double gamma;
  union {
    struct {
      int k, le;  // RADIX: the rank left to select; PAIR: the count <= the element
    };
    unsigned long long above;  // FPAIR: the smallest element above the prefix
  };
  int i0, shift, phase, pair;
};
// FPAIR: the prefix holds one element; one pass fetches it and the smallest element above it (the next order
// statistic).  PAIR: after a select down to the last byte.
enum { SEL_RADIX = 0, SEL_FETCH = 1, SEL_PAIR = 2, SEL_DONE = 3, SEL_FPAIR = 4 };
__device__ __forceinline__ void sel_init(SelSet& st, int n, double q) {
  const double qq = q / 100.0;
  const double vi = (double)n * qq + (1.0 + qq * (1.0 - 1.0 - 1.0)) - 1.0;  // numpy _compute_virtual_index
  int i0, i1;
  double gamma;
  if (vi >= (double)(n - 1)) {
    i0 = i1 = n - 1;
    gamma = 0.0;
  } else if (vi < 0.0) {
    i0 = i1 = 0;
    gamma = 0.0;
  } else {
    i0 = (int)floor(vi);
    i1 = i0 + 1;
    gamma = vi - floor(vi);
  }
  st.prefix = st.mask = 0ull;
  st.dsh = ~0ull;
  st.gamma = gamma;
  st.k = st.i0 = i0;
  st.shift = 56;
  st.phase = n > 0 ? SEL_RADIX : SEL_DONE;
  st.le = 0;
  st.pair = i1 != i0;
}
// A set's top-16-bit summary, OR-accumulated over its elements: high half the OR of each element's top 16 bits, low
// half the OR of their complements (so the AND of the top 16 bits is its complement).  Bits where the two agree are
// common to every element: oa_lo / oa_hi are bounds with those bits whose first differing byte (select_pair's start)
// is at or below the first byte where the elements' top 16 bits differ.
__device__ __forceinline__ uint32_t top16_oa(uint64_t bits) {
  const uint32_t t = (uint32_t)(bits >> 48);
  return (t << 16) | (~t & 0xFFFFu);
}
__device__ __forceinline__ uint64_t oa_lo(uint32_t oa) { return (uint64_t)(~oa & 0xFFFFu) << 48; }
__device__ __forceinline__ uint64_t oa_hi(uint32_t oa) { return ((uint64_t)(oa >> 16) << 48) | 0xFFFFFFFFFFFFull; }

// thr[s] for the sets [0, nsets); st: SB states, hist: SB x 256 u32 (16-B aligned), flag: 2 ints of LDS.  lo, hi
// (optional): each set's smallest and largest element bits -- its passes start at the first byte where they differ;
// or oa (optional): each set's top16_oa summary, the same from the bounds it gives.
template <int NT, int SB, class Visit>
__device__ void select_batch(Visit&& visit, int nsets, const int* n, double q, double* thr, SelSet* st, uint32_t* hist,
                             int* flag, const unsigned long long* lo = nullptr, const unsigned long long* hi = nullptr,
                             const uint32_t* oa = nullptr) {
  static_assert(NT / WAVE >= SB, "a wave per set of the batch");
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  for (int b0 = 0; b0 < nsets; b0 += SB) {
    const int nb = nsets - b0 < SB ? nsets - b0 : SB;
    if (tid < nb) {
      SelSet& S = st[tid];
      sel_init(S, n[b0 + tid], q);
      if (n[b0 + tid] == 0) thr[b0 + tid] = INFINITY;
      if ((lo != nullptr || oa != nullptr) && S.phase == SEL_RADIX) {
        const uint64_t l = lo != nullptr ? (uint64_t)lo[b0 + tid] : oa_lo(oa[b0 + tid]);
        const uint64_t d = l ^ (lo != nullptr ? (uint64_t)hi[b0 + tid] : oa_hi(oa[b0 + tid]));
        if (d == 0ull) {  // every element is the same value
          thr[b0 + tid] = __longlong_as_double((long long)l);
          S.phase = SEL_DONE;
        } else {
          const int top = (63 - __clzll((long long)d)) & ~7;
          S.shift = top;
          S.mask = top == 56 ? 0ull : ~((1ull << (top + 8)) - 1ull);
          S.prefix = l & S.mask;
        }
      }
    }
    for (int i = tid; i < SB * 256; i += NT) hist[i] = 0u;
    if (tid == 0) flag[0] = flag[1] = 1;
    __syncthreads();
    for (int round = 0; flag[round & 1]; ++round) {
      visit([&](int set, uint64_t bits) {
        const int j = set - b0;
        if ((unsigned)j >= (unsigned)nb) return;
        SelSet& S = st[j];
        const int ph = S.phase;
        if (ph == SEL_DONE) return;
        const uint64_t pre = S.prefix;
        if (ph == SEL_PAIR) {
          if (bits <= pre) atomicAdd(&S.le, 1);
          else atomicMin(&S.dsh, (unsigned long long)bits);
        } else {
          const uint64_t mb = bits & S.mask;
          if (mb == pre) {
            if (ph == SEL_RADIX) atomicAdd(&hist[j * 256 + ((bits >> S.shift) & 255u)], 1u);
            else S.dsh = bits;  // SEL_FETCH, SEL_FPAIR: the one element with the prefix
          } else if (ph == SEL_FPAIR && mb > pre) {
            atomicMin(&S.above, (unsigned long long)bits);
          }
        }
      });
      if (tid == 0) flag[(round + 1) & 1] = 0;
      __syncthreads();
      if (wid < nb) {
        SelSet& S = st[wid];
        const int ph = S.phase;  // (wave-uniform)
        bool done_now = false;
        if (ph == SEL_RADIX) {
          int k = S.k, cnt;
          const int d = hist_find(hist + wid * 256, k, cnt);
          reinterpret_cast<uint4*>(hist + wid * 256)[lane] = make_uint4(0u, 0u, 0u, 0u);
          if (lane == 0) {
            const int sh = S.shift;
            S.prefix |= (unsigned long long)d << sh;
            S.mask |= 255ull << sh;
            S.k = k;
            if (cnt == 1 && sh > 0) {
              S.phase = S.pair ? SEL_FPAIR : SEL_FETCH;
              if (S.pair) S.above = ~0ull;  // (k is spent)
            } else if (sh == 0) {
              done_now = true;
            } else {
              S.shift = sh - 8;
            }
          }
        } else if (ph == SEL_FETCH) {
          if (lane == 0) {
            S.prefix = S.dsh;
            done_now = true;
          }
        } else if (ph == SEL_FPAIR) {
          if (lane == 0) {
            const double a = __longlong_as_double((long long)S.dsh);
            const double b = __longlong_as_double((long long)S.above);  // i0 + 1 < n: an element lies above
            const double dd = b - a, g = S.gamma;
            thr[b0 + wid] = g >= 0.5 ? b - dd * (1.0 - g) : a + dd * g;
            S.phase = SEL_DONE;
          }
        } else if (ph == SEL_PAIR) {
          if (lane == 0) {
            const double a = __longlong_as_double((long long)S.prefix);
            const double b = S.le < S.i0 + 2 ? __longlong_as_double((long long)S.dsh) : a;
            const double dd = b - a, g = S.gamma;
            thr[b0 + wid] = g >= 0.5 ? b - dd * (1.0 - g) : a + dd * g;
            S.phase = SEL_DONE;
          }
        }
        if (lane == 0) {
          if (done_now) {  // the i0-th element is known: the pair pass next, or the threshold now
            if (S.pair) {
              S.phase = SEL_PAIR;
              S.le = 0;
              S.dsh = ~0ull;
            } else {
              thr[b0 + wid] = __longlong_as_double((long long)S.prefix);
              S.phase = SEL_DONE;
            }
          }
          if (S.phase != SEL_DONE) flag[(round + 1) & 1] = 1;
        }
      }
      __syncthreads();
    }
    // every thread has read the final flag (and is done with the batch's states) before the next batch, or the
    // next call, writes them: without this a thread still testing the loop condition sees the next batch's flag
    __syncthreads();
  }
}

// open-addressing f64 accumulators keyed by u32 (EMPTY = 0xFFFFFFFF); returns false when full

// (sum v, sum v^2 of unflagged points) over the points [i & ~63, i) of hit i's 64-point block
template <int FMT>
__device__ __forceinline__ double2 block_part(const Hits<FMT>& hits, int64_t i) {
  double2 c = make_double2(0.0, 0.0);
  const int64_t a = i & ~(int64_t)63;
  if constexpr (FMT == SMG_HITS_PACKED_F32) {  // 16-byte loads: two hits per load (a is even)
    const ulonglong2* h2 = reinterpret_cast<const ulonglong2*>(hits.h + a);
    const int m = (int)(i - a);
#pragma unroll 4  // (8 spilled 20 VGPRs in ion_desc8_kernel; 4 fits in 90, no scratch: ion stage -0.35 ms at config 3)
    for (int q = 0; q < (m >> 1); ++q) {
      const ulonglong2 hh = h2[q];
      const double v0 = Hits<FMT>::val(hh.x), v1 = Hits<FMT>::val(hh.y);
      c.x += v0;
      if (!Hits<FMT>::dup(hh.x)) c.y += v0 * v0;
      c.x += v1;
      if (!Hits<FMT>::dup(hh.y)) c.y += v1 * v1;
    }
    if (m & 1) {  // never reads past hit i - 1
      const uint64_t h = hits.h[i - 1];
      const double v = Hits<FMT>::val(h);
      c.x += v;
      if (!Hits<FMT>::dup(h)) c.y += v * v;
    }
    return c;
  }
#pragma unroll 4
  for (int64_t j = a; j < i; ++j) {
    const auto h = hits.load(j);
    const double v = Hits<FMT>::val(h);
    c.x += v;
    if (!Hits<FMT>::dup(h)) c.y += v * v;
  }
  return c;
}

// sums over the window [a, b): double-double block prefixes (smg_hit_prefix_sums) differenced, plus the partial
// blocks at either end -- accurate to the window's own magnitude, not to the intensity preceding it
template <int FMT>
__device__ __forceinline__ double2 window_sums(const Hits<FMT>& hits, const DD4* __restrict__ cum64, int64_t a,
                                               int64_t b) {
  const DD4 P1 = cum64[b >> 6], P0 = cum64[a >> 6];
  const double2 l1 = block_part<FMT>(hits, b), l0 = block_part<FMT>(hits, a);
  return make_double2(dd_diff(P1.xh, P1.xl, P0.xh, P0.xl) + (l1.x - l0.x),
                      dd_diff(P1.yh, P1.yl, P0.yh, P0.yl) + (l1.y - l0.y));
}

template <int FMT>
__global__ void ion_desc_kernel(Hits<FMT> hits, const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
                                const int64_t* __restrict__ ion_off, const double* __restrict__ theor,
                                const DD4* __restrict__ cum, const int64_t* __restrict__ ion_order,
                                int64_t n_ions, IonDesc* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_ions) return;
  const int64_t ion = ion_order ? ion_order[b] : b;
  const int64_t w0 = ion_off[ion];
  const int K = (int)(ion_off[ion + 1] - w0);
  IonDesc* d = out + b;
  int64_t g = 0;
  uint32_t has = 0;
  int64_t wb[MAXK];
  int32_t we[MAXK], wg[MAXK];
  double wt[MAXK], wy[MAXK], wyy[MAXK];
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    wb[k] = 0;
    we[k] = 0;
    wg[k] = 0x7FFFFFFF;
    wt[k] = wy[k] = wyy[k] = 0.0;
    if (k < K) {
      const int64_t a = lo[w0 + k], n = hi[w0 + k] - a;
      wt[k] = theor[w0 + k];
      const double2 ws = window_sums<FMT>(hits, cum, a, a + n);
      wy[k] = ws.x;
      wyy[k] = ws.y;
      if (n > 0) has = SMG_ION_HAS_HITS;
      if (k == 0) {
        wb[k] = a;
        we[k] = (int32_t)(n < 0x7FFFFFFF ? n : 0x7FFFFFFF);
        wg[k] = 0;
      } else {
        wb[k] = a - 64 * g;
        we[k] = (int32_t)(64 * g + n < 0x7FFFFFFF ? 64 * g + n : 0x7FFFFFFF);
        wg[k] = (int32_t)(g < 0x7FFFFFFF ? g : 0x7FFFFFFF);
        g += (n + 63) / 64;
      }
    }
  }
  for (int k = MAXK; k < K && k < MAXK_DENSE; ++k)
    if (hi[w0 + k] > lo[w0 + k]) has = SMG_ION_HAS_HITS;
#pragma unroll
  for (int k = 0; k < MAXK; k += 2) {
    reinterpret_cast<longlong2*>(d->base)[k / 2] = make_longlong2(wb[k], wb[k + 1]);
    reinterpret_cast<double2*>(d->theor)[k / 2] = make_double2(wt[k], wt[k + 1]);
    reinterpret_cast<double2*>(d->sy)[k / 2] = make_double2(wy[k], wy[k + 1]);
    reinterpret_cast<double2*>(d->syy)[k / 2] = make_double2(wyy[k], wyy[k + 1]);
  }
#pragma unroll
  for (int k = 0; k < MAXK; k += 4) {
    reinterpret_cast<int4*>(d->end)[k / 4] = make_int4(we[k], we[k + 1], we[k + 2], we[k + 3]);
    reinterpret_cast<int4*>(d->gs)[k / 4] = make_int4(wg[k], wg[k + 1], wg[k + 2], wg[k + 3]);
  }
  const int32_t ng = 64 * g < (1ll << 30) ? (int32_t)g : -1;
  reinterpret_cast<int4*>(&d->ion)[0] = make_int4((int32_t)ion, K, ng, (int)has);
#pragma unroll
  for (int i = 0; i < 3; ++i) reinterpret_cast<int4*>(d->pad)[i] = make_int4(0, 0, 0, 0);
}

// The same descriptors with eight lanes per ion, lane k = window k (k >= 8: the has-hits test of windows 8..31):
// the two partial 64-point blocks of every window are summed in parallel instead of one window after another.
template <int FMT>
__global__ void __launch_bounds__(256)
    ion_desc8_kernel(Hits<FMT> hits, const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
                     const int64_t* __restrict__ ion_off, const double* __restrict__ theor, const DD4* __restrict__ cum,
                     const int64_t* __restrict__ ion_order, int64_t n_ions, IonDesc* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = t >> 3;
  const int k = (int)(t & 7);
  const bool live = b < n_ions;
  const int64_t ion = live ? (ion_order ? ion_order[b] : b) : 0;
  const int64_t w0 = live ? ion_off[ion] : 0;
  const int K = live ? (int)(ion_off[ion + 1] - w0) : 0;
  int64_t a = 0, n = 0;
  double wt = 0.0, wy = 0.0, wyy = 0.0;
  if (k < K) {
    a = lo[w0 + k];
    n = hi[w0 + k] - a;
    wt = theor[w0 + k];
    const double2 ws = window_sums<FMT>(hits, cum, a, a + n);
    wy = ws.x;
    wyy = ws.y;
  }
  bool has = n > 0;
  for (int kk = k + MAXK; kk < K && kk < MAXK_DENSE; kk += MAXK) has |= hi[w0 + kk] > lo[w0 + kk];
  // groups of the tail windows 1..K-1: exclusive prefix over the eight lanes of this ion
  const int64_t gk = (k >= 1 && k < K) ? (n + 63) / 64 : 0;
  int64_t inc = gk;
#pragma unroll
  for (int d = 1; d < 8; d <<= 1) {
    const int64_t v = __shfl_up(inc, d, 8);
    if (k >= d) inc += v;
  }
  const int64_t g = inc - gk;            // first group of window k
  const int64_t ng_all = __shfl(inc, 7, 8);
  // any lane of the ion with a point: OR over the eight lanes
  uint32_t hv = has ? 1u : 0u;
#pragma unroll
  for (int d = 1; d < 8; d <<= 1) hv |= __shfl_xor(hv, d, 8);
  if (!live) return;
  IonDesc* d = out + b;
  int64_t wb = 0;
  int32_t we = 0, wg = 0x7FFFFFFF;
  if (k < K) {
    if (k == 0) {
      wb = a;
      we = (int32_t)(n < 0x7FFFFFFF ? n : 0x7FFFFFFF);
      wg = 0;
    } else {
      wb = a - 64 * g;
      we = (int32_t)(64 * g + n < 0x7FFFFFFF ? 64 * g + n : 0x7FFFFFFF);
      wg = (int32_t)(g < 0x7FFFFFFF ? g : 0x7FFFFFFF);
    }
  }
  d->base[k] = wb;
  d->end[k] = we;
  d->gs[k] = wg;
  d->theor[k] = wt;
  d->sy[k] = wy;
  d->syy[k] = wyy;
  if (k == 0) {
    const int32_t ng = 64 * ng_all < (1ll << 30) ? (int32_t)ng_all : -1;
    reinterpret_cast<int4*>(&d->ion)[0] = make_int4((int32_t)ion, K, ng, hv ? (int)SMG_ION_HAS_HITS : 0);
  } else if (k < 4) {
    reinterpret_cast<int4*>(d->pad)[k - 1] = make_int4(0, 0, 0, 0);
  }
}


// ---------------------------------------------------------------------------------------------
// LDS path: persistent, software-pipelined kernel.  Each workgroup scores a sequence of ions.  Iteration b
// scores ion b (phases 0-5), then issues the loads of ion b+1 (principal window, first two tail chunks)
// into the registers ion b no longer needs, then finishes ion b (duplicates, chaos, finalize) while those
// loads are in flight.  Barriers between phases:
//   0  initialise the LDS structures; thread 0 takes a ticket for ion b+1
//   1  principal bitmap (atomicOr), rank prefix, f64 values in rank order (duplicate-candidate points
//      zero their slot, then add atomically); ion b+1 resolved and its descriptor fetched
//   2  one fused reduction: sum x, sum x^2, sum x[x>0], #(x>0), max; level index per pixel
//   5  tail windows as one stream of 64-point groups (each group in one window; a wave sees windows in
//      increasing order; principal hits add into its LDS partials of the current window),
//      chunks of BLOCK*RC points, two register buffers, next chunk in flight; duplicate-candidate points
//      deferred to an LDS list.  Then the loads of ion b+1 are issued
//   d  deferred duplicates summed per (pixel, window) in an LDS table, squared into the partials
//   4a chaos candidates from the principal pixels (7x7 bit windows, isolation pre-filter), exact eL
//   4b Kruskal over eL with an LDS union-find
//   6  finalize (wave 0, one lane per window)
// measure_of_chaos by threshold decomposition: per-level dilate(cross)/erode(box) equals thresholding
// eL = erode_box(dilate_cross(L)), so sum_levels #components = sum_p eL(p) - weight(maximum spanning
// forest with edge weight min(eL)).
// Ions that do not fit (K > MAXK, principal window > CAPC, list/table overflows) go to `rej_list`: positions
// (SRC_RANGES pass, read by the big-ion pass) or ion indices (SRC_LIST pass, read by the dense kernel).
// ---------------------------------------------------------------------------------------------
template <int FMT, int LB, int LRMAX, int LRC, int WPE, int SRC, bool TWO, bool CLIP = false>
__global__ void __launch_bounds__(LB, WPE) ion_pipe_kernel(
    Hits<FMT> hits, IonDesc* __restrict__ desc, Sched S, Params P, double* __restrict__ oc,
    double* __restrict__ osp, double* __restrict__ osc, double* __restrict__ omsm, uint32_t* __restrict__ oflags,
    uint32_t* __restrict__ rej_list, uint32_t* __restrict__ rej_count SMG_CHK_PARAM) {
  constexpr int BLOCK = LB;
  constexpr int NW = LB / WAVE;
  constexpr int RMAX = LRMAX;
  constexpr int RC = LRC;
  constexpr int GPC = BLOCK * RC / 64;  // 64-point groups per chunk
  constexpr int CAPC = BLOCK * RMAX;
  using Reg = typename Hits<FMT>::Reg;
  using LY = std::conditional_t<TWO, Lay2<NW, CAPC>, Lay<NW, CAPC>>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* Hbm = reinterpret_cast<uint32_t*>(smem + LY::o_bm);  // a zero guard word in front, for bits7
  uint16_t* pf = reinterpret_cast<uint16_t*>(smem + P.o_pf);      // two-level: TP (top-level rank prefix)
  double* vals = reinterpret_cast<double*>(smem + LY::o_vals);
  uint8_t* Lv = reinterpret_cast<uint8_t*>(smem + LY::o_L);
  uint32_t* filtA = reinterpret_cast<uint32_t*>(smem + LY::o_filt);
  uint32_t* dkey = reinterpret_cast<uint32_t*>(smem + LY::o_dkey);
  double* dval = reinterpret_cast<double*>(smem + LY::o_dval);
  int* dcnt = reinterpret_cast<int*>(smem + LY::o_dcnt);
  uint32_t* tkey = reinterpret_cast<uint32_t*>(smem + LY::o_tkey);
  double* tval = reinterpret_cast<double*>(smem + LY::o_tval);
  double* part = reinterpret_cast<double*>(smem + LY::o_part);  // [MAXK][NW][4]: s_k, sy, syy, sxy
  double* red = reinterpret_cast<double*>(smem + LY::o_red);
  int* ctr = reinterpret_cast<int*>(smem + LY::o_ctr);
  int* wsc = reinterpret_cast<int*>(smem + LY::o_wsc);
  IonDesc* dsl = reinterpret_cast<IonDesc*>(smem + LY::o_desc);  // [2]: current / next
  // chaos-phase aliases.  The distinct principal pixels in rank order (olist) sit in the value region: right
  // behind the nnz values when 12*nnz <= 8*CAPC (written by their owners in phase 1), else at its start
  // (bitmap scan once the values are dead).  Candidates go to the (then dead) duplicate-list region.
  constexpr int OL_MAX = (2 * CAPC) / 3;
  uint32_t* epix = filtA;                                               // candidates, append order (4*CAPC)
  uint8_t* eL8 = reinterpret_cast<uint8_t*>(filtA) + (size_t)CAPC * 4;  // candidates' eL, append order
  uint32_t* epix_r = reinterpret_cast<uint32_t*>(vals);                 // E pixels, rank order
  uint8_t* eLr = Lv;                                                    // rank order
  uint32_t* par = reinterpret_cast<uint32_t*>(vals) + CAPC;             // rank order
  // CLIP (the hot-spot clip): the radix select's histogram and scalars, each window's threshold, positive count and
  // smallest / largest value bits, in the level region (free until the levels, which come after the tail)
  // (the level region and the duplicate lists behind it, which the clip does not use)
  constexpr int CSB = 4;  // tail windows per select batch
  static_assert(LY::o_tkey - LY::o_L >= 4336 + 24 + MAXK * 28 && CSB * sizeof(SelSet) <= 224,
                "clip scratch fits the level and duplicate-list regions");
  uint32_t* c_hist = reinterpret_cast<uint32_t*>(Lv);  // CSB x 256 bins (the principal's select: 2 x 256)
  SelSet* c_st = reinterpret_cast<SelSet*>(Lv + 4096);
  int* c_flag = reinterpret_cast<int*>(Lv + 4320);
  unsigned long long* c_dsh = reinterpret_cast<unsigned long long*>(Lv + 4328);  // 2
  int* c_sh = reinterpret_cast<int*>(Lv + 4344);
  double* c_thr = reinterpret_cast<double*>(Lv + 4360);
  unsigned long long* c_lo = reinterpret_cast<unsigned long long*>(Lv + 4360 + MAXK * 8);
  unsigned long long* c_hi = reinterpret_cast<unsigned long long*>(Lv + 4360 + MAXK * 16);
  int* c_n = reinterpret_cast<int*>(Lv + 4360 + MAXK * 24);

  // two-level pixel set (TWO): compact words W = Hbm as u64, their rank prefix B, top-level bitmap T
  const uint64_t* W64 = reinterpret_cast<const uint64_t*>(Hbm);
  uint16_t* Bpf = reinterpret_cast<uint16_t*>(smem + (TWO ? Lay2<NW, CAPC>::o_B : 0));
  uint32_t* T32 = reinterpret_cast<uint32_t*>(smem + (TWO ? Lay2<NW, CAPC>::o_T : 0));
  const uint64_t* T64 = reinterpret_cast<const uint64_t*>(T32);
  const int nT = TWO ? Lay2<NW, CAPC>::nT(P.npx) : 0;
  // two-level lookups: index r of word q among the non-empty words (-1: empty or outside the image)
  auto top_rank = [&](int q) -> int {
    if (q < 0) return -1;
    const uint64_t t = T64[q >> 6], b = 1ull << (q & 63);
    return (t & b) ? (int)pf[q >> 6] + __popcll(t & (b - 1ull)) : -1;
  };
  // word q (0 when empty) and the rank of its first pixel
  auto word2 = [&](int q, int& base) -> uint64_t {
    const int r = top_rank(q);
    base = r >= 0 ? (int)Bpf[r] : 0;
    return r >= 0 ? W64[r] : 0ull;
  };
  // rank of pixel p in the set (-1: not in it)
  auto rank2 = [&](int p) -> int {
    const int r = top_rank(p >> 6);
    if (r < 0) return -1;
    const uint64_t w = W64[r], b = 1ull << (p & 63);
    return (w & b) ? (int)Bpf[r] + __popcll(w & (b - 1ull)) : -1;
  };
  // builds the set from up to CAPC pixels (two passes: top-level bits, then the compact words); each(f) calls
  // f(j, p) for every pixel p (slot j) of this thread and records the slots for which f returns true (the
  // atomicOr of the second pass set the pixel's bit: its owner).  W and T are zero on entry.  Returns the
  // number of distinct pixels.
  auto build2 = [&](auto&& each) -> int {
    each([&](int, uint32_t p) {
      const uint32_t q = p >> 6;
      atomicOr(&T32[q >> 5], 1u << (q & 31));
      return false;
    });
    __syncthreads();
    const int nwords = prefix_words<NW, TOPCAP>(T64, pf, nT, wsc);
    (void)nwords;
    each([&](int, uint32_t p) {
      const int r = top_rank((int)(p >> 6));
      const uint32_t bit = 1u << (p & 31);
      return !(atomicOr(&Hbm[2 * r + ((p >> 5) & 1)], bit) & bit);
    });
    __syncthreads();
    return prefix_words<NW, CAPC>(W64, Bpf, nwords, wsc);
  };

  // tid and lane are laundered at the top of every ion iteration (SMG_LAUNDER): values derived from them are
  // then recomputed where they are used instead of being hoisted out of the ion loop and spilled to scratch
  int tid = threadIdx.x;
  int lane = tid & 63;
  const int wid = uni(tid >> 6);
  const int n64 = (P.npx + 63) / 64;
  const uint32_t big_flag = (SRC == SRC_LIST) ? SMG_ION_BIG : 0u;

  // Register buffers: the tail is streamed through a ring of four chunk buffers (pa, pb, pc, pd); the principal
  // window of the next ion arrives in pc, pd, pe (RMAX slots), which become tail buffers once phase 1 has
  // consumed it.  Issue order per ion: [principal, pa <- chunk 0, pb <- chunk 1] at the previous ion's issue
  // site, then [pc <- chunk 2, pd <- chunk 3] after phase 1, then each buffer is refilled four chunks ahead as
  // soon as it is processed, so every tail wait has exactly three younger buffers (3*RC loads) behind it.
  static_assert(RMAX >= 2 * RC, "principal slots double as two tail buffers");
  constexpr int RE = RMAX - 2 * RC > 0 ? RMAX - 2 * RC : 1;
  Reg pa[RC], pb[RC], pc[RC], pd[RC], pe[RE];
#pragma unroll
  for (int j = 0; j < RC; ++j) pa[j] = pb[j] = pc[j] = pd[j] = Hits<FMT>::zero();
#pragma unroll
  for (int j = 0; j < RE; ++j) pe[j] = Hits<FMT>::zero();
  auto hs = [&](int j) -> Reg& { return j < RC ? pc[j] : (j < 2 * RC ? pd[j - RC] : pe[j - 2 * RC]); };
  // Asynchronous (inline-asm, counted-wait) loads in the main pass only; the big-ion pass (~1% of the ions at
  // config 3) uses compiler-tracked loads: its 8-deep principal slots made the compiler copy in-flight registers
  constexpr bool ASYNC = (FMT == SMG_HITS_PACKED_F32) && LB <= 512 && !CLIP;
  // principal window (<= CAPC points, RMAX per thread).  Async form: every slot issues exactly one load
  // (clamped to the window's last point, or to hit 0 for an empty window) so that the counted waits hold.
  auto issue_principal = [&](const IonDesc* D) {
    const int n0 = D->end[0];
    const int64_t a = D->base[0];
    if constexpr (ASYNC) {
#pragma unroll
      for (int j = 0; j < RMAX; ++j) {
        const int i = tid + j * BLOCK;
#ifdef SMG_CHECK
        chk_load(CK, D->ion, 0, n0 > 0 ? a + min(i, n0 - 1) : 0, n0 <= 0);
#endif
        ld8_async_v(hs(j), hits.h + (n0 > 0 ? a + min(i, n0 - 1) : 0));
      }
    } else {
#pragma unroll
      for (int j = 0; j < RMAX; ++j) {
        const int i = tid + j * BLOCK;
#ifdef SMG_CHECK
        if (i < n0) chk_load(CK, D->ion, 0, a + i, false);
#endif
        if (i < n0) hs(j) = hits.load(a, i);
      }
    }
  };
  // tail chunk c: groups [c*GPC, (c+1)*GPC); slot j of wave w holds group c*GPC + j*NW + w.  Async form:
  // exactly RC loads per chunk; lanes past their window's end load its last point, groups past the tail
  // load hit 0 (consumers mask both).  Compiler form: such lanes hold a zero hit.
  auto issue_chunk = [&](const IonDesc* D, int c, Reg (&buf)[RC]) {
    // descriptor fields are read as broadcast LDS loads into VGPRs (no readfirstlane round trips)
    const int ng = D->ngroups;
    int gsv[MAXK];
#pragma unroll
    for (int kk = 2; kk < MAXK; ++kk) gsv[kk] = D->gs[kk];
#pragma unroll
    for (int j = 0; j < RC; ++j) {
      const int G = c * GPC + j * NW + wid;
      int k = 1;
#pragma unroll
      for (int kk = 2; kk < MAXK; ++kk) k += (G >= gsv[kk]) ? 1 : 0;
      if constexpr (ASYNC) {
        const int64_t bk = D->base[k];
        const int ek = D->end[k];
        const int64_t idx = G < ng ? bk + (int64_t)G * 64 + min(lane, ek - G * 64 - 1) : 0;
#ifdef SMG_CHECK
        chk_load(CK, D->ion, k, idx, G >= ng);
#endif
        ld8_async_v(buf[j], hits.h + idx);
      } else {
        buf[j] = Hits<FMT>::zero();
        if (G < ng) {
          const int i = G * 64 + lane;
#ifdef SMG_CHECK
          if (i < D->end[k]) chk_load(CK, D->ion, k, D->base[k] + i, false);
#endif
          if (i < D->end[k]) buf[j] = hits.load(D->base[k] + i);
        }
      }
    }
  };

  // scheduling runs one ion further ahead than the loads: iteration b scores pos, loads npos's descriptor and
  // data, and takes the ticket of the ion after npos
  STAMP_DECL();
  // The LDS structures start zeroed: the pixel set and the values here, then at the end of every ion that used
  // them (by the waves other than wave 0, while it writes the ion's record), so that no ion starts with a barrier of
  // its own; the window partials and the counters are zeroed in phase 1 before its first barrier, the duplicate
  // table before the tail stream's closing barrier.
  auto clear_set_vals = [&](int t0, int nt) {
    uint4* z = reinterpret_cast<uint4*>(smem + LY::o_guard);
    for (int i = t0; i < P.w32 / 4 + 1; i += nt) z[i] = make_uint4(0, 0, 0, 0);
    uint4* zv = reinterpret_cast<uint4*>(smem + LY::o_vals);
    for (int i = t0; i < CAPC / 2; i += nt) zv[i] = make_uint4(0, 0, 0, 0);
  };
  auto clear_table = [&]() {
    for (int i = tid; i < DTBL; i += BLOCK) {
      tkey[i] = 0xFFFFFFFFu;
      tval[i] = 0.0;
    }
  };
  clear_set_vals(tid, BLOCK);
  if (tid == 0) {
    int h0;
    const uint32_t t0 = sched_issue<SRC>(S, h0);
    ctr[C_NEXT] = (int)sched_resolve<SRC>(S, t0, h0);
  }
  __syncthreads();
  int64_t pos = -1;  // ion scored in this iteration (-1: none; the first iteration only issues loads)
  int64_t npos = uni(ctr[C_NEXT]);
  int cur = 0;
  while (true) {
#ifndef SMG_LAUNDER
#define SMG_LAUNDER 1
#endif
    if (SMG_LAUNDER) {
      asm volatile("" : "+v"(tid));
      asm volatile("" : "+v"(lane));
    }
    const IonDesc* D = &dsl[cur];
    IonDesc* DN = &dsl[cur ^ 1];
    // the ticket of the ion after npos: issued now, consumed after phase 1 (wave 0 issues after it exactly one
    // descriptor load, and the 2*RC loads of tail chunks 2 and 3 unless this iteration skips)
    uint32_t ticket = 0;
    int thome = 0;  // the XCD whose counter the ticket came from
    if constexpr (ASYNC) {
      if (tid == 0) sched_issue_async<SRC>(S, ticket, thome);
    } else {
      if (tid == 0) ticket = sched_issue<SRC>(S, thome);
    }
    // npos's descriptor: one async word per lane of wave 0 (exactly one load per lane, clamped), waited in
    // phase 2 behind the 2*RC loads of tail chunks 2 and 3
    uint64_t dword = 0;
    if ((tid >> 6) == 0) {
      if constexpr (ASYNC) {
        ld8_async_wave0(dword, reinterpret_cast<const uint64_t*>(desc + (npos >= 0 ? npos : 0)) +
                                   (lane < DESC_QWORDS ? lane : 0));
      } else {
        if (npos >= 0 && lane < DESC_QWORDS) dword = reinterpret_cast<const uint64_t*>(desc + npos)[lane];
      }
    }
    STAMP_INIT();
    bool skip = pos < 0;
    int K = 0, ion = 0, n0 = 0;
    // a reject beyond the list's capacity (impossible while every position is handed out once) is dropped
    auto reject = [&]() {
      if (tid == 0) {
        const uint32_t r = atomicAdd(rej_count, 1u);
        if (r < S.rej_cap) rej_list[r] = (SRC == SRC_RANGES) ? (uint32_t)pos : (uint32_t)ion;
#ifdef SMG_CHECK
        chk(CK, r < S.rej_cap, CHK_REJ, pos, r);
#endif
      }
    };
#ifdef SMG_CHECK
    if (!skip && wid == 0) chk_claim(CK, SRC == SRC_RANGES ? 0 : 1, pos);
#endif
    if (!skip) {
      K = uni(D->K);
      ion = uni(D->ion);
      n0 = uni(D->end[0]);
      if (K == 0) {
        if (tid == 0) {
          oc[ion] = osp[ion] = osc[ion] = omsm[ion] = 0.0;
          oflags[ion] = 0;
        }
        skip = true;
      } else if (!desc_lds_ok(D, CAPC)) {
#ifdef SMG_CHECK
        if (tid == 0) chk(CK, reinterpret_cast<const IonRec*>(D)->state == 0u, CHK_STATE, pos, 0);
#endif
        reject();
        skip = true;
      }
#ifdef SMG_CHECK
      else if (wid == 0) {
        chk_desc(CK, pos, D);
      }
#endif
    }

    const bool began = !skip;  // this ion uses the LDS structures (cleared again at its end)
    STAMP(0);

    // ---- phase 1: principal image -> bitmap, rank prefix, f64 values -----------------------------
    int nnz = 0;
    uint32_t* olist = nullptr;
    if (!skip) {
      // the window partials (first added to in the tail stream) and the counters (dup table, chaos), ordered before
      // their uses by phase 1's first barrier
      for (int i = tid; i < MAXK * NW * 4; i += BLOCK) part[i] = 0.0;
      if (tid < C_NEXT || tid == C_NS) ctr[tid] = 0;
      vm_wait<2 * RC>(pc);  // the principal window was issued before this ion's tail chunks 0 and 1
      vm_wait<2 * RC>(pd);
      vm_wait<2 * RC>(pe);
      uint32_t own = 0;     // slots whose atomicOr set the pixel's bit (one owner per distinct pixel)
      if constexpr (TWO) {
        nnz = build2([&](auto&& f) {
#pragma unroll
          for (int j = 0; j < RMAX; ++j) {
            const int i = tid + j * BLOCK;
            if (i < n0 && f(j, Hits<FMT>::pix(hs(j)))) own |= 1u << j;
          }
        });
      } else {
#pragma unroll
        for (int j = 0; j < RMAX; ++j) {
          const int i = tid + j * BLOCK;
          if (i < n0) {
            const uint32_t p = Hits<FMT>::pix(hs(j));
            const uint32_t bit = 1u << (p & 31);
            if (!(atomicOr(&Hbm[p >> 5], bit) & bit)) own |= 1u << j;
          }
        }
        __syncthreads();
        nnz = bm_build_prefix<NW>(Hbm, pf, n64, wsc);
      }
      olist = reinterpret_cast<uint32_t*>(vals) + (nnz <= OL_MAX ? ((2 * nnz + 3) & ~3) : 0);
      // A point without the duplicate-candidate flag is the only point of its pixel in this window
      // (smg_flag_duplicates), so it stores its value; flagged points (true duplicates and a few false
      // positives) add theirs atomically into the slot, zeroed in phase 0 (coo.toarray() sums duplicates).  The
      // pixel list behind the values (olist) lies past slot nnz - 1: no store of it meets a slot being summed.
#pragma unroll
      for (int j = 0; j < RMAX; ++j) {
        const int i = tid + j * BLOCK;
        if (i < n0) {
          const int r = TWO ? rank2((int)Hits<FMT>::pix(hs(j))) : bm_rank(Hbm, pf, (int)Hits<FMT>::pix(hs(j)));
          if (Hits<FMT>::dup(hs(j))) atomicAdd(&vals[r], Hits<FMT>::val(hs(j)));
          else vals[r] = Hits<FMT>::val(hs(j));
          if (nnz <= OL_MAX && ((own >> j) & 1u)) olist[r] = Hits<FMT>::pix(hs(j));
        }
      }
    }
    if (!skip && !CLIP) {  // the principal registers are consumed: tail chunks 2 and 3 go in flight
      issue_chunk(D, 2, pc);
      issue_chunk(D, 3, pd);
    } else if constexpr (ASYNC) {
      // the same number of loads (into the same registers, which the next principal overwrites): the waits for
      // the ticket and the descriptor below count 2*RC younger loads on every path
#pragma unroll
      for (int j = 0; j < RC; ++j) {
        ld8_async_v(pc[j], hits.h);
        ld8_async_v(pd[j], hits.h);
      }
    }
    STAMP(11);
    // wave 0: the ticket and npos's descriptor (issued at the top of this iteration, before chunks 2 and 3 or their
    // stand-ins): lane 0 resolves the ticket, the lanes store the descriptor for the end of the tail stream.  Counted
    // waits are per wave; the test is on the laundered tid (an exec-masked branch, not a scalar one), the form
    // scripts/check_async_regs.py recognises as wave-0 only
    if ((tid >> 6) == 0) {
      if constexpr (ASYNC) {
        vm_wait1<2 * RC>(ticket);
        vm_wait1<2 * RC>(dword);
      }
      if (tid == 0) ctr[C_NEXT] = (int)sched_resolve<SRC>(S, ticket, thome);
      if (npos >= 0 && lane < DESC_QWORDS) reinterpret_cast<uint64_t*>(DN)[lane] = dword;
    }
    __syncthreads();
    const int64_t n2pos = uni(ctr[C_NEXT]);
    STAMP(1);
    if constexpr (CLIP) {
      // the hot-spot clip of the principal image: its q-th percentile over the positive values, every value above
      // it lowered to it (each thread its own slots, as phase 2 reads them; the tail's lookups after a barrier)
      if (!skip) {
        int cnt = 0;
        uint64_t plo = ~0ull, phi = 0ull;
        for (int r = tid; r < nnz; r += BLOCK) {
          const double v = vals[r];
          if (v > 0.0) {
            const uint64_t b = (uint64_t)__double_as_longlong(v);
            ++cnt;
            plo = b < plo ? b : plo;
            phi = b > phi ? b : phi;
          }
        }
        if (tid == 0) {
          c_n[0] = 0;
          c_lo[0] = ~0ull;
          c_hi[0] = 0ull;
        }
        __syncthreads();
        if (cnt) {
          atomicAdd(&c_n[0], cnt);
          atomicMin(&c_lo[0], (unsigned long long)plo);
          atomicMax(&c_hi[0], (unsigned long long)phi);
        }
        __syncthreads();
        const int n0p = c_n[0];
        if (n0p > 0) {
          const double thr = percentile_of<BLOCK>(
              [&](auto&& f) {
                for (int r = tid; r < nnz; r += BLOCK)
                  if (vals[r] > 0.0) f((uint64_t)__double_as_longlong(vals[r]));
              },
              n0p, P.q, c_hist, c_sh, c_dsh, c_lo[0], c_hi[0]);
          for (int r = tid; r < nnz; r += BLOCK)
            if (vals[r] > thr) vals[r] = thr;
        }
      }
    }

    // ---- phase 2: fused principal-image statistics: each wave's sums into red, read after the tail stream's
    // closing barrier (nothing before it needs them), so no barrier of its own
    if (!skip) {
      double acc[5] = {0.0, 0.0, 0.0, 0.0, -INFINITY};
      for (int r = tid; r < nnz; r += BLOCK) {
        const double v = vals[r];
        acc[0] += v;
        acc[1] += v * v;
        if (v > 0.0) {
          acc[2] += v;
          acc[3] += 1.0;
        }
        acc[4] = v > acc[4] ? v : acc[4];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = wave_sum_dpp(acc[q]);
      acc[4] = wave_max_dpp(acc[4]);
      if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 5; ++q) red[q * NW + wid] = acc[q];
      }
    }
#ifndef SMG_ABL
#define SMG_ABL 0  // diagnostic ablations (timing only, wrong results): 1 = no chaos, 2 = no tail windows,
                   // 4 = tail chunk 0 only, 8 = no duplicate deferral, 16 = no principal lookups in the tail,
                   // 32 = no exact eL / Kruskal, 64 = no screen, 128 = no levels
#endif
    STAMP(2);

    // ---- phase 5: tail windows, one stream of window-aligned 64-point groups -------------------------
    if constexpr (CLIP) {
      // The hot-spot clip: each tail image is clipped at the q-th percentile of its positive pixels before its
      // sums, so Σy, Σy², Σxy, Σy[x>0] all come from the clipped pixel values (not from the prefix sums).  A
      // window's pixel values: its unflagged points' values (the only point of their pixel in the window,
      // smg_flag_duplicates) and the per-pixel sums of its flagged points (the duplicate table, keyed (pixel,
      // window)).  1. the flagged points into the table, positive unflagged points counted per window; 2. each
      // window's threshold by a radix select over both (its groups re-read once per pass); 3. the clipped
      // unflagged points into this wave's partials; 4. each flagged pixel's clipped sum (the same wide-pass scheme,
      // wide_clip_tail).  Groups are window-aligned: a group's window is uniform.
      if (!skip) {
        const int ng = uni(D->ngroups);
        int gsv[MAXK];
#pragma unroll
        for (int kk = 0; kk < MAXK; ++kk) gsv[kk] = D->gs[kk];
        auto win_of = [&](int G) {
          int k = 1;
#pragma unroll
          for (int kk = 2; kk < MAXK; ++kk) k += (G >= gsv[kk]) ? 1 : 0;
          return k;
        };
        auto xval = [&](uint32_t p) -> double {  // the (clipped) principal value at pixel p, 0 outside the image
          if constexpr (TWO) {
            const int r = rank2((int)p);
            return r >= 0 ? vals[r] : 0.0;
          } else {
            return bm_test(Hbm, (int)p) ? vals[bm_rank(Hbm, pf, (int)p)] : 0.0;
          }
        };
        auto bits_of = [](double v) { return (uint64_t)__double_as_longlong(v); };
        constexpr int GU = 4;  // groups per wave with loads in flight together
        // groups [g0, g1) in rounds of GU per wave: body(k, valid, hit) per group, uniform (k: the group's window)
        auto groups = [&](int g0, int g1, auto&& body) {
          for (int G0 = g0; G0 < g1; G0 += GU * NW) {
            Reg h[GU];
            int kg[GU];
            bool vg[GU];
#pragma unroll
            for (int u = 0; u < GU; ++u) {
              const int G = G0 + u * NW + wid;
              kg[u] = win_of(G);
              const int i = G * 64 + lane;
              vg[u] = G < g1 && i < D->end[kg[u]];
              h[u] = vg[u] ? hits.load(D->base[kg[u]] + i) : Hits<FMT>::zero();
            }
#pragma unroll
            for (int u = 0; u < GU; ++u)
              if (G0 + u * NW + wid < g1) body(kg[u], vg[u], h[u]);
          }
        };
        clear_table();  // (its space held the previous ion's chaos candidates)
        if (tid < MAXK) {
          c_n[tid] = 0;
          c_lo[tid] = ~0ull;
          c_hi[tid] = 0ull;
        }
        __syncthreads();  // (also: the clipped principal values before the lookups below)
        {  // 1.
          int cpos = 0, kc = -1;
          uint64_t plo = ~0ull, phi = 0ull;
          auto flush = [&]() {
            const int t = __builtin_amdgcn_readlane(wave_incl_scan_dpp(cpos), 63);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
              const uint64_t l2 = (uint64_t)__shfl_xor((unsigned long long)plo, o, WAVE);
              const uint64_t h2 = (uint64_t)__shfl_xor((unsigned long long)phi, o, WAVE);
              plo = l2 < plo ? l2 : plo;
              phi = h2 > phi ? h2 : phi;
            }
            if (lane == 0 && t) {
              atomicAdd(&c_n[kc], t);
              atomicMin(&c_lo[kc], (unsigned long long)plo);
              atomicMax(&c_hi[kc], (unsigned long long)phi);
            }
            cpos = 0;
            plo = ~0ull;
            phi = 0ull;
          };
          groups(0, ng, [&](int k, bool valid, const Reg& h) {
            if (k != kc) {
              if (kc >= 0) flush();
              kc = k;
            }
            const bool fl = valid && Hits<FMT>::dup(h);
            if (fl && !tbl_add<DTBL>(tkey, tval, (Hits<FMT>::pix(h) << 3) | (uint32_t)k, Hits<FMT>::val(h)))
              ctr[C_ABORT] = 1;
            if (valid && !fl && Hits<FMT>::val(h) > 0.0) {
              const uint64_t b = bits_of(Hits<FMT>::val(h));
              ++cpos;
              plo = b < plo ? b : plo;
              phi = b > phi ? b : phi;
            }
          });
          if (kc >= 0) flush();
        }
        __syncthreads();
        if (ctr[C_ABORT]) {  // more flagged pixels than the table holds: the next pass scores this ion
          reject();
          skip = true;
        } else {
          for (int i = tid; i < DTBL; i += BLOCK) {
            const uint32_t key = tkey[i];
            if (key != 0xFFFFFFFFu && tval[i] > 0.0) {
              const int k = (int)(key & 7u);
              atomicAdd(&c_n[k], 1);
              atomicMin(&c_lo[k], (unsigned long long)bits_of(tval[i]));
              atomicMax(&c_hi[k], (unsigned long long)bits_of(tval[i]));
            }
          }
          __syncthreads();
          // 2. (set s = window s + 1; every round reads the whole tail once for the batch's windows)
          select_batch<BLOCK, CSB>(
              [&](auto&& f) {
                groups(0, ng, [&](int k, bool valid, const Reg& h) {
                  if (valid && !Hits<FMT>::dup(h) && Hits<FMT>::val(h) > 0.0) f(k - 1, bits_of(Hits<FMT>::val(h)));
                });
                for (int i = tid; i < DTBL; i += BLOCK) {
                  const uint32_t key = tkey[i];
                  if (key != 0xFFFFFFFFu && tval[i] > 0.0) f((int)(key & 7u) - 1, bits_of(tval[i]));
                }
              },
              K - 1, c_n + 1, P.q, c_thr + 1, c_st, c_hist, c_flag, c_lo + 1, c_hi + 1);
          // 3. (a wave's partials of window k: part[k][wid], written by this wave only)
          groups(0, ng, [&](int k, bool valid, const Reg& h) {
            double a4[4] = {0.0, 0.0, 0.0, 0.0};
            if (valid && !Hits<FMT>::dup(h)) {
              const double thr = c_thr[k], v = Hits<FMT>::val(h);
              const double y = v > thr ? thr : v;
              const double x = xval(Hits<FMT>::pix(h));
              if (x > 0.0) a4[0] = y;
              a4[1] = y;
              a4[2] = y * y;
              a4[3] = x * y;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) a4[q] = wave_sum_dpp(a4[q]);
            if (lane == 0) {
              double* pk = part + ((size_t)k * NW + wid) * 4;
#pragma unroll
              for (int q = 0; q < 4; ++q) pk[q] += a4[q];
            }
          });
          __syncthreads();  // pass 3's plain partial updates before pass 4's atomics
          // 4. (the table is cleared by the same threads before the tail barrier)
          for (int i = tid; i < DTBL; i += BLOCK) {
            const uint32_t key = tkey[i];
            if (key != 0xFFFFFFFFu) {
              const int k = (int)(key & 7u);
              const double thr = c_thr[k], Y = tval[i];
              const double y = Y > thr ? thr : Y;
              const double x = xval(key >> 3);
              double* pk = part + (size_t)k * NW * 4;
              if (x > 0.0) atomicAdd(&pk[0], y);
              atomicAdd(&pk[1], y);
              atomicAdd(&pk[2], y * y);
              atomicAdd(&pk[3], x * y);
            }
          }
        }
        if (tid < NW) dcnt[tid] = 0;
      }
    } else if (!skip && !(SMG_ABL & 2)) {
      const int ng = uni(D->ngroups);
      // Window sums of y and y^2 come from the prefix sums (descriptor); the stream only joins the tail against
      // the principal image (sum xy, sum y[x>0]: nonzero for the few points whose pixel is in the principal
      // image) and collects duplicate-candidate points.
      int curk = 1;
      int nd = 0;  // this wave's deferred duplicate candidates (uniform)
      uint32_t* wdkey = dkey + wid * DSEG;
      double* wdval = dval + wid * DSEG;
      int gnext = uni(D->gs[2]);
      int wend = uni(D->end[1]);
      // Events: a principal hit (a tail point on a principal pixel, ~0.5% of the points: adds x*y and y[x>0] to
      // its window's partials) or a duplicate candidate (~1%: summed per (pixel, window) before squaring).
      // The stream only tests for them and parks up to two events per lane in registers (the raw hit and its
      // window); their LDS lookups, atomics and list appends run after the stream for all lanes at once.  A
      // lane's third and later events are handled in place (rare).  Partials: part[k][wid] (zeroed in phase 0),
      // written only by this wave, lanes of one instruction in hardware order -- deterministic.
#ifndef SMG_STASH
#define SMG_STASH 1
#endif
      Reg ev0 = Hits<FMT>::zero(), ev1 = Hits<FMT>::zero();
      int evk0 = 0, evk1 = 0, nev = 0;
      // handles one event per lane (pred); principal membership re-tested from the hit when `in` is unknown
      auto handle = [&](bool pred, const Reg& h, int k, bool known, bool in_known, uint64_t bwv, int brv) {
        const uint32_t p = Hits<FMT>::pix(h);
        const uint64_t bit = 1ull << (p & 63);
        bool in = false;
        int r = -1;
        if (pred) {
          if (known) {
            in = in_known;
            if (in) {
              if constexpr (TWO) r = (int)Bpf[brv] + __popcll(bwv & (bit - 1ull));
              else r = (int)pf[p >> 6] + __popcll(bwv & (bit - 1ull));
            }
          } else {
            if constexpr (TWO) r = rank2((int)p);
            else r = bm_test(Hbm, (int)p) ? bm_rank(Hbm, pf, (int)p) : -1;
            in = r >= 0;
          }
        }
        in = in && !(SMG_ABL & 16);
        if (__ballot(in)) {
          if (in) {
            const double x = vals[r];
            const double v = Hits<FMT>::val(h);
            double* pk = part + ((size_t)k * NW + wid) * 4;
            atomicAdd(&pk[3], x * v);
            if (x > 0.0) atomicAdd(&pk[0], v);
          }
        }
        // duplicate candidates: appended to this wave's list segment (ballot compaction, no atomics)
        const bool dup = pred && Hits<FMT>::dup(h) && !(SMG_ABL & 8);
        const uint64_t dm = __ballot(dup);
        if (dm) {
          const int e = nd + (int)__popcll(dm & ((1ull << lane) - 1ull));
          if (dup && e < DSEG) {
            wdkey[e] = (p << 3) | (uint32_t)k;
            wdval[e] = Hits<FMT>::val(h);
          }
          nd += (int)__popcll(dm);
        }
      };
      // Lanes past the end of their window hold a copy of its last point (masked by `valid`); groups past the
      // tail are skipped.  Stage 1 reads the bitmap words of every slot at once; stage 2 handles slot by slot.
      auto process = [&](int c, Reg (&buf)[RC]) {
        uint64_t bw[RC];
        int br[RC];  // two-level: index of the slot's word among the non-empty words
        if constexpr (TWO) {
          uint64_t tw[RC];
          int tp[RC];
#pragma unroll
          for (int j = 0; j < RC; ++j) {
            const uint32_t q = Hits<FMT>::pix(buf[j]) >> 6;
            tw[j] = T64[q >> 6];
            tp[j] = pf[q >> 6];
          }
#pragma unroll
          for (int j = 0; j < RC; ++j) {
            const uint32_t q = Hits<FMT>::pix(buf[j]) >> 6;
            const uint64_t b = 1ull << (q & 63);
            br[j] = (tw[j] & b) ? tp[j] + __popcll(tw[j] & (b - 1ull)) : -1;
            bw[j] = br[j] >= 0 ? W64[br[j]] : 0ull;
          }
        } else {
#pragma unroll
          for (int j = 0; j < RC; ++j) {
            bw[j] = reinterpret_cast<const uint64_t*>(Hbm)[Hits<FMT>::pix(buf[j]) >> 6];
            br[j] = 0;
          }
        }
#pragma unroll
        for (int j = 0; j < RC; ++j) {
          const int G = c * GPC + j * NW + wid;
          if (G < ng) {
            while (G >= gnext) {  // this wave moves on to a later window (uniform)
              ++curk;
              gnext = curk + 1 < MAXK ? uni(D->gs[curk + 1]) : 0x7FFFFFFF;
              wend = uni(D->end[curk]);
            }
            const bool valid = lane < wend - G * 64;
            const Reg h = buf[j];
            const uint32_t p = Hits<FMT>::pix(buf[j]);
            const bool in = valid && (bw[j] & (1ull << (p & 63))) != 0ull;
            const bool ev = in || (valid && Hits<FMT>::dup(buf[j]));
            if (SMG_STASH) {
              const bool s0 = ev && nev == 0, s1 = ev && nev == 1;
              ev0 = s0 ? h : ev0;
              evk0 = s0 ? curk : evk0;
              ev1 = s1 ? h : ev1;
              evk1 = s1 ? curk : evk1;
              const bool ovf = ev && nev >= 2;
              nev += ev ? 1 : 0;
              if (__ballot(ovf)) handle(ovf, h, curk, true, in, bw[j], br[j]);
            } else if (__ballot(ev)) {
              handle(ev, h, curk, true, in, bw[j], br[j]);
            }
          }
        }
      };
      // chunks 0 and 1 are in flight (issued during the previous iteration); later chunks one ahead
      // (refills are issued unconditionally so that exactly 3*RC loads follow each buffer's)
      for (int c = 0; c * GPC < ng; c += 4) {
        vm_wait<3 * RC>(pa);
        process(c, pa);
        issue_chunk(D, c + 4, pa);
        if ((c + 1) * GPC >= ng) break;
        vm_wait<3 * RC>(pb);
        process(c + 1, pb);
        issue_chunk(D, c + 5, pb);
        if ((c + 2) * GPC >= ng) break;
        vm_wait<3 * RC>(pc);
        process(c + 2, pc);
        issue_chunk(D, c + 6, pc);
        if ((c + 3) * GPC >= ng) break;
        vm_wait<3 * RC>(pd);
        process(c + 3, pd);
        issue_chunk(D, c + 7, pd);
      }
#ifndef SMG_PAIR
#define SMG_PAIR 1
#endif
      if (SMG_STASH && SMG_PAIR) {  // the parked events, both at once: lookups in flight together
        if (__ballot(nev > 0)) {
          const uint32_t p0 = Hits<FMT>::pix(ev0), p1 = Hits<FMT>::pix(ev1);
          int r0 = -1, r1 = -1;
          if constexpr (TWO) {
            if (nev > 0) r0 = rank2((int)p0);
            if (nev > 1) r1 = rank2((int)p1);
          } else {
            const uint64_t* bm64 = reinterpret_cast<const uint64_t*>(Hbm);
            const uint64_t w0 = nev > 0 ? bm64[p0 >> 6] : 0ull, w1 = nev > 1 ? bm64[p1 >> 6] : 0ull;
            const int f0 = pf[p0 >> 6], f1 = pf[p1 >> 6];
            const uint64_t b0 = 1ull << (p0 & 63), b1 = 1ull << (p1 & 63);
            r0 = (w0 & b0) ? f0 + __popcll(w0 & (b0 - 1ull)) : -1;
            r1 = (w1 & b1) ? f1 + __popcll(w1 & (b1 - 1ull)) : -1;
          }
          if (SMG_ABL & 16) r0 = r1 = -1;
          if (__ballot(r0 >= 0 || r1 >= 0)) {
            const double x0 = r0 >= 0 ? vals[r0] : 0.0, x1 = r1 >= 0 ? vals[r1] : 0.0;
            if (r0 >= 0) {
              const double v = Hits<FMT>::val(ev0);
              double* pk = part + ((size_t)evk0 * NW + wid) * 4;
              atomicAdd(&pk[3], x0 * v);
              if (x0 > 0.0) atomicAdd(&pk[0], v);
            }
            if (r1 >= 0) {
              const double v = Hits<FMT>::val(ev1);
              double* pk = part + ((size_t)evk1 * NW + wid) * 4;
              atomicAdd(&pk[3], x1 * v);
              if (x1 > 0.0) atomicAdd(&pk[0], v);
            }
          }
          const bool d0 = nev > 0 && Hits<FMT>::dup(ev0) && !(SMG_ABL & 8);
          const bool d1 = nev > 1 && Hits<FMT>::dup(ev1) && !(SMG_ABL & 8);
          const uint64_t m0 = __ballot(d0), m1 = __ballot(d1);
          if (m0 | m1) {
            const uint64_t below = (1ull << lane) - 1ull;
            const int e0 = nd + (int)__popcll(m0 & below);
            const int e1 = nd + (int)__popcll(m0) + (int)__popcll(m1 & below);
            if (d0 && e0 < DSEG) {
              wdkey[e0] = (p0 << 3) | (uint32_t)evk0;
              wdval[e0] = Hits<FMT>::val(ev0);
            }
            if (d1 && e1 < DSEG) {
              wdkey[e1] = (p1 << 3) | (uint32_t)evk1;
              wdval[e1] = Hits<FMT>::val(ev1);
            }
            nd += (int)(__popcll(m0) + __popcll(m1));
          }
        }
      } else if (SMG_STASH) {  // the parked events: membership and ranks re-read from the principal set
        if (__ballot(nev > 0)) handle(nev > 0, ev0, evk0, false, false, 0ull, 0);
        if (__ballot(nev > 1)) handle(nev > 1, ev1, evk1, false, false, 0ull, 0);
      }
      if (lane == 0) dcnt[wid] = nd;
    } else if (!skip && tid < NW) {
      dcnt[tid] = 0;
    }
    STAMP(8);
    // ---- the registers of ion b are dead: ion b+1's principal window and first two chunks go in flight
    if (npos >= 0 && desc_lds_ok(DN, CAPC)) {
      issue_principal(DN);
      if constexpr (!CLIP) {
        issue_chunk(DN, 0, pa);
        issue_chunk(DN, 1, pb);
      }
    }
    if (!skip) clear_table();  // for phase d (its space held the previous ion's chaos candidates)
    STAMP(10);
    __syncthreads();
    // the principal statistics (phase 2's per-wave sums, in wave order) and the level index per pixel
    double sx = 0.0, sxx = 0.0, s0 = 0.0, npx_pos = 0.0, vmax = 0.0;
    if (!skip) {
      double t[5] = {0.0, 0.0, 0.0, 0.0, -INFINITY};
#pragma unroll
      for (int w = 0; w < NW; ++w) {
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] += red[q * NW + w];
        t[4] = red[4 * NW + w] > t[4] ? red[4 * NW + w] : t[4];
      }
      sx = t[0];
      sxx = t[1];
      s0 = t[2];
      npx_pos = t[3];
      vmax = t[4];
    }
    const bool chaos_ok = !skip && (sx > 0.0) && (npx_pos >= 4.0) && !(SMG_ABL & 1);
    if (chaos_ok && nnz > OL_MAX && !(SMG_ABL & 128)) {  // else after the screen, if it finds candidates
      for (int r = tid; r < nnz; r += BLOCK) Lv[r] = (uint8_t)level_fast(vals[r], vmax, P);
      __syncthreads();  // the values are read here before the pixel list (olist) overwrites them in the chaos phase
    }
    STAMP(9);
    // ---- deferred duplicate candidates: exact per-(pixel, window) sums, squared into the partials --------
    // Thread t owns list slot t (segment t / DSEG, entry t % DSEG); the entries are summed per key in an LDS
    // table and each key's square goes to its window's partial (LDS f64 atomics: the few keys per ion make
    // the order of these additions immaterial at f64 precision).
    if (!skip) {
      int nd_tot = 0, nd_max = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        nd_tot += dcnt[w];
        nd_max = max(nd_max, dcnt[w]);
      }
      if (nd_max > DSEG) {
        reject();
        skip = true;
      } else if (nd_tot > 0 && !(SMG_ABL & 512)) {
        static_assert(NW * DSEG == BLOCK, "one list slot per thread");
        if ((tid % DSEG) < dcnt[tid / DSEG] && !tbl_add<DTBL>(tkey, tval, dkey[tid], dval[tid])) ctr[C_ABORT] = 1;
        __syncthreads();
        if (ctr[C_ABORT]) {
          reject();
          skip = true;
        } else {
          for (int i = tid; i < DTBL; i += BLOCK) {
            const uint32_t key = tkey[i];
            if (key != 0xFFFFFFFFu) {
              const double y = tval[i];
              atomicAdd(&part[(size_t)(key & 7u) * NW * 4 + 2], y * y);
            }
          }
          // SMG_NOB3: no barrier -- the chaos phase's first writes into this region (pass A's survivor list at
          // the bottom of the candidate array) stay below the table, and the partials are read after later ones
          if (!(SMG_NOB3 && SMG_SCREEN2P && chaos_ok && !P.erosion_border)) __syncthreads();
        }
      }
    }
    STAMP(3);

    // ---- phase 4a: chaos candidates (pixels with eL >= 1) from the principal pixels -----------------
    // (i) bit-level screen: a candidate p in cross(s) survives if its 3x3 box is covered by the
    //     dilated bitmap (superset of the exact condition) and s is its owner (smallest principal pixel
    //     of cross(p)); survivors go to an LDS list (the value region is free once L is computed).
    // (ii) exact eL for the survivors from the level indices.
    double chaos_raw = NAN;
    uint32_t flags = 0;
    if (!skip && chaos_ok) {
      if (nnz > OL_MAX) {
        // olist did not fit behind the values: the distinct principal pixels from the bitmap, rank order
        // (olist[pf[w] + i] = i-th set bit of word w); the values are dead
        if constexpr (TWO) {
          // top-level words strided over the threads; word q's pixels start at rank B[r]
          for (int tw = tid; tw < nT; tw += BLOCK) {
            uint64_t t = T64[tw];
            int r = pf[tw];
            while (t) {
              const int q = tw * 64 + __builtin_ctzll(t);
              uint64_t bits = W64[r];
              int o = Bpf[r];
              while (bits) {
                olist[o++] = (uint32_t)(q * 64 + __builtin_ctzll(bits));
                bits &= bits - 1;
              }
              ++r;
              t &= t - 1;
            }
          }
        } else {
          const uint64_t* bm64 = reinterpret_cast<const uint64_t*>(Hbm);
          constexpr int WPT = (NPX_LDS_MAX / 64 + BLOCK - 1) / BLOCK;
          uint64_t wb[WPT];
#pragma unroll
          for (int i = 0; i < WPT; ++i) wb[i] = (tid * WPT + i < n64) ? bm64[tid * WPT + i] : 0ull;
#pragma unroll
          for (int i = 0; i < WPT; ++i) {
            uint64_t bits = wb[i];
            if (!bits) continue;
            const int w = tid * WPT + i;
            int r = pf[w];
            while (bits) {
              olist[r++] = (uint32_t)(w * 64 + __builtin_ctzll(bits));
              bits &= bits - 1;
            }
          }
        }
        __syncthreads();
      }
      // the 7x7 window of principal pixel s: H[d] = columns cs-3..cs+3 of row rs-3+d
      auto rows7 = [&](int s, int& rs, int& cs, uint32_t& cv, uint32_t (&H)[7]) {
        rowcol(s, P, rs, cs);
        // valid-column mask of columns cs-3..cs+3
        const int clo = 3 - cs > 0 ? 3 - cs : 0, chi = P.ncols - cs + 3 < 7 ? P.ncols - cs + 3 : 7;
        cv = ((1u << chi) - 1u) & ~((1u << clo) - 1u);
#pragma unroll
        for (int d = 0; d < 7; ++d) {
          if constexpr (TWO) {
            // columns cs-3..cs+3 of row rs-3+d from words q and q+1 of the two-level set
            const int row = rs - 3 + d;
            const bool rv = (unsigned)row < (unsigned)P.nrows;
            const int st = (rv ? row : 0) * P.ncols + cs - 3;
            const int q = st >> 6, b = st & 63;  // st >= -3: q >= -1 (empty)
            int dummy;
            const uint64_t w0 = word2(q, dummy), w1 = b > 57 ? word2(q + 1, dummy) : 0ull;
            const uint32_t v = (uint32_t)((b ? ((w0 >> b) | (w1 << (64 - b))) : w0) & 0x7Full) & cv;
            H[d] = rv ? v : 0u;
          } else {
            H[d] = bits7(Hbm, rs - 3 + d, cs - 3, cv, P);
          }
        }
      };
      // sparsity pre-filter (erosion border = background only): an eL>0 pixel p in the cross of s has its 3x3
      // box covered by 4-crosses of principal pixels, which takes at least three of them (one cross meets at
      // most two corners of the box, and a cross through the centre none), all in p's 5x5, inside s's 7x7
#ifndef SMG_SCREEN3
#define SMG_SCREEN3 1
#endif
      auto sparse = [&](const uint32_t (&H)[7]) {
        return !P.erosion_border &&
               (SMG_SCREEN3 ? (__popc(H[0]) + __popc(H[1]) + __popc(H[2]) + __popc(H[3]) + __popc(H[4]) +
                               __popc(H[5]) + __popc(H[6])) < 3
                            : (H[0] | H[1] | H[2] | (H[3] & ~8u) | H[4] | H[5] | H[6]) == 0u);
      };
      // Pass A (erosion border 0): the principal pixels that pass the pre-filter (a few percent of a noise
      // image) are listed, wave-compacted, from the top of the candidate array down; pass B runs the full
      // screen over full waves of them only.  Candidates fill the array from the bottom (capacity CAPC - nsurv).


      const int nscreen = (SMG_ABL & 64) ? 0 : nnz;
      int nsurv = nscreen, ccap = CAPC, cbase = 0;
      // the survivor list stays below the duplicate table (its last readers may still run, SMG_NOB3)
      constexpr int SURV_CAP = (int)((LY::o_tkey - LY::o_filt) / 4);
      bool two_pass = SMG_SCREEN2P && !P.erosion_border;
      if (two_pass) {
        for (int ob = 0; ob < nscreen; ob += BLOCK) {  // uniform trip count
          const int oc_i = ob + tid;
          const int s0p = oc_i < nnz ? (int)olist[oc_i] : 0;
          int rs, cs;
          uint32_t cv, H[7];
          rows7(s0p, rs, cs, cv, H);
          const bool surv = oc_i < nnz && !sparse(H);
          const uint64_t m = __ballot(surv);
          if (m) {
            int wbase = 0;
            if (lane == 0) wbase = atomicAdd(&ctr[C_NS], (int)__popcll(m));
            const int idx = __builtin_amdgcn_readfirstlane(wbase) + (int)__popcll(m & ((1ull << lane) - 1ull));
            if (surv && idx < SURV_CAP) epix[idx] = (uint32_t)s0p;
          }
        }
        __syncthreads();
        nsurv = ctr[C_NS];
        ccap = CAPC - nsurv;
        cbase = nsurv;
        if (nsurv * 4 > CAPC || nsurv > SURV_CAP) {  // a dense image: its candidates need the whole array --
          two_pass = false;                          // screen every pixel
          nsurv = nscreen;
          ccap = CAPC;
          cbase = 0;
        }
      }
      uint32_t* ecand = epix + cbase;  // candidates (behind the survivor list)
      for (int ob = 0; ob < nsurv; ob += BLOCK) {  // uniform trip count: wave-compacted
        const int oc_i = ob + tid;
        const int s = oc_i < nsurv ? (int)(two_pass ? epix[oc_i] : olist[oc_i]) : 0;
        int rs, cs;
        uint32_t cv, H[7];
        rows7(s, rs, cs, cv, H);
        const bool isolated = sparse(H);
        uint32_t pass = 0;
        if (oc_i < nsurv && !isolated) {
        uint32_t Dl[7];
        Dl[0] = Dl[6] = 0;
#pragma unroll
        for (int d = 1; d <= 5; ++d) {
          const int row = rs - 3 + d;
          const bool rv = row >= 0 && row < P.nrows;
          uint32_t x = (H[d] | (H[d] << 1) | (H[d] >> 1) | H[d - 1] | H[d + 1]) & cv;
          if (!rv) x = 0;
          if (P.erosion_border) x |= rv ? (~cv & 0x7Fu) : 0x7Fu;
          Dl[d] = x & 0x7Fu;
        }
#define SMG_HB(dr, dc) ((H[3 + (dr)] >> (3 + (dc))) & 1u)
#define SMG_BOX(dr, dc) ((((Dl[2 + (dr)] >> (2 + (dc))) & 7u) == 7u) && (((Dl[3 + (dr)] >> (2 + (dc))) & 7u) == 7u) && \
                         (((Dl[4 + (dr)] >> (2 + (dc))) & 7u) == 7u))
        const bool in_l = cs > 0, in_r = cs + 1 < P.ncols, in_u = rs > 0, in_d = rs + 1 < P.nrows;
        if (SMG_BOX(0, 0) && !SMG_HB(-1, 0) && !SMG_HB(0, -1)) pass |= 1u;
        if (in_r && SMG_BOX(0, 1) && !SMG_HB(-1, 1)) pass |= 2u;
        if (in_l && SMG_BOX(0, -1) && !SMG_HB(-1, -1) && !SMG_HB(0, -2) && !SMG_HB(0, -1)) pass |= 4u;
        if (in_u && SMG_BOX(-1, 0) && !SMG_HB(-2, 0) && !SMG_HB(-1, -1) && !SMG_HB(-1, 0) && !SMG_HB(-1, 1))
          pass |= 8u;
        if (in_d && SMG_BOX(1, 0)) pass |= 16u;
#undef SMG_BOX
#undef SMG_HB
        }
        // wave-compacted append: one LDS atomic per wave
        const int cnt = __popc(pass);
        const int inc = wave_incl_scan_dpp(cnt);
        const int wtot = __builtin_amdgcn_readlane(inc, 63);
        if (wtot > 0) {
          int wbase = 0;
          if (lane == 63) wbase = atomicAdd(&ctr[C_NE], wtot);
          int idx = __builtin_amdgcn_readlane(wbase, 63) + inc - cnt;
          while (pass) {
            const int ci = __ffs(pass) - 1;
            pass &= pass - 1;
            const int p = s + (ci == 1 ? 1 : ci == 2 ? -1 : ci == 3 ? -P.ncols : ci == 4 ? P.ncols : 0);
            if (idx < ccap) ecand[idx] = (uint32_t)p;
            ++idx;
          }
        }
      }
      __syncthreads();
      STAMP(4);
      const int ncand = (SMG_ABL & 32) ? 0 : ctr[C_NE];
      if (ncand > ccap) {
        reject();
        skip = true;
      }
      // level index L: precomputed for every principal pixel when there are many candidates, else computed
      // on demand from the values (intact: olist sits behind them, candidates elsewhere) for the few principal
      // pixels around the candidates
      const bool lazyL = (nnz <= OL_MAX) && (ncand * 16 < nnz);
      if (!skip && ncand > 0 && nnz <= OL_MAX && !lazyL) {
        for (int r = tid; r < nnz; r += BLOCK) Lv[r] = (uint8_t)level_fast(vals[r], vmax, P);
        __syncthreads();
      }
      if (!skip) {
        // (ii) exact eL(p) = min_{q in box(p)} max_{q' in cross[q], in image} L(q').  The 21 pixels involved
        // (p's 5x5 neighbourhood without corners) come from five bitmap rows read at once; L is fetched only
        // for the principal pixels among them and packed six bits per column.
        int emax_local = 0;
        const uint64_t* bm64 = reinterpret_cast<const uint64_t*>(Hbm);
        for (int c = tid; c < ncand; c += BLOCK) {
          const int p = (int)ecand[c];
          int rp, cp;
          rowcol(p, P, rp, cp);
          const int clo = 2 - cp > 0 ? 2 - cp : 0, chi = P.ncols - cp + 2 < 5 ? P.ncols - cp + 2 : 5;
          const uint32_t cv5 = ((1u << chi) - 1u) & ~((1u << clo) - 1u);  // columns cp-2..cp+2 in the image
          uint64_t Lrow[5];  // 8 bits per column: level indices go up to nlevels <= 254
#pragma unroll
          for (int d = 0; d < 5; ++d) {
            const int row = rp - 2 + d;
            const bool rv = (unsigned)row < (unsigned)P.nrows;
            const int st = (rv ? row : 0) * P.ncols + cp - 2;  // >= -2: the guard word in front reads as zero
            const int w = st >> 6, b = st & 63;
            uint64_t w0, w1;
            int r0, r1;
            if constexpr (TWO) {
              w0 = word2(w, r0);
              w1 = word2(w + 1, r1);
            } else {
              w0 = bm64[w];
              w1 = bm64[w + 1];
              r0 = pf[w];
              r1 = pf[w + 1];
            }
            const uint32_t bits = rv ? (uint32_t)((b ? ((w0 >> b) | (w1 << (64 - b))) : w0) & 31u) & cv5 : 0u;
            uint64_t packed = 0;
            for (uint32_t rest = bits; rest; rest &= rest - 1u) {
              const int j = __builtin_ctz(rest);
              const int bj = b + j;  // bit of column cp-2+j in w0 (bj < 64) or w1
              const int r = bj < 64 ? r0 + __popcll(w0 & ((1ull << bj) - 1ull))
                                    : r1 + __popcll(w1 & ((1ull << (bj - 64)) - 1ull));
              const uint32_t L = lazyL ? (uint32_t)level_fast(vals[r], vmax, P) : (uint32_t)Lv[r];
              packed |= (uint64_t)L << (8 * j);
            }
            Lrow[d] = packed;
          }
#define SMG_L(r, cc) ((uint32_t)((Lrow[r] >> (8 * (cc))) & 0xFFull))
          int mn = 1 << 20;
          bool outside = false;
#pragma unroll
          for (int a2 = -1; a2 <= 1; ++a2) {
#pragma unroll
            for (int b2 = -1; b2 <= 1; ++b2) {
              const int rq = rp + a2, cq = cp + b2;
              if (rq < 0 || rq >= P.nrows || cq < 0 || cq >= P.ncols) {
                outside = true;
                continue;
              }
              const int R = 2 + a2, C = 2 + b2;
              uint32_t dl = SMG_L(R, C);
              dl = max(dl, SMG_L(R - 1, C));
              dl = max(dl, SMG_L(R + 1, C));
              dl = max(dl, SMG_L(R, C - 1));
              dl = max(dl, SMG_L(R, C + 1));
              mn = min(mn, (int)dl);
            }
          }
#undef SMG_L
          if (outside && !P.erosion_border) mn = 0;
          if (mn >= (1 << 20)) mn = 0;
          eL8[c] = (uint8_t)mn;
          emax_local = max(emax_local, mn);
        }
        if (emax_local > 0) atomicMax(&ctr[C_EMAX], emax_local);
        __syncthreads();
        STAMP(5);

        // ---- phase 4b: Kruskal over eL (levels descending) with an LDS union-find -------------------
        double sum_c = 0.0;
        const int emax_all = ctr[C_EMAX];
        if (emax_all > 0 && ncand <= WAVE) {
          // few candidates (most noise images): wave 0 alone, one candidate per lane; forward neighbours
          // found by comparing pixel indices across lanes, union-find over candidate indices in LDS; no
          // bitmap rebuild and no barrier.  Only wave 0 needs the result (finalize).
          if (wid == 0) {
            uint32_t* upar = reinterpret_cast<uint32_t*>(red);  // 64 entries (red is free until finalize)
            const bool act = lane < ncand;
            const int p = act ? (int)ecand[lane] : -1;
            const int e = act ? (int)eL8[lane] : 0;
            int rp = 0, cp = 0;
            rowcol(p < 0 ? 0 : p, P, rp, cp);
            int nb[4] = {-1, -1, -1, -1};
            for (int j = 0; j < ncand; ++j) {
              const int pj = __shfl(p, j, WAVE), ej = __shfl(e, j, WAVE);
              if (e >= 1 && ej >= 1) {
                if (cp + 1 < P.ncols && pj == p + 1) nb[0] = j;
                if (rp + 1 < P.nrows) {
                  if (pj == p + P.ncols) nb[1] = j;
                  if (P.connectivity == 8 && cp > 0 && pj == p + P.ncols - 1) nb[2] = j;
                  if (P.connectivity == 8 && cp + 1 < P.ncols && pj == p + P.ncols + 1) nb[3] = j;
                }
              }
            }
            int eq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int v = __shfl(e, nb[q] < 0 ? 0 : nb[q], WAVE);
              eq[q] = nb[q] < 0 ? 0 : (e < v ? e : v);  // edge weight min(eL)
            }
            upar[lane] = (uint32_t)lane;
            double wsum = 0.0;
            for (int t = emax_all; t >= 1; --t) {
#pragma unroll
              for (int q = 0; q < 4; ++q)
                if (eq[q] == t && uf_unite(upar, (uint32_t)lane, (uint32_t)nb[q])) wsum += (double)t;
            }
            sum_c = wave_sum_dpp(e >= 1 ? (double)e : 0.0) - wave_sum_dpp(wsum);
          }
        } else if (emax_all > 0) {
          uint4* z = reinterpret_cast<uint4*>(Hbm);  // two-level: W and T
          for (int i = tid; i < P.w32 / 4; i += BLOCK) z[i] = make_uint4(0, 0, 0, 0);  // guard stays zero
          __syncthreads();
          int m;
          if constexpr (TWO) {
            m = build2([&](auto&& f) {
              for (int i = tid; i < ncand; i += BLOCK)
                if (eL8[i]) f(0, ecand[i]);
            });
          } else {
            for (int i = tid; i < ncand; i += BLOCK)
              if (eL8[i]) atomicOr(&Hbm[ecand[i] >> 5], 1u << (ecand[i] & 31));
            __syncthreads();
            m = bm_build_prefix<NW>(Hbm, pf, n64, wsc);
          }
          for (int i = tid; i < ncand; i += BLOCK) {
            if (!eL8[i]) continue;
            const uint32_t p = ecand[i];
            const int r = TWO ? rank2((int)p) : bm_rank(Hbm, pf, (int)p);
            epix_r[r] = p;
            eLr[r] = eL8[i];
          }
          __syncthreads();
          for (int r = tid; r < m; r += BLOCK) par[r] = (uint32_t)r;
          __syncthreads();
          const int emax = emax_all;
          double wsum = 0.0, esum = 0.0;
          for (int r = tid; r < m; r += BLOCK) esum += (double)eLr[r];
          for (int t = emax; t >= 1; --t) {
            for (int r = tid; r < m; r += BLOCK) {
              const int e = eLr[r];
              if (e < t) continue;
              const int p = (int)epix_r[r];
              int rp, cp;
              rowcol(p, P, rp, cp);
              auto edge = [&](int q) {
                int rq;
                if constexpr (TWO) {
                  rq = rank2(q);
                  if (rq < 0) return;
                } else {
                  if (!bm_test(Hbm, q)) return;
                  rq = bm_rank(Hbm, pf, q);
                }
                const int eq = eLr[rq];
                if ((e < eq ? e : eq) == t) {
                  if (uf_unite(par, (uint32_t)r, (uint32_t)rq)) wsum += (double)t;
                }
              };
              if (cp + 1 < P.ncols) edge(p + 1);
              if (rp + 1 < P.nrows) {
                edge(p + P.ncols);
                if (P.connectivity == 8) {
                  if (cp > 0) edge(p + P.ncols - 1);
                  if (cp + 1 < P.ncols) edge(p + P.ncols + 1);
                }
              }
            }
            __syncthreads();
          }
          double acc[2] = {esum, wsum};
          block_sum<BLOCK, 2, true>(acc, red);
          sum_c = acc[0] - acc[1];
        }
        chaos_raw = 1.0 - sum_c / (double)P.nlevels / npx_pos;
        STAMP(6);
      }
    } else if (!skip) {
      flags |= SMG_ION_CHAOS_NAN;
    }

    // ---- the ion's sums -> its record (the descriptor's consumed fields, IonRec): ion_finalize_kernel turns them
    // into the scores after the pass (formula_img_validator.py:78-84 + the restated pyImagingMSpec functions), so
    // the f64 divisions and square roots stay out of this kernel.  Wave 0, lane k = window k.
    if (!skip && wid == 0) {
      IonRec* G = reinterpret_cast<IonRec*>(desc + pos);
      const int k = lane;
      if (k < K) {
        // Σy² + the squared per-pixel sums of duplicate candidates (CLIP: the clipped image's sums, Σy too)
        double sk = 0.0, syy = CLIP ? 0.0 : D->syy[k], sxy = 0.0, sy = 0.0;
        if (k == 0) {
          sk = s0;
        } else {
#pragma unroll
          for (int w = 0; w < NW; ++w) {
            const double* pk = part + ((size_t)k * NW + w) * 4;
            sk += pk[0];
            sy += pk[1];
            syy += pk[2];
            sxy += pk[3];
          }
        }
        G->s[k] = sk;
        G->sxy[k] = sxy;
        G->syy[k] = syy;
        if (CLIP && k > 0) G->sy[k] = sy;
      }
      if (lane == 0) {
        G->sx = sx;
        G->sxx = sxx;
        G->chaos = chaos_raw;
        G->flags = flags | big_flag | (TWO ? SMG_ION_TWO_LEVEL : 0u) | (uint32_t)D->hits;
        G->state = 1u;
      }
    }
    if (npos < 0) break;
    if (began && wid != 0) clear_set_vals(tid - WAVE, BLOCK - WAVE);  // (the chaos phase is done with both)
    pos = npos;
    npos = n2pos;
    cur ^= 1;
    __syncthreads();  // the next ion starts on cleared LDS structures
    STAMP(7);
  }
  STAMP_FLUSH();
  // no load of this wave outlives it
  vm_wait<0>(pa);
  vm_wait<0>(pb);
  vm_wait<0>(pc);
  vm_wait<0>(pd);
  vm_wait<0>(pe);
}

// Scores of the positions the LDS passes scored (IonRec state 1), from the sums they recorded (formula_img_validator.py
// :78-84 + the restated pyImagingMSpec functions, the arithmetic of finalize_ion): eight lanes per position, lane k
// = window k, so that a record's fields are read as coalesced 64-B runs; the sums over windows are taken in window
// order (lane 0 gathers them), as finalize_ion does.
__global__ void __launch_bounds__(256) ion_finalize_kernel(const IonRec* __restrict__ rec, int64_t n, double npx,
                                                           double* __restrict__ oc, double* __restrict__ osp,
                                                           double* __restrict__ osc, double* __restrict__ omsm,
                                                           uint32_t* __restrict__ oflags) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = t >> 3;
  const int k = (int)(t & 7);
  // every field this lane uses is read at once, before the record's state and K are known (one memory round trip
  // rather than three; k < 8 stays inside the record's arrays)
  const bool inr = i < n;
  const IonRec* R = rec + (inr ? i : 0);
  const uint32_t st = R->state;
  const int Kr = R->K;
  const double tk0 = R->theor[k], sk0 = R->s[k], sx = R->sx, sxx = R->sxx;
  const double sy = R->sy[k], syy = R->syy[k], sxy = R->sxy[k];
  const double chaos0 = R->chaos;
  const int32_t ion0 = R->ion;
  const uint32_t flags0 = R->flags;
  const bool live = inr && st == 1u;
  const int K = live ? Kr : 0;
  const bool act = live && k < K;
  const double tk = act ? tk0 : 0.0, sk = act ? sk0 : 0.0;
  double rt = 0.0;  // r_k * t_k of isotope_image_correlation (k >= 1)
  if (act && k >= 1 && K >= 2) {
    const double n1 = npx - 1.0;
    const double sd0 = sqrt((sxx - sx * sx / npx) / n1);
    const double syy_c = (syy - sy * sy / npx) / n1;
    const double sxy_c = (sxy - sx * sy / npx) / n1;
    double r = sxy_c / sqrt(syy_c) / sd0;
    if (!isnan(r)) r = r > 1.0 ? 1.0 : (r < -1.0 ? -1.0 : r);
    if (isinf(r)) r = 0.0;
    rt = r * tk;
  }
  // gather the eight lanes' terms in lane 0 of the group (window order)
  const int g0 = (threadIdx.x & 63) & ~7;
  double T[MAXK], S[MAXK], RT[MAXK], D[MAXK];
#pragma unroll
  for (int j = 0; j < MAXK; ++j) {
    T[j] = __shfl(tk, g0 + j, 64);
    S[j] = __shfl(sk, g0 + j, 64);
    RT[j] = __shfl(rt, g0 + j, 64);
  }
  // isotope_pattern_match: every lane of the group forms the two norms (same order, same values), lane k its own
  // term |t_k / |t| - s_k / |s||, and lane 0 sums the terms in window order
  double tt = 0.0, ss = 0.0;
  for (int j = 0; j < K; ++j) {
    tt += T[j] * T[j];
    ss += S[j] * S[j];
  }
  const double nt = sqrt(tt), ns = sqrt(ss);
  const double dk = act ? fabs(tk / nt - sk / ns) : 0.0;
#pragma unroll
  for (int j = 0; j < MAXK; ++j) D[j] = __shfl(dk, g0 + j, 64);
  if (!live || k != 0) return;
  double acc = 0.0;
  for (int j = 0; j < K; ++j) acc += D[j];
  double spectral = 1.0 - acc / (double)K;
  if (spectral == 1.0) spectral = 0.0;
  double spatial = 0.0;
  if (K >= 2) {
    double num = 0.0, den = 0.0;
    for (int j = 1; j < K; ++j) {
      num += RT[j];
      den += T[j];
    }
    spatial = num / den;
  }
  double chaos = chaos0;
  if (!isnan(chaos) && fabs(chaos - 1.0) <= 1e-8 + 1e-5) chaos = 0.0;  // np.isclose(moc, 1.0)
  chaos = clean(chaos);
  spatial = clean(spatial);
  spectral = clean(spectral);
  const int64_t ion = ion0;
  oc[ion] = chaos;
  osp[ion] = spatial;
  osc[ion] = spectral;
  omsm[ion] = chaos * spatial * spectral;
  oflags[ion] = flags0;
}

// position list -> ion list (when the big-ion pass is skipped, the dense kernel reads ion indices)
__global__ void pos_to_ion_kernel(const IonDesc* __restrict__ desc, const uint32_t* __restrict__ in,
                                  const uint32_t* __restrict__ count, uint32_t* __restrict__ out,
                                  uint32_t* __restrict__ out_count) {
  const uint32_t n = *count;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    out[i] = (uint32_t)desc[in[i]].ion;
  if (blockIdx.x == 0 && threadIdx.x == 0) *out_count = n;
}

// every position into the list (images too large for the main pass but not for the big-ion pass)
__global__ void list_positions_kernel(uint32_t* list, uint32_t* count, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) list[i] = (uint32_t)i;
  if (i == 0) *count = (uint32_t)n;
}



// ---------------------------------------------------------------------------------------------
// dense path: persistent workgroups, one global scratch slot each
// ---------------------------------------------------------------------------------------------
#ifndef SMG_DBLOCK
#define SMG_DBLOCK 1024
#endif
constexpr int DBLOCK = SMG_DBLOCK;  // dense kernel workgroup size
constexpr int DNW = DBLOCK / WAVE;
// Sparse over the slot's pixel-sized arrays: x / y (f64 images), L8 (level index) and E8 (eL) are zero
// between ions and only the pixels a window touches are written and cleared again, so an ion costs
// O(window points + chaos candidates), not O(K * N_px).  Each window lists its distinct pixels (plist: principal,
// ylist: current tail window); mark holds generation tags (one fresh tag per window) through which
// duplicate-flagged points claim their pixel.  par and elist are free until chaos and double as the clip's value
// list (vals, 8 B per pixel).
struct DenseSlot {
  double* x;
  double* y;
  uint32_t* par;
  uint32_t* elist;
  uint32_t* mark;
  uint32_t* plist;
  uint32_t* ylist;
  uint8_t* L8;
  uint8_t* E8;
  uint32_t* gbm;  // presence bitmap when it does not fit the LDS (npx bits)
  double* vals;   // aliases par + elist
};

static inline size_t dense_slot_bytes(int npx) {
  return al16((size_t)npx * 8) * 2 + al16((size_t)npx * 8) + al16((size_t)npx * 4) * 3 + al16((size_t)npx) * 2 +
         al16(((size_t)npx + 31) / 32 * 4 + 4) + 256;
}

__device__ __forceinline__ DenseSlot dense_slot(unsigned char* base, int npx) {
  DenseSlot S;
  auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  size_t o = 0;
  S.x = reinterpret_cast<double*>(base + o);
  o += a16((size_t)npx * 8);
  S.y = reinterpret_cast<double*>(base + o);
  o += a16((size_t)npx * 8);
  S.par = reinterpret_cast<uint32_t*>(base + o);  // par (npx u32) then elist (npx u32): 8*npx bytes
  S.elist = S.par + npx;
  S.vals = reinterpret_cast<double*>(base + o);
  o += a16((size_t)npx * 8);
  S.mark = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)npx * 4);
  S.plist = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)npx * 4);
  S.ylist = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)npx * 4);
  S.L8 = base + o;
  o += a16((size_t)npx);
  S.E8 = base + o;
  o += a16((size_t)npx);
  S.gbm = reinterpret_cast<uint32_t*>(base + o);
  return S;
}

// A slot is private to one workgroup (one CU, one XCD's L2): its global atomics complete in that L2 and its
// readers load past L1 (ld_agent), so phases only need every lane's memory operations acknowledged and a
// barrier -- no agent-scope fence (on gfx950 that writes back and invalidates the XCD's L2).
__device__ __forceinline__ void slot_sync() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t guf_find(uint32_t* par, uint32_t x) {
  while (true) {
    const uint32_t p = ld_agent(&par[x]);
    if (p == x) return x;
    const uint32_t g = ld_agent(&par[p]);
    if (g != p) __hip_atomic_store(&par[x], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x = g;
  }
}

__device__ __forceinline__ bool guf_unite(uint32_t* par, uint32_t a, uint32_t b) {
  while (true) {
    a = guf_find(par, a);
    b = guf_find(par, b);
    if (a == b) return false;
    if (a < b) {
      const uint32_t t = a;
      a = b;
      b = t;
    }
    const uint32_t old = atomicCAS(&par[a], a, b);
    if (old == a) return true;
  }
}

// block-wide sum of NV doubles for the 16-wave dense workgroup: wave partials in LDS, then every wave reduces
// the 16 partials with one lane each (same order everywhere; keeps the reduction out of the register budget)
template <int NV>
__device__ __forceinline__ void dblock_sum(double (&v)[NV], double* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = wave_sum(v[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) scratch[j * DNW + wid] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = wave_sum(lane < DNW ? scratch[j * DNW + lane] : 0.0);
  __syncthreads();
}

// index of this lane's item in a block-wide list when pred holds (wave-aggregated LDS counter)
__device__ __forceinline__ int wave_append(bool pred, int* cnt) {
  const uint64_t m = __ballot(pred);
  if (m == 0ull) return -1;
  const int lane = threadIdx.x & 63;
  const int first = __ffsll((unsigned long long)m) - 1;
  int base = 0;
  if (lane == first) base = atomicAdd(cnt, __popcll(m));
  base = __shfl(base, first);
  return pred ? base + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

// Presence bitmap of the principal image: in the LDS (ds ops; LDS = true) or, for images too large for it, in
// the slot's global memory, whose bits are set by atomics in L2 and read past L1.
template <bool LDS>
struct PresenceBits {
  uint32_t* w;
  __device__ __forceinline__ uint32_t word(int i) const {
    if constexpr (LDS) return w[i];
    else return ld_agent(&w[i]);
  }
  __device__ __forceinline__ bool test(uint32_t p) const { return (word((int)(p >> 5)) >> (p & 31)) & 1u; }
  __device__ __forceinline__ void set(uint32_t p) const { atomicOr(&w[p >> 5], 1u << (p & 31)); }
  __device__ __forceinline__ void clear_word_of(uint32_t p) const { w[p >> 5] = 0u; }
  // bits of columns c0-3 .. c0+3 of row r (bit j = column c0-3+j; 0 outside the image); one extra zero word
  // follows the bitmap
  __device__ __forceinline__ uint32_t row7(int r, int c0, int nr, int nc) const {
    if (r < 0 || r >= nr) return 0u;
    const int lc = c0 - 3;
    const int64_t g = (int64_t)r * nc + lc;
    uint32_t v;
    if (g >= 0) {
      const int wi = (int)(g >> 5);
      v = __builtin_amdgcn_alignbit(word(wi + 1), word(wi), (uint32_t)(g & 31));
    } else {
      v = word(0) << (uint32_t)(-g);
    }
    uint32_t cm = 0x7Fu;
    if (lc < 0) cm &= 0x7Fu << (uint32_t)(-lc);
    if (c0 + 3 >= nc) cm &= 0x7Fu >> (uint32_t)(c0 + 3 - (nc - 1));
    return v & cm;
  }
};

#ifndef SMG_DU
#define SMG_DU 4
#endif
constexpr int DU = SMG_DU;  // dense kernel: points per thread with loads in flight together

// The window's image into img (zero outside its listed pixels).  A point without the duplicate-candidate flag is
// alone on its pixel in the window: it stores its value and lists the pixel.  Flagged points add atomically and
// the first lane to tag the pixel with `gen` lists it; listed pixels go into the presence bitmap when one is given.
// Returns the number of listed pixels (ends with slot_sync: the image is complete in L2 for ld_agent readers).
template <int FMT, bool SET, bool LDS>
__device__ int scatter_window(const Hits<FMT>& hits, int64_t a, int64_t b, double* img, uint32_t* mark,
                              uint32_t gen, uint32_t* list, int* cnt, PresenceBits<LDS> bm) {
  using H = Hits<FMT>;
  if (threadIdx.x == 0) *cnt = 0;
  __syncthreads();
  for (int64_t i0 = a; i0 < b; i0 += (int64_t)DBLOCK * DU) {
    typename H::Reg r[DU];
#pragma unroll
    for (int u = 0; u < DU; ++u) {
      const int64_t i = i0 + (int64_t)u * DBLOCK + threadIdx.x;
      r[u] = i < b ? hits.load(i) : H::zero();
    }
#pragma unroll
    for (int u = 0; u < DU; ++u) {
      const int64_t i = i0 + (int64_t)u * DBLOCK + threadIdx.x;
      bool own = false;
      const uint32_t p = H::pix(r[u]);
      if (i < b) {
        const double v = H::val(r[u]);
        if (H::dup(r[u])) {
          atomicAdd(&img[p], v);
          own = atomicExch(&mark[p], gen) != gen;
        } else {
          img[p] = v;
          own = true;
        }
        if (SET && own) bm.set(p);
      }
      const int idx = wave_append(own, cnt);
      if (own) list[idx] = p;
    }
  }
  slot_sync();
  const int n = *cnt;
  __syncthreads();
  return n;
}

// The principal window without the clip: scatter_window plus the principal statistics.  An unflagged point's
// value is final (it is alone on its pixel): it goes to pvals[list index] and into acc / mx at once.  Flagged
// owners are listed by list index in fidx (their sums are complete only after the scatter): the caller reads
// them back from img.  Returns the number of listed pixels; *fcnt holds the number of flagged owners.
template <int FMT, bool LDS>
__device__ int scatter_principal(const Hits<FMT>& hits, int64_t a, int64_t b, double* img, uint32_t* mark,
                                 uint32_t gen, uint32_t* list, double* pvals, uint32_t* fidx, int* cnt, int* fcnt,
                                 PresenceBits<LDS> bm, double (&acc)[4], double& mx) {
  using H = Hits<FMT>;
  if (threadIdx.x == 0) *cnt = *fcnt = 0;
  __syncthreads();
  for (int64_t i0 = a; i0 < b; i0 += (int64_t)DBLOCK * DU) {
    typename H::Reg r[DU];
#pragma unroll
    for (int u = 0; u < DU; ++u) {
      const int64_t i = i0 + (int64_t)u * DBLOCK + threadIdx.x;
      r[u] = i < b ? hits.load(i) : H::zero();
    }
#pragma unroll
    for (int u = 0; u < DU; ++u) {
      const int64_t i = i0 + (int64_t)u * DBLOCK + threadIdx.x;
      bool own = false, fl = false;
      const uint32_t p = H::pix(r[u]);
      const double v = H::val(r[u]);
      if (i < b) {
        if (H::dup(r[u])) {
          atomicAdd(&img[p], v);
          own = fl = atomicExch(&mark[p], gen) != gen;
        } else {
          img[p] = v;
          own = true;
          acc[0] += v;
          acc[1] += v * v;
          if (v > 0.0) {
            acc[2] += v;
            acc[3] += 1.0;
          }
          mx = v > mx ? v : mx;
        }
        if (own) bm.set(p);
      }
      const int idx = wave_append(own, cnt);
      if (own) {
        list[idx] = p;
        if (!fl) pvals[idx] = v;
      }
      const int fi = wave_append(fl, fcnt);
      if (fl) fidx[fi] = (uint32_t)idx;
    }
  }
  slot_sync();
  const int n = *cnt;
  __syncthreads();
  return n;
}

// A tail window joined against the principal image x (presence bitmap bm) without materialising it: a point
// without the duplicate-candidate flag is alone on its pixel, so it adds (y, y^2, x*y, y[x>0]) to acc directly
// (x loaded only when the pixel is in the principal image).  Flagged points are summed per pixel into y and
// listed as with scatter_window; the caller adds their pixels.  Returns the number of listed pixels.
template <int FMT, bool LDS>
__device__ int tail_window(const Hits<FMT>& hits, int64_t a, int64_t b, const double* x, PresenceBits<LDS> bm,
                           double* y, uint32_t* mark, uint32_t gen, uint32_t* list, int* cnt, double (&acc)[4]) {
  using H = Hits<FMT>;
  if (threadIdx.x == 0) *cnt = 0;
  __syncthreads();
  for (int64_t i0 = a; i0 < b; i0 += (int64_t)DBLOCK * DU) {
    typename H::Reg r[DU];
#pragma unroll
    for (int u = 0; u < DU; ++u) {
      const int64_t i = i0 + (int64_t)u * DBLOCK + threadIdx.x;
      r[u] = i < b ? hits.load(i) : H::zero();
    }
#pragma unroll
    for (int u = 0; u < DU; ++u) {
      const int64_t i = i0 + (int64_t)u * DBLOCK + threadIdx.x;
      bool own = false;
      const uint32_t p = H::pix(r[u]);
      if (i < b) {
        const double v = H::val(r[u]);
        if (H::dup(r[u])) {
          atomicAdd(&y[p], v);
          own = atomicExch(&mark[p], gen) != gen;
        } else {
          const double xv = bm.test(p) ? ld_agent(&x[p]) : 0.0;
          acc[0] += v;
          acc[1] += v * v;
          acc[2] += xv * v;
          if (xv > 0.0) acc[3] += v;
        }
      }
      const int idx = wave_append(own, cnt);
      if (own) list[idx] = p;
    }
  }
  slot_sync();
  const int n = *cnt;
  __syncthreads();
  return n;
}

// Gated hot-spot clip (image_generation.do_preprocessing / q; the oracle's quantile_clip): every pixel above
// np.percentile(positive pixels, q) ('linear' method) is set to that value.  The image is zero outside its n
// listed pixels; vals is scratch for their values.
__device__ void clip_image(double* img, const uint32_t* list, int n_list, double* vals, double q, uint32_t* hist,
                           int* sh) {
  const int tid = threadIdx.x;
  if (tid == 0) sh[2] = 0;
  __syncthreads();
  for (int i0 = 0; i0 < n_list; i0 += DBLOCK) {
    const int i = i0 + tid;
    double v = 0.0;
    if (i < n_list) v = ld_agent(&img[list[i]]);
    const int idx = wave_append(v > 0.0, &sh[2]);
    if (v > 0.0) vals[idx] = v;
  }
  slot_sync();
  const int n = sh[2];
  __syncthreads();
  if (n == 0) return;
  __shared__ unsigned long long sel_u64[2];
  const double thr = percentile_of<DBLOCK>(
      [&](auto&& f) {
        for (int i = tid; i < n; i += DBLOCK) f((uint64_t)__double_as_longlong(ld_agent(&vals[i])));
      },
      n, q, hist, sh, sel_u64);
  for (int i = tid; i < n_list; i += DBLOCK) {
    const uint32_t p = list[i];
    const double v = ld_agent(&img[p]);
    if (v > thr) img[p] = thr;
  }
  slot_sync();
}

template <int FMT, bool BML>
__global__ void __launch_bounds__(DBLOCK) ion_dense_kernel(
    Hits<FMT> hits, const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
    const int64_t* __restrict__ ion_off, const double* __restrict__ theor, int64_t n_ions, Params P,
    const uint32_t* __restrict__ dense_list, const uint32_t* __restrict__ dense_count, uint32_t* next,
    unsigned char* scratch, size_t slot_bytes, double* __restrict__ oc, double* __restrict__ osp,
    double* __restrict__ osc, double* __restrict__ omsm, uint32_t* __restrict__ oflags) {
  extern __shared__ uint32_t dyn_bm[];  // presence bitmap of the principal image (when it fits)
  __shared__ double red[8 * DNW];
  __shared__ double kst[4 * MAXK_DENSE];
  __shared__ int sh_ion;
  __shared__ int sh_ctr[4];
  __shared__ __attribute__((aligned(16))) uint32_t sh_hist[512];
  __shared__ int sh_sel[4];
  const int tid = threadIdx.x;
  DenseSlot S = dense_slot(scratch + (size_t)blockIdx.x * slot_bytes, P.npx);
  const int npx = P.npx;
  const uint32_t total = *dense_count;
  bool fresh = true;
  uint32_t gen = 0;
  const PresenceBits<BML> bm{BML ? dyn_bm : S.gbm};
  const int nbw = (npx + 31) / 32 + 1;  // + one zero word for row7
  if (BML)
    for (int w = tid; w < nbw; w += DBLOCK) dyn_bm[w] = 0u;
  STAMP_DECL();

  while (true) {
    if (tid == 0) {
      const uint32_t k = atomicAdd(next, 1u);
      sh_ion = (k < total) ? (int)dense_list[k] : -1;
      sh_ctr[0] = 0;
      sh_ctr[1] = 0;
    }
    __syncthreads();
    const int64_t ion = sh_ion;
    if (ion < 0) break;
    STAMP(15);
    const int64_t w0 = ion_off[ion];
    const int K = (int)(ion_off[ion + 1] - w0);
    uint32_t flags = SMG_ION_DENSE;
    for (int k = 0; k < K && k < MAXK_DENSE; ++k)
      if (hi[w0 + k] > lo[w0 + k]) flags |= SMG_ION_HAS_HITS;
    if (K > MAXK_DENSE || K == 0) {
      if (tid == 0) {
        oc[ion] = osp[ion] = osc[ion] = omsm[ion] = 0.0;
        oflags[ion] = (K == 0) ? 0u : (flags | 0x80000000u);
      }
      __syncthreads();
      continue;
    }
    if (fresh) {  // the slot's first ion: clean images, levels, tags (plain stores land in L2 before atomics)
      for (int p = tid; p < npx; p += DBLOCK) {
        S.x[p] = 0.0;
        S.y[p] = 0.0;
        S.mark[p] = 0u;
        S.L8[p] = 0;
        S.E8[p] = 0;
      }
      if (!BML)
        for (int w = tid; w < nbw; w += DBLOCK) S.gbm[w] = 0u;
      slot_sync();
      fresh = false;
    }

    STAMP(10);
    // principal image
    // pvals (values in list order, for the levels) alias par + elist, which are free until the candidates
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    double mx = -INFINITY;
    int np;
    if (P.clip) {  // the clip needs the whole image first; statistics and levels then read x
      np = scatter_window<FMT, true>(hits, lo[w0], hi[w0], S.x, S.mark, ++gen, S.plist, &sh_ctr[2], bm);
      clip_image(S.x, S.plist, np, S.vals, P.q, sh_hist, sh_sel);
      for (int i = tid; i < np; i += DBLOCK) {
        const double v = ld_agent(&S.x[S.plist[i]]);
        acc[0] += v;
        acc[1] += v * v;
        if (v > 0.0) {
          acc[2] += v;
          acc[3] += 1.0;
        }
        mx = v > mx ? v : mx;
      }
    } else {
      np = scatter_principal<FMT>(hits, lo[w0], hi[w0], S.x, S.mark, ++gen, S.plist, S.vals, S.ylist, &sh_ctr[2],
                                  &sh_ctr[3], bm, acc, mx);
      const int nfl = sh_ctr[3];
      for (int j = tid; j < nfl; j += DBLOCK) {  // flagged owners: their per-pixel sums are complete now
        const uint32_t i = S.ylist[j];
        const double v = ld_agent(&S.x[S.plist[i]]);
        S.vals[i] = v;
        acc[0] += v;
        acc[1] += v * v;
        if (v > 0.0) {
          acc[2] += v;
          acc[3] += 1.0;
        }
        mx = v > mx ? v : mx;
      }
    }
    if (np < npx) mx = mx > 0.0 ? mx : 0.0;  // unlisted pixels are zero
    dblock_sum<4>(acc, red);
    const double sx = acc[0], sxx = acc[1], s0 = acc[2], npos = acc[3];
    const double vmax = block_max<DNW>(mx, red);
    const bool chaos_ok = (sx > 0.0) && (npos >= 4.0);

    STAMP(11);
    // other windows, joined against x through the dense principal image
    for (int k = 1; k < K; ++k) {
      double a2[4] = {0.0, 0.0, 0.0, 0.0};  // sy, syy, sxy, s (y[x > 0])
      int ny;
      if (P.clip) {  // the clip needs the whole tail image first
        ny = scatter_window<FMT, false>(hits, lo[w0 + k], hi[w0 + k], S.y, S.mark, ++gen, S.ylist, &sh_ctr[2], bm);
        clip_image(S.y, S.ylist, ny, S.vals, P.q, sh_hist, sh_sel);
      } else {
        ny = tail_window<FMT>(hits, lo[w0 + k], hi[w0 + k], S.x, bm, S.y, S.mark, ++gen, S.ylist, &sh_ctr[2], a2);
      }
      for (int i = tid; i < ny; i += DBLOCK) {
        const uint32_t p = S.ylist[i];
        const double y = ld_agent(&S.y[p]);
        const double x = bm.test(p) ? ld_agent(&S.x[p]) : 0.0;
        a2[0] += y;
        a2[1] += y * y;
        a2[2] += x * y;
        if (x > 0.0) a2[3] += y;
      }
      dblock_sum<4>(a2, red);
      if (tid == 0) {
        kst[0 * MAXK_DENSE + k] = a2[3];
        kst[1 * MAXK_DENSE + k] = a2[0];
        kst[2 * MAXK_DENSE + k] = a2[1];
        kst[3 * MAXK_DENSE + k] = a2[2];
      }
      for (int i = tid; i < ny; i += DBLOCK) S.y[S.ylist[i]] = 0.0;
      slot_sync();
    }
    __syncthreads();

    STAMP(12);
    double chaos_raw = NAN;
    int m = 0;
    if (chaos_ok) {
      const int nr = P.nrows, nc = P.ncols;
      for (int i = tid; i < np; i += DBLOCK) {  // with the clip, vals served the tail clips: read x
        const uint32_t p = S.plist[i];
        S.L8[p] = (uint8_t)level_of(P.clip ? ld_agent(&S.x[p]) : S.vals[i], vmax, P);
      }
      __syncthreads();
      // eL = erode_box(dilate_cross(L)) > 0 only on the 4-cross around a pixel with L > 0, i.e. around a
      // principal pixel: those are the candidates.  Candidate q is evaluated once, by the smallest-index
      // principal pixel on its 4-cross.  Each principal pixel s reads the 7x7 presence window around it from the
      // bitmap; a candidate survives only if every in-image pixel of its 3x3 box has a principal pixel on its
      // cross (presence is a superset of L > 0), and only survivors load the 7x7 level window for the exact eL.
      for (int i0 = 0; i0 < np; i0 += DBLOCK) {
        const int i = i0 + tid;
        const int p = (i < np) ? (int)S.plist[i] : -1;
        const int r0 = p >= 0 ? p / nc : 0, c0 = p >= 0 ? p - r0 * nc : 0;
        uint32_t B[7];  // bit (dc + 3) of B[dr + 3]: pixel (r0 + dr, c0 + dc) is in the image and principal
#pragma unroll
        for (int dr = -3; dr <= 3; ++dr) B[dr + 3] = p >= 0 ? bm.row7(r0 + dr, c0, nr, nc) : 0u;
        auto pres = [&](int wr, int wc) -> uint32_t { return (B[wr] >> wc) & 1u; };
        bool cand[5];
        bool any = false;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const int qr = (j == 1) ? -1 : (j == 2) ? 1 : 0, qc = (j == 3) ? -1 : (j == 4) ? 1 : 0;
          const int r = r0 + qr, c = c0 + qc;
          bool ok = p >= 0 && r >= 0 && r < nr && c >= 0 && c < nc;
          const int wr = qr + 3, wc = qc + 3;
          if (ok) {  // owner: the first principal pixel among q-nc, q-1, q, q+1, q+nc must be s
            int orr = 9, occ = 9;
            if (pres(wr + 1, wc)) orr = 1, occ = 0;
            if (pres(wr, wc + 1)) orr = 0, occ = 1;
            if (pres(wr, wc)) orr = 0, occ = 0;
            if (pres(wr, wc - 1)) orr = 0, occ = -1;
            if (pres(wr - 1, wc)) orr = -1, occ = 0;
            ok = (qr + orr == 0 && qc + occ == 0);
          }
          if (ok) {  // presence screen over the 3x3 box
#pragma unroll
            for (int a = -1; a <= 1; ++a)
#pragma unroll
              for (int b = -1; b <= 1; ++b) {
                const int rr = r + a, cc = c + b;
                if (rr < 0 || rr >= nr || cc < 0 || cc >= nc) {
                  if (!P.erosion_border) ok = false;
                  continue;
                }
                const int ur = wr + a, uc = wc + b;
                if (!(pres(ur, uc) | pres(ur - 1, uc) | pres(ur + 1, uc) | pres(ur, uc - 1) | pres(ur, uc + 1)))
                  ok = false;
              }
          }
          cand[j] = ok;
          any |= ok;
        }
        uint64_t WL[7];  // byte (dc + 3) of WL[dr + 3]: level of pixel (r0 + dr, c0 + dc), 0 outside the image
#pragma unroll
        for (int dr = 0; dr < 7; ++dr) WL[dr] = 0ull;
        if (any) {
#pragma unroll
          for (int dr = -3; dr <= 3; ++dr)
#pragma unroll
            for (int dc = -3; dc <= 3; ++dc) {
              const int rr = r0 + dr, cc = c0 + dc;
              const int rc = min(max(rr, 0), nr - 1), ccl = min(max(cc, 0), nc - 1);
              const uint64_t v = (rr == rc && cc == ccl) ? (uint64_t)S.L8[rc * nc + ccl] : 0ull;
              WL[dr + 3] |= v << (8 * (dc + 3));
            }
        }
        auto W = [&](int wr, int wc) -> int { return (int)((WL[wr] >> (8 * wc)) & 0xFFull); };
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const int qr = (j == 1) ? -1 : (j == 2) ? 1 : 0, qc = (j == 3) ? -1 : (j == 4) ? 1 : 0;
          const int r = r0 + qr, c = c0 + qc;
          const int q = cand[j] ? r * nc + c : -1;
          int e = 0;
          if (q >= 0) {
            e = 1 << 20;
#pragma unroll
            for (int a = -1; a <= 1; ++a)
#pragma unroll
              for (int b = -1; b <= 1; ++b) {
                const int rr = r + a, cc = c + b;
                if (rr < 0 || rr >= nr || cc < 0 || cc >= nc) {
                  if (!P.erosion_border) e = 0;
                  continue;
                }
                const int wr = qr + a + 3, wc = qc + b + 3;
                const int t = max(max(W(wr, wc), W(wr - 1, wc)), max(max(W(wr + 1, wc), W(wr, wc - 1)), W(wr, wc + 1)));
                e = min(e, t);
              }
            if (e >= (1 << 20)) e = 0;
          }
          const int idx = wave_append(e >= 1, &sh_ctr[0]);
          if (e >= 1) {
            S.E8[q] = (uint8_t)e;
            S.elist[idx] = (uint32_t)q;
            S.par[q] = (uint32_t)q;
            atomicMax(&sh_ctr[1], e);
          }
        }
      }
      slot_sync();
      m = sh_ctr[0];
      const int emax = sh_ctr[1];
      STAMP(13);
      double esum = 0.0, wsum = 0.0;
      for (int i = tid; i < m; i += DBLOCK) esum += (double)S.E8[S.elist[i]];
      for (int t = emax; t >= 1; --t) {
        for (int i = tid; i < m; i += DBLOCK) {
          const int p = (int)S.elist[i];
          const int e = S.E8[p];
          if (e < t) continue;
          const int r = p / nc, c = p - r * nc;
          auto edge = [&](int q) {
            const int eq = S.E8[q];
            if (eq >= 1 && (e < eq ? e : eq) == t) {
              if (guf_unite(S.par, (uint32_t)p, (uint32_t)q)) wsum += (double)t;
            }
          };
          if (c + 1 < nc) edge(p + 1);
          if (r + 1 < nr) {
            edge(p + nc);
            if (P.connectivity == 8) {
              if (c > 0) edge(p + nc - 1);
              if (c + 1 < nc) edge(p + nc + 1);
            }
          }
        }
        __syncthreads();
      }
      double a3[2] = {esum, wsum};
      dblock_sum<2>(a3, red);
      chaos_raw = 1.0 - (a3[0] - a3[1]) / (double)P.nlevels / npos;
    } else {
      flags |= SMG_ION_CHAOS_NAN;
    }

    STAMP(14);
    if (tid == 0) {  // per-window sums straight from LDS (kst rows: s, sy, syy, sxy; window 0 = principal)
      kst[0] = s0;
      kst[1 * MAXK_DENSE] = kst[2 * MAXK_DENSE] = kst[3 * MAXK_DENSE] = 0.0;
      finalize_ion(K, theor + w0, kst, sx, sxx, kst + MAXK_DENSE, kst + 2 * MAXK_DENSE, kst + 3 * MAXK_DENSE,
                   (double)npx, chaos_raw, ion, flags, oc, osp, osc, omsm, oflags);
    }
    // clean what this ion wrote
    for (int i = tid; i < m; i += DBLOCK) S.E8[S.elist[i]] = 0;
    for (int i = tid; i < np; i += DBLOCK) {
      const uint32_t p = S.plist[i];
      S.x[p] = 0.0;
      S.L8[p] = 0;
      bm.clear_word_of(p);  // every bit of the word belongs to this ion
    }
    slot_sync();
  }
  STAMP_FLUSH();
}

// ---------------------------------------------------------------------------------------------
// wide pass: dense-path ions of images whose presence bitmap and rank prefix fit the LDS (no clip)
// ---------------------------------------------------------------------------------------------
// The pixel-indexed slot above turns every window point into a random read-modify-write of a 38-B-per-pixel
// array far larger than the XCD's L2.  Here the principal image's presence bitmap lives in the LDS with a
// two-level rank prefix (u32 per 65536 pixels, u16 per 64): a principal pixel's value, level and plist entry sit
// at its dense rank in the slot's compact arrays (np entries, written in order of rank, L2-resident for ordinary
// windows).  Tail points without the duplicate-candidate flag read x at the rank of their pixel; flagged tail
// points are summed per pixel in a small open-addressing table that each window's owners clear again.  Chaos
// candidates get their own bitmap + ranks for Kruskal (the principal bitmap is no longer needed by then).  Nothing
// is pixel-indexed in global memory, so nothing has to be zeroed per slot; an ion whose flagged tail pixels
// overflow the table is handed to the pixel-indexed kernel.
//
// Diagnostic build only (-DSMG_WIDE_CHECK): index checks on the wide pass's global and table accesses; a failed
// check records (code, value) of its first occurrence and a count (smg_debug_wide_check) and the access is
// clamped, so a bad index is reported instead of faulting.  The shipped build compiles the plain expressions.
#ifdef SMG_WIDE_CHECK
__device__ unsigned long long g_wchk[4];  // [0] first code, [1] its value, [2] failures, [3] ions seen
__device__ __forceinline__ bool wchk(bool ok, int code, long long v) {
  if (!ok && atomicAdd(&g_wchk[2], 1ull) == 0ull) {
    g_wchk[0] = (unsigned long long)code;
    g_wchk[1] = (unsigned long long)v;
  }
  return ok;
}
#define WCK(ok, code, v) wchk((ok), (code), (long long)(v))
#else
#define WCK(ok, code, v) true
#endif
constexpr int WIDE_HT_LOG2 = 13;
constexpr int WIDE_HT = 1 << WIDE_HT_LOG2;  // tail duplicate table entries per slot
constexpr int WIDE_PROBES = 64;
constexpr int WIDE_DL = 2 * WIDE_HT;        // flagged tail points listed per ion (beyond the registers)
constexpr int WIDE_FLR = 3;                 // flagged tail points held in a lane's registers
constexpr uint32_t WIDE_EMPTY = 0xFFFFFFFFu;
#ifndef SMG_WDU
#define SMG_WDU 8
#endif
constexpr int WDU = SMG_WDU;  // wide pass: points per lane with loads in flight together
#ifndef SMG_TDU
#define SMG_TDU 4
#endif
constexpr int TDU = SMG_TDU;  // wide pass, pipelined tail stream: points per lane per batch
#ifndef SMG_TDEPTH
#define SMG_TDEPTH 2
#endif
constexpr int TDEPTH = SMG_TDEPTH;  // batches with loads in flight (the one processed and TDEPTH - 1 ahead)

struct WideSlot {
  double* vals;     // principal values by rank
  uint32_t* epix;   // chaos candidates in discovery order
  uint32_t* epr;    // chaos candidates by rank
  uint32_t* par;    // union-find over candidate ranks
  uint8_t* L;       // levels by principal rank
  uint8_t* eL;      // eL in discovery order
  uint8_t* eLr;     // eL by candidate rank
  uint32_t* hkey;   // tail duplicate table: (window, pixel) key, Σy, entries claimed for the ion
  double* hval;
  uint32_t* hown;
  uint32_t* dkey;   // flagged tail points of the ion: (window, pixel) key and value
  double* dval;
};

static inline size_t wide_slot_bytes(int npx) {
  return al16((size_t)npx * 8) + al16((size_t)npx * 4) * 3 + al16((size_t)npx) * 3 + al16((size_t)WIDE_HT * 4) * 2 +
         al16((size_t)WIDE_HT * 8) + al16((size_t)WIDE_DL * 4) + al16((size_t)WIDE_DL * 8) + 256;
}

__device__ __forceinline__ WideSlot wide_slot(unsigned char* base, int npx) {
  WideSlot S;
  auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  size_t o = 0;
  S.vals = reinterpret_cast<double*>(base + o);
  o += a16((size_t)npx * 8);
  S.epix = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)npx * 4);
  S.epr = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)npx * 4);
  S.par = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)npx * 4);
  S.L = base + o;
  o += a16((size_t)npx);
  S.eL = base + o;
  o += a16((size_t)npx);
  S.eLr = base + o;
  o += a16((size_t)npx);
  S.hval = reinterpret_cast<double*>(base + o);
  o += a16((size_t)WIDE_HT * 8);
  S.hkey = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)WIDE_HT * 4);
  S.hown = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)WIDE_HT * 4);
  S.dval = reinterpret_cast<double*>(base + o);
  o += a16((size_t)WIDE_DL * 8);
  S.dkey = reinterpret_cast<uint32_t*>(base + o);
  return S;
}

// the wide pass's LDS table of flagged tail points (summed per (window, pixel)); entries that find no free slot
// within WIDE_LT_PROBES go to the slot's global table
constexpr int WIDE_LT_LOG2 = 10;
constexpr int WIDE_LT = 1 << WIDE_LT_LOG2;
constexpr int WIDE_LT_PROBES = 32;

// LDS bytes of the wide pass: the bitmap (+ one zero word, padded to whole 4-word groups), superblock bases, group
// prefixes (one u16 per 4 words) and the flagged-point table
__host__ __device__ static inline size_t wide_n64p(int npx) { return ((((size_t)npx + 63) / 64 + 1) + 3) & ~(size_t)3; }
static inline size_t wide_lds_bytes(int npx) {
  const size_t n64 = ((size_t)npx + 63) / 64, n64p = wide_n64p(npx);
  return n64p * 8 + ((((n64 + 1023) / 1024) * 4 + 15) & ~(size_t)15) + (((n64p / 4) * 2 + 15) & ~(size_t)15) +
         (size_t)WIDE_LT * 4 + (size_t)WIDE_LT * 8;
}

// rank structure over the LDS bitmap: #set bits before word w = sb[w >> 10] + pf4[w >> 2] + the bits of words
// (w & ~3) .. w - 1 of its 4-word group.  A superblock of 1024 words (65536 bits, so pf4 fits 16 bits) is one
// wave's: its lanes read consecutive words (no bank conflicts) and scan them 64 at a time with DPP.  Needs
// n64 <= DNW * 1024.  Returns the bit count.  One prefix per 4 words (not per word) leaves the LDS room for the
// flagged-point table.
// With list != nullptr the set bits' pixels are also written to list (in no particular order; *lcount = 0 first).
__device__ uint32_t build_rank(const uint64_t* bm, uint16_t* pf, uint32_t* sb, int n64, uint32_t* sc,
                               uint32_t* list = nullptr, int* lcount = nullptr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int w0 = wid * 1024, w1 = min(w0 + 1024, n64);
  uint32_t run = 0;
  for (int c = w0; c < w1; c += 64) {
    const int w = c + lane;
    uint64_t bits = w < w1 ? bm[w] : 0ull;
    const int x = __popcll(bits);
    const int incl = wave_incl_scan_dpp(x);
    if (w < w1 && (w & 3) == 0) pf[w >> 2] = (uint16_t)(run + (uint32_t)(incl - x));
    const int tot = __builtin_amdgcn_readlane(incl, 63);
    run += (uint32_t)tot;
    if (list != nullptr) {
      int lb = 0;
      if (lane == 63) lb = atomicAdd(lcount, tot);
      lb = __shfl(lb, 63);
      int idx = lb + incl - x;
      while (bits != 0ull) {
        list[idx++] = (uint32_t)w * 64u + (uint32_t)(__ffsll((unsigned long long)bits) - 1);
        bits &= bits - 1ull;
      }
    }
  }
  if (lane == 0) sc[wid] = run;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < DNW; ++w) {
    const uint32_t t = sc[w];
    base += (w < wid) ? t : 0u;
    tot += t;
  }
  if (lane == 0 && w0 < n64) sb[wid] = base;
  __syncthreads();
  return tot;
}

// 8-byte load past L1 (agent scope, like ld_agent) issued asynchronously: waited for with vm_wait.  No memory
// clobber (the wide pass's loads read data made visible by an earlier slot_sync, whose asm orders them): the
// compiler may keep scheduling LDS and address work around them.
__device__ __forceinline__ void ld8_async_agent(uint64_t& r, const void* addr) {
  asm volatile("global_load_dwordx2 %0, %1, off sc1" : "+v"(r) : "v"(addr));
}
__device__ __forceinline__ void ld8_async_nm(uint64_t& r, const void* addr) {
  asm volatile("global_load_dwordx2 %0, %1, off" : "+v"(r) : "v"(addr));
}

struct RankBits {
  const uint64_t* bm;
  const uint16_t* pf;  // one prefix per 4-word group
  const uint32_t* sb;
  __device__ __forceinline__ bool test(uint32_t p) const { return (bm[p >> 6] >> (p & 63)) & 1ull; }
  __device__ __forceinline__ uint32_t rank(uint32_t p) const {  // number of set bits below pixel p
    const uint32_t w = p >> 6, j = w & 3u;
    const ulonglong2* g = reinterpret_cast<const ulonglong2*>(bm + (w & ~3u));
    const ulonglong2 a = g[0], b = g[1];  // the group's four words (two 16-B reads)
    const uint64_t m = (1ull << (p & 63)) - 1ull;
    const uint32_t c = (uint32_t)__popcll(j == 0 ? (a.x & m) : a.x) +
                       (j >= 1 ? (uint32_t)__popcll(j == 1 ? (a.y & m) : a.y) : 0u) +
                       (j >= 2 ? (uint32_t)__popcll(j == 2 ? (b.x & m) : b.x) : 0u) +
                       (j == 3 ? (uint32_t)__popcll(b.y & m) : 0u);
    return sb[w >> 10] + (uint32_t)pf[w >> 2] + c;
  }
};

// The wide pass's tail windows under the hot-spot clip (CLIP, image_generation.do_preprocessing): each tail image is
// clipped at the q-th percentile of its positive pixels before its sums, so its Σy, Σy², Σxy and Σy[x>0] come from
// the clipped pixel values, not from the hit prefix sums.  A window's pixel values are its unflagged points' values
// (the only point of their pixel in the window, smg_flag_duplicates) and the per-pixel sums of its flagged points.
//  1. one stream over the tail: flagged points summed per (window, pixel) in the tables (LDS, then the slot's global
//     table; an overflow sends the ion to the pixel-indexed kernel), positive unflagged points counted per window;
//  2. per window, its threshold by an MSD radix select over those values (select_pair: the window's points and the
//     tables, re-read once per pass);
//  3. a second stream: the clipped unflagged points' sums, x gathered by rank;
//  4. the table entries: each flagged pixel's clipped sum into its window's sums, then the entry released.
// kst rows as in the kernel: 0 Σy[x>0], 1 Σy, 2 Σy², 3 Σxy (window k at column k).
template <int FMT>
__device__ void wide_clip_tail(const Hits<FMT>& hits, int K, double q, int npx, const RankBits& R, const WideSlot& S,
                               const int64_t* sh_tb, const int64_t* sh_tlo, const int64_t* sh_tn, uint32_t* ltkey,
                               double* ltval, double* kst, int* sh_nown, int* sh_ctr, uint32_t* c_hist, int* c_sh,
                               unsigned long long* c_dsh, double* c_thr, int* c_n, SelSet* c_st, int* c_flag,
                               uint32_t* c_oa) {
  using H = Hits<FMT>;
  const int tid = threadIdx.x, lane = tid & 63;
  constexpr int U = FMT == SMG_HITS_PACKED_F32 ? TDU : WDU;
  constexpr int64_t TSTEP = (int64_t)DBLOCK * U;  // the kernel's batch (sh_tb pads each window to a whole batch)
  const int64_t T = sh_tb[K - 1];
  if (tid < MAXK_DENSE) {
    c_n[tid] = 0;
    c_oa[tid] = 0u;
  }
  __syncthreads();
  auto insert_global = [&](uint32_t key, double y) {
    uint32_t h = (key * 0x9E3779B1u) >> (32 - WIDE_HT_LOG2);
    bool own = false, done = false;
    for (int t = 0; t < WIDE_PROBES; ++t) {
      const uint32_t old = atomicCAS(&S.hkey[h], WIDE_EMPTY, key);
      if (old == WIDE_EMPTY || old == key) {
        atomicAdd(&S.hval[h], y);
        own = old == WIDE_EMPTY;
        done = true;
        break;
      }
      h = (h + 1) & (WIDE_HT - 1);
    }
    if (!done) sh_ctr[3] = 1;
    return own ? (int)h : -1;
  };
  auto insert = [&](bool act, uint32_t key, double y) {  // uniform call: act = this lane has an entry
    bool placed = !act;
    if (act) {
      uint32_t h = (key * 0x9E3779B1u) >> (32 - WIDE_LT_LOG2);
      for (int t = 0; t < WIDE_LT_PROBES; ++t) {
        const uint32_t old = atomicCAS(&ltkey[h], WIDE_EMPTY, key);
        if (old == WIDE_EMPTY || old == key) {
          atomicAdd(&ltval[h], y);
          placed = true;
          break;
        }
        h = (h + 1) & (WIDE_LT - 1);
      }
    }
    int gh = -1;
    if (__ballot(!placed)) {
      if (!placed) gh = insert_global(key, y);
    }
    const int idx = wave_append(gh >= 0, sh_nown);
    if (gh >= 0) S.hown[idx] = (uint32_t)gh;
  };
  // batches of U points per lane, each inside one window (uniform kb); body(kb, off, n, r)
  auto stream = [&](auto&& body) {
    int kb = 0;
    for (int64_t v0 = 0; v0 < T; v0 += TSTEP) {
      while (v0 >= sh_tb[kb + 1]) ++kb;
      kb = __builtin_amdgcn_readfirstlane(kb);
      const int64_t off = v0 - sh_tb[kb], n = sh_tn[kb], a = sh_tlo[kb];
      typename H::Reg r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t lv = off + (int64_t)u * DBLOCK + tid;
        r[u] = hits.load(a + (lv < n ? lv : n - 1));
      }
      body(kb, off, n, r);
    }
  };
  auto bits_of = [](double v) { return (uint64_t)__double_as_longlong(v); };

  // 1. flagged points -> tables; positive unflagged points counted per window (and their top16_oa summary)
  {
    int cpos = 0, kc = 0;
    uint32_t oa = 0u;
    auto flush = [&]() {
      const int t = __builtin_amdgcn_readlane(wave_incl_scan_dpp(cpos), 63);
      if (lane == 0 && t) atomicAdd(&c_n[kc + 1], t);
      if (oa) atomicOr(&c_oa[kc + 1], oa);
      cpos = 0;
      oa = 0u;
    };
    stream([&](int kb, int64_t off, int64_t n, const typename H::Reg (&r)[U]) {
      if (kb != kc) {
        flush();
        kc = kb;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool valid = off + (int64_t)u * DBLOCK + tid < n;
        const bool fl = valid && H::dup(r[u]);
        insert(fl, (uint32_t)kb * (uint32_t)npx + H::pix(r[u]), fl ? (double)H::val(r[u]) : 0.0);
        const bool pos = valid && !H::dup(r[u]) && H::val(r[u]) > 0.0;
        cpos += pos ? 1 : 0;
        oa |= pos ? top16_oa(bits_of((double)H::val(r[u]))) : 0u;
      }
    });
    flush();
  }
  slot_sync();  // the tables' sums are complete (LDS; L2 for the global entries)
  const int no = *sh_nown;
  auto count_entry = [&](uint32_t key, double y) {
    if (y > 0.0) {
      const int k = (int)(key / (uint32_t)npx) + 1;
      atomicAdd(&c_n[k], 1);
      atomicOr(&c_oa[k], top16_oa(bits_of(y)));
    }
  };
  for (int i = tid; i < WIDE_LT; i += DBLOCK) {
    const uint32_t key = ltkey[i];
    if (key != WIDE_EMPTY) count_entry(key, ltval[i]);
  }
  for (int j = tid; j < no; j += DBLOCK) {
    const uint32_t sl = S.hown[j];
    count_entry(ld_agent(&S.hkey[sl]), ld_agent(&S.hval[sl]));
  }
  __syncthreads();

  // 2. thresholds: every window's radix select, four windows per batch advancing together (each round reads the
  // whole tail once); set s = window s + 1
  if (!sh_ctr[3]) {
    select_batch<DBLOCK, 4>(
        [&](auto&& f) {
          stream([&](int kb, int64_t off, int64_t n, const typename H::Reg (&r)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u)
              if (off + (int64_t)u * DBLOCK + tid < n && !H::dup(r[u]) && H::val(r[u]) > 0.0)
                f(kb, bits_of((double)H::val(r[u])));
          });
          for (int i = tid; i < WIDE_LT; i += DBLOCK) {
            const uint32_t key = ltkey[i];
            if (key != WIDE_EMPTY && ltval[i] > 0.0) f((int)(key / (uint32_t)npx), bits_of(ltval[i]));
          }
          for (int j = tid; j < no; j += DBLOCK) {
            const uint32_t sl = S.hown[j];
            const double y = ld_agent(&S.hval[sl]);
            if (y > 0.0) f((int)(ld_agent(&S.hkey[sl]) / (uint32_t)npx), bits_of(y));
          }
        },
        K - 1, c_n + 1, q, c_thr + 1, c_st, c_hist, c_flag, nullptr, nullptr, c_oa + 1);
  }

  // 3. the clipped unflagged points
  {
    double as = 0.0, axy = 0.0, ay = 0.0, ayy = 0.0;
    int kacc = 0;
    auto flush = [&]() {
      const double t0 = wave_sum_dpp(as), t1 = wave_sum_dpp(ay), t2 = wave_sum_dpp(ayy), t3 = wave_sum_dpp(axy);
      if (lane == 0) {
        atomicAdd(&kst[0 * MAXK_DENSE + kacc + 1], t0);
        atomicAdd(&kst[1 * MAXK_DENSE + kacc + 1], t1);
        atomicAdd(&kst[2 * MAXK_DENSE + kacc + 1], t2);
        atomicAdd(&kst[3 * MAXK_DENSE + kacc + 1], t3);
      }
      as = axy = ay = ayy = 0.0;
    };
    stream([&](int kb, int64_t off, int64_t n, const typename H::Reg (&r)[U]) {
      if (kb != kacc) {
        flush();
        kacc = kb;
      }
      const double thr = c_thr[kb + 1];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool valid = off + (int64_t)u * DBLOCK + tid < n;
        if (valid && !H::dup(r[u])) {
          const double v = H::val(r[u]);
          const double y = v > thr ? thr : v;
          const uint32_t p = H::pix(r[u]);
          const double x = R.test(p) ? ld_agent(&S.vals[R.rank(p)]) : 0.0;
          if (x > 0.0) as += y;
          axy += x * y;
          ay += y;
          ayy += y * y;
        }
      }
    });
    flush();
  }

  // 4. the flagged pixels' clipped sums; the entries are released for the next ion
  auto add_pixel = [&](uint32_t key, double Y) {
    const uint32_t kk = key / (uint32_t)npx, p = key - kk * (uint32_t)npx;
    const int k = (int)kk + 1;
    const double thr = c_thr[k];
    const double y = Y > thr ? thr : Y;
    const double x = R.test(p) ? ld_agent(&S.vals[R.rank(p)]) : 0.0;
    if (x > 0.0) atomicAdd(&kst[0 * MAXK_DENSE + k], y);
    atomicAdd(&kst[1 * MAXK_DENSE + k], y);
    atomicAdd(&kst[2 * MAXK_DENSE + k], y * y);
    atomicAdd(&kst[3 * MAXK_DENSE + k], x * y);
  };
  for (int i = tid; i < WIDE_LT; i += DBLOCK) {
    const uint32_t key = ltkey[i];
    if (key != WIDE_EMPTY) {
      add_pixel(key, ltval[i]);
      ltkey[i] = WIDE_EMPTY;
      ltval[i] = 0.0;
    }
  }
  for (int j = tid; j < no; j += DBLOCK) {
    const uint32_t sl = S.hown[j];
    add_pixel(ld_agent(&S.hkey[sl]), ld_agent(&S.hval[sl]));
    S.hkey[sl] = WIDE_EMPTY;
    S.hval[sl] = 0.0;
  }
  __syncthreads();  // (released entries reach L2 before the next ion's inserts: slot_syncs lie between)
}

constexpr int PRV = 4;  // wide pass clip: principal values per lane held in registers (np <= PRV * DBLOCK)
template <int FMT, bool CLIP>
__global__ void __launch_bounds__(DBLOCK) ion_wide_kernel(
    Hits<FMT> hits, const DD4* __restrict__ cum, const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
    const int64_t* __restrict__ ion_off, const double* __restrict__ theor, Params P,
    const uint32_t* __restrict__ list, const uint32_t* __restrict__ count, uint32_t* next, uint32_t* rej_list,
    uint32_t* rej_count, unsigned char* scratch, size_t slot_bytes, double* __restrict__ oc,
    double* __restrict__ osp, double* __restrict__ osc, double* __restrict__ omsm, uint32_t* __restrict__ oflags) {
  using H = Hits<FMT>;
  extern __shared__ __attribute__((aligned(16))) uint64_t wide_dyn[];
  __shared__ double red[8 * DNW];
  __shared__ double kst[4 * MAXK_DENSE];
  __shared__ uint32_t sc[DNW];
  __shared__ int sh_ion;
  __shared__ int sh_ctr[4];  // candidates, max eL, listed flagged tail points, list / table overflow
  __shared__ int sh_nown;    // claimed table entries
  __shared__ int sh_ncand;   // screened chaos candidates
  __shared__ int sh_anyfl;   // the ion's tail stream met a flagged point
  __shared__ double sh_st[5];  // principal sums: x, x^2, x[x > 0], #(x > 0); max
  __shared__ int64_t sh_tb[MAXK_DENSE + 1];  // tail stream: offset of window k at k - 1 (+ the total)
  __shared__ int64_t sh_tlo[MAXK_DENSE];     // first point of window k at k - 1
  __shared__ int64_t sh_tn[MAXK_DENSE];      // length of window k at k - 1
  // CLIP (do_preprocessing): the radix select's histogram and scalars, each window's threshold and positive count
  __shared__ __attribute__((aligned(16))) uint32_t c_hist[CLIP ? 1024 : 4];
  __shared__ SelSet c_st[CLIP ? 4 : 1];
  __shared__ int c_flag[2];
  __shared__ int c_sh[4];
  __shared__ unsigned long long c_dsh[2];
  __shared__ double c_thr[CLIP ? MAXK_DENSE : 1];
  __shared__ int c_n[CLIP ? MAXK_DENSE : 1];
  __shared__ uint32_t c_oa[CLIP ? MAXK_DENSE : 1];  // top16_oa of the positive values: the principal at 0, window k at k
  const int tid = threadIdx.x;
  const int npx = P.npx, n64 = (npx + 63) / 64, nsb = (n64 + 1023) / 1024;
  const int n64p = (int)wide_n64p(npx);  // n64 words + zero words to a whole 4-word group (row7 reads one past)
  uint64_t* bm = wide_dyn;
  uint32_t* bm32 = reinterpret_cast<uint32_t*>(bm);
  uint32_t* sb = reinterpret_cast<uint32_t*>(bm + n64p);
  uint16_t* pf = reinterpret_cast<uint16_t*>(reinterpret_cast<unsigned char*>(sb) + (((size_t)nsb * 4 + 15) & ~(size_t)15));
  uint32_t* ltkey = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(pf) +
                                                ((((size_t)n64p / 4) * 2 + 15) & ~(size_t)15));
  double* ltval = reinterpret_cast<double*>(ltkey + WIDE_LT);
  const RankBits R{bm, pf, sb};
  const PresenceBits<true> pres{bm32};
  WideSlot S = wide_slot(scratch + (size_t)blockIdx.x * slot_bytes, npx);
  const uint32_t total = *count;
  for (int i = tid; i < WIDE_HT; i += DBLOCK) {
    S.hkey[i] = WIDE_EMPTY;
    S.hval[i] = 0.0;
  }
  for (int i = tid; i < WIDE_LT; i += DBLOCK) {
    ltkey[i] = WIDE_EMPTY;
    ltval[i] = 0.0;
  }
  slot_sync();
  const int nr = P.nrows, nc = P.ncols;
  STAMP_DECL();

  while (true) {
    if (tid == 0) {
      const uint32_t k = atomicAdd(next, 1u);
      sh_ion = (k < total) ? (int)list[k] : -1;
      sh_ctr[0] = sh_ctr[1] = sh_ctr[2] = sh_ctr[3] = 0;
      sh_nown = 0;
      sh_ncand = 0;
      sh_anyfl = 0;
    }
    __syncthreads();
    const int64_t ion = sh_ion;
    if (ion < 0) break;
#ifdef SMG_WIDE_CHECK
    if (tid == 0) atomicAdd(&g_wchk[3], 1ull);
    if (!WCK(ion < (int64_t)total, 1, ion)) {
      __syncthreads();
      continue;
    }
#endif
    const int64_t w0 = ion_off[ion];
    const int K = (int)(ion_off[ion + 1] - w0);
    uint32_t flags = SMG_ION_DENSE | SMG_ION_WIDE;
    for (int k = 0; k < K && k < MAXK_DENSE; ++k)
      if (hi[w0 + k] > lo[w0 + k]) flags |= SMG_ION_HAS_HITS;
    if (K > MAXK_DENSE || K == 0) {
      if (tid == 0) {
        oc[ion] = osp[ion] = osc[ion] = omsm[ion] = 0.0;
        oflags[ion] = (K == 0) ? 0u : (flags | 0x80000000u);
      }
      __syncthreads();
      continue;
    }

    STAMP(15);
    // principal image: presence bits, ranks, then values and pixels at their ranks
    for (int w = tid; w < n64p; w += DBLOCK) bm[w] = 0ull;
    __syncthreads();
    const int64_t a0 = lo[w0];
    int64_t b0 = hi[w0];
    if (!WCK(a0 >= 0 && a0 <= b0 && b0 < (1ll << 36), 3, b0 - a0)) b0 = a0;
    for (int64_t i0 = a0; i0 < b0; i0 += (int64_t)DBLOCK * WDU) {
      typename H::Reg r[WDU];
#pragma unroll
      for (int u = 0; u < WDU; ++u) {  // unconditional loads (clamped index): counted waits, not vmcnt(0)
        const int64_t i = i0 + (int64_t)u * DBLOCK + tid;
        r[u] = hits.load(i < b0 ? i : b0 - 1);
      }
#pragma unroll
      for (int u = 0; u < WDU; ++u) {
        const int64_t i = i0 + (int64_t)u * DBLOCK + tid;
        bool dup_own = false;
        uint32_t p = 0u;
        if (i < b0 && WCK(H::pix(r[u]) < (uint32_t)npx, 4, H::pix(r[u]))) {
          p = H::pix(r[u]);
          const uint32_t bit = 1u << (p & 31);
          // a flagged point that sets its pixel's bit lists the pixel: one entry per pixel with duplicates
          dup_own = !(atomicOr(&bm32[p >> 5], bit) & bit) && H::dup(r[u]);
        }
        const int idx = wave_append(dup_own, &sh_ctr[2]);
        if (dup_own && idx < WIDE_DL) S.dkey[idx] = p;
      }
    }
    __syncthreads();
    const int np = (int)build_rank(bm, pf, sb, n64, sc, S.par, &sh_ncand);  // principal pixels listed in par
    STAMP(10);
    // Values by rank.  An unflagged point is the only point of its pixel in the window (smg_flag_duplicates), so it
    // stores its value and enters the statistics at once; the pixels with flagged points (listed above, ~1-2%) are
    // zeroed first, summed by atomics and counted after.  (Too many of them for the list: every rank is zeroed and
    // the statistics re-read all values.)
    const int ndp = sh_ctr[2];
    const bool fused = ndp <= WIDE_DL;
    if (CLIP && tid == 0) c_oa[0] = 0u;  // (read after the statistics' block reduction)
    if (fused) {
      for (int j = tid; j < ndp; j += DBLOCK) S.vals[R.rank(ld_agent(&S.dkey[j]))] = 0.0;
    } else {
      for (int r = tid; r < np; r += DBLOCK) S.vals[r] = 0.0;
    }
    slot_sync();
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    double mx = -INFINITY;
    uint32_t poa = 0u;  // CLIP: top16_oa of the positive values
    for (int64_t i0 = a0; i0 < b0; i0 += (int64_t)DBLOCK * WDU) {
      typename H::Reg r[WDU];
#pragma unroll
      for (int u = 0; u < WDU; ++u) {  // unconditional loads (clamped index): counted waits, not vmcnt(0)
        const int64_t i = i0 + (int64_t)u * DBLOCK + tid;
        r[u] = hits.load(i < b0 ? i : b0 - 1);
      }
#pragma unroll
      for (int u = 0; u < WDU; ++u) {
        const int64_t i = i0 + (int64_t)u * DBLOCK + tid;
        if (i < b0 && WCK(H::pix(r[u]) < (uint32_t)npx, 4, H::pix(r[u]))) {
          const uint32_t p = H::pix(r[u]);
          uint32_t k = R.rank(p);
          if (!WCK(k < (uint32_t)np, 5, k)) k = 0;
          const double v = H::val(r[u]);
          if (H::dup(r[u])) {
            atomicAdd(&S.vals[k], v);
          } else {
            S.vals[k] = v;
            if (fused) {
              acc[0] += v;
              acc[1] += v * v;
              if (v > 0.0) {
                acc[2] += v;
                acc[3] += 1.0;
                if constexpr (CLIP) poa |= top16_oa((uint64_t)__double_as_longlong(v));
              }
              mx = v > mx ? v : mx;
            }
          }
        }
      }
    }
    slot_sync();
    if (fused) {  // the summed pixels, once each
      for (int j = tid; j < ndp; j += DBLOCK) {
        const double v = ld_agent(&S.vals[R.rank(ld_agent(&S.dkey[j]))]);
        acc[0] += v;
        acc[1] += v * v;
        if (v > 0.0) {
          acc[2] += v;
          acc[3] += 1.0;
          if constexpr (CLIP) poa |= top16_oa((uint64_t)__double_as_longlong(v));
        }
        mx = v > mx ? v : mx;
      }
    } else {
      for (int r0 = tid; r0 < np; r0 += DBLOCK * WDU) {  // WDU loads in flight per lane
        uint64_t vb[WDU];
#pragma unroll
        for (int j = 0; j < WDU; ++j) {
          vb[j] = 0ull;
          vb[j] = (uint64_t)__double_as_longlong(ld_agent(&S.vals[(r0 + j * DBLOCK < np) ? r0 + j * DBLOCK : 0]));
        }
#pragma unroll
        for (int j = 0; j < WDU; ++j) {
          if (r0 + j * DBLOCK >= np) continue;
          const double v = __longlong_as_double((long long)vb[j]);
          acc[0] += v;
          acc[1] += v * v;
          if (v > 0.0) {
            acc[2] += v;
            acc[3] += 1.0;
            if constexpr (CLIP) poa |= top16_oa(vb[j]);
          }
          mx = v > mx ? v : mx;
        }
      }
    }
    if (np < npx) mx = mx > 0.0 ? mx : 0.0;  // unlisted pixels are zero
    if (CLIP && poa) atomicOr(&c_oa[0], poa);
    dblock_sum<4>(acc, red);
    if constexpr (CLIP) {
      // the hot-spot clip of the principal image: its q-th percentile over the acc[3] positive values, every value
      // above it lowered to it, then the statistics again
      const int n0 = (int)acc[3];
      if (n0 > 0) {
        // the bits common to the positive values' top 16 (gathered with the statistics) skip the select's first
        // pass or two
        const uint32_t oa = c_oa[0];
        acc[0] = acc[1] = acc[2] = acc[3] = 0.0;
        mx = -INFINITY;
        auto clip_one = [&](int r, double v, double thr) {
          if (v > thr) {
            v = thr;
            S.vals[r] = thr;
          }
          acc[0] += v;
          acc[1] += v * v;
          if (v > 0.0) {
            acc[2] += v;
            acc[3] += 1.0;
          }
          mx = v > mx ? v : mx;
        };
        if (np <= PRV * DBLOCK) {
          // up to PRV values per lane: held in registers for the select's passes and the clip (one read)
          uint64_t pv[PRV];
#pragma unroll
          for (int j = 0; j < PRV; ++j) {
            const int r = tid + j * DBLOCK;
            pv[j] = r < np ? (uint64_t)__double_as_longlong(ld_agent(&S.vals[r])) : 0ull;
          }
          const double thr = percentile_of<DBLOCK>(
              [&](auto&& f) {
#pragma unroll
                for (int j = 0; j < PRV; ++j)
                  if ((int64_t)pv[j] > 0) f(pv[j]);  // v > 0 (sign clear, not +0)
              },
              n0, P.q, c_hist, c_sh, c_dsh, oa_lo(oa), oa_hi(oa));
#pragma unroll
          for (int j = 0; j < PRV; ++j)
            if (tid + j * DBLOCK < np) clip_one(tid + j * DBLOCK, __longlong_as_double((long long)pv[j]), thr);
        } else {
          const double thr = percentile_of<DBLOCK>(
              [&](auto&& f) {
                for (int r = tid; r < np; r += DBLOCK) {
                  const double v = ld_agent(&S.vals[r]);
                  if (v > 0.0) f((uint64_t)__double_as_longlong(v));
                }
              },
              n0, P.q, c_hist, c_sh, c_dsh, oa_lo(oa), oa_hi(oa));
          for (int r = tid; r < np; r += DBLOCK) clip_one(r, ld_agent(&S.vals[r]), thr);
        }
        if (np < npx) mx = mx > 0.0 ? mx : 0.0;
        dblock_sum<4>(acc, red);
        slot_sync();  // the clipped values are visible to the tail's gathers
      }
    }
    {
      const double vmax = block_max<DNW>(mx, red);
      if (tid == 0) {  // kept in the LDS until chaos / finalize (frees registers for the tail stream)
        sh_ctr[2] = 0;   // the principal's flagged-pixel count: the tail stream's list count from here
        sh_st[0] = acc[0];
        sh_st[1] = acc[1];
        sh_st[2] = acc[2];
        sh_st[3] = acc[3];
        sh_st[4] = vmax;
      }
    }

    STAMP(11);
    // tail windows.  Σy and Σy² per window come from the hit prefix sums (one thread per window; their Σy² covers
    // the points without the duplicate-candidate flag); Σxy and Σy[x>0] are linear in the points, so one stream
    // over the windows' concatenated points (a lane's window index only grows along it) adds x·y and [x>0]·y of
    // every point whose pixel is principal, x gathered by rank.  Flagged points are listed and summed per
    // (window, pixel) in the table, which adds (Σy)² of each entry to Σy².
    // the stream runs over the tail windows in batches of TSTEP positions (one per lane and u); each window starts
    // on a batch boundary (its length padded), so a batch lies in one window: the window index is uniform
    constexpr int64_t TSTEP = (int64_t)DBLOCK * (FMT == SMG_HITS_PACKED_F32 ? TDU : WDU);
    if (tid < 4 * MAXK_DENSE) kst[tid] = 0.0;
    if (tid <= K - 1) {
      int64_t n = 0;
      for (int k = 1; k <= tid; ++k) {
        WCK(hi[w0 + k] >= lo[w0 + k] && lo[w0 + k] >= 0, 6, hi[w0 + k] - lo[w0 + k]);
        n += (hi[w0 + k] - lo[w0 + k] + TSTEP - 1) / TSTEP * TSTEP;
      }
      sh_tb[tid] = n;  // sh_tb[k - 1]: stream offset of window k (padded lengths before it)
      if (tid < K - 1) {
        sh_tlo[tid] = lo[w0 + 1 + tid];
        sh_tn[tid] = hi[w0 + 1 + tid] - lo[w0 + 1 + tid];
      }
    }
    __syncthreads();
    if (!CLIP && tid < K - 1) {  // (CLIP: Σy, Σy² of the clipped images come from the clip stream below)
      const double2 ws = window_sums<FMT>(hits, cum, lo[w0 + 1 + tid], hi[w0 + 1 + tid]);
      kst[1 * MAXK_DENSE + tid + 1] = ws.x;
      kst[2 * MAXK_DENSE + tid + 1] = ws.y;
    }
    if constexpr (CLIP) {
      wide_clip_tail<FMT>(hits, K, P.q, npx, R, S, sh_tb, sh_tlo, sh_tn, ltkey, ltval, kst, &sh_nown, sh_ctr, c_hist, c_sh,
                          c_dsh, c_thr, c_n, c_st, c_flag, c_oa);
    } else {
      const int64_t T = sh_tb[K - 1];
      double as = 0.0, axy = 0.0;  // the lane's Σy[x > 0], Σxy in window kacc
      int kacc = 0;
      auto wflush = [&]() {  // uniform: the wave's sums of window kacc into its LDS row
        const double t0 = wave_sum_dpp(as), t1 = wave_sum_dpp(axy);
        if ((tid & 63) == 0) {
          atomicAdd(&kst[0 * MAXK_DENSE + kacc + 1], t0);
          atomicAdd(&kst[3 * MAXK_DENSE + kacc + 1], t1);
        }
        as = axy = 0.0;
      };
      // the flagged points of a batch (bit u of flm: point u) stay in the lane's registers (WIDE_FLR of them;
      // ~2% of the points are flagged): no stores in the stream, whose counted waits would then wait for them.
      // A lane's further flagged points go to the global list (rare).
      using YT = std::conditional_t<FMT == SMG_HITS_PACKED_F32, float, double>;  // exact: packed values are f32
      uint32_t fk[WIDE_FLR];
      YT fv[WIDE_FLR];
      int fc = 0;
#pragma unroll
      for (int j = 0; j < WIDE_FLR; ++j) {
        fk[j] = 0u;
        fv[j] = (YT)0;
      }
      auto append = [&](uint32_t flm, int kw, const auto& rs, int n) {
        for (int u = 0; u < n; ++u)
          if ((flm >> u) & 1u) {
            const uint32_t key = (uint32_t)kw * (uint32_t)npx + H::pix(rs[u]);
            const YT y = (YT)H::val(rs[u]);
            if (fc < WIDE_FLR) {
#pragma unroll
              for (int j = 0; j < WIDE_FLR; ++j)
                if (fc == j) {
                  fk[j] = key;
                  fv[j] = y;
                }
            } else {
              const int idx = atomicAdd(&sh_ctr[2], 1);
              if (idx < WIDE_DL) {
                S.dkey[idx] = key;
                S.dval[idx] = (double)y;
              } else {
                sh_ctr[3] = 1;
              }
            }
            ++fc;
            sh_anyfl = 1;
          }
      };
      if constexpr (FMT == SMG_HITS_PACKED_F32) {
        // software pipeline over batches of TDU points per lane, two register sets: a batch first issues the next
        // batch's loads, then waits for its own (all but the TDU youngest operations).  A batch only tests its
        // points against the principal bitmap (LDS) and the duplicate flag; a principal hit (~1-2% of the points)
        // is parked in registers (two per lane, with its window) and its x gathered after the stream, all lanes at
        // once, so the stream has one memory round trip per batch, not two.  A lane's third and later hits gather
        // in place (rare).  Every lane issues every load (a clamped index) so that the counted waits hold per wave.
        const uint64_t* hb = hits.h;
        uint64_t rA[TDU], rB[TDU], rC[TDU];
#pragma unroll
        for (int u = 0; u < TDU; ++u) rA[u] = rB[u] = rC[u] = 0ull;
        uint64_t ev0 = 0ull, ev1 = 0ull;
        int evk0 = 0, evk1 = 0, nev = 0;
        int ki = 0;  // window of the last batch issued (uniform)
        auto issue = [&](int64_t v0, uint64_t (&r)[TDU]) -> int {
          while (v0 >= sh_tb[ki + 1]) ++ki;
          ki = __builtin_amdgcn_readfirstlane(ki);
#ifdef SMG_WIDE_CHECK
          if (!WCK(ki <= K - 2, 7, ki)) ki = 0;
#endif
          const int64_t off = v0 - sh_tb[ki], n = sh_tn[ki], a = sh_tlo[ki];
#pragma unroll
          for (int u = 0; u < TDU; ++u) {
            const int64_t lv = off + (int64_t)u * DBLOCK + tid;
#ifdef SMG_WIDE_CHECK
            const int64_t ix = a + (lv < n ? lv : n - 1);
            r[u] = hb[WCK(ix >= 0 && ix < (1ll << 36), 8, ix) ? ix : 0];
#else
            r[u] = hb[a + (lv < n ? lv : n - 1)];
#endif
          }
          return ki;
        };
        // a batch first issues the batch TDEPTH - 1 ahead (TDEPTH register sets in rotation)
        auto batch = [&](int64_t v0, uint64_t (&r)[TDU], int kb, uint64_t (&rn)[TDU], int& kn) {
          if (v0 + (TDEPTH - 1) * TSTEP < T) kn = issue(v0 + (TDEPTH - 1) * TSTEP, rn);
          const int64_t off = v0 - sh_tb[kb], n = sh_tn[kb];
          uint32_t flm = 0u;
#pragma unroll
          for (int u = 0; u < TDU; ++u) {
            const bool valid = off + (int64_t)u * DBLOCK + tid < n && WCK(H::pix(r[u]) < (uint32_t)npx, 9, H::pix(r[u]));
            const uint32_t p = H::pix(r[u]);
            const bool pr = valid && R.test(p);
            const bool s0 = pr && nev == 0, s1 = pr && nev == 1;
            ev0 = s0 ? r[u] : ev0;
            evk0 = s0 ? kb : evk0;
            ev1 = s1 ? r[u] : ev1;
            evk1 = s1 ? kb : evk1;
            nev += pr ? 1 : 0;
            flm |= (uint32_t)(valid && H::dup(r[u])) << u;
            flm |= (uint32_t)(pr && nev > 2) << (16 + u);
          }
          if (__ballot((flm >> 16) != 0u)) {  // rare: a lane's third and later hits gather in place
#pragma unroll
            for (int u = 0; u < TDU; ++u)
              if ((flm >> (16 + u)) & 1u && WCK(R.rank(H::pix(r[u])) < (uint32_t)np, 11, R.rank(H::pix(r[u])))) {
                const double xv = ld_agent(&S.vals[R.rank(H::pix(r[u]))]);
                const double y = H::val(r[u]);
                atomicAdd(&kst[3 * MAXK_DENSE + kb + 1], xv * y);
                if (xv > 0.0) atomicAdd(&kst[0 * MAXK_DENSE + kb + 1], y);
              }
          }
          append(flm & 0xFFFFu, kb, r, TDU);
        };
        int kA = 0, kB = 0, kC = 0;
        if (T > 0) kA = issue(0, rA);
        if constexpr (TDEPTH == 3) {
          if (TSTEP < T) kB = issue(TSTEP, rB);
          for (int64_t v0 = 0; v0 < T; v0 += 3 * TSTEP) {
            batch(v0, rA, kA, rC, kC);
            if (v0 + TSTEP >= T) break;
            batch(v0 + TSTEP, rB, kB, rA, kA);
            if (v0 + 2 * TSTEP >= T) break;
            batch(v0 + 2 * TSTEP, rC, kC, rB, kB);
          }
        } else {
          for (int64_t v0 = 0; v0 < T; v0 += 2 * TSTEP) {
            batch(v0, rA, kA, rB, kB);
            if (v0 + TSTEP >= T) break;
            batch(v0 + TSTEP, rB, kB, rA, kA);
          }
        }
        // the parked principal hits: ranks, both x gathers in flight together, then the window partials
        if (__ballot(nev > 0)) {
          const uint32_t p0 = H::pix(ev0), p1 = H::pix(ev1);
#ifdef SMG_WIDE_CHECK
          const uint32_t k0 = nev > 0 && WCK(R.rank(p0) < (uint32_t)np, 10, R.rank(p0)) ? R.rank(p0) : 0u;
          const uint32_t k1 = nev > 1 && WCK(R.rank(p1) < (uint32_t)np, 10, R.rank(p1)) ? R.rank(p1) : 0u;
          const double x0 = nev > 0 ? ld_agent(&S.vals[k0]) : 0.0;
          const double x1 = nev > 1 ? ld_agent(&S.vals[k1]) : 0.0;
#else
          const double x0 = nev > 0 ? ld_agent(&S.vals[R.rank(p0)]) : 0.0;
          const double x1 = nev > 1 ? ld_agent(&S.vals[R.rank(p1)]) : 0.0;
#endif
          if (nev > 0) {
            const double y = H::val(ev0);
            atomicAdd(&kst[3 * MAXK_DENSE + evk0 + 1], x0 * y);
            if (x0 > 0.0) atomicAdd(&kst[0 * MAXK_DENSE + evk0 + 1], y);
          }
          if (nev > 1) {
            const double y = H::val(ev1);
            atomicAdd(&kst[3 * MAXK_DENSE + evk1 + 1], x1 * y);
            if (x1 > 0.0) atomicAdd(&kst[0 * MAXK_DENSE + evk1 + 1], y);
          }
        }
      } else {
        int kb = 0;
        for (int64_t v0 = 0; v0 < T; v0 += TSTEP) {
          while (v0 >= sh_tb[kb + 1]) ++kb;
          kb = __builtin_amdgcn_readfirstlane(kb);
          if (kb != kacc) {
            wflush();
            kacc = kb;
          }
          const int64_t off = v0 - sh_tb[kb], n = sh_tn[kb], a = sh_tlo[kb];
          typename H::Reg r[WDU];
#pragma unroll
          for (int u = 0; u < WDU; ++u) {
            const int64_t lv = off + (int64_t)u * DBLOCK + tid;
            r[u] = hits.load(a + (lv < n ? lv : n - 1));
          }
          uint32_t flm = 0u;
#pragma unroll
          for (int u = 0; u < WDU; ++u) {
            const bool valid = off + (int64_t)u * DBLOCK + tid < n;
            const uint32_t p = H::pix(r[u]);
            const double xv = (valid && R.test(p)) ? ld_agent(&S.vals[R.rank(p)]) : 0.0;
            const double y = H::val(r[u]);
            if (xv > 0.0) as += y;
            axy += xv * y;
            flm |= (uint32_t)(valid && H::dup(r[u])) << u;
          }
          append(flm, kb, r, WDU);
        }
      }
      wflush();
      __syncthreads();
      const int nd = min(sh_ctr[2], WIDE_DL);
      if (sh_anyfl) {
        if (nd > 0) slot_sync();  // the overflow list is complete in L2
        // sum the flagged points per key: in the LDS table (LDS atomics), an entry that finds no free slot within
        // WIDE_LT_PROBES in the slot's global table (one atomic round trip per entry held); the lane that claims a
        // global entry lists it
        auto insert_global = [&](uint32_t key, double y) {
          uint32_t h = (key * 0x9E3779B1u) >> (32 - WIDE_HT_LOG2);
          bool own = false, done = false;
          for (int t = 0; t < WIDE_PROBES; ++t) {
            const uint32_t old = atomicCAS(&S.hkey[h], WIDE_EMPTY, key);
            if (old == WIDE_EMPTY || old == key) {
              atomicAdd(&S.hval[h], y);
              own = old == WIDE_EMPTY;
              done = true;
              break;
            }
            h = (h + 1) & (WIDE_HT - 1);
          }
          if (!done) sh_ctr[3] = 1;
          return own ? (int)h : -1;
        };
        auto insert = [&](bool act, uint32_t key, double y) {  // uniform call: act = this lane has an entry
          bool placed = !act;
          if (act) {
            uint32_t h = (key * 0x9E3779B1u) >> (32 - WIDE_LT_LOG2);
            for (int t = 0; t < WIDE_LT_PROBES; ++t) {
              const uint32_t old = atomicCAS(&ltkey[h], WIDE_EMPTY, key);
              if (old == WIDE_EMPTY || old == key) {
                atomicAdd(&ltval[h], y);
                placed = true;
                break;
              }
              h = (h + 1) & (WIDE_LT - 1);
            }
          }
          int gh = -1;
          if (__ballot(!placed)) {
            if (!placed) gh = insert_global(key, y);
          }
          const int idx = wave_append(gh >= 0, &sh_nown);
          if (gh >= 0) S.hown[idx] = (uint32_t)gh;
        };
#pragma unroll
        for (int j = 0; j < WIDE_FLR; ++j) insert(j < fc, fk[j], (double)fv[j]);
        for (int j0 = 0; j0 < nd; j0 += DBLOCK) {
          const int j = j0 + tid;
          insert(j < nd, j < nd ? ld_agent(&S.dkey[j]) : 0u, j < nd ? ld_agent(&S.dval[j]) : 0.0);
        }
        slot_sync();  // the tables' sums are complete (LDS; L2 for the global entries)
        for (int i = tid; i < WIDE_LT; i += DBLOCK) {  // LDS entries: add their pixel's (Σy)², then release them
          const uint32_t key = ltkey[i];
          if (key != WIDE_EMPTY && WCK(key / (uint32_t)npx + 1 < (uint32_t)MAXK_DENSE, 12, key)) {
            const double y = ltval[i];
            atomicAdd(&kst[2 * MAXK_DENSE + key / (uint32_t)npx + 1], y * y);
            ltkey[i] = WIDE_EMPTY;
            ltval[i] = 0.0;
          }
        }
        const int no = sh_nown;
        for (int j = tid; j < no; j += DBLOCK) {  // claimed entries: add their pixel's (Σy)², then release them
          const uint32_t s = S.hown[j];
          const uint32_t key = ld_agent(&S.hkey[s]);
          const double y = ld_agent(&S.hval[s]);
          const uint32_t k = key / (uint32_t)npx;
          if (WCK(k + 1 < (uint32_t)MAXK_DENSE, 12, key)) atomicAdd(&kst[2 * MAXK_DENSE + k + 1], y * y);
          S.hkey[s] = WIDE_EMPTY;
          S.hval[s] = 0.0;
        }
        __syncthreads();  // (released entries reach L2 before the next ion's inserts: slot_syncs lie between)
      }
    }
    if (sh_ctr[3]) {  // the table overflowed: the pixel-indexed kernel scores this ion
      if (tid == 0) rej_list[atomicAdd(rej_count, 1u)] = (uint32_t)ion;
      __syncthreads();
      continue;
    }

    STAMP(12);
    double chaos_raw = NAN;
    const double npos = sh_st[3];
    if ((sh_st[0] > 0.0) && (npos >= 4.0)) {
      const double vmax = sh_st[4];
      STAMP(13);
      // candidates: eL = erode_box(dilate_cross(L)) >= 1 only where erode_box(dilate_cross(presence)) is set
      // (presence is a superset of L >= 1).  That screen is computed 64 pixels at a time on the flat LDS bitmap
      // (E = erode_box(dilate_cross(P)) with the image border, from presence rows r-2 .. r+2), E's pixels listed;
      // the exact eL of each listed pixel reads the levels of its 5x5 neighbourhood by rank.
      // per principal pixel p (listed in par, any order): presence rows r-3 .. r+3 of its 7-column window give
      // D = dilate_cross and E = erode_box(D) (with the image border) for the five pixels of p's 4-cross by
      // row-parallel bit operations; each pixel of E is listed once, by the first principal pixel on its cross
      STAMP(8);
      if (tid == 0) sh_ncand = 0;
      __syncthreads();
      // the candidate list is staged in the LDS table's space (free until the next ion's tail stream), the rest
      // in the slot (S.epr); the next iteration's principal pixel is loaded one iteration ahead
      uint32_t* lcand = ltkey;
      constexpr int LCAND = WIDE_LT * 3;  // ltkey + ltval: 12 B per table entry
      int pnext = (tid < np) ? (int)ld_agent(&S.par[tid]) : -1;
      for (int i0 = 0; i0 < np; i0 += DBLOCK) {  // uniform trip count: DPP scan below
        const int p = pnext;
        pnext = (i0 + DBLOCK + tid < np) ? (int)ld_agent(&S.par[i0 + DBLOCK + tid]) : -1;
        uint32_t cm = 0u;  // bit j: cross pixel j (0 centre, 1 up, 2 down, 3 left, 4 right) is listed by p
        int r0 = 0, c0 = 0;
        if (p >= 0) {
          rowcol(p, P, r0, c0);
          uint32_t B[7], IM[7];
          uint32_t imc = 0x7Fu;  // columns c0-3 .. c0+3 inside the image
          if (c0 - 3 < 0) imc &= 0x7Fu << (uint32_t)(3 - c0);
          if (c0 + 3 >= nc) imc &= 0x7Fu >> (uint32_t)(c0 + 3 - (nc - 1));
#pragma unroll
          for (int dr = -3; dr <= 3; ++dr) {
            B[dr + 3] = pres.row7(r0 + dr, c0, nr, nc);
            IM[dr + 3] = (r0 + dr >= 0 && r0 + dr < nr) ? imc : 0u;
          }
          // sparsity pre-filter (erosion border 0): a candidate's 3x3 box is covered by 4-crosses of principal
          // pixels only if at least three of them lie in its 5x5, inside p's 7x7
          const bool sparse = !P.erosion_border && (__popc(B[0]) + __popc(B[1]) + __popc(B[2]) + __popc(B[3]) +
                                                    __popc(B[4]) + __popc(B[5]) + __popc(B[6])) < 3;
          if (!sparse) {
          uint32_t Eh[7];
#pragma unroll
          for (int k = 1; k <= 5; ++k) {
            const uint32_t d = B[k] | (B[k] << 1) | (B[k] >> 1) | B[k - 1] | B[k + 1];
            const uint32_t dm = (P.erosion_border ? (d | ~IM[k]) : (d & IM[k])) & 0x7Fu;
            Eh[k] = dm & (dm << 1) & (dm >> 1);
          }
          auto E = [&](int k, int j) -> uint32_t { return (Eh[k - 1] & Eh[k] & Eh[k + 1] & IM[k]) >> j & 1u; };
          auto pr = [&](int k, int j) -> uint32_t { return (B[k] >> j) & 1u; };
#pragma unroll
          for (int t = 0; t < 5; ++t) {
            const int qr = (t == 1) ? -1 : (t == 2) ? 1 : 0, qc = (t == 3) ? -1 : (t == 4) ? 1 : 0;
            const int wr = qr + 3, wc = qc + 3;
            // the first principal pixel among q-nc, q-1, q, q+1, q+nc must be p
            int orr = 9, occ = 9;
            if (pr(wr + 1, wc)) orr = 1, occ = 0;
            if (pr(wr, wc + 1)) orr = 0, occ = 1;
            if (pr(wr, wc)) orr = 0, occ = 0;
            if (pr(wr, wc - 1)) orr = 0, occ = -1;
            if (pr(wr - 1, wc)) orr = -1, occ = 0;
            if (qr + orr == 0 && qc + occ == 0 && E(wr, wc)) cm |= 1u << t;
          }
          }
        }
        const int cnt = __popc(cm);
        const int incl = wave_incl_scan_dpp(cnt);
        int wbase = 0;
        if ((tid & 63) == 63 && incl > 0) wbase = atomicAdd(&sh_ncand, incl);
        wbase = __shfl(wbase, 63);
        int idx = wbase + incl - cnt;
        while (cm != 0u) {
          const int t = __ffs(cm) - 1;
          const int qr = (t == 1) ? -1 : (t == 2) ? 1 : 0, qc = (t == 3) ? -1 : (t == 4) ? 1 : 0;
          const uint32_t q = (uint32_t)((r0 + qr) * nc + c0 + qc);
          if (idx < LCAND) lcand[idx] = q;
          else if (WCK(idx < npx, 13, idx)) S.epr[idx] = q;
          ++idx;
          cm &= cm - 1u;
        }
      }
      slot_sync();
      STAMP(9);
#ifdef SMG_WIDE_CHECK
      const int nscr = WCK(sh_ncand <= npx, 14, sh_ncand) ? sh_ncand : 0;
#else
      const int nscr = sh_ncand;
#endif
      if (nscr > 0) {  // level index per principal pixel, needed only around screened candidates
        for (int r0 = tid; r0 < np; r0 += DBLOCK * WDU) {
          uint64_t vb[WDU];
#pragma unroll
          for (int j = 0; j < WDU; ++j) {
            vb[j] = 0ull;
            vb[j] = (uint64_t)__double_as_longlong(ld_agent(&S.vals[(r0 + j * DBLOCK < np) ? r0 + j * DBLOCK : 0]));
          }
#pragma unroll
          for (int j = 0; j < WDU; ++j)
            if (r0 + j * DBLOCK < np)
              S.L[r0 + j * DBLOCK] = (uint8_t)level_fast(__longlong_as_double((long long)vb[j]), vmax, P);
        }
        slot_sync();
      }
      for (int i0 = 0; i0 < nscr; i0 += DBLOCK) {
        const int i = i0 + tid;
        const int q = (i < nscr) ? (int)(i < LCAND ? lcand[i] : ld_agent(&S.epr[i])) : -1;
        int e = 0;
        if (q >= 0) {
          int r0, c0;
          rowcol(q, P, r0, c0);
          uint64_t WL[7];  // byte (dc + 3) of WL[dr + 3]: level of pixel (r0 + dr, c0 + dc), 0 outside / absent
          WL[0] = WL[6] = 0ull;
#pragma unroll
          for (int dr = -2; dr <= 2; ++dr) {
            const uint32_t row = pres.row7(r0 + dr, c0, nr, nc);
            uint64_t wv = 0ull;
            if (row != 0u) {
              // the row's present pixels have consecutive ranks: their levels are L[base .. base + popc(row))
              uint32_t rb = R.rank((uint32_t)((r0 + dr) * nc + max(c0 - 3, 0)));
              if (!WCK(rb <= (uint32_t)np, 16, rb)) rb = 0;
              const uint64_t* la = reinterpret_cast<const uint64_t*>(S.L + (rb & ~7u));
              const uint64_t l0 = la[0], l1 = la[1];
              const uint32_t sh = (rb & 7u) * 8u;
              uint64_t packed = sh ? ((l0 >> sh) | (l1 << (64u - sh))) : l0;
#pragma unroll
              for (int j = 0; j < 7; ++j)
                if ((row >> j) & 1u) {
                  wv |= (packed & 0xFFull) << (8 * j);
                  packed >>= 8;
                }
            }
            WL[dr + 3] = wv;
          }
          auto W = [&](int wr, int wc) -> int { return (int)((WL[wr] >> (8 * wc)) & 0xFFull); };
          e = 1 << 20;
#pragma unroll
          for (int a = -1; a <= 1; ++a)
#pragma unroll
            for (int b = -1; b <= 1; ++b) {
              const int rr = r0 + a, cc = c0 + b;
              if (rr < 0 || rr >= nr || cc < 0 || cc >= nc) {
                if (!P.erosion_border) e = 0;
                continue;
              }
              const int wr = a + 3, wc = b + 3;
              const int t = max(max(W(wr, wc), W(wr - 1, wc)), max(max(W(wr + 1, wc), W(wr, wc - 1)), W(wr, wc + 1)));
              e = min(e, t);
            }
          if (e >= (1 << 20)) e = 0;
        }
        const int idx = wave_append(e >= 1, &sh_ctr[0]);
        if (e >= 1) {
          S.epix[idx] = (uint32_t)q;
          S.eL[idx] = (uint8_t)e;
          atomicMax(&sh_ctr[1], e);
        }
      }
      slot_sync();
      // the staged candidates are consumed: the LDS table is empty again for the next ion's tail stream
      for (int i = tid; i < min(nscr, LCAND); i += DBLOCK) lcand[i] = i < WIDE_LT ? WIDE_EMPTY : 0u;
#ifdef SMG_WIDE_CHECK
      const int m = WCK(sh_ctr[0] <= npx, 15, sh_ctr[0]) ? sh_ctr[0] : 0;
#else
      const int m = sh_ctr[0];
#endif
      const int emax = sh_ctr[1];
      STAMP(14);
      double esum = 0.0, wsum = 0.0;
      for (int i = tid; i < m; i += DBLOCK) esum += (double)S.eL[i];
      if (m > 0) {  // Kruskal over the candidates, indexed by their rank in a candidate bitmap
        for (int w = tid; w < n64p; w += DBLOCK) bm[w] = 0ull;
        __syncthreads();
        for (int i = tid; i < m; i += DBLOCK) {
          const uint32_t q = S.epix[i];
          atomicOr(&bm32[q >> 5], 1u << (q & 31));
        }
        __syncthreads();
        build_rank(bm, pf, sb, n64, sc);
        for (int i = tid; i < m; i += DBLOCK) {
          const uint32_t q = S.epix[i];
          uint32_t k = R.rank(q);
          if (!WCK(k < (uint32_t)m && q < (uint32_t)npx, 17, k)) k = 0;
          S.epr[k] = q;
          S.eLr[k] = S.eL[i];
          S.par[k] = k;
        }
        slot_sync();
        for (int t = emax; t >= 1; --t) {
          for (int i = tid; i < m; i += DBLOCK) {
            const int e = S.eLr[i];
            if (e < t) continue;
            const int p = (int)S.epr[i];
            const int r = p / nc, c = p - r * nc;
            auto edge = [&](int q) {
              if (!R.test((uint32_t)q)) return;
              const uint32_t kq = R.rank((uint32_t)q);
              const int eq = S.eLr[kq];
              if ((e < eq ? e : eq) == t && guf_unite(S.par, (uint32_t)i, kq)) wsum += (double)t;
            };
            if (c + 1 < nc) edge(p + 1);
            if (r + 1 < nr) {
              edge(p + nc);
              if (P.connectivity == 8) {
                if (c > 0) edge(p + nc - 1);
                if (c + 1 < nc) edge(p + nc + 1);
              }
            }
          }
          __syncthreads();
        }
      }
      double a3[2] = {esum, wsum};
      dblock_sum<2>(a3, red);
      chaos_raw = 1.0 - (a3[0] - a3[1]) / (double)P.nlevels / npos;
    } else {
      flags |= SMG_ION_CHAOS_NAN;
    }

    if (tid == 0) {
      kst[0] = sh_st[2];
      kst[1 * MAXK_DENSE] = kst[2 * MAXK_DENSE] = kst[3 * MAXK_DENSE] = 0.0;
      finalize_ion(K, theor + w0, kst, sh_st[0], sh_st[1], kst + MAXK_DENSE, kst + 2 * MAXK_DENSE, kst + 3 * MAXK_DENSE,
                   (double)npx, chaos_raw, ion, flags, oc, osp, osc, omsm, oflags);
    }
    STAMP(15);
    __syncthreads();
  }
  STAMP_FLUSH();
}

// ---------------------------------------------------------------------------------------------
// wide pass without per-pixel arrays in global memory (round 6): ion_wide_join_kernel
// ---------------------------------------------------------------------------------------------
// ion_wide_kernel keeps the principal image's values, pixel list and levels at the pixels' ranks in its slot: at
// config 5 (~8.5k principal pixels per ion) that is ~110 KB stored per ion, 77 GB per rank-0 launch
// (profiles/round4/traffic_wide_r4.json), of which only ~450 values per ion are ever read back -- the tail's hits on
// principal pixels (mean 386) and the principal pixels within two of a chaos candidate (mean 59;
// profiles/round6/r6c5s_c5_stats.txt).  This pass stores none of them.  Per ion:
//  1. one stream over the principal window: presence bits (LDS bitmap), the statistics of the unflagged points (each
//     alone on its pixel, smg_flag_duplicates), the flagged points summed per pixel in an LDS table (PD), then the
//     statistics of PD's pixels;
//  2. the tail stream of ion_wide_kernel; a lane parks its first two hits on principal pixels in registers, later
//     ones go to a list in the slot; flagged tail points into the LT table (+ the slot's table) for Σy²;
//  3. the chaos screen of ion_wide_kernel per principal pixel, the pixels walked from the bitmap (every DNW-th word
//     per wave, per-wave work lists in the LT table's space, no barrier); candidates listed in the slot;
//  4. a hash (JH) over the dead bitmap / rank / LT space holds the tail hits' pixels and every candidate's 5x5 minus
//     its corners (images of up to 12,288 pixels index x by pixel instead); a second stream over the principal
//     window fills each entry's x (an unflagged point's value, a flagged pixel's PD sum; 0 without a point);
//  5. the hits' Σxy and Σy[x>0] from JH; each candidate's eL from its 5x5's levels; Kruskal as in
//     ion_wide_kernel (candidate bitmap + ranks over the bitmap's space) with its arrays and union-find in the LDS
//     (up to WJ_LK candidates, else in the slot), visiting only the levels some candidate has.
// An ion whose tables overflow goes to the pixel-indexed kernel (rej_list), as from ion_wide_kernel.
// LDS (fixed, WJ_LDS): [bitmap n64p*8][superblock bases][group prefixes][LT 12 KB] ... [PD at the end];
// JH = keys (u32) then x (f64), WJ_JH entries over [0, PD); images of up to WJ_JH * 12 / 8 pixels index x by pixel
// instead (every pixel's x, absent pixels 0), so that no image of that size overflows JH.  PD takes what JH and the
// LT table leave (1024 .. 8192 entries: 1024 at 2^20 pixels, 8192 on small images, whose flagged pixels can be many).
constexpr size_t WJ_LDS = 160 * 1024 - 4096;  // dynamic LDS of the join pass (static arrays ~3 KB)
constexpr int WJ_JH_LOG2 = 13;
constexpr int WJ_JH = 1 << WJ_JH_LOG2;       // hit pixels and candidates' neighbourhoods per ion
constexpr int WJ_WL = 128;                   // per-wave work list entries (principal pixels of the screen)
constexpr int WJ_LK = 1024;                  // candidates whose eL / Kruskal arrays stay in the LDS
static_assert(DNW * (WJ_WL + WAVE) * 4 <= WIDE_LT * 12, "work and survivor lists in the LT space");
static_assert(WJ_LK * 9 <= WIDE_LT * 12 && WJ_LK * 5 <= 1024 * 12, "Kruskal arrays in LT, eL lists in PD");
static_assert(DNW * WJ_WL * 4 <= WIDE_LT * 12, "work lists in the LT space");

__host__ __device__ static inline size_t wj_lt_off(int npx) {  // offset of the LT table: bitmap, sb, pf before it
  const size_t n64 = ((size_t)npx + 63) / 64, n64p = wide_n64p(npx);
  return n64p * 8 + ((((n64 + 1023) / 1024) * 4 + 15) & ~(size_t)15) + (((n64p / 4) * 2 + 15) & ~(size_t)15);
}
struct WjGeom {
  bool jdirect;   // x by pixel (over the bitmap's space)
  bool jafter;    // JH after the bitmap (over the LT table's space): the bitmap stays live while JH is filled
  int pd_log2;    // PD entries (log2)
  size_t jh_off;  // JH's offset
  size_t pd_off;
};
__host__ __device__ static inline WjGeom wj_geom(int npx) {
  WjGeom g;
  const size_t lt_off = wj_lt_off(npx), lt_end = lt_off + (size_t)WIDE_LT * 12, jhb = (size_t)WJ_JH * 12;
  g.jdirect = (size_t)npx * 8 <= jhb;
  g.jafter = !g.jdirect && lt_off + jhb + (size_t)12 * 1024 <= WJ_LDS;
  g.jh_off = g.jafter ? lt_off : 0;
  const size_t jh_end = g.jdirect ? (size_t)npx * 8 : g.jh_off + jhb;
  const size_t used = lt_end > jh_end ? lt_end : jh_end;
  const size_t room = used < WJ_LDS ? WJ_LDS - used : 0;
  g.pd_log2 = 0;
  while (g.pd_log2 < 13 && ((size_t)12 << (g.pd_log2 + 1)) <= room) ++g.pd_log2;
  g.pd_off = WJ_LDS - ((size_t)12 << g.pd_log2);
  return g;
}
// the join pass applies where its layout leaves PD >= 1024 entries and build_rank covers the bitmap (n64 <= DNW * 1024)
static inline bool wide_join_fits(int npx) {
  return ((size_t)npx + 63) / 64 <= (size_t)DNW * 1024 && wj_geom(npx).pd_log2 >= 10 &&
         wj_lt_off(npx) + (size_t)WIDE_LT * 12 <= wj_geom(npx).pd_off;
}

// union-find over LDS parents (the join pass's Kruskal): find with path halving, unite the larger root under the smaller
__device__ __forceinline__ uint32_t luf_find(uint32_t* par, uint32_t x) {
  volatile uint32_t* vp = par;
  while (true) {
    const uint32_t p = vp[x];
    if (p == x) return x;
    const uint32_t g = vp[p];
    if (g != p) vp[x] = g;
    x = g;
  }
}
__device__ __forceinline__ bool luf_unite(uint32_t* par, uint32_t a, uint32_t b) {
  while (true) {
    a = luf_find(par, a);
    b = luf_find(par, b);
    if (a == b) return false;
    if (a < b) {
      const uint32_t t = a;
      a = b;
      b = t;
    }
    if (atomicCAS(&par[a], a, b) == a) return true;
  }
}

// open-addressing u32 -> slot hash in LDS (empty WIDE_EMPTY): the slot of key or of its insertion (-1: full)
__device__ __forceinline__ int wj_insert(uint32_t* keys, int cap_log2, uint32_t key) {
  const int cap = 1 << cap_log2;
  uint32_t h = (key * 0x9E3779B1u) >> (32 - cap_log2);
  for (int t = 0; t < cap; ++t) {
    const uint32_t old = atomicCAS(&keys[h], WIDE_EMPTY, key);
    if (old == WIDE_EMPTY || old == key) return (int)h;
    h = (h + 1) & (uint32_t)(cap - 1);
  }
  return -1;
}
__device__ __forceinline__ uint32_t wj_hash(uint32_t key, int cap_log2) { return (key * 0x9E3779B1u) >> (32 - cap_log2); }
// wj_find with the first probe's slot h and key k0 already read
__device__ __forceinline__ int wj_find_from(const uint32_t* keys, int cap_log2, uint32_t key, uint32_t h, uint32_t k0) {
  if (k0 == key) return (int)h;
  if (k0 == WIDE_EMPTY) return -1;
  const int cap = 1 << cap_log2;
  for (int t = 1; t < cap; ++t) {
    h = (h + 1) & (uint32_t)(cap - 1);
    const uint32_t k = keys[h];
    if (k == key) return (int)h;
    if (k == WIDE_EMPTY) return -1;
  }
  return -1;
}
__device__ __forceinline__ int wj_find(const uint32_t* keys, int cap_log2, uint32_t key) {
  const int cap = 1 << cap_log2;
  uint32_t h = (key * 0x9E3779B1u) >> (32 - cap_log2);
  for (int t = 0; t < cap; ++t) {
    const uint32_t k = keys[h];
    if (k == key) return (int)h;
    if (k == WIDE_EMPTY) return -1;
    h = (h + 1) & (uint32_t)(cap - 1);
  }
  return -1;
}

// presence bits of columns c0-3 .. c0+3 of rows r0-3 .. r0+3 from the LDS bitmap (B[k]: row r0+k-3, bit j = column
// c0-3+j; 0 outside the image), branch-free: the 14 words are read together (one wait), then aligned and masked.
// One zero word follows the bitmap.
__device__ __forceinline__ void wj_rows7(const uint32_t* w, int r0, int c0, int nr, int nc, uint32_t (&B)[7]) {
  uint32_t lo[7], hi[7];
  int g[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int rr = r0 + k - 3;
    g[k] = (rr >= 0 && rr < nr) ? rr * nc + c0 - 3 : 0;
    const int wi = (g[k] > 0 ? g[k] : 0) >> 5;
    lo[k] = w[wi];
    hi[k] = w[wi + 1];
  }
  uint32_t cm = 0x7Fu;  // columns inside the image
  if (c0 - 3 < 0) cm &= 0x7Fu << (uint32_t)(3 - c0);
  if (c0 + 3 >= nc) cm &= 0x7Fu >> (uint32_t)(c0 + 3 - (nc - 1));
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int rr = r0 + k - 3;
    const uint32_t v = g[k] >= 0 ? __builtin_amdgcn_alignbit(hi[k], lo[k], (uint32_t)(g[k] & 31)) : lo[k] << (uint32_t)(-g[k]);
    B[k] = (rr >= 0 && rr < nr) ? (v & cm) : 0u;
  }
}

__global__ void __launch_bounds__(DBLOCK) ion_wide_join_kernel(
    Hits<SMG_HITS_PACKED_F32> hits, const DD4* __restrict__ cum, const int64_t* __restrict__ lo,
    const int64_t* __restrict__ hi, const int64_t* __restrict__ ion_off, const double* __restrict__ theor, Params P,
    const uint32_t* __restrict__ list, const uint32_t* __restrict__ count, uint32_t* next, uint32_t* rej_list,
    uint32_t* rej_count, uint32_t rej_cap, unsigned char* scratch, size_t slot_bytes, double* __restrict__ oc,
    double* __restrict__ osp, double* __restrict__ osc, double* __restrict__ omsm, uint32_t* __restrict__ oflags) {
  using H = Hits<SMG_HITS_PACKED_F32>;
  extern __shared__ __attribute__((aligned(16))) uint64_t wide_dyn[];
  __shared__ double red[8 * DNW];
  __shared__ double kst[4 * MAXK_DENSE];
  __shared__ uint32_t sc[DNW];
  __shared__ int sh_ion;
  __shared__ int sh_ctr[4];  // candidates with eL >= 1, max eL, listed flagged tail points, overflow (-> pixel kernel)
  __shared__ int sh_nown;    // claimed global table entries
  __shared__ int sh_ncand;   // screened chaos candidates (listed in S.epr)
  __shared__ int sh_anyfl;   // the tail stream met a flagged point
  __shared__ int sh_nov;     // tail hits beyond the registers (listed in the slot)
  __shared__ int sh_anyhit;  // some lane parked a hit
  __shared__ int sh_rs;      // the hit list overflowed on an image with x by pixel: the tail is streamed again
  __shared__ uint32_t sh_lvm[8];  // the candidates' eL values (bit e)
  __shared__ double sh_th[MAXK_DENSE];  // the ion's theoretical intensities (read during the tail, used by finalize)
  __shared__ int sh_K;       // the ion's windows, first window, principal bounds (fetched during the previous ion)
  __shared__ int64_t sh_w0, sh_a0, sh_b0;
  __shared__ double sh_st[5];  // principal sums: x, x^2, x[x > 0], #(x > 0); max
  __shared__ int64_t sh_tb[MAXK_DENSE + 1];
  __shared__ int64_t sh_tlo[MAXK_DENSE];
  __shared__ int64_t sh_tn[MAXK_DENSE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int npx = P.npx, n64 = (npx + 63) / 64, nsb = (n64 + 1023) / 1024;
  const int n64p = (int)wide_n64p(npx);
  unsigned char* const lds = reinterpret_cast<unsigned char*>(wide_dyn);
  uint64_t* bm = wide_dyn;
  uint32_t* bm32 = reinterpret_cast<uint32_t*>(bm);
  uint32_t* sb = reinterpret_cast<uint32_t*>(lds + (size_t)n64p * 8);
  uint16_t* pf = reinterpret_cast<uint16_t*>(reinterpret_cast<unsigned char*>(sb) + (((size_t)nsb * 4 + 15) & ~(size_t)15));
  uint32_t* ltkey = reinterpret_cast<uint32_t*>(lds + wj_lt_off(npx));
  double* ltval = reinterpret_cast<double*>(ltkey + WIDE_LT);
  const WjGeom G = wj_geom(npx);
  const int pd_log2 = G.pd_log2, npd = 1 << pd_log2;
  uint32_t* pdkey = reinterpret_cast<uint32_t*>(lds + G.pd_off);
  double* pdval = reinterpret_cast<double*>(pdkey + npd);
  // JH (after the screen), or x by pixel on small images
  const bool jdirect = G.jdirect, jafter = G.jafter;
  uint32_t* jkey = reinterpret_cast<uint32_t*>(lds + G.jh_off);
  double* jx = reinterpret_cast<double*>(lds + (jdirect ? (size_t)0 : G.jh_off + (size_t)WJ_JH * 4));
  auto jslot = [&](uint32_t p) -> int { return jdirect ? (int)p : wj_find(jkey, WJ_JH_LOG2, p); };
  const RankBits R{bm, pf, sb};
  WideSlot S = wide_slot(scratch + (size_t)blockIdx.x * slot_bytes, npx);
  uint64_t* ovh = reinterpret_cast<uint64_t*>(S.vals);  // tail hits beyond the registers (their windows in S.L)
  const PresenceBits<true> pres{bm32};
  uint32_t* wlist = ltkey + wid * WJ_WL;  // the screen's per-wave work lists (LT space)
  uint32_t* slist = ltkey + DNW * WJ_WL + wid * WAVE;  // the screen's per-wave survivor lists (LT space)
  auto cand = [&](int i) -> uint32_t { return ld_agent(&S.epr[i]); };
  const uint32_t total = *count;
  for (int i = tid; i < WIDE_HT; i += DBLOCK) {
    S.hkey[i] = WIDE_EMPTY;
    S.hval[i] = 0.0;
  }
  for (int i = tid; i < WIDE_LT; i += DBLOCK) {
    ltkey[i] = WIDE_EMPTY;
    ltval[i] = 0.0;
  }
  for (int i = tid; i < npd; i += DBLOCK) {
    pdkey[i] = WIDE_EMPTY;
    pdval[i] = 0.0;
  }
  slot_sync();
  const int nr = P.nrows, nc = P.ncols;
  STAMP_DECL();
  // the next ion (ticket, list entry, windows, principal bounds) is fetched by thread 0 one dependent load per phase
  // of the current ion, so that the chain's round trips overlap its streams; nst = the last stage done
  // (thread 0's state in the LDS: registers held across the ion by every lane would spill)
  __shared__ uint32_t nx_k;
  __shared__ int nx_ion, nx_st;
  __shared__ int64_t nx_w0, nx_w1, nx_a0, nx_b0;
  auto nx_start = [&]() {
    nx_k = atomicAdd(next, 1u);
    nx_ion = -1;
    nx_w0 = nx_w1 = nx_a0 = nx_b0 = 0;
    nx_st = 0;
  };
  auto nx_step = [&]() {
    const int st = nx_st;
    if (st == 0) {
      const uint32_t k = nx_k;
      nx_ion = k < total ? (int)list[k] : -1;
    } else if (st == 1) {
      const int i = nx_ion;
      if (i >= 0) {
        nx_w0 = ion_off[i];
        nx_w1 = ion_off[i + 1];
      }
    } else if (st == 2) {
      const int64_t w = nx_w0;
      if (nx_ion >= 0 && nx_w1 > w) {
        nx_a0 = lo[w];
        nx_b0 = hi[w];
      }
    }
    nx_st = st < 3 ? st + 1 : 3;
  };
  auto nx_publish = [&]() {
    while (nx_st < 3) nx_step();
    sh_ion = nx_ion;
    sh_w0 = nx_w0;
    sh_K = (int)(nx_w1 - nx_w0);
    sh_a0 = nx_a0;
    sh_b0 = nx_b0;
  };
  if (tid == 0) {
    nx_start();
    nx_publish();
  }

  while (true) {
    if (tid == 0) {
      sh_ctr[0] = sh_ctr[1] = sh_ctr[2] = sh_ctr[3] = 0;
      sh_nown = 0;
      sh_ncand = 0;
      sh_anyfl = 0;
      sh_nov = 0;
      sh_anyhit = 0;
      sh_rs = 0;
      for (int j = 0; j < 8; ++j) sh_lvm[j] = 0u;
    }
    __syncthreads();
    const int64_t ion = sh_ion;
    if (ion < 0) break;
    const int64_t w0 = sh_w0, a0 = sh_a0, b0 = sh_b0;
    const int K = sh_K;
    if (tid == 0) nx_start();
    uint32_t flags = SMG_ION_DENSE | SMG_ION_WIDE;
    if (K > MAXK_DENSE || K == 0) {
      for (int k = 0; k < K && k < MAXK_DENSE; ++k)
        if (hi[w0 + k] > lo[w0 + k]) flags |= SMG_ION_HAS_HITS;
      if (tid == 0) {
        oc[ion] = osp[ion] = osc[ion] = omsm[ion] = 0.0;
        oflags[ion] = (K == 0) ? 0u : (flags | 0x80000000u);
        nx_publish();
      }
      __syncthreads();
      continue;
    }
    STAMP(15);
    // ---- 1. principal image: presence bits, statistics, flagged pixels summed in PD ----------------------------
    for (int w = tid; w < n64p; w += DBLOCK) bm[w] = 0ull;
    __syncthreads();
    double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // Σx, Σx², Σx[x>0], #(x>0), #pixels
    double mx = -INFINITY;
    auto stat = [&](double v) {
      acc[0] += v;
      acc[1] += v * v;
      if (v > 0.0) {
        acc[2] += v;
        acc[3] += 1.0;
      }
      acc[4] += 1.0;
      mx = v > mx ? v : mx;
    };
    for (int64_t i0 = a0; i0 < b0; i0 += (int64_t)DBLOCK * WDU) {
      uint64_t r[WDU];
#pragma unroll
      for (int u = 0; u < WDU; ++u) {
        const int64_t i = i0 + (int64_t)u * DBLOCK + tid;
        r[u] = hits.load(i < b0 ? i : b0 - 1);
      }
#pragma unroll
      for (int u = 0; u < WDU; ++u) {
        const int64_t i = i0 + (int64_t)u * DBLOCK + tid;
        if (i < b0) {
          const uint32_t p = H::pix(r[u]);
          if (p >= (uint32_t)npx) {  // (only a caller-supplied hit can carry one)
            sh_ctr[3] = 1;
            continue;
          }
          atomicOr(&bm32[p >> 5], 1u << (p & 31));
          const double v = H::val(r[u]);
          if (H::dup(r[u])) {
            const int s = wj_insert(pdkey, pd_log2, p);
            if (s >= 0) atomicAdd(&pdval[s], v);
            else sh_ctr[3] = 1;
          } else {
            stat(v);
          }
        }
      }
    }
    if (tid == 0) nx_step();
    __syncthreads();
    for (int s = tid; s < npd; s += DBLOCK)
      if (pdkey[s] != WIDE_EMPTY) stat(pdval[s]);
    dblock_sum<5>(acc, red);
    if (acc[4] < (double)npx) mx = mx > 0.0 ? mx : 0.0;  // pixels outside the principal image are zero
    {
      const double vmax = block_max<DNW>(mx, red);
      if (tid == 0) {
        sh_st[0] = acc[0];
        sh_st[1] = acc[1];
        sh_st[2] = acc[2];
        sh_st[3] = acc[3];
        sh_st[4] = vmax;
      }
    }
    STAMP(10);
    // ---- 2. tail windows (ion_wide_kernel's packed stream; hits parked, none gathered) -------------------------
    constexpr int64_t TSTEP = (int64_t)DBLOCK * TDU;
    if (tid < 4 * MAXK_DENSE) kst[tid] = 0.0;
    if (tid <= K - 1) {
      int64_t n = 0;
      for (int k = 1; k <= tid; ++k) n += (hi[w0 + k] - lo[w0 + k] + TSTEP - 1) / TSTEP * TSTEP;
      sh_tb[tid] = n;
      if (tid < K - 1) {
        sh_tlo[tid] = lo[w0 + 1 + tid];
        sh_tn[tid] = hi[w0 + 1 + tid] - lo[w0 + 1 + tid];
      }
    }
    __syncthreads();
    if (tid < K) sh_th[tid] = theor[w0 + tid];
    if (tid < K - 1) {
      const double2 ws = window_sums<SMG_HITS_PACKED_F32>(hits, cum, lo[w0 + 1 + tid], hi[w0 + 1 + tid]);
      kst[1 * MAXK_DENSE + tid + 1] = ws.x;
      kst[2 * MAXK_DENSE + tid + 1] = ws.y;
    }
    const int64_t T = sh_tb[K - 1];
    uint32_t fk[WIDE_FLR];
    float fv[WIDE_FLR];
    int fc = 0;
#pragma unroll
    for (int j = 0; j < WIDE_FLR; ++j) {
      fk[j] = 0u;
      fv[j] = 0.0f;
    }
    auto append = [&](uint32_t flm, int kw, const uint64_t (&rs)[TDU]) {
      for (int u = 0; u < TDU; ++u)
        if ((flm >> u) & 1u) {
          const uint32_t key = (uint32_t)kw * (uint32_t)npx + H::pix(rs[u]);
          const float y = __uint_as_float((uint32_t)(rs[u] >> 32));
          if (fc < WIDE_FLR) {
#pragma unroll
            for (int j = 0; j < WIDE_FLR; ++j)
              if (fc == j) {
                fk[j] = key;
                fv[j] = y;
              }
          } else {
            const int idx = atomicAdd(&sh_ctr[2], 1);
            if (idx < WIDE_DL) {
              S.dkey[idx] = key;
              S.dval[idx] = (double)y;
            } else {
              sh_ctr[3] = 1;
            }
          }
          ++fc;
          sh_anyfl = 1;
        }
    };
    const uint64_t* hb = hits.h;
    uint64_t rA[TDU], rB[TDU];
#pragma unroll
    for (int u = 0; u < TDU; ++u) rA[u] = rB[u] = 0ull;
    uint64_t ev0 = 0ull, ev1 = 0ull;
    int evk0 = 0, evk1 = 0, nev = 0;
    int ki = 0;
    auto issue = [&](int64_t v0, uint64_t (&r)[TDU]) -> int {
      while (v0 >= sh_tb[ki + 1]) ++ki;
      ki = __builtin_amdgcn_readfirstlane(ki);
      const int64_t off = v0 - sh_tb[ki], n = sh_tn[ki], a = sh_tlo[ki];
#pragma unroll
      for (int u = 0; u < TDU; ++u) {
        const int64_t lv = off + (int64_t)u * DBLOCK + tid;
        r[u] = hb[a + (lv < n ? lv : n - 1)];
      }
      return ki;
    };
    auto batch = [&](int64_t v0, uint64_t (&r)[TDU], int kb, uint64_t (&rn)[TDU], int& kn) {
      if (v0 + TSTEP < T) kn = issue(v0 + TSTEP, rn);
      const int64_t off = v0 - sh_tb[kb], n = sh_tn[kb];
      uint32_t flm = 0u;
#pragma unroll
      for (int u = 0; u < TDU; ++u) {
        const uint32_t p = H::pix(r[u]);
        const bool valid = off + (int64_t)u * DBLOCK + tid < n && p < (uint32_t)npx;
        const bool pr = valid && R.test(p);
        const bool s0 = pr && nev == 0, s1 = pr && nev == 1;
        ev0 = s0 ? r[u] : ev0;
        evk0 = s0 ? kb : evk0;
        ev1 = s1 ? r[u] : ev1;
        evk1 = s1 ? kb : evk1;
        nev += pr ? 1 : 0;
        flm |= (uint32_t)(valid && H::dup(r[u])) << u;
        flm |= (uint32_t)(pr && nev > 2) << (16 + u);
      }
      if (__ballot((flm >> 16) != 0u)) {  // a lane's third and later hits: listed in the slot (rare)
#pragma unroll
        for (int u = 0; u < TDU; ++u)
          if ((flm >> (16 + u)) & 1u) {
            const int idx = atomicAdd(&sh_nov, 1);
            if (idx < npx) {
              ovh[idx] = r[u];
              S.L[idx] = (uint8_t)kb;
            } else if (jdirect) {
              sh_rs = 1;
            } else {
              sh_ctr[3] = 1;
            }
          }
      }
      append(flm & 0xFFFFu, kb, r);
    };
    int kA = 0, kB = 0;
    if (T > 0) kA = issue(0, rA);
    for (int64_t v0 = 0; v0 < T; v0 += 2 * TSTEP) {
      batch(v0, rA, kA, rB, kB);
      if (v0 + TSTEP >= T) break;
      batch(v0 + TSTEP, rB, kB, rA, kA);
    }
    if (nev > 0) sh_anyhit = 1;
    if (tid == 0) nx_step();
    __syncthreads();
    // flagged tail points summed per (window, pixel): LDS table, then the slot's table; (Σy)² of each entry into Σy²
    const int nd = min(sh_ctr[2], WIDE_DL);
    if (sh_anyfl) {
      if (nd > 0) slot_sync();
      auto insert_global = [&](uint32_t key, double y) {
        uint32_t h = (key * 0x9E3779B1u) >> (32 - WIDE_HT_LOG2);
        bool own = false, done = false;
        for (int t = 0; t < WIDE_PROBES; ++t) {
          const uint32_t old = atomicCAS(&S.hkey[h], WIDE_EMPTY, key);
          if (old == WIDE_EMPTY || old == key) {
            atomicAdd(&S.hval[h], y);
            own = old == WIDE_EMPTY;
            done = true;
            break;
          }
          h = (h + 1) & (WIDE_HT - 1);
        }
        if (!done) sh_ctr[3] = 1;
        return own ? (int)h : -1;
      };
      auto insert = [&](bool act, uint32_t key, double y) {
        bool placed = !act;
        if (act) {
          uint32_t h = (key * 0x9E3779B1u) >> (32 - WIDE_LT_LOG2);
          for (int t = 0; t < WIDE_LT_PROBES; ++t) {
            const uint32_t old = atomicCAS(&ltkey[h], WIDE_EMPTY, key);
            if (old == WIDE_EMPTY || old == key) {
              atomicAdd(&ltval[h], y);
              placed = true;
              break;
            }
            h = (h + 1) & (WIDE_LT - 1);
          }
        }
        int gh = -1;
        if (__ballot(!placed)) {
          if (!placed) gh = insert_global(key, y);
        }
        const int idx = wave_append(gh >= 0, &sh_nown);
        if (gh >= 0) S.hown[idx] = (uint32_t)gh;
      };
#pragma unroll
      for (int j = 0; j < WIDE_FLR; ++j) insert(j < fc, fk[j], (double)fv[j]);
      for (int j0 = 0; j0 < nd; j0 += DBLOCK) {
        const int j = j0 + tid;
        insert(j < nd, j < nd ? ld_agent(&S.dkey[j]) : 0u, j < nd ? ld_agent(&S.dval[j]) : 0.0);
      }
      slot_sync();
      for (int i = tid; i < WIDE_LT; i += DBLOCK) {
        const uint32_t key = ltkey[i];
        if (key != WIDE_EMPTY) {
          const double y = ltval[i];
          atomicAdd(&kst[2 * MAXK_DENSE + key / (uint32_t)npx + 1], y * y);
          ltkey[i] = WIDE_EMPTY;
          ltval[i] = 0.0;
        }
      }
      const int no = sh_nown;
      for (int j = tid; j < no; j += DBLOCK) {
        const uint32_t s = S.hown[j];
        const uint32_t key = ld_agent(&S.hkey[s]);
        const double y = ld_agent(&S.hval[s]);
        atomicAdd(&kst[2 * MAXK_DENSE + key / (uint32_t)npx + 1], y * y);
        S.hkey[s] = WIDE_EMPTY;
        S.hval[s] = 0.0;
      }
      __syncthreads();
    }
    if (sh_ctr[3]) {  // an overflow: the pixel-indexed kernel scores this ion
      if (tid == 0) {
        const uint32_t r = atomicAdd(rej_count, 1u);
        if (r < rej_cap) rej_list[r] = (uint32_t)ion;
        nx_publish();
      }
      for (int s = tid; s < npd; s += DBLOCK) {
        pdkey[s] = WIDE_EMPTY;
        pdval[s] = 0.0;
      }
      __syncthreads();
      continue;
    }
    STAMP(12);
    // ---- 3. chaos screen per principal pixel, walked from the bitmap -------------------------------------------
    const double npos = sh_st[3];
    const bool chaos_ok = (sh_st[0] > 0.0) && (npos >= 4.0);
    if (chaos_ok) {
      // uniform call: the candidates on p's 4-cross, each listed by the first principal pixel on its cross (as in
      // ion_wide_kernel), from presence rows r-3 .. r+3
      auto screen_px = [&](bool act, int p) {
#ifdef SMG_STAMPS
        {
          const uint64_t am = __ballot(act);
          if (lane == 0) {
            atomicAdd(&_sacc[0], 1ull);
            atomicAdd(&_sacc[1], (unsigned long long)__popcll(am));
          }
        }
#endif
        uint32_t cm = 0u;
        int r0 = 0, c0 = 0;
#ifdef SMG_WJ_ABL  // diagnostic (timing only, wrong chaos): the walk without the screen itself
        act = act && (SMG_WJ_ABL == 0);
#endif
        if (act) {
          rowcol(p, P, r0, c0);
          uint32_t B[7], IM[7];
          uint32_t imc = 0x7Fu;  // columns c0-3 .. c0+3 inside the image
          if (c0 - 3 < 0) imc &= 0x7Fu << (uint32_t)(3 - c0);
          if (c0 + 3 >= nc) imc &= 0x7Fu >> (uint32_t)(c0 + 3 - (nc - 1));
          int cnt = 0;
          wj_rows7(bm32, r0, c0, nr, nc, B);
#pragma unroll
          for (int k = 0; k < 7; ++k) {
            IM[k] = (r0 + k - 3 >= 0 && r0 + k - 3 < nr) ? imc : 0u;
            cnt += __popc(B[k]);
          }
          // a candidate's 3x3 box is covered by 4-crosses of principal pixels only if >= 3 of them lie in its 5x5
          if (P.erosion_border || cnt >= 3) {
            uint32_t Eh[7];
#pragma unroll
            for (int k = 1; k <= 5; ++k) {
              const uint32_t d = B[k] | (B[k] << 1) | (B[k] >> 1) | B[k - 1] | B[k + 1];
              const uint32_t dm = (P.erosion_border ? (d | ~IM[k]) : (d & IM[k])) & 0x7Fu;
              Eh[k] = dm & (dm << 1) & (dm >> 1);
            }
            auto Ebit = [&](int k, int j) -> uint32_t { return (Eh[k - 1] & Eh[k] & Eh[k + 1] & IM[k]) >> j & 1u; };
            auto prb = [&](int k, int j) -> uint32_t { return (B[k] >> j) & 1u; };
#pragma unroll
            for (int t = 0; t < 5; ++t) {
              const int qr = (t == 1) ? -1 : (t == 2) ? 1 : 0, qc = (t == 3) ? -1 : (t == 4) ? 1 : 0;
              const int wr = qr + 3, wc = qc + 3;
              int orr = 9, occ = 9;  // the first principal pixel among q-nc, q-1, q, q+1, q+nc must be p
              if (prb(wr + 1, wc)) orr = 1, occ = 0;
              if (prb(wr, wc + 1)) orr = 0, occ = 1;
              if (prb(wr, wc)) orr = 0, occ = 0;
              if (prb(wr, wc - 1)) orr = 0, occ = -1;
              if (prb(wr - 1, wc)) orr = -1, occ = 0;
              if (qr + orr == 0 && qc + occ == 0 && Ebit(wr, wc)) cm |= 1u << t;
            }
          }
        }
        const int cnt = __popc(cm);
        const int incl = wave_incl_scan_dpp(cnt);
        int wbase = 0;
        if (lane == 63 && incl > 0) wbase = atomicAdd(&sh_ncand, incl);
        wbase = __shfl(wbase, 63);
        int idx = wbase + incl - cnt;
        while (cm != 0u) {
          const int t = __ffs(cm) - 1;
          const int qr = (t == 1) ? -1 : (t == 2) ? 1 : 0, qc = (t == 3) ? -1 : (t == 4) ? 1 : 0;
          const uint32_t qq = (uint32_t)((r0 + qr) * nc + c0 + qc);
          if (idx < npx) S.epr[idx] = qq;
          ++idx;
          cm &= cm - 1u;
        }
      };
      // pass A of the screen (as in ion_sparse_kernel): a principal pixel with fewer than three principal pixels in its
      // 7x7 (itself included) cannot list a candidate (erosion border 0); the survivors (~6 % at config 5) go to the
      // wave's survivor list, which gets the full screen (screen_px) 64 at a time, so that its ~200 instructions do not
      // run for every list of pixels with a survivor somewhere in it
      int sn = 0;  // survivors listed (uniform)
      auto screen_list = [&](bool act, int p) {
        bool sv = act;
        if (act && !P.erosion_border) {
          int r0, c0;
          rowcol(p, P, r0, c0);
          uint32_t B[7];
          wj_rows7(bm32, r0, c0, nr, nc, B);
          int cnt = 0;
#pragma unroll
          for (int k = 0; k < 7; ++k) cnt += __popc(B[k]);
          sv = cnt >= 3;
        }
        const uint64_t m = __ballot(sv);
        const int c = (int)__popcll(m);
        if (sn + c > WAVE) {
          __builtin_amdgcn_wave_barrier();
          screen_px(lane < sn, lane < sn ? (int)slist[lane] : 0);
          __builtin_amdgcn_wave_barrier();
          sn = 0;
        }
        if (sv) slist[sn + (int)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)p;
        sn += c;
      };
      // each wave takes one word of every DNW (lane j of wave w: word c0 + j * DNW + ((w + j) mod DNW): a permutation
      // within each group, so the lanes' 8-byte reads spread over the LDS banks), so that a blob's rows are spread
      // over all waves; a lane pops its word's bits one per round into the wave's list, which is screened 64 entries
      // (one per lane) at a time.  No barrier: the candidates' stores stay in flight until the slot_sync after the
      // walk.
      int wn = 0;  // listed entries (uniform)
      for (int c0 = 0; c0 < n64; c0 += DBLOCK) {
        const int w = c0 + lane * DNW + ((wid + lane) & (DNW - 1));
        uint64_t bits = w < n64 ? bm[w] : 0ull;
        while (true) {
          const bool has = bits != 0ull;
          const uint64_t m = __ballot(has);
          if (m == 0ull) break;
          if (has) {
            const int b = __ffsll((unsigned long long)bits) - 1;
            bits &= bits - 1ull;
            wlist[wn + (int)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)(w * 64 + b);
          }
          wn += (int)__popcll(m);
          if (wn >= WAVE) {
            __builtin_amdgcn_wave_barrier();
            screen_list(true, (int)wlist[lane]);
            __builtin_amdgcn_wave_barrier();
            wn -= WAVE;
            const uint32_t mv = lane < wn ? wlist[WAVE + lane] : 0u;
            __builtin_amdgcn_wave_barrier();
            if (lane < wn) wlist[lane] = mv;
            __builtin_amdgcn_wave_barrier();
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (wn > 0) screen_list(lane < wn, lane < wn ? (int)wlist[lane] : 0);
      __builtin_amdgcn_wave_barrier();
      if (sn > 0) screen_px(lane < sn, lane < sn ? (int)slist[lane] : 0);
    }
    if (tid == 0) nx_step();
    slot_sync();  // (candidates listed in L2; every bitmap reader done)
    const int nscr = chaos_ok ? min(sh_ncand, npx) : 0;
    STAMP(8);
    // ---- 4. JH over the dead bitmap / rank / LT space: the needed and the hit pixels, x from a second stream ----
    const int nov = min(sh_nov, npx);
    const bool rs = sh_rs != 0;
    const bool anyhit = sh_anyhit != 0 || nov > 0 || rs;
    if (anyhit || nscr > 0) {
      if (jdirect) {
        for (int i = tid; i < npx; i += DBLOCK) jx[i] = 0.0;
      } else {
        for (int i = tid; i < WJ_JH; i += DBLOCK) {
          jkey[i] = WIDE_EMPTY;
          jx[i] = 0.0;  // (pixels of a candidate's neighbourhood without a point keep x = 0)
        }
        __syncthreads();
        if (nev > 0 && wj_insert(jkey, WJ_JH_LOG2, H::pix(ev0)) < 0) sh_ctr[3] = 1;
        if (nev > 1 && wj_insert(jkey, WJ_JH_LOG2, H::pix(ev1)) < 0) sh_ctr[3] = 1;
        for (int j = tid; j < nov; j += DBLOCK)
          if (wj_insert(jkey, WJ_JH_LOG2, H::pix(ld_agent(&ovh[j]))) < 0) sh_ctr[3] = 1;
        // every candidate's 5x5 minus its corners (what its eL reads), in the image (and present, while the bitmap
        // lives: JH after it)
        for (int j = tid; j < nscr * 21; j += DBLOCK) {
          const int i = j / 21, o = j - i * 21;
          const int oo = o + (o >= 18 ? 3 : o >= 3 ? 2 : 1);  // offsets 1..3, 5..19, 21..23 of 0..24
          const int dr = oo / 5 - 2, dc = oo % 5 - 2;
          int r0, c0;
          rowcol((int)cand(i), P, r0, c0);
          const int rr = r0 + dr, cc = c0 + dc;
          if (rr >= 0 && rr < nr && cc >= 0 && cc < nc && (!jafter || pres.test((uint32_t)(rr * nc + cc))) &&
              wj_insert(jkey, WJ_JH_LOG2, (uint32_t)(rr * nc + cc)) < 0)
            sh_ctr[3] = 1;
        }
      }
      __syncthreads();
      for (int64_t i0 = a0; i0 < b0; i0 += (int64_t)DBLOCK * WDU) {
        uint64_t r[WDU];
#pragma unroll
        for (int u = 0; u < WDU; ++u) {
          const int64_t i = i0 + (int64_t)u * DBLOCK + tid;
          r[u] = hits.load(i < b0 ? i : b0 - 1);
        }
        // every point's first probe read together (one wait), then the rare collisions probed on
        uint32_t h0[WDU], k0[WDU];
#pragma unroll
        for (int u = 0; u < WDU; ++u) {
          h0[u] = jdirect ? H::pix(r[u]) : wj_hash(H::pix(r[u]), WJ_JH_LOG2);
          k0[u] = jdirect ? 0u : jkey[h0[u]];
        }
#pragma unroll
        for (int u = 0; u < WDU; ++u) {
          const int64_t i = i0 + (int64_t)u * DBLOCK + tid;
          if (i < b0) {
            const uint32_t p = H::pix(r[u]);
            const int s = jdirect ? (int)p : wj_find_from(jkey, WJ_JH_LOG2, p, h0[u], k0[u]);
            if (s >= 0) {
              double x = H::val(r[u]);
              if (H::dup(r[u])) {
                const int t = wj_find(pdkey, pd_log2, p);
                x = t >= 0 ? pdval[t] : 0.0;
              }
              jx[s] = x;  // (every point of a pixel stores the same value)
            }
          }
        }
      }
      __syncthreads();
      STAMP(11);
      // ---- 5a. the hits' Σxy and Σy[x>0] -----------------------------------------------------------------------
      auto hit = [&](uint64_t h, int kb) {
        const int s = jslot(H::pix(h));
        const double xv = s >= 0 ? jx[s] : 0.0;
        const double y = H::val(h);
        atomicAdd(&kst[3 * MAXK_DENSE + kb + 1], xv * y);
        if (xv > 0.0) atomicAdd(&kst[0 * MAXK_DENSE + kb + 1], y);
      };
      if (!rs) {
        if (nev > 0) hit(ev0, evk0);
        if (nev > 1) hit(ev1, evk1);
        for (int j = tid; j < nov; j += DBLOCK) hit(ld_agent(&ovh[j]), (int)S.L[j]);
      } else {  // more hits than pixels (x by pixel, absent pixels 0): every tail point again, none listed
        int kb = 0;
        for (int64_t v0 = 0; v0 < T; v0 += TSTEP) {
          while (v0 >= sh_tb[kb + 1]) ++kb;
          kb = __builtin_amdgcn_readfirstlane(kb);
          const int64_t off = v0 - sh_tb[kb], n = sh_tn[kb], a = sh_tlo[kb];
          uint64_t r[TDU];
#pragma unroll
          for (int u = 0; u < TDU; ++u) {
            const int64_t lv = off + (int64_t)u * DBLOCK + tid;
            r[u] = hb[a + (lv < n ? lv : n - 1)];
          }
#pragma unroll
          for (int u = 0; u < TDU; ++u)
            if (off + (int64_t)u * DBLOCK + tid < n && H::pix(r[u]) < (uint32_t)npx && jx[H::pix(r[u])] != 0.0)
              hit(r[u], kb);
        }
      }
    }
    STAMP(13);
    // ---- 5b. eL of every screened candidate from its 5x5's levels (absent pixels: level 0), then Kruskal --------
    // Up to WJ_LK candidates keep their arrays in the LDS: eL in discovery order over PD's space (dead after the join
    // stream), the arrays by rank over the LT space (JH is dead by then), union-find with LDS atomics; more go to
    // the slot.  Kruskal visits only the levels some candidate has (sh_lvm).
    double chaos_raw = NAN;
    if (chaos_ok && !sh_ctr[3]) {
      const double vmax = sh_st[4], rcp = 1.0 / vmax;  // (x <= vmax: sp_level's domain)
      const bool lk = nscr <= WJ_LK;
      uint32_t* lepix = pdkey;  // (PD: >= WJ_LK * 12 B)
      uint8_t* leL = reinterpret_cast<uint8_t*>(pdkey + WJ_LK);
      uint32_t* lepr = ltkey;   // (LT: 12 KB)
      uint32_t* lpar = ltkey + WJ_LK;
      uint8_t* leLr = reinterpret_cast<uint8_t*>(ltkey + 2 * WJ_LK);
      for (int i0 = 0; i0 < nscr; i0 += DBLOCK) {
        const int i = i0 + tid;
        const int q = (i < nscr) ? (int)cand(i) : -1;
        int e = 0;
        if (q >= 0) {
          int r0, c0;
          rowcol(q, P, r0, c0);
          // the levels of q's 5x5 minus corners (0 outside the image or absent): the 21 first probes read together,
          // then the rare collisions probed on, then the 21 values read together
          int Lv[5][5];
          uint32_t pk[5][5], ph[5][5], pv[5][5];
          int ps[5][5];
#pragma unroll
          for (int a = 0; a < 5; ++a)
#pragma unroll
            for (int b = 0; b < 5; ++b) {
              const int rr = r0 + a - 2, cc = c0 + b - 2;
              const bool in = rr >= 0 && rr < nr && cc >= 0 && cc < nc && !((a == 0 || a == 4) && (b == 0 || b == 4));
              pk[a][b] = in ? (uint32_t)(rr * nc + cc) : WIDE_EMPTY;
              ph[a][b] = jdirect ? (in ? pk[a][b] : 0u) : wj_hash(pk[a][b], WJ_JH_LOG2);
              pv[a][b] = jdirect ? 0u : jkey[ph[a][b]];
            }
#pragma unroll
          for (int a = 0; a < 5; ++a)
#pragma unroll
            for (int b = 0; b < 5; ++b)
              ps[a][b] = pk[a][b] == WIDE_EMPTY ? -1 : jdirect ? (int)ph[a][b] :
                         wj_find_from(jkey, WJ_JH_LOG2, pk[a][b], ph[a][b], pv[a][b]);
          double xv[5][5];
#pragma unroll
          for (int a = 0; a < 5; ++a)
#pragma unroll
            for (int b = 0; b < 5; ++b) xv[a][b] = ps[a][b] >= 0 ? jx[ps[a][b]] : 0.0;
#pragma unroll
          for (int a = 0; a < 5; ++a)
#pragma unroll
            for (int b = 0; b < 5; ++b) Lv[a][b] = ps[a][b] >= 0 ? sp_level(xv[a][b], vmax, rcp, P) : 0;
          e = 1 << 20;
#pragma unroll
          for (int a = -1; a <= 1; ++a)
#pragma unroll
            for (int b = -1; b <= 1; ++b) {
              const int rr = r0 + a, cc = c0 + b;
              if (rr < 0 || rr >= nr || cc < 0 || cc >= nc) {
                if (!P.erosion_border) e = 0;
                continue;
              }
              const int A = a + 2, Bc = b + 2;
              const int t = max(max(Lv[A][Bc], Lv[A - 1][Bc]), max(max(Lv[A + 1][Bc], Lv[A][Bc - 1]), Lv[A][Bc + 1]));
              e = min(e, t);
            }
          if (e >= (1 << 20)) e = 0;
        }
        const int idx = wave_append(e >= 1, &sh_ctr[0]);
        if (e >= 1) {
          if (lk) {
            lepix[idx] = (uint32_t)q;
            leL[idx] = (uint8_t)e;
          } else {
            S.epix[idx] = (uint32_t)q;
            S.eL[idx] = (uint8_t)e;
          }
          atomicOr(&sh_lvm[(e >> 5) & 7], 1u << (e & 31));
        }
      }
      if (lk) __syncthreads();
      else slot_sync();
      STAMP(14);
      const int m = sh_ctr[0];
      double esum = 0.0, wsum = 0.0;
      for (int i = tid; i < m; i += DBLOCK) esum += (double)(lk ? leL[i] : S.eL[i]);
      if (m > 0 && lk && m <= WAVE) {
        // up to 64 candidates: wave 0 alone, one candidate per lane, its forward neighbours found in a 128-slot
        // pixel hash over the LT space (JH is dead), the levels in sequence without a block barrier
        if (wid == 0) {
          uint32_t* hk = ltkey;           // 128 keys
          uint32_t* hv = ltkey + 2 * WAVE;  // their candidate indices
          uint32_t* lp = ltkey + 4 * WAVE;  // union-find parents
          hk[lane] = WIDE_EMPTY;
          hk[lane + WAVE] = WIDE_EMPTY;
          __builtin_amdgcn_wave_barrier();
          const bool mine = lane < m;
          const uint32_t q = mine ? lepix[lane] : 0u;
          const int e = mine ? (int)leL[lane] : 0;
          if (mine) {
            const int h = wj_insert(hk, 7, q);
            hv[h] = (uint32_t)lane;  // (distinct candidates: the table has room for all)
            lp[lane] = (uint32_t)lane;
          }
          __builtin_amdgcn_wave_barrier();
          const int r = mine ? (int)q / nc : 0, c = mine ? (int)q - r * nc : 0;
          auto nbr = [&](bool ok, int qq) -> int {  // candidate index of pixel qq, -1 if none
            if (!ok) return -1;
            const int h = wj_find(hk, 7, (uint32_t)qq);
            return h >= 0 ? (int)hv[h] : -1;
          };
          // the forward neighbours (right, down, and with 8-connectivity down-left, down-right), found once
          const int n0 = nbr(mine && c + 1 < nc, (int)q + 1);
          const int n1 = nbr(mine && r + 1 < nr, (int)q + nc);
          const int n2 = nbr(mine && P.connectivity == 8 && r + 1 < nr && c > 0, (int)q + nc - 1);
          const int n3 = nbr(mine && P.connectivity == 8 && r + 1 < nr && c + 1 < nc, (int)q + nc + 1);
          const int e0 = n0 >= 0 ? (int)leL[n0] : 0, e1 = n1 >= 0 ? (int)leL[n1] : 0;
          const int e2 = n2 >= 0 ? (int)leL[n2] : 0, e3 = n3 >= 0 ? (int)leL[n3] : 0;
          uint32_t lvm[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) lvm[j] = sh_lvm[j];
          for (int t = 255; t >= 1; --t) {  // (uniform: the levels some candidate has, from the highest)
            const int wj = t >> 5;
            const uint32_t word = wj == 7 ? lvm[7] : wj == 6 ? lvm[6] : wj == 5 ? lvm[5] : wj == 4 ? lvm[4] :
                                  wj == 3 ? lvm[3] : wj == 2 ? lvm[2] : wj == 1 ? lvm[1] : lvm[0];
            const uint32_t below = word & ((2u << (t & 31)) - 1u);
            if (below == 0u) {
              t = wj * 32;
              continue;
            }
            t = wj * 32 + 31 - __clz(below);
            if (t < 1) break;
            if (mine && e >= t) {
              if (n0 >= 0 && min(e, e0) == t && luf_unite(lp, (uint32_t)lane, (uint32_t)n0)) wsum += (double)t;
              if (n1 >= 0 && min(e, e1) == t && luf_unite(lp, (uint32_t)lane, (uint32_t)n1)) wsum += (double)t;
              if (n2 >= 0 && min(e, e2) == t && luf_unite(lp, (uint32_t)lane, (uint32_t)n2)) wsum += (double)t;
              if (n3 >= 0 && min(e, e3) == t && luf_unite(lp, (uint32_t)lane, (uint32_t)n3)) wsum += (double)t;
            }
            __builtin_amdgcn_wave_barrier();
          }
        }
      } else if (m > 0) {  // Kruskal over the candidates, indexed by their rank in a candidate bitmap (ion_wide_kernel's)
        for (int w = tid; w < n64p; w += DBLOCK) bm[w] = 0ull;
        __syncthreads();
        for (int i = tid; i < m; i += DBLOCK) {
          const uint32_t q = lk ? lepix[i] : S.epix[i];
          atomicOr(&bm32[q >> 5], 1u << (q & 31));
        }
        __syncthreads();
        build_rank(bm, pf, sb, n64, sc);
        for (int i = tid; i < m; i += DBLOCK) {
          const uint32_t q = lk ? lepix[i] : S.epix[i];
          const uint32_t k = R.rank(q);
          if (lk) {
            lepr[k] = q;
            leLr[k] = leL[i];
            lpar[k] = k;
          } else {
            S.epr[k] = q;
            S.eLr[k] = S.eL[i];
            S.par[k] = k;
          }
        }
        if (lk) __syncthreads();
        else slot_sync();
        uint32_t lvm[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) lvm[j] = sh_lvm[j];
        for (int t = 255; t >= 1; --t) {  // (uniform: the levels some candidate has, from the highest)
          const int wj = t >> 5;
          const uint32_t word = wj == 7 ? lvm[7] : wj == 6 ? lvm[6] : wj == 5 ? lvm[5] : wj == 4 ? lvm[4] :
                                wj == 3 ? lvm[3] : wj == 2 ? lvm[2] : wj == 1 ? lvm[1] : lvm[0];
          const uint32_t below = word & ((2u << (t & 31)) - 1u);  // levels <= t in this word (bit 31: 2u << 31 = 0 -> ~0)
          if (below == 0u) {  // none at or below t in this word: jump to the word's start
            t = wj * 32;
            continue;
          }
          t = wj * 32 + 31 - __clz(below);  // the highest present level <= t
          if (t < 1) break;
          for (int i = tid; i < m; i += DBLOCK) {
            const int e = lk ? leLr[i] : S.eLr[i];
            if (e < t) continue;
            const int p = (int)(lk ? lepr[i] : S.epr[i]);
            const int r = p / nc, c = p - r * nc;
            auto edge = [&](int q) {
              if (!R.test((uint32_t)q)) return;
              const uint32_t kq = R.rank((uint32_t)q);
              const int eq = lk ? leLr[kq] : S.eLr[kq];
              if ((e < eq ? e : eq) == t && (lk ? luf_unite(lpar, (uint32_t)i, kq) : guf_unite(S.par, (uint32_t)i, kq)))
                wsum += (double)t;
            };
            if (c + 1 < nc) edge(p + 1);
            if (r + 1 < nr) {
              edge(p + nc);
              if (P.connectivity == 8) {
                if (c > 0) edge(p + nc - 1);
                if (c + 1 < nc) edge(p + nc + 1);
              }
            }
          }
          __syncthreads();
        }
      }
      double a3[2] = {esum, wsum};
      dblock_sum<2>(a3, red);
      chaos_raw = 1.0 - (a3[0] - a3[1]) / (double)P.nlevels / npos;
    } else if (!chaos_ok) {
      flags |= SMG_ION_CHAOS_NAN;
    }
    STAMP(9);
    __syncthreads();  // (the hits' kst sums; every JH and LT-space reader done)
    const bool over = sh_ctr[3] != 0;
    // the LT space (work lists, JH) and PD back to empty for the next ion
    for (int i = tid; i < WIDE_LT; i += DBLOCK) {
      ltkey[i] = WIDE_EMPTY;
      ltval[i] = 0.0;
    }
    for (int s = tid; s < npd; s += DBLOCK) {
      pdkey[s] = WIDE_EMPTY;
      pdval[s] = 0.0;
    }
    bool hh = b0 > a0;
    for (int j = 0; j < K - 1; ++j) hh = hh || sh_tn[j] > 0;
    if (hh) flags |= SMG_ION_HAS_HITS;
    if (tid == 0) {
      nx_publish();
      if (over) {  // JH or a list overflowed after the tail: the pixel-indexed kernel scores this ion
        const uint32_t r = atomicAdd(rej_count, 1u);
        if (r < rej_cap) rej_list[r] = (uint32_t)ion;
      } else {
        kst[0] = sh_st[2];
        kst[1 * MAXK_DENSE] = kst[2 * MAXK_DENSE] = kst[3 * MAXK_DENSE] = 0.0;
        finalize_ion(K, sh_th, kst, sh_st[0], sh_st[1], kst + MAXK_DENSE, kst + 2 * MAXK_DENSE,
                     kst + 3 * MAXK_DENSE, (double)npx, chaos_raw, ion, flags, oc, osp, osc, omsm, oflags);
      }
    }
    __syncthreads();
  }
  STAMP_FLUSH();
}

__global__ void list_all_kernel(uint32_t* list, uint32_t* count, const int64_t* ion_order, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) list[i] = (uint32_t)(ion_order ? ion_order[i] : i);
  if (i == 0) *count = (uint32_t)n;
}

#ifndef SMG_DENSE_SLOTS
#define SMG_DENSE_SLOTS 256
#endif
static constexpr int DENSE_SLOTS = SMG_DENSE_SLOTS;  // dense-path workgroups (one scratch slot each)
static constexpr size_t DENSE_BM_LDS_MAX = 152 * 1024;  // dense kernel: LDS presence bitmap up to this size
static constexpr size_t WIDE_LDS_MAX = 160 * 1024 - 4096;  // wide pass: dynamic LDS (static arrays ~2.9 KB)
static constexpr size_t WIDE_LDS_MAX_CLIP = 160 * 1024 - 8192;  // its CLIP instantiation (static arrays ~7.7 KB)
// workspace: header (pass counters at word 0.., per-XCD range counters at word 64..), two ion lists,
// the ion descriptors, dense scratch slots
static constexpr size_t WS_HEADER = 2048;
static constexpr int HDR_XCD = 64;
// LDS-path geometries: the main pass (two 512-thread workgroups per CU) and the big-ion pass over its
// rejects (one 1024-thread workgroup per CU with the whole LDS)
#ifndef SMG_MAIN_CFG
#define SMG_MAIN_CFG 512, 5, 2, 4
#endif
// main LDS pass: threads, principal points per thread, chunk points per thread, min waves per SIMD
static constexpr int MAIN_CFG[4] = {SMG_MAIN_CFG};
static constexpr int MAIN_BLOCK = MAIN_CFG[0], MAIN_RMAX = MAIN_CFG[1], MAIN_RC = MAIN_CFG[2],
                     MAIN_WPE = MAIN_CFG[3];
static constexpr int BIG_BLOCK = 1024, BIG_RMAX = 8, BIG_RC = 2;
#ifndef SMG_MAIN_WGPCU
#define SMG_MAIN_WGPCU 2
#endif
static constexpr int MAIN_WGPCU = SMG_MAIN_WGPCU;  // main pass: resident workgroups per CU
static constexpr size_t MAIN_LDS = (160 * 1024) / MAIN_WGPCU, BIG_LDS = 160 * 1024 - 512;

// the wide pass and the pixel-indexed kernel run one after the other over the same slots
static size_t slot_bytes_for(int npx) {
  const size_t a = dense_slot_bytes(npx), b = wide_slot_bytes(npx);
  return a > b ? a : b;
}

// SMG_CHECK builds: two claimed-bit sets (main pass, big-ion pass) behind the slots, zeroed per launch
static size_t chk_words(int64_t n_ions) { return (size_t)((n_ions + 31) / 32 + 1); }
static size_t chk_bytes(int64_t n_ions) {
#ifdef SMG_CHECK
  return al16(2 * chk_words(n_ions) * 4);
#else
  (void)n_ions;
  return 0;
#endif
}

static size_t ws_bytes_for(int64_t n_ions, int npx) {
  return WS_HEADER + 2 * al16((size_t)n_ions * 4) + (size_t)n_ions * sizeof(IonDesc) +
         (size_t)DENSE_SLOTS * slot_bytes_for(npx) + chk_bytes(n_ions);
}

// SMG_CHECK: the counters (persistent device buffer) and the hit count the checks index against
#ifdef SMG_CHECK
static unsigned long long* g_chk_cnt = nullptr;
#endif
static int64_t g_chk_points = INT64_MAX;

using MainLay = Lay<MAIN_BLOCK / WAVE, MAIN_BLOCK * MAIN_RMAX>;
using BigLay = Lay<BIG_BLOCK / WAVE, BIG_BLOCK * BIG_RMAX>;
// two-level passes: the big-ion pass takes principal windows of up to 4096 points (W needs 8 B per point)
static constexpr int BIG2_RMAX = 4;
using Main2Lay = Lay2<MAIN_BLOCK / WAVE, MAIN_BLOCK * MAIN_RMAX>;
using Big2Lay = Lay2<BIG_BLOCK / WAVE, BIG_BLOCK * BIG2_RMAX>;
static int g_main_kernel = 1;      // smg_debug_main_kernel: 1 the sparse main pass where it applies, 0 ion_pipe_kernel
static int g_force_two_level = 0;  // smg_debug_force_two_level: two-level passes for every image size
static int g_force_dense = 0;      // smg_debug_force_dense: 1 every ion on the dense path, 2 pixel-indexed only
static int g_wide_impl = 1;        // smg_debug_wide_impl: 1 ion_wide_join_kernel where it applies, 0 ion_wide_kernel
// smg_debug_time_main_pass: HIP events recorded on the launch stream around every pass launch of
// smg_ion_metrics (descriptors, main LDS pass, big-ion pass, wide pass, pixel-indexed pass), so a benchmark
// measures each kernel itself and prices each pass's own window points against its own time
static int g_time_main = 0;
static std::mutex g_ev_mu;
struct PassEvents {
  int pass;
  hipEvent_t ev0, ev1;
};
static std::vector<PassEvents> g_pass_events;
// drained events are kept for reuse: after the first timed searches no event is created (a creation can reach the
// device while a persistent pass runs)
static std::vector<hipEvent_t> g_ev_pool;
static hipEvent_t ev_take() {
  {
    std::lock_guard<std::mutex> g(g_ev_mu);
    if (!g_ev_pool.empty()) {
      hipEvent_t e = g_ev_pool.back();
      g_ev_pool.pop_back();
      return e;
    }
  }
  hipEvent_t e = nullptr;
  return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}
static void ev_give(hipEvent_t e) {  // caller holds g_ev_mu
  if (!e) return;
  if (g_ev_pool.size() < 4096) g_ev_pool.push_back(e);
  else (void)hipEventDestroy(e);
}

// opens a timed region for one pass launch on `st` (no-op unless smg_debug_time_main_pass is on)
struct PassTimer {
  int pass;
  hipStream_t st;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  PassTimer(int p, hipStream_t s) : pass(p), st(s) {
    if (!g_time_main) return;
    ev0 = ev_take();
    if (!ev0) return;
    ev1 = ev_take();
    if (!ev1 || hipEventRecord(ev0, st) != hipSuccess) release();
  }
  ~PassTimer() {
    if (!ev0) return;
    if (hipEventRecord(ev1, st) != hipSuccess) {
      release();
      return;
    }
    std::lock_guard<std::mutex> g(g_ev_mu);
    if (g_pass_events.size() >= kMaxPassEvents) {  // nobody drains them: drop the oldest record
      (void)hipEventDestroy(g_pass_events.front().ev0);
      (void)hipEventDestroy(g_pass_events.front().ev1);
      g_pass_events.erase(g_pass_events.begin());
    }
    g_pass_events.push_back({pass, ev0, ev1});
  }
  void release() {  // returns whatever was taken; no record is kept
    std::lock_guard<std::mutex> g(g_ev_mu);
    ev_give(ev0);
    ev_give(ev1);
    ev0 = ev1 = nullptr;
  }
  static constexpr size_t kMaxPassEvents = 16384;
};

static int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || cus <= 0)
    cus = 256;
  return cus;
}

template <int FMT>
static int launch_metrics(Hits<FMT> hits, const double* hit_cum, const int64_t* lo, const int64_t* hi,
                          const int64_t* ion_off,
                          const double* theor, const int64_t* ion_order, int64_t n_ions, const Params& P,
                          double* oc, double* osp, double* osc, double* omsm, uint32_t* oflags,
                          unsigned char* ws, hipStream_t st) {
  // header words: [0] count A, [1] cursor A, [2] count B, [3] cursor B, [4] count / [5] cursor of the wide
  // pass's rejects (list A again), [HDR_XCD + x*CTR_STRIDE] range x
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ws);
  uint32_t* list_a = reinterpret_cast<uint32_t*>(ws + WS_HEADER);
  uint32_t* list_b = reinterpret_cast<uint32_t*>(ws + WS_HEADER + al16((size_t)n_ions * 4));
  IonDesc* desc = reinterpret_cast<IonDesc*>(ws + WS_HEADER + 2 * al16((size_t)n_ions * 4));
  unsigned char* slots = reinterpret_cast<unsigned char*>(desc) + (size_t)n_ions * sizeof(IonDesc);
  const size_t slot_bytes = slot_bytes_for(P.npx);
  SMG_HIP(hipMemsetAsync(ws, 0, WS_HEADER, st));
  ChkCtx ck{lo, hi, ion_off, ion_order, nullptr, (int64_t)chk_words(n_ions), g_chk_points, nullptr};
#ifdef SMG_CHECK
  if (!g_chk_cnt) {
    SMG_HIP(hipMalloc(&g_chk_cnt, CHK_N * sizeof(unsigned long long)));
    SMG_HIP(hipMemset(g_chk_cnt, 0, CHK_N * sizeof(unsigned long long)));
  }
  ck.cnt = g_chk_cnt;
  ck.claim = reinterpret_cast<uint32_t*>(slots + (size_t)DENSE_SLOTS * slot_bytes);
  SMG_HIP(hipMemsetAsync(ck.claim, 0, chk_bytes(n_ions), st));
#endif
  // images above NPX_LDS_MAX pixels (or forced, smg_debug_force_two_level) take the two-level LDS passes
  const bool two = (P.npx > NPX_LDS_MAX || g_force_two_level) && P.npx <= NPX_TWO_MAX;
  Params PM = P, PB = P;
  PM.w32 = two ? Main2Lay::w32(P.npx) : MainLay::w32(P.npx);
  PM.o_pf = two ? Main2Lay::o_pf(P.npx) : MainLay::o_pf(P.npx);
  PB.w32 = two ? Big2Lay::w32(P.npx) : BigLay::w32(P.npx);
  PB.o_pf = two ? Big2Lay::o_pf(P.npx) : BigLay::o_pf(P.npx);
  size_t lds_main = two ? Main2Lay::bytes(P.npx) : MainLay::bytes(P.npx);
#ifdef SMG_MAIN_LDS_MIN  // diagnostic: reserve at least this much LDS per main-pass workgroup (fewer per CU)
  if (lds_main < (size_t)SMG_MAIN_LDS_MIN) lds_main = SMG_MAIN_LDS_MIN;
#endif
  const size_t lds_big = two ? Big2Lay::bytes(P.npx) : BigLay::bytes(P.npx);
  // the hot-spot clip (do_preprocessing) clips every image before its sums: the LDS passes and the wide pass have
  // CLIP instantiations (ion_pipe_kernel<..., CLIP>, ion_wide_kernel<FMT, true>), the pixel-indexed kernel clips
  // its images in place.  Images above NPX_LDS_MAX pixels go to
  // the rank-indexed wide pass when its LDS bitmap fits: it outruns the two-level LDS passes on them (config-5
  // rank shard: the big two-level pass scored 3,958 ions in 18.4 ms, the wide pass 586k in 255 ms, and the main
  // two-level pass spent 6.7 ms rejecting every ion, profiles/round3/r3c5_*); smg_debug_force_two_level keeps
  // the two-level passes for the parity suite
  const size_t wide_max = P.clip ? WIDE_LDS_MAX_CLIP : WIDE_LDS_MAX;
  // (build_rank ranks at most DNW * 1024 bitmap words: images up to 2^20 pixels)
  const bool wide_fits = g_force_dense != 2 && wide_lds_bytes(P.npx) <= wide_max &&
                         ((int64_t)P.npx + 63) / 64 <= (int64_t)DNW * 1024;
  const bool lds_ok = two ? (!wide_fits || g_force_two_level) : P.npx <= NPX_LDS_MAX;
  // the main pass: ion_sparse_kernel (four 256-thread workgroups per CU, a sparse principal set) where it applies,
  // else ion_pipe_kernel<512>; either hands its rejects (positions) to the big-ion pass
  const bool sparse = FMT == SMG_HITS_PACKED_F32 && g_main_kernel == 1 && !g_force_dense && !two &&
                      sparse_main_fits(P);
  const bool main_ok = !g_force_dense && lds_ok && (sparse || lds_main <= MAIN_LDS);
  const bool big_ok = !g_force_dense && lds_ok && lds_big <= BIG_LDS;
  const int cus = device_cus();
  if (main_ok || big_ok) {
#ifndef SMG_DESC8
#define SMG_DESC8 1
#endif
    PassTimer tm(SMG_PASS_DESC, st);
    if (SMG_DESC8)
      hipLaunchKernelGGL(ion_desc8_kernel<FMT>, dim3((unsigned)((n_ions * 8 + 255) / 256)), dim3(256), 0, st, hits,
                         lo, hi, ion_off, theor, reinterpret_cast<const DD4*>(hit_cum), ion_order, n_ions, desc);
    else
      hipLaunchKernelGGL(ion_desc_kernel<FMT>, dim3((unsigned)((n_ions + 255) / 256)), dim3(256), 0, st, hits, lo,
                         hi, ion_off, theor, reinterpret_cast<const DD4*>(hit_cum), ion_order, n_ions, desc);
    SMG_LAUNCH_CHECK();
  }
  if (main_ok && sparse) {
    Sched SA{n_ions, hdr + HDR_XCD, nullptr, nullptr, (uint32_t)n_ions};
    PassTimer tm(SMG_PASS_MAIN, st);
    if constexpr (FMT == SMG_HITS_PACKED_F32) {
      const int rc = launch_sparse_main(hits, desc, SA, P, oc, osp, osc, omsm, oflags, list_a, hdr + 0, cus, st, ck);
      if (rc != SMG_OK) return rc;
    }
  } else if (main_ok) {
    Sched SA{n_ions, hdr + HDR_XCD, nullptr, nullptr, (uint32_t)n_ions};
    auto k1 =P.clip ? (two ? &ion_pipe_kernel<FMT, MAIN_BLOCK, MAIN_RMAX, MAIN_RC, MAIN_WPE, SRC_RANGES, true, true>
                            : &ion_pipe_kernel<FMT, MAIN_BLOCK, MAIN_RMAX, MAIN_RC, MAIN_WPE, SRC_RANGES, false, true>)
                     : (two ? &ion_pipe_kernel<FMT, MAIN_BLOCK, MAIN_RMAX, MAIN_RC, MAIN_WPE, SRC_RANGES, true>
                            : &ion_pipe_kernel<FMT, MAIN_BLOCK, MAIN_RMAX, MAIN_RC, MAIN_WPE, SRC_RANGES, false>);
    SMG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k1), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_main));
    // MAIN_WGPCU resident workgroups per CU, a multiple of the XCD count
    int64_t nwg = (int64_t)cus * MAIN_WGPCU;
    if (nwg > n_ions) nwg = ((n_ions + XCDS - 1) / XCDS) * XCDS;
    PassTimer tm(SMG_PASS_MAIN, st);
    hipLaunchKernelGGL(k1, dim3((unsigned)nwg), dim3(MAIN_BLOCK), lds_main, st, hits, desc, SA, PM, oc, osp, osc,
                       omsm, oflags, list_a, hdr + 0 SMG_CHK_ARG(ck));
    SMG_LAUNCH_CHECK();
  } else if (big_ok) {
    hipLaunchKernelGGL(list_positions_kernel, dim3((unsigned)((n_ions + 255) / 256)), dim3(256), 0, st, list_a,
                       hdr + 0, n_ions);
    SMG_LAUNCH_CHECK();
  }
  if (big_ok) {
    Sched SB{0, hdr + 1, list_a, hdr + 0, (uint32_t)n_ions};
    auto k2 = P.clip ? (two ? &ion_pipe_kernel<FMT, BIG_BLOCK, BIG2_RMAX, BIG_RC, 1, SRC_LIST, true, true>
                            : &ion_pipe_kernel<FMT, BIG_BLOCK, BIG_RMAX, BIG_RC, 1, SRC_LIST, false, true>)
                     : (two ? &ion_pipe_kernel<FMT, BIG_BLOCK, BIG2_RMAX, BIG_RC, 1, SRC_LIST, true>
                            : &ion_pipe_kernel<FMT, BIG_BLOCK, BIG_RMAX, BIG_RC, 1, SRC_LIST, false>);
    SMG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k2), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_big));
    const int nwg2 = (int)(n_ions < cus ? n_ions : cus);
    PassTimer tm(SMG_PASS_BIG, st);
    hipLaunchKernelGGL(k2, dim3((unsigned)nwg2), dim3(BIG_BLOCK), lds_big, st, hits, desc, SB, PB, oc, osp, osc,
                       omsm, oflags, list_b, hdr + 2 SMG_CHK_ARG(ck));
    SMG_LAUNCH_CHECK();
  } else if (main_ok) {
    hipLaunchKernelGGL(pos_to_ion_kernel, dim3(64), dim3(256), 0, st, desc, list_a, hdr + 0, list_b, hdr + 2);
    SMG_LAUNCH_CHECK();
  } else {
    hipLaunchKernelGGL(list_all_kernel, dim3((unsigned)((n_ions + 255) / 256)), dim3(256), 0, st, list_b, hdr + 2,
                       ion_order, n_ions);
    SMG_LAUNCH_CHECK();
  }
  if (main_ok || big_ok) {  // the scores of every position the LDS passes scored
    PassTimer tm(SMG_PASS_FINALIZE, st);
    hipLaunchKernelGGL(ion_finalize_kernel, dim3((unsigned)((n_ions * 8 + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<const IonRec*>(desc), n_ions, (double)P.npx, oc, osp, osc, omsm, oflags);
    SMG_LAUNCH_CHECK();
  }
  const int nslots = (int)(n_ions < DENSE_SLOTS ? n_ions : DENSE_SLOTS);
  // dense path: the rank-indexed wide pass where the image's bitmap + rank prefix fit the LDS (with the clip: its
  // CLIP instantiation); the pixel-indexed kernel takes its rejects (or everything)
  const uint32_t* dlist = list_b;
  uint32_t* dcount = hdr + 2;
  uint32_t* dnext = hdr + 3;
  const size_t wide_lds = wide_lds_bytes(P.npx);
  // packed hits without the clip: the join variant (no per-pixel arrays in the slot) where its LDS fits
  const bool wide_join = FMT == SMG_HITS_PACKED_F32 && !P.clip && g_wide_impl == 1 && wide_join_fits(P.npx);
  if (wide_fits && wide_join) {
    if constexpr (FMT == SMG_HITS_PACKED_F32) {
      const size_t jl = WJ_LDS;
      SMG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&ion_wide_join_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)jl));
      PassTimer tm(SMG_PASS_WIDE, st);
      hipLaunchKernelGGL(ion_wide_join_kernel, dim3((unsigned)nslots), dim3(DBLOCK), jl, st, hits,
                         reinterpret_cast<const DD4*>(hit_cum), lo, hi, ion_off, theor, P, list_b, hdr + 2, hdr + 3,
                         list_a, hdr + 4, (uint32_t)n_ions, slots, slot_bytes, oc, osp, osc, omsm, oflags);
      SMG_LAUNCH_CHECK();
    }
    dlist = list_a;
    dcount = hdr + 4;
    dnext = hdr + 5;
  } else if (wide_fits) {
    auto kw = P.clip ? &ion_wide_kernel<FMT, true> : &ion_wide_kernel<FMT, false>;
    SMG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kw), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)wide_lds));
    PassTimer tm(SMG_PASS_WIDE, st);
    hipLaunchKernelGGL(kw, dim3((unsigned)nslots), dim3(DBLOCK), wide_lds, st, hits,
                       reinterpret_cast<const DD4*>(hit_cum), lo, hi, ion_off,
                       theor, P, list_b, hdr + 2, hdr + 3, list_a, hdr + 4, slots, slot_bytes, oc, osp, osc, omsm,
                       oflags);
    SMG_LAUNCH_CHECK();
    dlist = list_a;
    dcount = hdr + 4;
    dnext = hdr + 5;
  }
  // the principal presence bitmap lives in the LDS when it fits (images up to ~1.2M pixels)
  const size_t bm_bytes = (((size_t)P.npx + 31) / 32 + 1) * 4;
  PassTimer tm(SMG_PASS_DENSE, st);
  if (bm_bytes <= DENSE_BM_LDS_MAX) {
    SMG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&ion_dense_kernel<FMT, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)bm_bytes));
    hipLaunchKernelGGL((ion_dense_kernel<FMT, true>), dim3((unsigned)nslots), dim3(DBLOCK), bm_bytes, st, hits, lo,
                       hi, ion_off, theor, n_ions, P, dlist, dcount, dnext, slots, slot_bytes, oc, osp, osc, omsm,
                       oflags);
  } else {
    hipLaunchKernelGGL((ion_dense_kernel<FMT, false>), dim3((unsigned)nslots), dim3(DBLOCK), 0, st, hits, lo, hi,
                       ion_off, theor, n_ions, P, dlist, dcount, dnext, slots, slot_bytes, oc, osp, osc, omsm,
                       oflags);
  }
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}


}  // namespace smg

using namespace smg;

extern "C" {

int smg_debug_stamps(unsigned long long* host_out, int n) {
#ifdef SMG_STAMPS
  SMG_HIP(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * (n < 16 ? n : 16)));
  unsigned long long z[16] = {0};
  SMG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)));
  return SMG_OK;
#else
  (void)host_out;
  (void)n;
  set_error("library built without -DSMG_STAMPS");
  return SMG_ERR_UNSUPPORTED;
#endif
}

#ifdef SMG_WIDE_CHECK
// diagnostic build only: the wide pass's index checks (first code, its value, failures, ions seen); resets them
int smg_debug_wide_check(unsigned long long* host_out) {
  SMG_HIP(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wchk), sizeof(unsigned long long) * 4));
  unsigned long long z[4] = {0, 0, 0, 0};
  SMG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wchk), z, sizeof(z)));
  return SMG_OK;
}
#endif

int smg_debug_check_points(int64_t n_points) {
  SMG_CHECK_ARG(n_points >= 0, "negative n_points");
  g_chk_points = n_points;
  return SMG_OK;
}

int smg_debug_check_read(unsigned long long* host_out, int32_t n) {
#ifdef SMG_CHECK
  SMG_CHECK_ARG(host_out != nullptr && n >= 0, "bad arguments");
  unsigned long long z[CHK_N] = {0};
  if (!g_chk_cnt) {  // no checked launch yet
    for (int i = 0; i < n && i < CHK_N; ++i) host_out[i] = 0;
    return SMG_OK;
  }
  SMG_HIP(hipDeviceSynchronize());
  SMG_HIP(hipMemcpy(z, g_chk_cnt, sizeof(z), hipMemcpyDeviceToHost));
  for (int i = 0; i < n && i < CHK_N; ++i) host_out[i] = z[i];
  SMG_HIP(hipMemset(g_chk_cnt, 0, sizeof(z)));
  return SMG_OK;
#else
  (void)host_out;
  (void)n;
  set_error("library built without -DSMG_CHECK");
  return SMG_ERR_UNSUPPORTED;
#endif
}

int smg_debug_main_kernel(int32_t which) {
  SMG_CHECK_ARG(which == 0 || which == 1, "main kernel must be 0 (ion_pipe_kernel) or 1 (ion_sparse_kernel)");
  g_main_kernel = which;
  return SMG_OK;
}

int smg_debug_sparse_stamps(unsigned long long* host_out, int n) { return sparse_read_stamps(host_out, n); }

int smg_debug_force_two_level(int32_t on) {
  g_force_two_level = on ? 1 : 0;
  return SMG_OK;
}

int smg_debug_time_main_pass(int32_t on) {
  g_time_main = on ? 1 : 0;
  if (on) {  // events for ~170 searches made now, not while a pass runs
    std::lock_guard<std::mutex> g(g_ev_mu);
    while (g_ev_pool.size() < 2048) {
      hipEvent_t e = nullptr;
      if (hipEventCreate(&e) != hipSuccess) break;
      g_ev_pool.push_back(e);
    }
  }
  return SMG_OK;
}

// waits for the recorded launches, hands out those of pass `only` (-1: every pass) and forgets them all
static int drain_pass_times(int only, int32_t* pass, double* ms, int32_t cap, int32_t* n) {
  std::lock_guard<std::mutex> g(g_ev_mu);
  int32_t k = 0;
  int rc = SMG_OK;
  for (auto& e : g_pass_events) {
    float t = 0.0f;
    if (rc == SMG_OK && (hipEventSynchronize(e.ev1) != hipSuccess ||
                         hipEventElapsedTime(&t, e.ev0, e.ev1) != hipSuccess)) {
      set_error("pass timing events failed");
      rc = SMG_ERR_HIP;
    }
    if (only < 0 || e.pass == only) {
      if (k < cap) {
        ms[k] = (double)t;
        if (pass) pass[k] = e.pass;
      }
      ++k;
    }
    ev_give(e.ev0);
    ev_give(e.ev1);
  }
  g_pass_events.clear();
  *n = k;
  return rc;
}

int smg_debug_main_pass_times(double* ms, int32_t cap, int32_t* n) {
  SMG_CHECK_ARG(n != nullptr && (ms != nullptr || cap == 0), "bad arguments");
  return drain_pass_times(SMG_PASS_MAIN, nullptr, ms, cap, n);
}

int smg_debug_pass_times(int32_t* pass, double* ms, int32_t cap, int32_t* n) {
  SMG_CHECK_ARG(n != nullptr && ((ms != nullptr && pass != nullptr) || cap == 0), "bad arguments");
  return drain_pass_times(-1, pass, ms, cap, n);
}

int smg_debug_force_dense(int32_t on) {
  g_force_dense = (on == 1 || on == 2) ? on : 0;
  return SMG_OK;
}

int smg_debug_wide_impl(int32_t which) {
  SMG_CHECK_ARG(which == 0 || which == 1, "wide pass must be 0 (ion_wide_kernel) or 1 (ion_wide_join_kernel)");
  g_wide_impl = which;
  return SMG_OK;
}

int smg_ion_metrics_workspace_size(int64_t n_ions, int32_t nrows, int32_t ncols, size_t* bytes) {
  SMG_CHECK_ARG(bytes && n_ions >= 0 && nrows > 0 && ncols > 0, "bad arguments");
  SMG_CHECK_ARG((int64_t)nrows * ncols < (1ll << 31), "image too large");
  *bytes = ws_bytes_for(n_ions, nrows * ncols);
  return SMG_OK;
}

int smg_ion_metrics(int32_t hit_format, const void* hits, const double* hit_vals, const double* hit_cum,
                    const int64_t* lo,
                    const int64_t* hi, const int64_t* ion_win_off, const double* theor_int,
                    const int64_t* ion_order, int64_t n_ions, int32_t nrows, int32_t ncols, int32_t nlevels,
                    double q, int32_t do_preprocessing, int32_t connectivity, int32_t erosion_border,
                    double* out_chaos, double* out_spatial, double* out_spectral, double* out_msm,
                    uint32_t* out_flags, void* workspace, size_t workspace_bytes, void* stream) {
  SMG_CHECK_ARG(n_ions >= 0 && n_ions < (1ll << 31), "n_ions out of range");
  if (n_ions == 0) return SMG_OK;
  SMG_CHECK_ARG(nrows > 0 && ncols > 0 && (int64_t)nrows * ncols < (1ll << 31), "bad image shape");
  SMG_CHECK_ARG(nlevels >= 1 && nlevels <= 254, "nlevels must be in [1, 254]");
  SMG_CHECK_ARG(connectivity == 4 || connectivity == 8, "connectivity must be 4 or 8");
  SMG_CHECK_ARG(erosion_border == 0 || erosion_border == 1, "erosion_border must be 0 or 1");
  SMG_CHECK_ARG(hit_format == SMG_HITS_PACKED_F32 || hit_format == SMG_HITS_SPLIT_F64, "bad hit_format");
  SMG_CHECK_ARG(hit_cum && lo && hi && ion_win_off && theor_int && out_chaos && out_spatial && out_spectral &&
                    out_msm && out_flags && workspace,
                "null pointer");
  SMG_CHECK_ARG(!do_preprocessing || (q >= 0.0 && q <= 100.0), "q must be in [0, 100]");
  const size_t need = ws_bytes_for(n_ions, nrows * ncols);
  if (workspace_bytes < need) {
    set_error("ion_metrics workspace too small: %zu < %zu", workspace_bytes, need);
    return SMG_ERR_WORKSPACE;
  }
  Params P;
  P.nrows = nrows;
  P.ncols = ncols;
  P.npx = nrows * ncols;
  P.nlevels = nlevels;
  P.connectivity = connectivity;
  P.erosion_border = erosion_border;
  P.step = nlevels > 1 ? 1.0 / (double)(nlevels - 1) : 0.0;
  P.inv_ncols = 1.0f / (float)ncols;
  P.w32 = 0;
  P.o_pf = 0;
  P.q = q;
  P.clip = do_preprocessing ? 1 : 0;
  unsigned char* ws = reinterpret_cast<unsigned char*>(workspace);
  hipStream_t st = as_stream(stream);
  if (hit_format == SMG_HITS_PACKED_F32) {
    SMG_CHECK_ARG(hits != nullptr, "null hits");
    Hits<SMG_HITS_PACKED_F32> h{reinterpret_cast<const uint64_t*>(hits), nullptr};
    return launch_metrics<SMG_HITS_PACKED_F32>(h, hit_cum, lo, hi, ion_win_off, theor_int, ion_order, n_ions, P, out_chaos,
                                               out_spatial, out_spectral, out_msm, out_flags, ws, st);
  }
  SMG_CHECK_ARG(hits != nullptr && hit_vals != nullptr, "null hits");
  Hits<SMG_HITS_SPLIT_F64> h{reinterpret_cast<const uint32_t*>(hits), hit_vals};
  return launch_metrics<SMG_HITS_SPLIT_F64>(h, hit_cum, lo, hi, ion_win_off, theor_int, ion_order, n_ions, P, out_chaos,
                                            out_spatial, out_spectral, out_msm, out_flags, ws, st);
}

}  // extern "C"
