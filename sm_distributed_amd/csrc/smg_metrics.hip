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
// Two paths:
//  * LDS path (ion_lds_kernel): one 256-thread workgroup per ion.  The principal image lives in LDS
//    as a pixel bitmap + per-64-bit-word popcount prefix (rank) + f64 values in rank order.  The
//    other isotope windows are streamed once and joined against it (spectral sums, Pearson sums);
//    their own duplicate pixels are found with a hashed two-bit filter.  measure_of_chaos uses the
//    threshold decomposition of flat morphology: the per-level dilate(cross)/erode(box) equals
//    thresholding eL = erode_box(dilate_cross(L)) of the per-pixel level index L, so
//    sum_levels #components = sum_p eL(p) - weight(maximum spanning forest), computed with one
//    Kruskal pass (levels descending) over an LDS union-find.  Candidates for eL > 0 are found from
//    7x7 bit windows of the bitmap, so isolated pixels cost ~14 LDS reads.
//  * dense path (ion_dense_kernel): persistent workgroups with a global-memory scratch slot of
//    N_px-sized images, for ions that do not fit the LDS path (principal window > CAP points, too
//    many E pixels / suspects, images larger than 2^18 pixels).
#include <stdarg.h>

#include "smg_common.hpp"

namespace smg {

constexpr int BLOCK = 256;           // dense (global-scratch) kernel
constexpr int NW = BLOCK / WAVE;
constexpr int MAXK = 8;              // windows per ion on the LDS path
constexpr int MAXK_DENSE = 32;       // windows per ion supported at all
constexpr int TBL = 1024;             // duplicate-candidate table slots ((pixel, window)-keyed f64 sums)
constexpr int SIDE = 256;             // principal duplicate-pixel table slots (rank-keyed f64 sums)
constexpr int NPX_LDS_MAX = 1 << 18; // images up to 262144 pixels use the LDS path

enum { C_NE = 0, C_EMAX, C_ABORT, C_NOWN, C_NCTR = 8 };

// Diagnostic build only (-DSMG_STAMPS): per-phase wall cycles of the LDS kernel, summed over workgroups
// into a buffer of their own (read back by smg_debug_stamps); the shipped build executes no stamp.
#ifdef SMG_STAMPS
__device__ unsigned long long g_stamps[16];
#define STAMP_INIT() unsigned long long _st0 = __builtin_amdgcn_s_memtime(), _st1
#define STAMP(i)                                                                   \
  do {                                                                             \
    if (threadIdx.x == 0) {                                                        \
      _st1 = __builtin_amdgcn_s_memtime();                                         \
      atomicAdd(&g_stamps[i], _st1 - _st0);                                        \
      _st0 = _st1;                                                                 \
    }                                                                              \
  } while (0)
#else
#define STAMP_INIT()
#define STAMP(i)
#endif

struct Params {
  int32_t nrows, ncols, npx;
  int32_t nlevels;
  int32_t connectivity;
  int32_t erosion_border;
  double step;      // np.linspace(0, 1, nlevels) step
  float inv_ncols;  // 1/ncols for the LDS path's row/column split (npx < 2^24)
};

// row and column of pixel p < 2^24 from a float reciprocal: the estimate is off by at most one row
__device__ __forceinline__ void rowcol(int p, const Params& P, int& r, int& c) {
  r = (int)((float)p * P.inv_ncols);
  c = p - r * P.ncols;
  if (c < 0) {
    --r;
    c += P.ncols;
  } else if (c >= P.ncols) {
    ++r;
    c -= P.ncols;
  }
}

template <int FMT>
struct Hits;

template <>
struct Hits<SMG_HITS_PACKED_F32> {
  const uint64_t* h;
  const double* unused;
  using Reg = uint64_t;
  __device__ __forceinline__ Reg load(int64_t i) const { return h[i]; }
  // scalar base + 32-bit lane offset (saddr addressing)
  __device__ __forceinline__ Reg load(int64_t base, int i) const { return (h + base)[i]; }
  static __device__ __forceinline__ uint32_t pix(Reg r) { return (uint32_t)r & 0x7FFFFFFFu; }
  static __device__ __forceinline__ bool dup(Reg r) { return ((uint32_t)r >> 31) != 0u; }
  static __device__ __forceinline__ double val(Reg r) { return (double)__uint_as_float((uint32_t)(r >> 32)); }
  __device__ __forceinline__ void get(int64_t i, uint32_t& p, double& v) const {
    const uint64_t x = h[i];
    p = (uint32_t)x & 0x7FFFFFFFu;
    v = (double)__uint_as_float((uint32_t)(x >> 32));
  }
};

struct PixVal {
  uint32_t p;
  double v;
};

template <>
struct Hits<SMG_HITS_SPLIT_F64> {
  const uint32_t* pa;
  const double* va;
  using Reg = PixVal;
  __device__ __forceinline__ Reg load(int64_t i) const { return PixVal{pa[i], va[i]}; }
  __device__ __forceinline__ Reg load(int64_t base, int i) const { return PixVal{(pa + base)[i], (va + base)[i]}; }
  static __device__ __forceinline__ uint32_t pix(Reg r) { return r.p & 0x7FFFFFFFu; }
  static __device__ __forceinline__ bool dup(Reg r) { return (r.p >> 31) != 0u; }
  static __device__ __forceinline__ double val(Reg r) { return r.v; }
  __device__ __forceinline__ void get(int64_t i, uint32_t& p, double& v) const {
    p = pa[i] & 0x7FFFFFFFu;
    v = va[i];
  }
};

// level index L = #{i : linspace(0,1,n)[i] < v/vmax}  (measure_of_chaos: bw = im_clean > level)
__device__ __forceinline__ int level_of(double v, double vmax, const Params& P) {
  const double norm = v / vmax;
  int L = 0;
  for (int i = 0; i < P.nlevels; ++i) {
    const double lev = (P.nlevels > 1 && i == P.nlevels - 1) ? 1.0 : (double)i * P.step;
    L += (lev < norm) ? 1 : 0;
  }
  return L;
}

__device__ __forceinline__ double clean(double v) {  // ImgMeasures._replace_nan
  return (v == 0.0 || isnan(v) || isinf(v)) ? 0.0 : v;
}

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

// exclusive popcount prefix over the first n64 64-bit words: each wave scans a contiguous range
// 64 words at a time (lane-parallel), then wave offsets are added.  Returns the total.
template <int NW_>
__device__ int bm_build_prefix(const uint32_t* bm, uint16_t* pf, int n64, int* wscratch) {
  constexpr int NW = NW_;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t* bm64 = reinterpret_cast<const uint64_t*>(bm);
  const int span = ((n64 + NW - 1) / NW + 63) & ~63;
  const int a = wid * span;
  const int b = min(n64, a + span);
  int carry = 0;
  for (int base = a; base < b; base += 64) {
    const int j = base + lane;
    const int c = (j < b) ? __popcll(bm64[j]) : 0;
    const int inc = wave_incl_scan_dpp(c);
    if (j < b) pf[j] = (uint16_t)(carry + inc - c);
    carry += __builtin_amdgcn_readlane(inc, 63);
  }
  if (lane == 0) wscratch[wid] = carry;
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < NW; ++w) {
    const int c = wscratch[w];
    if (w < wid) off += c;
    tot += c;
  }
  if (off) {
    for (int j = a + lane; j < b; j += 64) pf[j] = (uint16_t)(pf[j] + off);
  }
  __syncthreads();
  return tot;
}

// bits of image row `row`, columns c0..c0+6 (bit j <-> column c0+j), masked by the valid-column mask cv;
// 0 outside the image.  c0 >= -3: the bitmap has a zero guard word in front (LdsLayout::o_hbm).
__device__ __forceinline__ uint32_t bits7(const uint32_t* bm, int row, int c0, uint32_t cv, const Params& P) {
  const bool rv = (unsigned)row < (unsigned)P.nrows;
  const int st = (rv ? row : 0) * P.ncols + c0;
  const int w = st >> 5;
  const uint32_t v = __builtin_amdgcn_alignbit(bm[w + 1], bm[w], (uint32_t)(st & 31)) & cv;
  return rv ? v : 0u;
}

__device__ __forceinline__ uint32_t uf_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ uint32_t uf_find(uint32_t* par, uint32_t x) {
  while (true) {
    const uint32_t p = uf_load(&par[x]);
    if (p == x) return x;
    const uint32_t g = uf_load(&par[p]);
    if (g != p) __hip_atomic_store(&par[x], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    x = g;
  }
}

// returns true if a and b were in different trees (one successful link)
__device__ __forceinline__ bool uf_unite(uint32_t* par, uint32_t a, uint32_t b) {
  while (true) {
    a = uf_find(par, a);
    b = uf_find(par, b);
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

struct LdsLayout {
  int w32;        // bitmap words incl. padding (multiple of 4)
  int cap;        // max principal-window points on the LDS path (runtime, <= CAP_MAX)
  size_t o_pf, o_vals, o_L, o_dupb, o_side_k, o_side_v, o_filt, o_tkey, o_tval, o_part, o_red, o_ctr, o_wsc,
      bytes;
};

static inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS carve for an image of npx pixels and principal values of val_bytes each.  The principal-image
// capacity is whatever fits the per-workgroup budget (LDS_BUDGET -> two workgroups per CU), capped by
// CAP_MAX and by the chaos phase's reuse of the filter + table region (rank-ordered E pixels: 5 B each).
static LdsLayout lds_layout(int npx, int val_bytes, int NW, int CAP_MAX, size_t LDS_BUDGET) {
  LdsLayout L;
  const int words = (npx + 31) / 32 + 2;
  L.w32 = (words + 3) & ~3;
  const size_t region_ft0 = al16((size_t)TBL * 4) + al16((size_t)TBL * 8);
  const size_t fixed = 16 + al16((size_t)L.w32 * 4) + al16((size_t)(L.w32 / 2) * 2) + al16((size_t)SIDE * 4) +
                       al16((size_t)SIDE * 8) + al16((size_t)MAXK * NW * 4 * 8) + al16((size_t)8 * NW * 8) +
                       al16((size_t)C_NCTR * 4) + al16((size_t)NW * 4) + 256;
  // largest cap (multiple of 64, <= CAP_MAX) whose carve fits the budget; the filter + table region
  // doubles as the chaos phase's E-pixel storage (5 B per point) and grows with cap when needed
  int cap = CAP_MAX & ~63;
  size_t region_ft = region_ft0;
  for (; cap >= 64; cap -= 64) {
    region_ft = region_ft0 > al16((size_t)5 * cap) ? region_ft0 : al16((size_t)5 * cap);
    const size_t need = fixed + region_ft + al16((size_t)cap * (val_bytes < 4 ? 4 : val_bytes)) + al16((size_t)cap) +
                        al16((size_t)((cap + 31) / 32) * 4);
    if (need <= LDS_BUDGET) break;
  }
  if (cap < 64) cap = 0;
  L.cap = cap;
  size_t o = 16 + al16((size_t)L.w32 * 4);  // zero guard word(s), then the bitmap at offset 16
  L.o_pf = o;
  o = al16(o + (size_t)(L.w32 / 2) * 2);
  L.o_vals = o;
  o = al16(o + (size_t)cap * (val_bytes < 4 ? 4 : val_bytes));
  L.o_L = o;
  o = al16(o + (size_t)cap);
  L.o_dupb = o;
  o = al16(o + (size_t)((cap + 31) / 32) * 4);
  L.o_side_k = o;
  o = al16(o + (size_t)SIDE * 4);
  L.o_side_v = o;
  o = al16(o + (size_t)SIDE * 8);
  L.o_filt = o;  // region shared by the duplicate table and (later) the chaos phase's E arrays
  L.o_tkey = o;
  o = al16(o + (size_t)TBL * 4);
  L.o_tval = o;
  o = al16(o + (size_t)TBL * 8);
  if (o - L.o_filt < region_ft) o = L.o_filt + region_ft;
  L.o_part = o;
  o = al16(o + (size_t)MAXK * NW * 4 * 8);
  L.o_red = o;
  o = al16(o + (size_t)8 * NW * 8);
  L.o_ctr = o;
  o = al16(o + (size_t)C_NCTR * 4);
  L.o_wsc = o;
  o = al16(o + (size_t)NW * 4);
  L.bytes = o;
  return L;
}


// open-addressing f64 accumulators keyed by u32 (EMPTY = 0xFFFFFFFF); returns false when full
template <int NSLOT>
__device__ __forceinline__ bool tbl_add(uint32_t* keys, double* vals, uint32_t key, double v) {
  uint32_t h = (key * 2654435761u) >> (32 - __builtin_ctz(NSLOT));
  for (int probe = 0; probe < NSLOT; ++probe) {
    const uint32_t old = atomicCAS(&keys[h], 0xFFFFFFFFu, key);
    if (old == 0xFFFFFFFFu || old == key) {
      atomicAdd(&vals[h], v);
      return true;
    }
    h = (h + 1) & (NSLOT - 1);
  }
  return false;
}

template <int NSLOT>
__device__ __forceinline__ int tbl_find(const uint32_t* keys, uint32_t key) {
  uint32_t h = (key * 2654435761u) >> (32 - __builtin_ctz(NSLOT));
  for (int probe = 0; probe < NSLOT; ++probe) {
    const uint32_t k = keys[h];
    if (k == key) return (int)h;
    if (k == 0xFFFFFFFFu) return -1;
    h = (h + 1) & (NSLOT - 1);
  }
  return -1;
}

// level index via the closed form of np.linspace(0, 1, n): lev_i = i*step (i < n-1), lev_{n-1} = 1.0;
// L = #{i : lev_i < norm}; the estimate is corrected with exact comparisons so it equals the loop.
__device__ __forceinline__ int level_fast(double v, double vmax, const Params& P) {
  const double norm = v / vmax;
  const int n = P.nlevels;
  if (n == 1) return (0.0 < norm) ? 1 : 0;
  if (!(norm > 0.0)) return 0;
  int j = (int)(norm * (double)(n - 1));  // candidate count of i*step < norm among i < n-1
  j = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
  while (j > 0 && !((double)(j - 1) * P.step < norm)) --j;
  while (j < n - 1 && (double)j * P.step < norm) ++j;
  return j + ((1.0 < norm) ? 1 : 0);
}

template <int FMT>
struct ValStore;
template <>
struct ValStore<SMG_HITS_PACKED_F32> {
  using T = float;  // a single f32 hit is exact in f32; duplicate pixels use the f64 side table
};
template <>
struct ValStore<SMG_HITS_SPLIT_F64> {
  using T = double;
};

// ---------------------------------------------------------------------------------------------
// LDS path kernel (one workgroup per ion; two workgroups per CU).  Phases, barriers between:
//   0  issue the loads of the principal window (<= cap points, RMAX per thread) and of the first
//      chunk of window 1 into registers; initialise the LDS structures meanwhile
//   1  principal bitmap (atomicOr; the thread that sets a bit owns the pixel), rank prefix, values in
//      rank order (f32 for single hits, exact f64 side table for duplicate pixels)
//   2  one fused reduction: sum x, sum x^2, sum x[x>0], #(x>0), max; then level index per pixel
//   5  for k >= 1: stream window k (registers, next window prefetched), join against the principal
//      image; duplicate pixels of window k found by a hashed 2-bit filter and summed in an LDS table
//   4a chaos candidates from owned principal pixels (7x7 bit windows, isolation pre-filter), exact eL
//   4b Kruskal over eL with an LDS union-find
//   6  finalize (thread 0)
// ---------------------------------------------------------------------------------------------
template <int FMT, int LB, int LRMAX, int LRC>
__device__ __forceinline__ void process_ion_lds(
    int64_t ion, const Hits<FMT>& hits, const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
    const int64_t* __restrict__ ion_off, const double* __restrict__ theor, const Params& P, const LdsLayout& LL,
    double* __restrict__ oc, double* __restrict__ osp, double* __restrict__ osc, double* __restrict__ omsm,
    uint32_t* __restrict__ oflags, uint32_t* __restrict__ dense_list, uint32_t* __restrict__ dense_count) {
  constexpr int BLOCK = LB;
  constexpr int NW = LB / WAVE;
  constexpr int RMAX = LRMAX;
  constexpr int RC = LRC;
  constexpr int CAP_MAX = BLOCK * RMAX;
  using Reg = typename Hits<FMT>::Reg;
  using VT = typename ValStore<FMT>::T;
  constexpr bool SIDE_TABLE = (FMT == SMG_HITS_PACKED_F32);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* Hbm = reinterpret_cast<uint32_t*>(smem + 16);  // smem[0..16): zero guard for bits7
  uint16_t* pf = reinterpret_cast<uint16_t*>(smem + LL.o_pf);
  VT* vals = reinterpret_cast<VT*>(smem + LL.o_vals);
  uint8_t* Lv = reinterpret_cast<uint8_t*>(smem + LL.o_L);
  uint32_t* dupb = reinterpret_cast<uint32_t*>(smem + LL.o_dupb);
  uint32_t* side_k = reinterpret_cast<uint32_t*>(smem + LL.o_side_k);
  double* side_v = reinterpret_cast<double*>(smem + LL.o_side_v);
  uint32_t* filtA = reinterpret_cast<uint32_t*>(smem + LL.o_filt);  // base of the table / E region
  uint32_t* tkey = reinterpret_cast<uint32_t*>(smem + LL.o_tkey);
  double* tval = reinterpret_cast<double*>(smem + LL.o_tval);
  double* part = reinterpret_cast<double*>(smem + LL.o_part);  // [MAXK][NW][4]: s_k, sy, syy, sxy
  double* red = reinterpret_cast<double*>(smem + LL.o_red);
  int* ctr = reinterpret_cast<int*>(smem + LL.o_ctr);
  int* wsc = reinterpret_cast<int*>(smem + LL.o_wsc);
  const int cap = LL.cap;
  // chaos-phase aliases (the value, filter and table regions are dead by then)
  uint32_t* epix = reinterpret_cast<uint32_t*>(vals);                  // candidates, append order
  uint32_t* epix_r = filtA;                                            // E pixels, rank order (4*cap)
  uint8_t* eL8 = reinterpret_cast<uint8_t*>(filtA) + (size_t)cap * 4;  // candidates' eL, append order
  uint8_t* eLr = Lv;                                                   // rank order
  uint32_t* par = reinterpret_cast<uint32_t*>(vals);                   // rank order (after epix consumed)

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int64_t w0 = ion_off[ion];
  const int K = (int)(ion_off[ion + 1] - w0);

  uint32_t flags = (LB >= 1024) ? SMG_ION_BIG : 0u;
  for (int k = 0; k < K && k < MAXK_DENSE; ++k)
    if (hi[w0 + k] > lo[w0 + k]) flags |= SMG_ION_HAS_HITS;
  if (K == 0) {
    if (tid == 0) {
      oc[ion] = osp[ion] = osc[ion] = omsm[ion] = 0.0;
      oflags[ion] = 0;
    }
    return;
  }
  const int64_t lo0 = lo[w0];
  const int n0 = (int)min<int64_t>(hi[w0] - lo0, (int64_t)CAP_MAX + 1);
  if (K > MAXK || n0 > cap) {
    if (tid == 0) dense_list[atomicAdd(dense_count, 1u)] = (uint32_t)ion;
    return;
  }

  // ---- phase 0: loads in flight, LDS initialisation meanwhile -----------------------------------
  STAMP_INIT();
  Reg h0[RMAX];
#pragma unroll
  for (int j = 0; j < RMAX; ++j) {
    const int i = tid + j * BLOCK;
    if (i < n0) h0[j] = hits.load(lo0, i);
  }
  // windows 1..K-1 are streamed in chunks of BLOCK*RC points that never span two windows; a chunk is
  // (window k, offset base).  The first chunk (A) is issued here with the principal window, the second (B)
  // right after phase 1, so both are in flight during phases 1-3.
  constexpr int CH = BLOCK * RC;
  auto skip_empty = [&](int& k, int64_t& base) {
    while (k < K && base >= hi[w0 + k] - lo[w0 + k]) {
      ++k;
      base = 0;
    }
  };
  auto load_chunk = [&](int k, int64_t base, Reg (&buf)[RC]) {
    const int64_t a = lo[w0 + k];
    const int64_t n = hi[w0 + k] - a;
    const int rem = (int)min<int64_t>(n - base, (int64_t)CH);
#pragma unroll
    for (int j = 0; j < RC; ++j) {
      const int i = tid + j * BLOCK;
      if (i < rem) buf[j] = hits.load(a + base, i);
    }
  };
  Reg ra[RC], rb[RC];
  int ka = 1, kb = K;
  int64_t ba = 0, bb = 0;
  skip_empty(ka, ba);
  if (ka < K) load_chunk(ka, ba, ra);
  {
    uint4* z = reinterpret_cast<uint4*>(smem);
    for (int i = tid; i < LL.w32 / 4 + 1; i += BLOCK) z[i] = make_uint4(0, 0, 0, 0);
    for (int i = tid; i < TBL; i += BLOCK) {
      tkey[i] = 0xFFFFFFFFu;
      tval[i] = 0.0;
    }
    for (int i = tid; i < SIDE; i += BLOCK) {
      side_k[i] = 0xFFFFFFFFu;
      side_v[i] = 0.0;
    }
    for (int i = tid; i < (cap + 31) / 32; i += BLOCK) dupb[i] = 0u;
    if (tid < C_NCTR) ctr[tid] = 0;
  }
  __syncthreads();
  STAMP(0);

  // ---- phase 1: principal image -> bitmap (+ ownership), rank prefix, values --------------------
  uint32_t own = 0;
  uint32_t hp[RMAX];
#pragma unroll
  for (int j = 0; j < RMAX; ++j) {
    const int i = tid + j * BLOCK;
    hp[j] = 0;
    if (i < n0) {
      const uint32_t p = Hits<FMT>::pix(h0[j]);
      hp[j] = p;
      const uint32_t bit = 1u << (p & 31);
      const uint32_t old = atomicOr(&Hbm[p >> 5], bit);
      if (!(old & bit)) own |= 1u << j;
    }
  }
  __syncthreads();
  const int n64 = (P.npx + 63) / 64;
  const int nnz = bm_build_prefix<NW>(Hbm, pf, n64, wsc);
  if constexpr (SIDE_TABLE) {
    // A point without the duplicate-candidate flag is the only point of its pixel in this window
    // (smg_flag_duplicates), so its f32 value is the pixel value exactly.  Flagged points (true duplicates
    // and a few false positives) are summed per rank in the f64 side table, marked in dupb.
#pragma unroll
    for (int j = 0; j < RMAX; ++j) {
      const int i = tid + j * BLOCK;
      if (i < n0) {
        const int r = bm_rank(Hbm, pf, (int)hp[j]);
        if (!Hits<FMT>::dup(h0[j])) {
          vals[r] = (VT)Hits<FMT>::val(h0[j]);
        } else {
          atomicOr(&dupb[r >> 5], 1u << (r & 31));
          if (!tbl_add<SIDE>(side_k, side_v, (uint32_t)r, Hits<FMT>::val(h0[j]))) ctr[C_ABORT] = 1;
        }
      }
    }
  } else {
    for (int r = tid; r < nnz; r += BLOCK) vals[r] = (VT)0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RMAX; ++j) {
      const int i = tid + j * BLOCK;
      if (i < n0) atomicAdd(&vals[bm_rank(Hbm, pf, (int)hp[j])], Hits<FMT>::val(h0[j]));
    }
  }
  if (ka < K) {
    kb = ka;
    bb = ba + CH;
    skip_empty(kb, bb);
    if (kb < K) load_chunk(kb, bb, rb);
  }
  __syncthreads();
  if (ctr[C_ABORT]) {  // more duplicate pixels than the side table holds
    if (tid == 0) dense_list[atomicAdd(dense_count, 1u)] = (uint32_t)ion;
    return;
  }
  auto value_at = [&](int r) -> double {
    if constexpr (SIDE_TABLE) {
      if ((dupb[r >> 5] >> (r & 31)) & 1u) return side_v[tbl_find<SIDE>(side_k, (uint32_t)r)];
    }
    return (double)vals[r];
  };
  STAMP(1);

  // ---- phase 2: fused principal-image statistics, then level index per pixel -------------------
  double sx, sxx, s0, npos, vmax;
  {
    double acc[5] = {0.0, 0.0, 0.0, 0.0, -INFINITY};
    for (int r = tid; r < nnz; r += BLOCK) {
      const double v = value_at(r);
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
    __syncthreads();
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
    npos = t[3];
    vmax = t[4];
  }
#ifndef SMG_ABL
#define SMG_ABL 0  // diagnostic ablations (timing only, wrong results): 1 = no chaos, 2 = no windows k >= 1
#endif
  const bool chaos_ok = (sx > 0.0) && (npos >= 4.0) && !(SMG_ABL & 1);
  if (chaos_ok) {
    for (int r = tid; r < nnz; r += BLOCK) Lv[r] = (uint8_t)level_fast(value_at(r), vmax, P);
  }
  STAMP(2);

  // ---- phase 5: other isotope windows in one streaming pass, joined against the principal image -----
  // Chunks of BLOCK*RC points walk windows 1..K-1 in order with the next chunk prefetched into the other
  // register buffer; there is no barrier between windows.  Per-window partial sums are reduced per wave at
  // the window's last chunk.  A point whose duplicate-candidate flag is set (smg_flag_duplicates: it has a
  // same-spectrum neighbour within a window width) goes to the pixel-keyed f64 table so that duplicate
  // pixels are summed before squaring (sum y^2 over pixels); every other point contributes v^2 directly.
  {
    double psk = 0.0, psy = 0.0, psyy = 0.0, psxy = 0.0;
    auto flush = [&](int k) {
      const double a0 = wave_sum_dpp(psk), a1 = wave_sum_dpp(psy), a2 = wave_sum_dpp(psyy), a3 = wave_sum_dpp(psxy);
      if (lane == 0) {
        double* pk = part + ((size_t)k * NW + wid) * 4;
        pk[0] = a0;
        pk[1] = a1;
        pk[2] = a2;
        pk[3] = a3;
      }
      psk = psy = psyy = psxy = 0.0;
    };
    auto process = [&](int k, int64_t base, Reg (&buf)[RC]) {
      const int64_t n = hi[w0 + k] - lo[w0 + k];
      const int rem = (int)min<int64_t>(n - base, (int64_t)BLOCK * RC);
#pragma unroll
      for (int j = 0; j < RC; ++j) {
        if (tid + j * BLOCK < rem) {
          const uint32_t p = Hits<FMT>::pix(buf[j]);
          const double v = Hits<FMT>::val(buf[j]);
          double x = 0.0;
          if (bm_test(Hbm, (int)p)) x = value_at(bm_rank(Hbm, pf, (int)p));
          psy += v;
          psxy += x * v;
          if (x > 0.0) psk += v;
          if (!Hits<FMT>::dup(buf[j])) {
            psyy += v * v;
          } else if (!tbl_add<TBL>(tkey, tval, (p << 3) | (uint32_t)k, v)) {
            ctr[C_ABORT] = 1;
          }
        }
      }
      if (base + (int64_t)BLOCK * RC >= n) flush(k);  // last chunk of window k
    };
    // windows 1..K-1 with zero points still need their (zero) partials
    for (int k = 1; k < K; ++k)
      if (hi[w0 + k] <= lo[w0 + k] && lane == 0) {
        double* pk = part + ((size_t)k * NW + wid) * 4;
        pk[0] = pk[1] = pk[2] = pk[3] = 0.0;
      }
    // ra holds chunk A, rb chunk B (when they exist); each buffer is refilled as soon as it is consumed
    while (ka < K && !(SMG_ABL & 2)) {
      process(ka, ba, ra);
      if (kb >= K) break;
      ka = kb;
      ba = bb + CH;
      skip_empty(ka, ba);
      if (ka < K) load_chunk(ka, ba, ra);
      process(kb, bb, rb);
      if (ka >= K) break;
      kb = ka;
      bb = ba + CH;
      skip_empty(kb, bb);
      if (kb < K) load_chunk(kb, bb, rb);
    }
  }
  __syncthreads();
  if (ctr[C_ABORT]) {  // duplicate-candidate table full
    if (tid == 0) dense_list[atomicAdd(dense_count, 1u)] = (uint32_t)ion;
    return;
  }
  // drain the duplicate-candidate table: exact per-(pixel, window) sums, squared, into per-wave partials
  {
    double dq[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) dq[k] = 0.0;
    for (int sl = tid; sl < TBL; sl += BLOCK) {
      const uint32_t key = tkey[sl];
      if (key != 0xFFFFFFFFu) {
        const double y = tval[sl];
        const int k = (int)(key & 7u);
#pragma unroll
        for (int kk = 1; kk < MAXK; ++kk)
          if (kk == k) dq[kk] += y * y;
      }
    }
#pragma unroll
    for (int kk = 1; kk < MAXK; ++kk) {
      if (kk < K) {
        const double t = wave_sum_dpp(dq[kk]);
        if (lane == 0) part[((size_t)kk * NW + wid) * 4 + 2] += t;
      }
    }
  }
  STAMP(3);

  // ---- phase 4a: chaos candidates (pixels with eL >= 1) from owned principal pixels --------------
  // (i) bit-level screen: a candidate p in cross(s) survives if its 3x3 box is covered by the
  //     dilated bitmap (superset of the exact condition) and s is its owner (smallest principal pixel
  //     of cross(p)); survivors go to an LDS list (the value region is free once L is computed).
  // (ii) exact eL for the survivors from the level indices.
  double chaos_raw = NAN;
  if (chaos_ok) {
    __syncthreads();  // values and the duplicate table are dead: the table region takes the owned list
    // compact the owned principal pixels (one per distinct pixel) into a dense list so that every lane of
    // the screen below has a pixel: the register slots are only ~half owned
    uint32_t* olist = filtA;
    {
      const int cnt = __popc(own);
      const int inc = wave_incl_scan_dpp(cnt);
      int wbase = 0;
      if (lane == 63) wbase = atomicAdd(&ctr[C_NOWN], inc);
      int pos = __builtin_amdgcn_readlane(wbase, 63) + inc - cnt;
#pragma unroll
      for (int j = 0; j < RMAX; ++j)
        if ((own >> j) & 1u) olist[pos++] = hp[j];
    }
    __syncthreads();
    for (int oc_i = tid; oc_i < nnz; oc_i += BLOCK) {
      const int s = (int)olist[oc_i];
      int rs, cs;
      rowcol(s, P, rs, cs);
      // valid-column mask of columns cs-3..cs+3
      const int clo = 3 - cs > 0 ? 3 - cs : 0, chi = P.ncols - cs + 3 < 7 ? P.ncols - cs + 3 : 7;
      const uint32_t cv = ((1u << chi) - 1u) & ~((1u << clo) - 1u);
      uint32_t H[7];
#pragma unroll
      for (int d = 0; d < 7; ++d) H[d] = bits7(Hbm, rs - 3 + d, cs - 3, cv, P);
      // isolation pre-filter (erosion border = background only): an eL>0 pixel in the cross of s needs
      // another principal pixel in s's 7x7, since the 4-cross of s alone cannot cover a 3x3 box
      if (!P.erosion_border && (H[0] | H[1] | H[2] | (H[3] & ~8u) | H[4] | H[5] | H[6]) == 0u) continue;
      uint32_t D[7];
      D[0] = D[6] = 0;
#pragma unroll
      for (int d = 1; d <= 5; ++d) {
        const int row = rs - 3 + d;
        const bool rv = row >= 0 && row < P.nrows;
        uint32_t x = (H[d] | (H[d] << 1) | (H[d] >> 1) | H[d - 1] | H[d + 1]) & cv;
        if (!rv) x = 0;
        if (P.erosion_border) x |= rv ? (~cv & 0x7Fu) : 0x7Fu;
        D[d] = x & 0x7Fu;
      }
#define SMG_HB(dr, dc) ((H[3 + (dr)] >> (3 + (dc))) & 1u)
#define SMG_BOX(dr, dc) ((((D[2 + (dr)] >> (2 + (dc))) & 7u) == 7u) && (((D[3 + (dr)] >> (2 + (dc))) & 7u) == 7u) && \
                         (((D[4 + (dr)] >> (2 + (dc))) & 7u) == 7u))
      const bool in_l = cs > 0, in_r = cs + 1 < P.ncols, in_u = rs > 0, in_d = rs + 1 < P.nrows;
      uint32_t pass = 0;
      if (SMG_BOX(0, 0) && !SMG_HB(-1, 0) && !SMG_HB(0, -1)) pass |= 1u;
      if (in_r && SMG_BOX(0, 1) && !SMG_HB(-1, 1)) pass |= 2u;
      if (in_l && SMG_BOX(0, -1) && !SMG_HB(-1, -1) && !SMG_HB(0, -2) && !SMG_HB(0, -1)) pass |= 4u;
      if (in_u && SMG_BOX(-1, 0) && !SMG_HB(-2, 0) && !SMG_HB(-1, -1) && !SMG_HB(-1, 0) && !SMG_HB(-1, 1))
        pass |= 8u;
      if (in_d && SMG_BOX(1, 0)) pass |= 16u;
#undef SMG_BOX
#undef SMG_HB
      while (pass) {
        const int ci = __ffs(pass) - 1;
        pass &= pass - 1;
        const int p = s + (ci == 1 ? 1 : ci == 2 ? -1 : ci == 3 ? -P.ncols : ci == 4 ? P.ncols : 0);
        const int idx = atomicAdd(&ctr[C_NE], 1);
        if (idx < cap) epix[idx] = (uint32_t)p;
      }
    }
    __syncthreads();
    STAMP(4);
    const int ncand = ctr[C_NE];
    if (ncand > cap) {
      if (tid == 0) dense_list[atomicAdd(dense_count, 1u)] = (uint32_t)ion;
      return;
    }
    // (ii) exact eL(p) = min_{q in N9(p)} max_{q' in N4[q] in image} L(q')
    int emax_local = 0;
    for (int c = tid; c < ncand; c += BLOCK) {
      const int p = (int)epix[c];
      int rp, cp;
      rowcol(p, P, rp, cp);
      int mn = 1 << 20;
      for (int qa = -1; qa <= 1; ++qa) {
        for (int qb = -1; qb <= 1; ++qb) {
          const int rq = rp + qa, cq = cp + qb;
          if (rq < 0 || rq >= P.nrows || cq < 0 || cq >= P.ncols) {
            if (!P.erosion_border) mn = 0;
            continue;
          }
          int dl = 0;
          for (int t = 0; t < 5; ++t) {
            const int r2 = rq + (t == 1 ? -1 : t == 2 ? 1 : 0);
            const int c2 = cq + (t == 3 ? -1 : t == 4 ? 1 : 0);
            if (r2 < 0 || r2 >= P.nrows || c2 < 0 || c2 >= P.ncols) continue;
            const int q = r2 * P.ncols + c2;
            if (bm_test(Hbm, q)) dl = max(dl, (int)Lv[bm_rank(Hbm, pf, q)]);
          }
          mn = min(mn, dl);
        }
      }
      if (mn >= (1 << 20)) mn = 0;
      eL8[c] = (uint8_t)mn;
      emax_local = max(emax_local, mn);
    }
    if (emax_local > 0) atomicMax(&ctr[C_EMAX], emax_local);
    __syncthreads();
    STAMP(5);

    // ---- phase 4b: Kruskal over eL (levels descending) with an LDS union-find -------------------
    double sum_c = 0.0;
    if (ctr[C_EMAX] > 0) {
      uint4* z = reinterpret_cast<uint4*>(Hbm);
      for (int i = tid; i < LL.w32 / 4; i += BLOCK) z[i] = make_uint4(0, 0, 0, 0);  // guard stays zero
      __syncthreads();
      for (int i = tid; i < ncand; i += BLOCK)
        if (eL8[i]) atomicOr(&Hbm[epix[i] >> 5], 1u << (epix[i] & 31));
      __syncthreads();
      const int m = bm_build_prefix<NW>(Hbm, pf, n64, wsc);
      for (int i = tid; i < ncand; i += BLOCK) {
        if (!eL8[i]) continue;
        const uint32_t p = epix[i];
        const int r = bm_rank(Hbm, pf, (int)p);
        epix_r[r] = p;
        eLr[r] = eL8[i];
      }
      __syncthreads();
      for (int r = tid; r < m; r += BLOCK) par[r] = (uint32_t)r;
      __syncthreads();
      const int emax = ctr[C_EMAX];
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
            if (!bm_test(Hbm, q)) return;
            const int rq = bm_rank(Hbm, pf, q);
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
    chaos_raw = 1.0 - sum_c / (double)P.nlevels / npos;
    STAMP(6);
  } else {
    flags |= SMG_ION_CHAOS_NAN;
  }

  if (tid == 0) {
    // s, sy, syy, sxy per window from the per-wave partials (wave order: deterministic)
    double* st = red;  // reuse: [4][MAXK]
    for (int k = 0; k < K; ++k) {
      double a4[4] = {0.0, 0.0, 0.0, 0.0};
      if (k > 0) {
        for (int w = 0; w < NW; ++w)
          for (int q = 0; q < 4; ++q) a4[q] += part[((size_t)k * NW + w) * 4 + q];
      } else {
        a4[0] = s0;
      }
      for (int q = 0; q < 4; ++q) st[q * MAXK + k] = a4[q];
    }
    finalize_ion(K, theor + w0, st, sx, sxx, st + MAXK, st + 2 * MAXK, st + 3 * MAXK, (double)P.npx, chaos_raw,
                 ion, flags, oc, osp, osc, omsm, oflags);
  }
}


template <int FMT, int LB, int LRMAX, int LRC, int WPE>
__global__ void __launch_bounds__(LB, WPE) ion_lds_kernel(
    Hits<FMT> hits, const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
    const int64_t* __restrict__ ion_off, const double* __restrict__ theor, const int64_t* __restrict__ ion_order,
    int64_t n_ions, Params P, LdsLayout LL, double* __restrict__ oc, double* __restrict__ osp,
    double* __restrict__ osc, double* __restrict__ omsm, uint32_t* __restrict__ oflags,
    uint32_t* __restrict__ next_list, uint32_t* __restrict__ next_count) {
  const int64_t ion = ion_order ? ion_order[blockIdx.x] : (int64_t)blockIdx.x;
  if (ion >= n_ions) return;
  process_ion_lds<FMT, LB, LRMAX, LRC>(ion, hits, lo, hi, ion_off, theor, P, LL, oc, osp, osc, omsm, oflags,
                                       next_list, next_count);
}

// persistent variant over a device list of ions (the rejects of a smaller-geometry pass)
template <int FMT, int LB, int LRMAX, int LRC>
__global__ void __launch_bounds__(LB, 4) ion_lds_list_kernel(
    Hits<FMT> hits, const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
    const int64_t* __restrict__ ion_off, const double* __restrict__ theor, const uint32_t* __restrict__ list,
    const uint32_t* __restrict__ count, uint32_t* __restrict__ cursor, Params P, LdsLayout LL,
    double* __restrict__ oc, double* __restrict__ osp, double* __restrict__ osc, double* __restrict__ omsm,
    uint32_t* __restrict__ oflags, uint32_t* __restrict__ next_list, uint32_t* __restrict__ next_count) {
  __shared__ int sh_ion;
  const uint32_t total = *count;
  while (true) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t k = atomicAdd(cursor, 1u);
      sh_ion = (k < total) ? (int)list[k] : -1;
    }
    __syncthreads();
    const int ion = sh_ion;
    if (ion < 0) break;
    process_ion_lds<FMT, LB, LRMAX, LRC>(ion, hits, lo, hi, ion_off, theor, P, LL, oc, osp, osc, omsm, oflags,
                                         next_list, next_count);
  }
}

// ---------------------------------------------------------------------------------------------
// dense path: persistent workgroups, one global scratch slot each
// ---------------------------------------------------------------------------------------------
struct DenseSlot {
  double* x;
  double* y;
  uint32_t* par;
  uint32_t* elist;
  uint8_t* L8;
  uint8_t* T8;
  uint8_t* E8;
};

static inline size_t dense_slot_bytes(int npx) {
  return al16((size_t)npx * 8) * 2 + al16((size_t)npx * 4) * 2 + al16((size_t)npx) * 3 + 256;
}

__device__ __forceinline__ DenseSlot dense_slot(unsigned char* base, int npx) {
  DenseSlot S;
  auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  size_t o = 0;
  S.x = reinterpret_cast<double*>(base + o);
  o += a16((size_t)npx * 8);
  S.y = reinterpret_cast<double*>(base + o);
  o += a16((size_t)npx * 8);
  S.par = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)npx * 4);
  S.elist = reinterpret_cast<uint32_t*>(base + o);
  o += a16((size_t)npx * 4);
  S.L8 = base + o;
  o += a16((size_t)npx);
  S.T8 = base + o;
  o += a16((size_t)npx);
  S.E8 = base + o;
  return S;
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

template <int FMT>
__device__ void scatter_window(const Hits<FMT>& hits, int64_t a, int64_t b, double* img) {
  for (int64_t i = a + threadIdx.x; i < b; i += BLOCK) {
    uint32_t p;
    double v;
    hits.get(i, p, v);
    atomicAdd(&img[p], v);
  }
}

template <int FMT>
__global__ void __launch_bounds__(BLOCK) ion_dense_kernel(
    Hits<FMT> hits, const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
    const int64_t* __restrict__ ion_off, const double* __restrict__ theor, int64_t n_ions, Params P,
    const uint32_t* __restrict__ dense_list, const uint32_t* __restrict__ dense_count, uint32_t* next,
    unsigned char* scratch, size_t slot_bytes, double* __restrict__ oc, double* __restrict__ osp,
    double* __restrict__ osc, double* __restrict__ omsm, uint32_t* __restrict__ oflags) {
  __shared__ double red[8 * NW];
  __shared__ double kst[4 * MAXK_DENSE];
  __shared__ int sh_ion;
  __shared__ int sh_ctr[4];
  const int tid = threadIdx.x;
  DenseSlot S = dense_slot(scratch + (size_t)blockIdx.x * slot_bytes, P.npx);
  const int npx = P.npx;
  const uint32_t total = *dense_count;

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

    // principal image (agent fences: plain zero stores must land in L2 before the L2 atomics,
    // and the atomics before the loads that follow)
    for (int p = tid; p < npx; p += BLOCK) S.x[p] = 0.0;
    __threadfence();
    __syncthreads();
    scatter_window<FMT>(hits, lo[w0], hi[w0], S.x);
    __threadfence();
    __syncthreads();
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    double mx = -INFINITY;
    for (int p = tid; p < npx; p += BLOCK) {
      const double v = ld_agent(&S.x[p]);
      acc[0] += v;
      acc[1] += v * v;
      if (v > 0.0) {
        acc[2] += v;
        acc[3] += 1.0;
      }
      mx = v > mx ? v : mx;
    }
    block_sum<BLOCK, 4>(acc, red);
    const double sx = acc[0], sxx = acc[1], s0 = acc[2], npos = acc[3];
    const double vmax = block_max(mx, red);
    const bool chaos_ok = (sx > 0.0) && (npos >= 4.0);

    // other windows
    for (int k = 1; k < K; ++k) {
      for (int p = tid; p < npx; p += BLOCK) S.y[p] = 0.0;
      __threadfence();
      __syncthreads();
      scatter_window<FMT>(hits, lo[w0 + k], hi[w0 + k], S.y);
      __threadfence();
      __syncthreads();
      double a2[4] = {0.0, 0.0, 0.0, 0.0};
      for (int p = tid; p < npx; p += BLOCK) {
        const double y = ld_agent(&S.y[p]);
        const double x = ld_agent(&S.x[p]);
        a2[0] += y;
        a2[1] += y * y;
        a2[2] += x * y;
        if (x > 0.0) a2[3] += y;
      }
      block_sum<BLOCK, 4>(a2, red);
      if (tid == 0) {
        kst[0 * MAXK_DENSE + k] = a2[3];
        kst[1 * MAXK_DENSE + k] = a2[0];
        kst[2 * MAXK_DENSE + k] = a2[1];
        kst[3 * MAXK_DENSE + k] = a2[2];
      }
    }
    __syncthreads();

    double chaos_raw = NAN;
    if (chaos_ok) {
      const int nr = P.nrows, nc = P.ncols;
      for (int p = tid; p < npx; p += BLOCK) S.L8[p] = (uint8_t)level_of(ld_agent(&S.x[p]), vmax, P);
      __syncthreads();
      for (int p = tid; p < npx; p += BLOCK) {  // dilation with the 4-cross (outside = 0)
        const int r = p / nc, c = p - r * nc;
        int d = S.L8[p];
        if (r > 0) d = max(d, (int)S.L8[p - nc]);
        if (r + 1 < nr) d = max(d, (int)S.L8[p + nc]);
        if (c > 0) d = max(d, (int)S.L8[p - 1]);
        if (c + 1 < nc) d = max(d, (int)S.L8[p + 1]);
        S.T8[p] = (uint8_t)d;
      }
      __syncthreads();
      for (int p = tid; p < npx; p += BLOCK) {  // erosion with the 3x3 box
        const int r = p / nc, c = p - r * nc;
        int e = 1 << 20;
        for (int a = -1; a <= 1; ++a)
          for (int b = -1; b <= 1; ++b) {
            const int rr = r + a, cc = c + b;
            if (rr < 0 || rr >= nr || cc < 0 || cc >= nc) {
              if (!P.erosion_border) e = 0;
              continue;
            }
            e = min(e, (int)S.T8[rr * nc + cc]);
          }
        if (e >= (1 << 20)) e = 0;
        S.E8[p] = (uint8_t)e;
        if (e >= 1) {
          const int idx = atomicAdd(&sh_ctr[0], 1);
          S.elist[idx] = (uint32_t)p;
          S.par[p] = (uint32_t)p;
          atomicMax(&sh_ctr[1], e);
        }
      }
      __threadfence();
      __syncthreads();
      const int m = sh_ctr[0], emax = sh_ctr[1];
      double esum = 0.0, wsum = 0.0;
      for (int i = tid; i < m; i += BLOCK) esum += (double)S.E8[S.elist[i]];
      for (int t = emax; t >= 1; --t) {
        for (int i = tid; i < m; i += BLOCK) {
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
      block_sum<BLOCK, 2>(a3, red);
      chaos_raw = 1.0 - (a3[0] - a3[1]) / (double)P.nlevels / npos;
    } else {
      flags |= SMG_ION_CHAOS_NAN;
    }

    if (tid == 0) {
      double t[MAXK_DENSE], s[MAXK_DENSE], sy[MAXK_DENSE], syy[MAXK_DENSE], sxy[MAXK_DENSE];
      for (int k = 0; k < K; ++k) {
        t[k] = theor[w0 + k];
        if (k == 0) {
          s[k] = s0;
          sy[k] = syy[k] = sxy[k] = 0.0;
        } else {
          s[k] = kst[0 * MAXK_DENSE + k];
          sy[k] = kst[1 * MAXK_DENSE + k];
          syy[k] = kst[2 * MAXK_DENSE + k];
          sxy[k] = kst[3 * MAXK_DENSE + k];
        }
      }
      finalize_ion(K, t, s, sx, sxx, sy, syy, sxy, (double)npx, chaos_raw, ion, flags, oc, osp, osc, omsm,
                   oflags);
    }
    __syncthreads();
  }
}

__global__ void list_all_kernel(uint32_t* list, uint32_t* count, const int64_t* ion_order, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) list[i] = (uint32_t)(ion_order ? ion_order[i] : i);
  if (i == 0) *count = (uint32_t)n;
}

static constexpr int DENSE_SLOTS = 256;
static constexpr size_t WS_HEADER = 256;
// LDS-path geometries: the main pass (two 512-thread workgroups per CU) and the big-ion pass over its
// rejects (one 1024-thread workgroup per CU with the whole LDS)
#ifndef SMG_MAIN_CFG
#define SMG_MAIN_CFG 512, 8, 4, 4
#endif
// main LDS pass: threads, principal points per thread, chunk points per thread, min waves per SIMD
static constexpr int MAIN_CFG[4] = {SMG_MAIN_CFG};
static constexpr int MAIN_BLOCK = MAIN_CFG[0], MAIN_RMAX = MAIN_CFG[1], MAIN_RC = MAIN_CFG[2],
                     MAIN_WPE = MAIN_CFG[3];
static constexpr int BIG_BLOCK = 1024, BIG_RMAX = 8, BIG_RC = 4;
static constexpr size_t MAIN_LDS = 80 * 1024, BIG_LDS = 160 * 1024 - 512;

static size_t ws_bytes_for(int64_t n_ions, int npx) {
  return WS_HEADER + 2 * al16((size_t)n_ions * 4) + (size_t)DENSE_SLOTS * dense_slot_bytes(npx);
}

static LdsLayout main_layout(int npx, int vb) { return lds_layout(npx, vb, MAIN_BLOCK / WAVE, MAIN_BLOCK * MAIN_RMAX, MAIN_LDS); }
static LdsLayout big_layout(int npx, int vb) { return lds_layout(npx, vb, BIG_BLOCK / WAVE, BIG_BLOCK * BIG_RMAX, BIG_LDS); }

template <int FMT>
static int launch_metrics(Hits<FMT> hits, const int64_t* lo, const int64_t* hi, const int64_t* ion_off,
                          const double* theor, const int64_t* ion_order, int64_t n_ions, const Params& P,
                          double* oc, double* osp, double* osc, double* omsm, uint32_t* oflags,
                          unsigned char* ws, hipStream_t st) {
  // header: [0] count A, [1] cursor A, [2] count B, [3] cursor B
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ws);
  uint32_t* list_a = reinterpret_cast<uint32_t*>(ws + WS_HEADER);
  uint32_t* list_b = reinterpret_cast<uint32_t*>(ws + WS_HEADER + al16((size_t)n_ions * 4));
  unsigned char* slots = ws + WS_HEADER + 2 * al16((size_t)n_ions * 4);
  const size_t slot_bytes = dense_slot_bytes(P.npx);
  SMG_HIP(hipMemsetAsync(ws, 0, WS_HEADER, st));
  const int vb = FMT == SMG_HITS_PACKED_F32 ? 4 : 8;
  LdsLayout LM = main_layout(P.npx, vb);
  LdsLayout LB = big_layout(P.npx, vb);
  const bool lds_ok = P.npx <= NPX_LDS_MAX && LM.cap >= 256;
  if (lds_ok) {
    auto k1 = &ion_lds_kernel<FMT, MAIN_BLOCK, MAIN_RMAX, MAIN_RC, MAIN_WPE>;
    SMG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k1), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)LM.bytes));
    hipLaunchKernelGGL(k1, dim3((unsigned)n_ions), dim3(MAIN_BLOCK), LM.bytes, st, hits, lo, hi, ion_off, theor,
                       ion_order, n_ions, P, LM, oc, osp, osc, omsm, oflags, list_a, hdr + 0);
    SMG_LAUNCH_CHECK();
    if (LB.cap > LM.cap) {
      auto k2 = &ion_lds_list_kernel<FMT, BIG_BLOCK, BIG_RMAX, BIG_RC>;
      SMG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k2), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)LB.bytes));
      const int nwg = (int)(n_ions < 256 ? n_ions : 256);
      hipLaunchKernelGGL(k2, dim3((unsigned)nwg), dim3(BIG_BLOCK), LB.bytes, st, hits, lo, hi, ion_off, theor,
                         list_a, hdr + 0, hdr + 1, P, LB, oc, osp, osc, omsm, oflags, list_b, hdr + 2);
      SMG_LAUNCH_CHECK();
    } else {
      SMG_HIP(hipMemcpyAsync(list_b, list_a, (size_t)n_ions * 4, hipMemcpyDeviceToDevice, st));
      SMG_HIP(hipMemcpyAsync(hdr + 2, hdr + 0, 4, hipMemcpyDeviceToDevice, st));
    }
  } else {
    hipLaunchKernelGGL(list_all_kernel, dim3((unsigned)((n_ions + 255) / 256)), dim3(256), 0, st, list_b, hdr + 2,
                       ion_order, n_ions);
    SMG_LAUNCH_CHECK();
  }
  const int nslots = (int)(n_ions < DENSE_SLOTS ? n_ions : DENSE_SLOTS);
  hipLaunchKernelGGL(ion_dense_kernel<FMT>, dim3((unsigned)nslots), dim3(BLOCK), 0, st, hits, lo, hi, ion_off,
                     theor, n_ions, P, list_b, hdr + 2, hdr + 3, slots, slot_bytes, oc, osp, osc, omsm, oflags);
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

int smg_ion_metrics_workspace_size(int64_t n_ions, int32_t nrows, int32_t ncols, size_t* bytes) {
  SMG_CHECK_ARG(bytes && n_ions >= 0 && nrows > 0 && ncols > 0, "bad arguments");
  SMG_CHECK_ARG((int64_t)nrows * ncols < (1ll << 31), "image too large");
  *bytes = ws_bytes_for(n_ions, nrows * ncols);
  return SMG_OK;
}

int smg_ion_metrics(int32_t hit_format, const void* hits, const double* hit_vals, const int64_t* lo,
                    const int64_t* hi, const int64_t* ion_win_off, const double* theor_int,
                    const int64_t* ion_order, int64_t n_ions, int32_t nrows, int32_t ncols, int32_t nlevels,
                    double q, int32_t do_preprocessing, int32_t connectivity, int32_t erosion_border,
                    double* out_chaos, double* out_spatial, double* out_spectral, double* out_msm,
                    uint32_t* out_flags, void* workspace, size_t workspace_bytes, void* stream) {
  (void)q;
  SMG_CHECK_ARG(n_ions >= 0 && n_ions < (1ll << 31), "n_ions out of range");
  if (n_ions == 0) return SMG_OK;
  SMG_CHECK_ARG(nrows > 0 && ncols > 0 && (int64_t)nrows * ncols < (1ll << 31), "bad image shape");
  SMG_CHECK_ARG(nlevels >= 1 && nlevels <= 254, "nlevels must be in [1, 254]");
  SMG_CHECK_ARG(connectivity == 4 || connectivity == 8, "connectivity must be 4 or 8");
  SMG_CHECK_ARG(erosion_border == 0 || erosion_border == 1, "erosion_border must be 0 or 1");
  SMG_CHECK_ARG(hit_format == SMG_HITS_PACKED_F32 || hit_format == SMG_HITS_SPLIT_F64, "bad hit_format");
  SMG_CHECK_ARG(lo && hi && ion_win_off && theor_int && out_chaos && out_spatial && out_spectral && out_msm &&
                    out_flags && workspace,
                "null pointer");
  if (do_preprocessing) {
    set_error("do_preprocessing (q-percentile hot-spot clip) is not implemented on the device path yet");
    return SMG_ERR_UNSUPPORTED;
  }
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
  unsigned char* ws = reinterpret_cast<unsigned char*>(workspace);
  hipStream_t st = as_stream(stream);
  if (hit_format == SMG_HITS_PACKED_F32) {
    SMG_CHECK_ARG(hits != nullptr, "null hits");
    Hits<SMG_HITS_PACKED_F32> h{reinterpret_cast<const uint64_t*>(hits), nullptr};
    return launch_metrics<SMG_HITS_PACKED_F32>(h, lo, hi, ion_win_off, theor_int, ion_order, n_ions, P, out_chaos,
                                               out_spatial, out_spectral, out_msm, out_flags, ws, st);
  }
  SMG_CHECK_ARG(hits != nullptr && hit_vals != nullptr, "null hits");
  Hits<SMG_HITS_SPLIT_F64> h{reinterpret_cast<const uint32_t*>(hits), hit_vals};
  return launch_metrics<SMG_HITS_SPLIT_F64>(h, lo, hi, ion_win_off, theor_int, ion_order, n_ions, P, out_chaos,
                                            out_spatial, out_spectral, out_msm, out_flags, ws, st);
}

}  // extern "C"
