// Sparse-set main pass (ion_sparse_kernel): the fused imaging + MSM scoring of ion_pipe_kernel (smg_metrics.hip)
// with a per-ion LDS footprint that does not grow with the image.
//
// Replaces, in frulo/SM_distributed (the same rows as ion_pipe_kernel):
//   formula_imager_segm.py:84-92   per-window COO construction   (_gen_iso_images)
//   formula_img_validator.py:72-84 compute(): spectral / spatial / chaos (pyImagingMSpec / cpyImagingMSpec restated)
//
// Why: ion_pipe_kernel keeps the principal image as an image-sized presence bitmap + rank prefix (39 KB at 500x500
// px) plus f64 values: 78 KB per 512-thread workgroup, two per CU.  The same code at 256 threads and four
// workgroups per CU ran 1.47x faster where its LDS fits (profiles/round5/r5_occupancy_ab.txt).  This kernel gets
// there at 500x500 px: 40,448 B per 256-thread workgroup, four per CU.
//
// Per-ion structures (LDS):
//  * entries: the principal window's points grouped by bucket (a counting sort: bucket counts, their scan, each point
//    at its bucket's arrival slot), one u32 key per point, pixel << 12 | window position; bit 31 marks every point
//    after the first of its pixel (a "hole": coo.toarray() sums it into the first);
//  * dir: a bucket directory over 2^bs-pixel buckets (<= 1024 of them): entries [dir[b], dir[b+1]) hold bucket b's
//    points.  A pixel's entry (its first point: lowest window position) is found by a short scan of its bucket;
//  * values: f32 per entry (the packed hits carry f32 intensities, so a single point's value is exact); a pixel
//    with several points keeps its f64 sum -- summed in window order, as coo.toarray() adds them -- in a side table
//    its entry points to;
//  * a direct-mapped filter F (bit p mod 2^16 for principal pixel p, 8 KB) answers the tail stream's membership test
//    with one LDS read; its positives (~2% false at 500x500 px) are resolved exactly after the stream, as
//    ion_pipe_kernel resolves its parked principal hits;
//  * chaos: the level index per entry (u8); the 7x7 screen reads presence rows from F where F is exact (images up to
//    2^16 pixels), else from band bitmaps of image rows rebuilt in the LDS; candidates' exact eL and the Kruskal pass
//    look pixels up in the directory / a candidate hash, never in an image-sized array.
// Everything else (software pipeline with counted waits, the tail stream of window-aligned 64-point groups with
// parked events, the flagged-point lists and table, the threshold-decomposition chaos, the record for
// ion_finalize_kernel) is ion_pipe_kernel's.
#include <type_traits>

#include "smg_common.hpp"
#include "smg_ion.hpp"

namespace smg {

#ifdef SMG_STAMPS
__device__ unsigned long long g_sp_stamps[16];
#define SP_STAMP_DECL()                                            \
  __shared__ unsigned long long _sacc[16];                         \
  unsigned long long _st0 = 0, _st1 = 0;                           \
  if (threadIdx.x == 0) {                                          \
    for (int _i = 0; _i < 16; ++_i) _sacc[_i] = 0;                 \
    _st0 = __builtin_amdgcn_s_memtime();                           \
  }
#define SP_STAMP(i)                                                \
  do {                                                             \
    if (threadIdx.x == 0) {                                        \
      _st1 = __builtin_amdgcn_s_memtime();                         \
      _sacc[i] += _st1 - _st0;                                     \
      _st0 = _st1;                                                 \
    }                                                              \
  } while (0)
#define SP_STAMP_FLUSH()                                           \
  do {                                                             \
    if (threadIdx.x == 0)                                          \
      for (int _i = 0; _i < 16; ++_i) atomicAdd(&g_sp_stamps[_i], _sacc[_i]); \
  } while (0)
// wave 0's cycles inside the tail stream's counted waits (part of the tail-stream phase), in slot 12
#define SP_WAIT_BEGIN() const unsigned long long _tw0 = __builtin_amdgcn_s_memtime()
#define SP_WAIT_END()                                              \
  do {                                                             \
    if (threadIdx.x == 0) _sacc[12] += __builtin_amdgcn_s_memtime() - _tw0; \
  } while (0)
// wave 0's cycles in a marked region (inside a phase) into slot i (13: the marked events' resolution, 14: the
// in-place event handling inside the tail stream, 15: the tail stream's refills)
#define SP_MARK_BEGIN(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define SP_MARK_END(v, i)                                          \
  do {                                                             \
    if (threadIdx.x == 0) _sacc[i] += __builtin_amdgcn_s_memtime() - v; \
  } while (0)
#else
#define SP_STAMP_DECL()
#define SP_STAMP(i)
#define SP_STAMP_FLUSH()
#define SP_WAIT_BEGIN()
#define SP_WAIT_END()
#define SP_MARK_BEGIN(v)
#define SP_MARK_END(v, i)
#endif

namespace {

#ifndef SMG_SP_RC
// tail points per thread per chunk (four chunks in flight): 1 since round 6 (ion stage 25.80 -> 25.47 ms at config 3,
// profiles/round6/r6spv2_*, r6spv3_*; 3: 26.41 ms)
#define SMG_SP_RC 1
#endif
// timing ablations (wrong results; diagnostic builds only): 1 no chaos, 2 no tail stream, 4 no levels, 8 no chaos
// pass B (no candidates), 16 no band bitmaps, 32 no chaos screen, 64 no eL / Kruskal, 128 no collision scans
#ifndef SMG_SP_ABL
#define SMG_SP_ABL 0
#endif
// The points that may share a pixel with another point of the principal window: 1 (round 6) its duplicate-candidate
// points (the hit's flag: every pair of points of one pixel inside a window carries it; ~1.2% of the points at config
// 3, against ~5% whose filter bit was set twice), 0 the filter's collision bits (round 5; A/B: 27.15 vs 26.46 ms for
// the ion stage at config 3, profiles/round6/r6var1_variants.txt)
#ifndef SMG_SP_DUPCOLL
#define SMG_SP_DUPCOLL 1
#endif
#ifndef SMG_SP_EVB
#define SMG_SP_EVB 1  // rounds of 64 listed tail events resolved together (their points read again together)
#endif
constexpr int SP_EVB = SMG_SP_EVB;
// geometry (diagnostic variants override it): principal points per thread, resident workgroups per CU (also the
// launch bound's waves per SIMD), LDS bytes per workgroup, filter words, side-table entries
#ifndef SMG_SP_RMAX
#define SMG_SP_RMAX 10
#endif
#ifndef SMG_SP_WGPCU
#define SMG_SP_WGPCU 4
#endif
// round 6: a 2^16-bit filter (half the tail stream's false positives; ion stage 26.46 -> 25.97 ms at config 3,
// profiles/round6/r6var3_variants.txt), paid for by a 48-entry side table (the principal windows of config 3 have at most
// 38 pixels with two or more points), f32 deferred values and the whole 40 KiB of LDS a workgroup can have at four per CU
#ifndef SMG_SP_LDS
#define SMG_SP_LDS 40960
#endif
#ifndef SMG_SP_FWORDS
#define SMG_SP_FWORDS 2048
#endif
#ifndef SMG_SP_HASH_AT_F
#define SMG_SP_HASH_AT_F 1
#endif
#ifndef SMG_SP_SIDE
#define SMG_SP_SIDE 48
#endif
// deferred flagged tail points' values as f32 (exact: packed hits carry f32 intensities) instead of f64
#ifndef SMG_SP_DV32
#define SMG_SP_DV32 1
#endif
using SpDv = std::conditional_t<SMG_SP_DV32 != 0, float, double>;
constexpr int SP_BLOCK = 256, SP_RMAX = SMG_SP_RMAX, SP_RC = SMG_SP_RC, SP_WPE = SMG_SP_WGPCU,
              SP_WGPCU = SMG_SP_WGPCU;
constexpr int SP_NW = SP_BLOCK / WAVE;
constexpr int SP_CAPC = SP_BLOCK * SP_RMAX;  // principal points per ion (more: the big-ion pass)
constexpr int SP_NBMAX = 1024;               // bucket directory entries
constexpr int SP_FWORDS = SMG_SP_FWORDS;     // Bloom filter: 2^16 bits
constexpr int SP_DSEG = 64;                  // deferred flagged tail points per wave
constexpr int SP_DTBL = 256;                 // their (pixel, window)-keyed sums
constexpr int SP_SIDE = SMG_SP_SIDE;         // f64 sums of pixels with >= 2 principal points
constexpr int SP_CLW = 2 * WAVE;               // colliding principal points listed per wave
constexpr int SP_EVCAP = 192;               // tail events listed per wave (resolved when it fills)
constexpr int SP_CCAP = 768;                 // chaos survivors + candidates
constexpr int SP_HSZ = 2048;                 // Kruskal: candidate hash
constexpr int SP_BMAX = 128;                 // points per bucket (more: the big-ion pass)
constexpr uint32_t SP_HOLE = 0x80000000u;
constexpr uint32_t SP_SIDEREF = 0xFFF00000u;  // an f32 NaN pattern: the entry's value is side[w & 0xFFFFF]
constexpr uint32_t SP_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t SP_LDS_BYTES = SMG_SP_LDS;  // 4 x 40,960 B = 160 KiB: four workgroups per CU
enum { S_NE = 0, S_EMAX, S_ABORT, S_SIDE, S_NEXT, S_MAXB, S_NCTR = 8 };

constexpr uint32_t c16(uint32_t x) { return (x + 15u) & ~15u; }

// LDS carve (bytes).  A persistent part, then a region U with two views: the principal / tail view (Bloom filter,
// values, bucket counters inside the values' space, flagged-point lists and table, side sums) and the chaos view (the
// filter, still read; the candidate hash + union-find in the values' space; the survivor / candidate lists at U's
// end).  The end-of-ion clear zeroes the filter and the counters only: the chaos list stays intact for wave 0's
// few-candidate Kruskal while the other waves clear.
struct SpLay {
  static constexpr uint32_t o_ekey = 0;
  static constexpr uint32_t o_L = o_ekey + SP_CAPC * 4;
  static constexpr uint32_t o_dir = c16(o_L + SP_CAPC);
  static constexpr uint32_t o_part = c16(o_dir + (SP_NBMAX + 2) * 2);
  static constexpr uint32_t o_red = c16(o_part + MAXK * SP_NW * 4 * 8);
  static constexpr uint32_t o_ctr = c16(o_red + 8 * SP_NW * 8);
  static constexpr uint32_t o_wsc = c16(o_ctr + S_NCTR * 4);
  static constexpr uint32_t o_desc = c16(o_wsc + SP_NW * 4);
  static constexpr uint32_t o_U = c16(o_desc + 2 * 384);
  // principal / tail view
  static constexpr uint32_t o_F = o_U;
  static constexpr uint32_t o_evals = o_F + SP_FWORDS * 4;
  static constexpr uint32_t o_cnt = o_evals;  // bucket counters: build only (the values are written after)
  static constexpr uint32_t o_dkey = c16(o_evals + SP_CAPC * 4);
  static constexpr uint32_t o_coll = o_dkey;  // filter collisions: build only (the tail's lists are written after)
  static constexpr uint32_t o_dval = c16(o_dkey + SP_NW * SP_DSEG * 4);
  static constexpr uint32_t o_dcnt = c16(o_dval + SP_NW * SP_DSEG * sizeof(SpDv));
  static constexpr uint32_t o_tkey = c16(o_dcnt + SP_NW * 4);
  static constexpr uint32_t o_tval = c16(o_tkey + SP_DTBL * 4);
  static constexpr uint32_t o_side = c16(o_tval + SP_DTBL * 8);  // read until the levels are computed
  static constexpr uint32_t o_tend = c16(o_side + SP_SIDE * 8);
  // colliding points' work lists (entries phase): behind the collision bits, or at their place without them
  static constexpr uint32_t o_clw = SMG_SP_DUPCOLL ? o_dkey : c16(o_coll + SP_FWORDS * 4);
  // chaos view
  static constexpr uint32_t o_cel = SP_LDS_BYTES - SP_CCAP;
  static constexpr uint32_t o_clist = o_cel - SP_CCAP * 4;
  static constexpr uint32_t o_wsurv = o_clist - SP_NW * WAVE * 4;  // per-wave survivor lists (chaos screen)
  static constexpr uint32_t o_band = o_U;                          // band bitmaps (images above 2^16 pixels)
  static constexpr int band_bits = (int)(o_wsurv - o_band) * 8;
  static_assert(o_band % 16 == 0, "band bitmaps are zeroed as uint4");
  // the Kruskal's candidate hash: after the screen (which reads F for images up to SP_FWORDS * 32 pixels), so it may
  // start at F (SMG_SP_HASH_AT_F) or behind it
  static constexpr uint32_t o_hash = SMG_SP_HASH_AT_F ? o_F : o_evals;
  static constexpr uint32_t o_par = o_hash + SP_HSZ * 4;
  static_assert(o_tend <= SP_LDS_BYTES, "principal / tail view fits");
  static_assert(o_cnt + SP_NBMAX * 4 <= o_dkey, "bucket counters inside the values' space");
  static_assert(SMG_SP_DUPCOLL || (o_coll + SP_FWORDS * 4 <= o_tval + 8 * 8 &&
                                   o_coll + SP_FWORDS * 4 <= SP_LDS_BYTES - SP_CCAP * 5 - SP_NW * WAVE * 4),
                "collision bits below the chaos lists");
  static_assert(o_hash >= o_F && o_par + SP_CCAP * 4 <= o_wsurv, "hash + union-find below the lists");
  static_assert(o_F + SP_FWORDS * 4 <= o_wsurv && o_cnt + SP_NBMAX * 4 <= o_wsurv, "cleared words below the lists");
  static_assert(SP_LDS_BYTES % 512 == 0 && SP_WGPCU * SP_LDS_BYTES <= 160 * 1024, "SP_WGPCU workgroups per CU");
  static_assert(SP_NW == 4, "the chaos screen merges four partial survivor lists");
  static_assert(o_clw + SP_NW * SP_CLW * 4 <= o_side, "collision work lists between the collision bits and the side table");
  static_assert(SP_NW * SP_EVCAP * 4 == SP_DTBL * 12 && o_tval == o_tkey + SP_DTBL * 4 && SP_EVCAP % WAVE == 0,
                "the event lists tile the dup table's space");
  static_assert(o_U + SP_NW * WAVE * 8 <= o_wsurv && SP_NW * WAVE * 8 <= SP_FWORDS * 4 && SP_NW * WAVE >= 2 * WAVE, "eL row blocks over the screen's bitmaps, the small Kruskal's hash over the survivor lists");
};

struct SpGeo {
  int32_t bs;         // bucket = pixel >> bs
  int32_t band_rows;  // image rows screened per chaos band (images above 2^16 pixels)
};

// the number of lanes below this one whose bit is set in the wave mask m (v_mbcnt)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// the filter F: bit p mod 2^16 for every principal pixel p (direct-mapped: a row segment of pixels is a run of bits, so
// the chaos pre-filter reads it too)
__device__ __forceinline__ uint32_t sp_fword(uint32_t p) { return (p >> 5) & (uint32_t)(SP_FWORDS - 1); }
__device__ __forceinline__ uint32_t sp_fmask(uint32_t p) { return 1u << (p & 31u); }

__device__ __forceinline__ double sp_val(uint32_t w, const double* side) {
  return (w & 0xFFF00000u) == SP_SIDEREF ? side[w & 0xFFFFFu] : (double)__uint_as_float(w);
}

// entry index of principal pixel p (-1: not in the principal image): among its bucket's entries of pixel p (keys
// pixel << 12 | window position, in arrival order) the one with the lowest window position, the pixel's first point,
// which holds the pixel's value (a marked hole has bit 31 set and never matches)
__device__ __forceinline__ int sp_lookup(const uint32_t* ekey, const uint16_t* dir, uint32_t p, int bs) {
  const uint32_t b = p >> bs;
  const int s0 = dir[b], e = dir[b + 1];
  int r = -1;
  uint32_t best = 0xFFFFFFFFu;
  // two entries per step, read together (one LDS round trip per pair: the loop is bound by their latency); the
  // second of a bucket with an odd count is the next bucket's or the level bytes' and is not tested
  for (int i = s0; i < e; i += 2) {
    const uint32_t w0 = ekey[i], w1 = ekey[i + 1];
    if ((w0 >> 12) == p && w0 < best) {
      best = w0;
      r = i;
    }
    if (i + 1 < e && (w1 >> 12) == p && w1 < best) {
      best = w1;
      r = i + 1;
    }
  }
  return r;
}

template <int LB, int RMAX, int RC, int WPE>
__global__ void __launch_bounds__(LB, WPE) ion_sparse_kernel(
    Hits<SMG_HITS_PACKED_F32> hits, IonDesc* __restrict__ desc, Sched S, Params P, SpGeo G, double* __restrict__ oc,
    double* __restrict__ osp, double* __restrict__ osc, double* __restrict__ omsm, uint32_t* __restrict__ oflags,
    uint32_t* __restrict__ rej_list, uint32_t* __restrict__ rej_count SMG_CHK_PARAM) {
  using H = Hits<SMG_HITS_PACKED_F32>;
  using Reg = uint64_t;
  constexpr int BLOCK = LB;
  constexpr int NW = LB / WAVE;
  constexpr int GPC = BLOCK * RC / 64;  // 64-point groups per chunk
  constexpr int CAPC = BLOCK * RMAX;
  static_assert(CAPC == SP_CAPC && NW == SP_NW, "layout geometry");
  static_assert(RMAX >= 2 * RC, "principal slots double as two tail buffers");
  static_assert(NW * SP_DSEG == BLOCK, "one deferred-list slot per thread");
  static_assert(SP_NBMAX == 16 * WAVE, "sixteen bucket counters per lane of wave 0");
  static_assert(CAPC <= 4096, "window positions in 12 bits of the sort key");
  using LY = SpLay;
  // static LDS (the kernel's only variable besides the stamps' accumulators): its offset is a compile-time constant,
  // so LDS addresses fold into the instructions' offsets (dynamic LDS costs an add of a relocated base per access)
  __shared__ __attribute__((aligned(16))) unsigned char smem[SP_LDS_BYTES];
  uint32_t* ekey = reinterpret_cast<uint32_t*>(smem + LY::o_ekey);
  uint8_t* L8 = smem + LY::o_L;
  uint16_t* dir = reinterpret_cast<uint16_t*>(smem + LY::o_dir);
  double* part = reinterpret_cast<double*>(smem + LY::o_part);  // [MAXK][NW][4]: s_k, sy, syy, sxy
  double* red = reinterpret_cast<double*>(smem + LY::o_red);
  double* side = reinterpret_cast<double*>(smem + LY::o_side);
  int* ctr = reinterpret_cast<int*>(smem + LY::o_ctr);
  IonDesc* dsl = reinterpret_cast<IonDesc*>(smem + LY::o_desc);
  uint32_t* F = reinterpret_cast<uint32_t*>(smem + LY::o_F);
  uint32_t* evals = reinterpret_cast<uint32_t*>(smem + LY::o_evals);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem + LY::o_cnt);
  uint32_t* coll = reinterpret_cast<uint32_t*>(smem + LY::o_coll);
  uint32_t* dkey = reinterpret_cast<uint32_t*>(smem + LY::o_dkey);
  SpDv* dval = reinterpret_cast<SpDv*>(smem + LY::o_dval);
  int* dcnt = reinterpret_cast<int*>(smem + LY::o_dcnt);
  uint32_t* tkey = reinterpret_cast<uint32_t*>(smem + LY::o_tkey);
  double* tval = reinterpret_cast<double*>(smem + LY::o_tval);
  uint32_t* clist = reinterpret_cast<uint32_t*>(smem + LY::o_clist);
  uint8_t* cel = smem + LY::o_cel;
  uint32_t* wsurv = reinterpret_cast<uint32_t*>(smem + LY::o_wsurv) + (threadIdx.x >> 6) * WAVE;
  int* wsc = reinterpret_cast<int*>(smem + LY::o_wsc);  // the chaos screen's partial survivor counts per wave
  uint32_t* band = reinterpret_cast<uint32_t*>(smem + LY::o_band);
  uint32_t* htab = reinterpret_cast<uint32_t*>(smem + LY::o_hash);
  uint32_t* par = reinterpret_cast<uint32_t*>(smem + LY::o_par);

  // tid and lane are laundered at the top of every ion iteration (as in ion_pipe_kernel)
  int tid = threadIdx.x;
  int lane = tid & 63;
  const int wid = uni(tid >> 6);
  const int bs = G.bs;
  const int nr = P.nrows, ncl = P.ncols;

  // register buffers: tail chunks through a ring of four (pa, pb, pc, pd); the next ion's principal window arrives
  // in pc, pd, pe (RMAX slots), which become tail buffers once the principal build has consumed them
  constexpr int RE = RMAX - 2 * RC > 0 ? RMAX - 2 * RC : 1;
  Reg pa[RC], pb[RC], pc[RC], pd[RC], pe[RE];
#pragma unroll
  for (int j = 0; j < RC; ++j) pa[j] = pb[j] = pc[j] = pd[j] = 0ull;
#pragma unroll
  for (int j = 0; j < RE; ++j) pe[j] = 0ull;
  auto hs = [&](int j) -> Reg& { return j < RC ? pc[j] : (j < 2 * RC ? pd[j - RC] : pe[j - 2 * RC]); };
  // every slot issues exactly one load (clamped to the window's last point, or hit 0 for an empty window), so that
  // the counted waits hold on every path
  auto issue_principal = [&](const IonDesc* D) {
    const int n0 = uni(D->end[0]);
    const int64_t a = uni64(D->base[0]);
#pragma unroll
    for (int j = 0; j < RMAX; ++j) {
      const int i = tid + j * BLOCK;
      const int64_t idx = n0 > 0 ? a + min(i, n0 - 1) : 0;
#ifdef SMG_CHECK
      chk_load(CK, D->ion, 0, idx, n0 <= 0);
#endif
      ld8_async_v(hs(j), hits.h + idx);
    }
  };
  // tail chunk c: groups [c*GPC, (c+1)*GPC); slot j of wave w holds group c*GPC + j*NW + w; exactly RC loads
  auto issue_chunk = [&](const IonDesc* D, int c, Reg (&buf)[RC]) {  // (descriptor fields and group uniform: scalar)
    const int ng = uni(D->ngroups);
    int gsv[MAXK];
#pragma unroll
    for (int kk = 2; kk < MAXK; ++kk) gsv[kk] = uni(D->gs[kk]);
#pragma unroll
    for (int j = 0; j < RC; ++j) {
      const int Gi = c * GPC + j * NW + wid;
      int k = 1;
#pragma unroll
      for (int kk = 2; kk < MAXK; ++kk) k += (Gi >= gsv[kk]) ? 1 : 0;
      const int64_t bk = uni64(D->base[k]);
      const int ek = uni(D->end[k]);
      const int64_t idx = Gi < ng ? bk + (int64_t)Gi * 64 + min(lane, ek - Gi * 64 - 1) : 0;
#ifdef SMG_CHECK
      chk_load(CK, D->ion, k, idx, Gi >= ng);
#endif
      ld8_async_v(buf[j], hits.h + idx);
    }
  };

  SP_STAMP_DECL();
  // the Bloom filter and the bucket counters start zeroed (here, then at the end of every ion that used them, by the
  // waves other than wave 0 while it writes the record); the counters too
  auto clear_fc = [&](int t0, int nt) {
    uint4* zf = reinterpret_cast<uint4*>(F);
    uint4* zc = reinterpret_cast<uint4*>(cnt);
    uint4* zl = reinterpret_cast<uint4*>(coll);
    for (int i = t0; i < SP_FWORDS / 4; i += nt) zf[i] = make_uint4(0, 0, 0, 0);
    for (int i = t0; i < SP_NBMAX / 4; i += nt) zc[i] = make_uint4(0, 0, 0, 0);
    if (!SMG_SP_DUPCOLL)
      for (int i = t0; i < SP_FWORDS / 4; i += nt) zl[i] = make_uint4(0, 0, 0, 0);
    if (t0 < S_NCTR && t0 != S_NEXT) ctr[t0] = 0;
  };
  // the dup table (keys all ones, values zero), cleared by each wave over the words of its own tail-event list (the
  // two share the space), so that a wave done with its stream never touches the list of one still streaming
  auto clear_table = [&]() {
#pragma unroll
    for (int q = 0; q < SP_EVCAP / WAVE; ++q) {
      const int i = wid * SP_EVCAP + q * WAVE + (int)(threadIdx.x & 63u);
      tkey[i] = i < SP_DTBL ? 0xFFFFFFFFu : 0u;
    }
  };
  clear_fc(tid, BLOCK);
  if (tid == 0) {
    int h0;
    const uint32_t t0 = sched_issue<SRC_RANGES>(S, h0);
    ctr[S_NEXT] = (int)sched_resolve<SRC_RANGES>(S, t0, h0);
  }
  __syncthreads();
  int64_t pos = -1;  // ion scored in this iteration (-1: none; the first iteration only issues loads)
  int64_t npos = uni(ctr[S_NEXT]);
  int cur = 0;
  while (true) {
    asm volatile("" : "+v"(tid));
    asm volatile("" : "+v"(lane));
    const IonDesc* D = &dsl[cur];
    IonDesc* DN = &dsl[cur ^ 1];
    // the ticket of the ion after npos, consumed after the principal build (wave 0 issues after it exactly one
    // descriptor load, then the 2*RC loads of tail chunks 2 and 3 or their stand-ins)
    uint32_t ticket = 0;
    int thome = 0;  // the XCD whose counter the ticket came from (sched_resolve)
    if (tid == 0) sched_issue_async<SRC_RANGES>(S, ticket, thome);
    uint64_t dword = 0;
    if ((tid >> 6) == 0)
      ld8_async_wave0(dword, reinterpret_cast<const uint64_t*>(desc + (npos >= 0 ? npos : 0)) +
                                 (lane < DESC_QWORDS ? lane : 0));
    bool skip = pos < 0;
    int K = 0, ion = 0, n0 = 0;
    // a reject beyond the list's capacity (impossible while every position is handed out once) is dropped, never
    // written past the list
    auto reject = [&]() {
      if (tid == 0) {
        const uint32_t r = atomicAdd(rej_count, 1u);
        if (r < S.rej_cap) rej_list[r] = (uint32_t)pos;
#ifdef SMG_CHECK
        chk(CK, r < S.rej_cap, CHK_REJ, pos, r);
#endif
      }
    };
#ifdef SMG_CHECK
    if (!skip && wid == 0) chk_claim(CK, 0, pos);
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
    const bool began = !skip;  // this ion uses the filter and the counters (cleared again at its end)
    SP_STAMP(0);

    // ---- principal image -> sorted entries, bucket directory, Bloom filter, values -------------------------------
    // the principal statistics (sum x, sum x^2, sum x[x>0], #(x>0), max) over the image's pixels, per thread in a fixed
    // order: single-point pixels from the registers, summed pixels by their first entry
    double acc[5] = {0.0, 0.0, 0.0, 0.0, -INFINITY};
    int npos_l = 0;  // #(x > 0) of this lane (acc[3] after an integer wave sum)
    auto stat = [&](double v) {
      acc[0] += v;
      acc[1] += v * v;
      if (v > 0.0) {
        acc[2] += v;
        ++npos_l;
      }
      acc[4] = v > acc[4] ? v : acc[4];
    };
    uint32_t aw[RMAX];  // a point's arrival index in its bucket, later its entry index (a register each)
#pragma unroll
    for (int j = 0; j < RMAX; ++j) aw[j] = 0u;
    auto aw_get = [&](int j) -> uint32_t { return aw[j]; };
    auto aw_set = [&](int j, uint32_t v) { aw[j] = v; };
    // the principal window was issued before this ion's tail chunks 0 and 1.  Waited on every path (a skipped
    // position has nothing older in flight; the wait only gets stricter), so that the wait dominates every use of
    // the principal registers in the separate blocks below
    vm_wait<2 * RC>(pc);
    vm_wait<2 * RC>(pd);
    vm_wait<2 * RC>(pe);
    if (!skip) {
      for (int i = tid; i < MAXK * NW * 4; i += BLOCK) part[i] = 0.0;
      bool bad = false;
#pragma unroll
      for (int j = 0; j < RMAX; ++j) {
        const int i = tid + j * BLOCK;
        if (i < n0) {
          const uint32_t p = H::pix(hs(j));
          const float v = __uint_as_float((uint32_t)(hs(j) >> 32));
          if ((v != v) || p >= (uint32_t)P.npx) {  // NaN intensities / foreign pixels: the big-ion pass (f64 values)
            bad = true;
          } else {
            // a filter bit set twice: the two points may share a pixel (only those scan their bucket below)
            if (SMG_SP_DUPCOLL) atomicOr(&F[sp_fword(p)], sp_fmask(p));
            else if (atomicOr(&F[sp_fword(p)], sp_fmask(p)) & sp_fmask(p)) atomicOr(&coll[sp_fword(p)], sp_fmask(p));
            aw_set(j, atomicAdd(&cnt[p >> bs], 1u));
          }
        }
      }
      if (bad) ctr[S_ABORT] = 1;
      __syncthreads();
      if (ctr[S_ABORT]) {
        reject();
        skip = true;
      }
    }
    if (!skip) {
      // exclusive scan of the bucket counts -> dir, and the largest bucket: wave 0 alone (16 counters per lane), one
      // barrier
      if (wid == 0) {
        const uint4* c4 = reinterpret_cast<const uint4*>(cnt) + lane * 4;
        uint32_t c[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 v = c4[q];
          c[4 * q] = v.x;
          c[4 * q + 1] = v.y;
          c[4 * q + 2] = v.z;
          c[4 * q + 3] = v.w;
        }
        uint32_t tot = 0, mx = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          tot += c[q];
          mx = max(mx, c[q]);
        }
        const int inc = wave_incl_scan_dpp((int)tot);
        uint32_t run = (uint32_t)inc - tot, d[8];
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
          const uint32_t a = run;
          run += c[q];
          d[q / 2] = a | (run << 16);
          run += c[q + 1];
        }
        uint4* dd = reinterpret_cast<uint4*>(dir) + lane * 2;
        dd[0] = make_uint4(d[0], d[1], d[2], d[3]);
        dd[1] = make_uint4(d[4], d[5], d[6], d[7]);
        if (lane == 63) dir[SP_NBMAX] = (uint16_t)inc;
        if (__ballot(mx > (uint32_t)SP_BMAX)) ctr[S_MAXB] = 1;
      }
      __syncthreads();
      if (ctr[S_MAXB]) {  // a crowded bucket (the sort below is quadratic in it): the big-ion pass
        reject();
        skip = true;
      }
    }
    SP_STAMP(1);
    if (!skip) {
      // every point's key (pixel << 12 | window position) and value at its bucket's arrival slot (entry index); its
      // hole mark (L8, until the levels overwrite it) cleared
#pragma unroll
      for (int j = 0; j < RMAX; ++j) {
        const int i = tid + j * BLOCK;
        if (i < n0) {
          const uint32_t p = H::pix(hs(j));
          const int f = (int)dir[p >> bs] + (int)aw_get(j);
          ekey[f] = (p << 12) | (uint32_t)i;
          evals[f] = (uint32_t)(hs(j) >> 32);
          L8[f] = 0;
          aw_set(j, (uint32_t)f);
        }
      }
      __syncthreads();
      // ... then each point whose filter bit was set twice scans its bucket for points of its pixel: none (a single
      // point, like every point with a filter bit of its own: its value enters the statistics), only later ones (the
      // pixel's first point: it sums them all, in window order as coo.toarray() does, into the side table), or an
      // earlier one (a hole: L8 = 1, marked in ekey after the ticket barrier).  The colliding points are listed per
      // wave (entry indices, compacted over the lanes by ballot) and scanned 64 at a time, one per lane.
      uint32_t* wcl = reinterpret_cast<uint32_t*>(smem + LY::o_clw) + wid * SP_CLW;
      auto coll_round = [&](int cnt) {  // lanes < cnt take wcl[lane] (cnt uniform)
        __builtin_amdgcn_wave_barrier();  // (the list was written by this wave's lanes)
        const bool ok = lane < cnt;
        const uint32_t f = ok ? wcl[lane] : 0u;
        const uint32_t key = ekey[f], p = key >> 12;
        int b0 = 0, b1 = 0;
        if (ok) {
          b0 = dir[p >> bs];
          b1 = dir[(p >> bs) + 1];
        }
        uint32_t st = 0u;
        for (int k = b0; k < b1; k += 2) {  // (pairs read together, as in sp_lookup)
          const uint32_t w0 = ekey[k], w1 = ekey[k + 1];
          const bool same0 = (w0 >> 12) == p, same1 = k + 1 < b1 && (w1 >> 12) == p;
          st |= (same0 && w0 < key ? 2u : 0u) | (same0 && w0 > key ? 1u : 0u);
          st |= (same1 && w1 < key ? 2u : 0u) | (same1 && w1 > key ? 1u : 0u);
        }
        if (ok) {
          const float v0 = __uint_as_float(evals[f]);
          if (st & 2u) {
            L8[f] = 1;
          } else if (st == 0u) {
            stat((double)v0);
          } else {  // the first point of a pixel with several: their sum in window order
            double sum = (double)v0;
            uint32_t last = key;
            while (true) {  // the next point of the pixel by window position
              uint32_t nk = 0xFFFFFFFFu;
              int ni = -1;
              for (int k = b0; k < b1; ++k) {
                const uint32_t w = ekey[k];
                if ((w >> 12) == p && w > last && w < nk) {
                  nk = w;
                  ni = k;
                }
              }
              if (ni < 0) break;
              sum += (double)__uint_as_float(evals[ni]);
              last = nk;
            }
            const int slot = atomicAdd(&ctr[S_SIDE], 1);
            if (slot < SP_SIDE) {
              side[slot] = sum;
              evals[f] = SP_SIDEREF | (uint32_t)slot;
            } else {
              ctr[S_ABORT] = 1;
            }
            stat(sum);
          }
        }
        __builtin_amdgcn_wave_barrier();  // (the list is rewritten after this)
      };
      int ncw = 0;  // (uniform)
#pragma unroll
      for (int j = 0; j < RMAX; ++j) {
        const int i = tid + j * BLOCK;
        bool col = false;
        if (i < n0) {
          const uint32_t p = H::pix(hs(j));
          col = !(SMG_SP_ABL & 128) &&
                (SMG_SP_DUPCOLL ? H::dup(hs(j)) : (coll[sp_fword(p)] & sp_fmask(p)) != 0u);
          if (!col) stat((double)__uint_as_float((uint32_t)(hs(j) >> 32)));  // (no other point has its pixel)
        }
        const uint64_t m = __ballot(col);
        if (m) {  // (uniform)
          if (col) wcl[ncw + (int)lanes_below(m)] = aw_get(j);
          ncw += (int)__popcll(m);
          if (ncw >= WAVE) {
            coll_round(WAVE);
            ncw -= WAVE;
            if (lane < ncw) wcl[lane] = wcl[WAVE + lane];
          }
        }
      }
      if (ncw > 0) coll_round(ncw);
    }
    // the principal registers are consumed: tail chunks 2 and 3 go in flight (or the same number of stand-in loads, so
    // that the waits below count 2*RC younger loads on every path)
    if (!skip) {
      issue_chunk(D, 2, pc);
      issue_chunk(D, 3, pd);
    } else {
#pragma unroll
      for (int j = 0; j < RC; ++j) {
        ld8_async_v(pc[j], hits.h);
        ld8_async_v(pd[j], hits.h);
      }
    }
    // the statistics' per-wave sums into red (every thread reads them after the ticket barrier)
    if (!skip) {
#pragma unroll
      for (int q = 0; q < 3; ++q) acc[q] = wave_sum_dpp(acc[q]);
      acc[3] = (double)__builtin_amdgcn_readlane(wave_incl_scan_dpp(npos_l), 63);
      acc[4] = wave_max_dpp(acc[4]);
      if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 5; ++q) red[q * NW + wid] = acc[q];
      }
    }
    SP_STAMP(2);
    // wave 0: the ticket and npos's descriptor (issued at the top of this iteration, before chunks 2 and 3 or their
    // stand-ins); the test is on the laundered tid (an exec-masked branch: scripts/check_async_regs.py's wave-0 form)
    if ((tid >> 6) == 0) {
      vm_wait1<2 * RC>(ticket);
      vm_wait1<2 * RC>(dword);
      if (tid == 0) ctr[S_NEXT] = (int)sched_resolve<SRC_RANGES>(S, ticket, thome);
      if (npos >= 0 && lane < DESC_QWORDS) reinterpret_cast<uint64_t*>(DN)[lane] = dword;
    }
    __syncthreads();
    const int64_t n2pos = uni(ctr[S_NEXT]);
    if (!skip && ctr[S_ABORT]) {  // more summed pixels than the side table holds
      reject();
      skip = true;
    }
    // the principal statistics (per-wave sums, in wave order)
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
    const bool chaos_ok = !skip && (sx > 0.0) && (npx_pos >= 4.0) && !(SMG_SP_ABL & 1);
    // the holes (L8 = 1) mark their entries (no scan reads the keys any more; a lookup before the mark sees the
    // pixel's first point anyway: it takes the lowest window position), and the other entries get their level index
    // for the chaos phase (the values' space later holds its candidate hash): computed here, while tail chunks 2 and
    // 3 are in flight
    if (!skip) {
      const bool lv = chaos_ok && !(SMG_SP_ABL & 4);
      const double rcp = lv ? 1.0 / vmax : 0.0;
      for (int i = tid; i < n0; i += BLOCK) {
        if (L8[i]) ekey[i] |= SP_HOLE;
        else if (lv) L8[i] = (uint8_t)sp_level(sp_val(evals[i], side), vmax, rcp, P);
      }
    }
    SP_STAMP(3);

    // ---- tail windows, one stream of window-aligned 64-point groups ------------------------------------------------
    if (!skip) {
      const int ng = (SMG_SP_ABL & 2) ? 0 : uni(D->ngroups);
      int curk = 1;
      int nd = 0;  // this wave's deferred flagged points (uniform)
      uint32_t* wdkey = dkey + wid * SP_DSEG;
      SpDv* wdval = dval + wid * SP_DSEG;
      int gnext = uni(D->gs[2]);
      int wend = uni(D->end[1]);
      // Events: a filter positive (the point's pixel may be principal: Σxy, Σy[x>0]) or a flagged point (summed per
      // (pixel, window) before squaring).  The stream only lists them, compacted over the wave's lanes (one list entry
      // per event, so that resolving them takes ceil(events / 64) rounds rather than the busiest lane's count); the
      // list is resolved when it fills and after the stream.  Partials: part[k][wid], written only by this wave, lanes
      // of one instruction in hardware order -- deterministic.
      // the wave's event list (t << 6 | lane, t = chunk * RC + slot), in the dup table's space (written only
      // after the stream; the filter collisions overlapping it were read before the ticket barrier)
      uint32_t* evl = tkey + wid * SP_EVCAP;
      int nev = 0;  // (uniform)
      int gsv[MAXK];
#pragma unroll
      for (int kk = 2; kk < MAXK; ++kk) gsv[kk] = uni(D->gs[kk]);
      auto add_x = [&](bool hit, int r, const Reg& h, int k) {
        if (__ballot(hit)) {
          if (hit) {
            const double x = sp_val(evals[r], side);
            const double v = H::val(h);
            double* pk = part + ((size_t)k * NW + wid) * 4;
            atomicAdd(&pk[3], x * v);
            if (x > 0.0) atomicAdd(&pk[0], v);
          }
        }
      };
      // the listed events, SP_EVB rounds of 64 together (their points read again, an L2 hit: streamed just now), in
      // list order -- stream order, then lane order
      auto resolve = [&]() {
        __builtin_amdgcn_wave_barrier();  // (the list was written by this wave's lanes)
        for (int e0 = 0; e0 < nev; e0 += SP_EVB * WAVE) {  // uniform
          Reg hq[SP_EVB];
          int kq[SP_EVB];
          bool hasq[SP_EVB];
#pragma unroll
          for (int q = 0; q < SP_EVB; ++q) {
            const int e = e0 + q * WAVE + lane;
            hasq[q] = e < nev;
            const uint32_t ent = hasq[q] ? evl[e] : 0u;
            const int t = (int)(ent >> 6);
            const int Gi = (t / RC) * GPC + (t % RC) * NW + wid;
            int k = 1;
#pragma unroll
            for (int kk = 2; kk < MAXK; ++kk) k += (Gi >= gsv[kk]) ? 1 : 0;
            kq[q] = k;
#ifdef SMG_CHECK
            if (hasq[q]) chk_load(CK, ion, k, D->base[k] + (int64_t)Gi * 64 + (ent & 63u), false);
#endif
            hq[q] = hasq[q] ? hits.h[D->base[k] + (int64_t)Gi * 64 + (ent & 63u)] : 0ull;
          }
#pragma unroll
          for (int q = 0; q < SP_EVB; ++q) {
            const Reg h = hq[q];
            const uint32_t p = H::pix(h);
            // (tested again: not in the entry; a pixel outside the image -- only a caller-supplied hit can carry one --
            // is no principal pixel and never indexes the directory)
            const bool in = hasq[q] && p < (uint32_t)P.npx && (F[sp_fword(p)] & sp_fmask(p)) != 0u;
            const int r = in ? sp_lookup(ekey, dir, p, bs) : -1;
            add_x(r >= 0, r, h, kq[q]);
            const bool dq = hasq[q] && H::dup(h);
            const uint64_t mq = __ballot(dq);
            if (mq) {
              const int e = nd + (int)lanes_below(mq);
              if (dq && e < SP_DSEG) {
                wdkey[e] = (p << 3) | (uint32_t)kq[q];
                wdval[e] = (SpDv)H::val(h);
              }
              nd += (int)__popcll(mq);
            }
          }
        }
        nev = 0;
      };
      auto process = [&](int c, Reg (&buf)[RC]) {
        uint32_t fw[RC], fm[RC];
#pragma unroll
        for (int j = 0; j < RC; ++j) {
          const uint32_t pj = H::pix(buf[j]);
          fw[j] = F[sp_fword(pj)];
          fm[j] = sp_fmask(pj);
        }
#pragma unroll
        for (int j = 0; j < RC; ++j) {
          const int Gi = c * GPC + j * NW + wid;
          if (Gi < ng) {
            while (Gi >= gnext) {  // this wave moves on to a later window (uniform)
              ++curk;
              gnext = curk + 1 < MAXK ? uni(D->gs[curk + 1]) : 0x7FFFFFFF;
              wend = uni(D->end[curk]);
            }
            const bool valid = lane < wend - Gi * 64;
            const Reg h = buf[j];
            const bool in = valid && (fw[j] & fm[j]) != 0u;
            const bool evt = in || (valid && H::dup(h));
            const uint64_t em = __ballot(evt);
            if (em) {  // (uniform)
              const uint32_t t = (uint32_t)(c * RC + j);
              if (evt) evl[nev + (int)lanes_below(em)] = (t << 6) | (uint32_t)lane;
              nev += (int)__popcll(em);
              if (nev > SP_EVCAP - WAVE) {
                SP_MARK_BEGIN(_th0);
                resolve();
                SP_MARK_END(_th0, 14);
              }
            }
          }
        }
      };
      // chunks 0 and 1 are in flight (issued during the previous iteration); later chunks one ahead (refills are
      // issued unconditionally so that exactly 3*RC loads follow each buffer's)
      // refills of this ion's later chunks: the window of the next group to load is tracked like the stream's (groups
      // only grow along a wave's issues), so that a refill reads the descriptor only when the window changes
      int ik = 1, ign = uni(D->gs[2]), iend = uni(D->end[1]);
      int64_t ibase = uni64(D->base[1]);
      auto refill = [&](int c, Reg (&buf)[RC]) {
        SP_MARK_BEGIN(_tr0);
#pragma unroll
        for (int j = 0; j < RC; ++j) {
          const int Gi = c * GPC + j * NW + wid;
          while (Gi >= ign) {  // (uniform)
            ++ik;
            ign = ik + 1 < MAXK ? uni(D->gs[ik + 1]) : 0x7FFFFFFF;
            iend = uni(D->end[ik]);
            ibase = uni64(D->base[ik]);
          }
          const int64_t idx = Gi < ng ? ibase + (int64_t)Gi * 64 + min(lane, iend - Gi * 64 - 1) : 0;
#ifdef SMG_CHECK
          chk_load(CK, ion, ik, idx, Gi >= ng);
#endif
          ld8_async_v(buf[j], hits.h + idx);
        }
        SP_MARK_END(_tr0, 15);
      };
      for (int c = 0; c * GPC < ng; c += 4) {
        {
          SP_WAIT_BEGIN();
          vm_wait<3 * RC>(pa);
          SP_WAIT_END();
        }
        process(c, pa);
        refill(c + 4, pa);
        if ((c + 1) * GPC >= ng) break;
        {
          SP_WAIT_BEGIN();
          vm_wait<3 * RC>(pb);
          SP_WAIT_END();
        }
        process(c + 1, pb);
        refill(c + 5, pb);
        if ((c + 2) * GPC >= ng) break;
        {
          SP_WAIT_BEGIN();
          vm_wait<3 * RC>(pc);
          SP_WAIT_END();
        }
        process(c + 2, pc);
        refill(c + 6, pc);
        if ((c + 3) * GPC >= ng) break;
        {
          SP_WAIT_BEGIN();
          vm_wait<3 * RC>(pd);
          SP_WAIT_END();
        }
        process(c + 3, pd);
        refill(c + 7, pd);
      }
      // the events still listed
      SP_MARK_BEGIN(_tp0);
      if (nev) resolve();
      if (lane == 0) dcnt[wid] = nd;
      SP_MARK_END(_tp0, 13);
    }
    SP_STAMP(4);
    // ---- the registers of ion b are dead: ion b+1's principal window and first two chunks go in flight
    if (npos >= 0 && desc_lds_ok(DN, CAPC)) {
      issue_principal(DN);
      issue_chunk(DN, 0, pa);
      issue_chunk(DN, 1, pb);
    }
    if (!skip) clear_table();
    __syncthreads();
    SP_STAMP(5);
    // ---- deferred flagged points: exact per-(pixel, window) sums, squared into the partials -----------------------
    if (!skip) {
      int nd_tot = 0, nd_max = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        nd_tot += dcnt[w];
        nd_max = max(nd_max, dcnt[w]);
      }
      if (nd_max > SP_DSEG) {
        reject();
        skip = true;
      } else if (nd_tot > 0) {
        if ((tid % SP_DSEG) < dcnt[tid / SP_DSEG] && !tbl_add<SP_DTBL>(tkey, tval, dkey[tid], (double)dval[tid]))
          ctr[S_ABORT] = 1;
        __syncthreads();
        if (ctr[S_ABORT]) {
          reject();
          skip = true;
        } else {
          for (int i = tid; i < SP_DTBL; i += BLOCK) {
            const uint32_t key = tkey[i];
            if (key != 0xFFFFFFFFu) {
              const double y = tval[i];
              atomicAdd(&part[(size_t)(key & 7u) * NW * 4 + 2], y * y);
            }
          }
          __syncthreads();  // (the table's space becomes the chaos lists)
        }
      }
    }
    SP_STAMP(6);

    // ---- measure_of_chaos by threshold decomposition (ion_pipe_kernel's scheme) ----------------------------------
    double chaos_raw = NAN;
    uint32_t flags = 0;
    if (!skip && chaos_ok) {
      SP_STAMP(7);
      // (i) the 7x7 screen over presence bitmaps: the filter F itself where it is exact (images up to 2^16 pixels: bit
      //     p for pixel p), else band bitmaps of image rows rebuilt in the LDS the values and the flagged-point lists
      //     leave behind (two bands at 500x500 px): the band's words zeroed, then a bit set per entry.  Pass A: a
      //     principal pixel with fewer than three principal pixels in its 7x7 (itself included) cannot own a
      //     candidate (erosion border 0); the others go to the wave's own survivor list, and pass B runs the full
      //     screen over each full list (no barrier) and over the waves' partial lists together at the range's end
      //     (after one), appending candidates (owned pixels of the dilated-covered boxes) to the chaos list.
      auto rowcv = [&](int s, int& rs, int& cs, uint32_t& cv) {
        rowcol(s, P, rs, cs);
        const int clo = 3 - cs > 0 ? 3 - cs : 0, chi = ncl - cs + 3 < 7 ? ncl - cs + 3 : 7;
        cv = ((1u << chi) - 1u) & ~((1u << clo) - 1u);
      };
      // passes A and B over the entries [i0, i1) whose pixels lie in [q0, q1), rows read from bm (origin org)
      auto screen_range = [&](const uint32_t* bm, int org, int wmax, int i0, int i1, uint32_t q0, uint32_t q1) {
        // presence rows rs-3 .. rs+3 of pixel s, columns cs-3 .. cs+3 (masked by cv; 0 outside the image), from bm
        // whose bit 0 is pixel org.  The bit of column cs-3 in row rs is st0 = s - 3 - org, row rs+e's is st0 + e*ncl;
        // word indices are clamped into [-1, wmax] (a row outside the image reads some word of the bitmap's space and
        // is zeroed by its row mask).  Branch-free.  Bits
        // outside the image's columns are masked, so the words around the bitmap may hold anything.
        auto rows7 = [&](int s, int& rs, int& cs, uint32_t& cv, uint32_t (&Hh)[7]) {
          rowcv(s, rs, cs, cv);
          const int st0 = s - 3 - org;
          const int dlo = 3 - rs > 0 ? 3 - rs : 0, dhi = nr + 2 - rs < 6 ? nr + 2 - rs : 6;
          const uint32_t vmask = ((2u << dhi) - 1u) & ~((1u << dlo) - 1u);  // rows d in [dlo, dhi] lie in the image
          uint32_t a[7], b[7];
          int st[7];
#pragma unroll
          for (int d = 0; d < 7; ++d) {
            st[d] = st0 + (d - 3) * ncl;
            const int w = min(max(st[d] >> 5, -1), wmax);
            a[d] = bm[w];
            b[d] = bm[w + 1];
          }
#pragma unroll
          for (int d = 0; d < 7; ++d) {
            const uint32_t rm = (uint32_t)((int)(vmask << (31 - d)) >> 31);  // all ones if row d is in the image
            Hh[d] = __builtin_amdgcn_alignbit(b[d], a[d], (uint32_t)st[d]) & cv & rm;
          }
        };
        // pass B on survivor s of each lane where ok (wave-uniform call)
        auto screen_s = [&](const bool ok, const int s) {
          if constexpr ((SMG_SP_ABL & 8) != 0) return;
          int rs, cs;
          uint32_t cv, Hh[7];
          rows7(s, rs, cs, cv, Hh);
          uint32_t pass = 0;
          if (ok) {
            uint32_t Dl[7];
            Dl[0] = Dl[6] = 0;
#pragma unroll
            for (int d = 1; d <= 5; ++d) {
              const int row = rs - 3 + d;
              const bool rv = row >= 0 && row < nr;
              uint32_t x = (Hh[d] | (Hh[d] << 1) | (Hh[d] >> 1) | Hh[d - 1] | Hh[d + 1]) & cv;
              if (!rv) x = 0;
              if (P.erosion_border) x |= rv ? (~cv & 0x7Fu) : 0x7Fu;
              Dl[d] = x & 0x7Fu;
            }
#define SP_HB(dr, dc) ((Hh[3 + (dr)] >> (3 + (dc))) & 1u)
#define SP_BOX(dr, dc) ((((Dl[2 + (dr)] >> (2 + (dc))) & 7u) == 7u) && (((Dl[3 + (dr)] >> (2 + (dc))) & 7u) == 7u) && \
                        (((Dl[4 + (dr)] >> (2 + (dc))) & 7u) == 7u))
            const bool in_l = cs > 0, in_r = cs + 1 < ncl, in_u = rs > 0, in_d = rs + 1 < nr;
            if (SP_BOX(0, 0) && !SP_HB(-1, 0) && !SP_HB(0, -1)) pass |= 1u;
            if (in_r && SP_BOX(0, 1) && !SP_HB(-1, 1)) pass |= 2u;
            if (in_l && SP_BOX(0, -1) && !SP_HB(-1, -1) && !SP_HB(0, -2) && !SP_HB(0, -1)) pass |= 4u;
            if (in_u && SP_BOX(-1, 0) && !SP_HB(-2, 0) && !SP_HB(-1, -1) && !SP_HB(-1, 0) && !SP_HB(-1, 1))
              pass |= 8u;
            if (in_d && SP_BOX(1, 0)) pass |= 16u;
#undef SP_BOX
#undef SP_HB
          }
          const int cnt1 = __popc(pass);
          const int inc = wave_incl_scan_dpp(cnt1);
          const int wtot = __builtin_amdgcn_readlane(inc, 63);
          if (wtot > 0) {
            int wbase = 0;
            if (lane == 63) wbase = atomicAdd(&ctr[S_NE], wtot);
            int idx = __builtin_amdgcn_readlane(wbase, 63) + inc - cnt1;
            while (pass) {
              const int ci = __ffs(pass) - 1;
              pass &= pass - 1;
              const int p = s + (ci == 1 ? 1 : ci == 2 ? -1 : ci == 3 ? -ncl : ci == 4 ? ncl : 0);
              if (idx < SP_CCAP) clist[idx] = (uint32_t)p;
              else ctr[S_ABORT] = 1;
              ++idx;
            }
          }
        };
        // pass B on this wave's full survivor list wsurv[0, wcnt) (lane i takes survivor i)
        auto screen = [&](int wcnt) {
          __builtin_amdgcn_wave_barrier();  // (the survivor list was written by this wave's lanes)
          const bool ok = lane < wcnt;
          screen_s(ok, ok ? (int)wsurv[lane] : (int)q0);
          __builtin_amdgcn_wave_barrier();  // (the list is refilled after this)
        };
        int wcnt = 0;  // (wave-uniform)
        for (int ob = i0; ob < i1; ob += BLOCK) {  // uniform trip count
          const int i = ob + tid;
          const uint32_t w = i < i1 ? ekey[i] >> 12 : 0xFFFFFFFFu;  // the pixel (a hole's: >= 2^19)
          const bool ok = w >= q0 && w < q1;
          // pass A counts the 7x7 window's bits without the column and row masks: a window at the image's left or
          // right edge also counts bits of the neighbouring row, one at its top or bottom whatever its clamped reads
          // find -- only ever more, never fewer, so a pixel it lets through gets the exact screen in pass B, and
          // one it drops has fewer than three principal pixels in its 7x7
          bool surv = ok;
          if (!P.erosion_border) {  // (uniform)
            const int st0 = (ok ? (int)w : (int)q0) - 3 - org;
            uint32_t a[7], b[7];
            int st[7];
#pragma unroll
            for (int d = 0; d < 7; ++d) {
              st[d] = st0 + (d - 3) * ncl;
              const int wd = min(max(st[d] >> 5, -1), wmax);
              a[d] = bm[wd];
              b[d] = bm[wd + 1];
            }
            int cnt = 0;
#pragma unroll
            for (int d = 0; d < 7; ++d) cnt += __popc(__builtin_amdgcn_alignbit(b[d], a[d], (uint32_t)st[d]) & 0x7Fu);
            surv = ok && cnt >= 3;
          }
          const uint64_t m = __ballot(surv);
          const int c = (int)__popcll(m);
          if (wcnt + c > WAVE) {
            screen(wcnt);
            wcnt = 0;
          }
          if (surv) wsurv[wcnt + (int)lanes_below(m)] = w;
          wcnt += c;
        }
        // the waves' partial lists (up to 63 survivors each) are screened together: their counts, a barrier, then
        // wave w takes survivors [64w, 64w + 64) of the four lists laid end to end -- one pass B per range and
        // chunk of 64 survivors rather than one per wave
        if (lane == 0) wsc[wid] = wcnt;
        __syncthreads();
        const int c0 = wsc[0], c1 = c0 + wsc[1], c2 = c1 + wsc[2], tot = c2 + wsc[3];
        const uint32_t* wall = reinterpret_cast<const uint32_t*>(smem + SpLay::o_wsurv);
        if (wid * WAVE < tot) {  // (wave-uniform)
          const int g = wid * WAVE + lane;
          const int at = g < c0 ? g : g < c1 ? WAVE + g - c0 : g < c2 ? 2 * WAVE + g - c1 : 3 * WAVE + g - c2;
          const bool ok = g < tot;
          screen_s(ok, ok ? (int)wall[at] : (int)q0);
        }
      };
      if (P.npx <= SP_FWORDS * 32) {  // F is the principal image's presence bitmap
        if (!(SMG_SP_ABL & 32)) screen_range(F, 0, SP_FWORDS - 2, 0, n0, 0u, (uint32_t)P.npx);
        __syncthreads();
      } else {
        const int B = G.band_rows;
        for (int r0 = 0; r0 < nr; r0 += B) {  // uniform
          const int r1 = min(r0 + B, nr), rb = max(r0 - 3, 0), re = min(r1 + 3, nr);
          const int b0 = (rb * ncl) >> bs, b1 = (re * ncl - 1) >> bs, org = b0 << bs;
          // rows [rb, re) of the band bitmap: zeroed, then a bit per entry (holes and the partial buckets' foreign
          // rows fall outside)
          const uint32_t span = (uint32_t)(re * ncl - org);
          const int nw4 = (int)((span + 127u) >> 7);
          for (int k = tid; k < nw4 && !(SMG_SP_ABL & 16); k += BLOCK)
            reinterpret_cast<uint4*>(band)[k] = make_uint4(0u, 0u, 0u, 0u);
          __syncthreads();
          const int e1 = (SMG_SP_ABL & 16) ? 0 : dir[b1 + 1];
          for (int i = dir[b0] + tid; i < e1; i += BLOCK) {
            const uint32_t q = (ekey[i] >> 12) - (uint32_t)org;
            if (q < span) atomicOr(&band[q >> 5], 1u << (q & 31u));
          }
          __syncthreads();
          const uint32_t q0 = (uint32_t)(r0 * ncl), q1 = (uint32_t)(r1 * ncl);
          if (!(SMG_SP_ABL & 32))
            screen_range(band, org, SpLay::band_bits / 32 - 2, dir[q0 >> bs], dir[((q1 - 1) >> bs) + 1], q0, q1);
          __syncthreads();
        }
      }
      SP_STAMP(8);
      const int ncand = (SMG_SP_ABL & 64) ? 0 : ctr[S_NE];
      if (ctr[S_ABORT] || ncand > SP_CCAP) {  // more candidates than the list holds: the big-ion pass
        reject();
        skip = true;
      }
      if (!skip) {
        // (ii) exact eL(p) = min_{q in box(p)} max_{q' in cross[q], in image} L(q') for every candidate, the levels of
        //      its 5x5 neighbourhood's principal pixels found in the directory (entries are in pixel order), packed 8
        //      bits per column
        int emax_local = 0;
        // one lane per (candidate, window row), so that the five rows' directory scans run side by side: wave w
        // takes candidates w, w + 4, ... in rounds of 12; the rows meet in a wave-private block where the screen's
        // bitmaps were (free now: F is cleared whole by the next ion's build)
        uint64_t* lrow = reinterpret_cast<uint64_t*>(smem + SpLay::o_U) + wid * WAVE;
        const int eslot = lane % 12, erow = lane / 12;  // lanes 60..63 idle
        for (int cb = 0; cb < ncand; cb += SP_NW * 12) {  // uniform trip count
          const int c = cb + eslot * SP_NW + wid;
          uint64_t packed = 0;
          if (erow < 5 && c < ncand) {
            const int p = (int)clist[c];
            int rp, cp;
            rowcol(p, P, rp, cp);
            const int row = rp - 2 + erow;
            if ((unsigned)row < (unsigned)nr) {
              const int base = row * ncl + cp - 2;  // pixel of window column 0
              const uint32_t lo = (uint32_t)(row * ncl + max(cp - 2, 0)), hi = (uint32_t)(row * ncl + min(cp + 2, ncl - 1));
              const int e1 = dir[(hi >> bs) + 1];
              for (int i = dir[lo >> bs]; i < e1; i += 2) {  // (pairs read together, as in sp_lookup)
                const uint32_t w0 = ekey[i] >> 12, w1 = ekey[i + 1] >> 12;  // (a hole's: >= 2^19, outside the range)
                const uint64_t l0 = L8[i], l1 = L8[i + 1];
                if (w0 >= lo && w0 <= hi) packed |= l0 << (8 * (int)(w0 - (uint32_t)base));
                if (i + 1 < e1 && w1 >= lo && w1 <= hi) packed |= l1 << (8 * (int)(w1 - (uint32_t)base));
              }
            }
          }
          lrow[lane] = packed;
          __builtin_amdgcn_wave_barrier();
          const int c2 = cb + lane * SP_NW + wid;
          if (lane < 12 && c2 < ncand) {
            const int p = (int)clist[c2];
            int rp, cp;
            rowcol(p, P, rp, cp);
            uint64_t Lrow[5];
#pragma unroll
            for (int d = 0; d < 5; ++d) Lrow[d] = lrow[d * 12 + lane];
#define SP_L(r, cc) ((int)((Lrow[r] >> (8 * (cc))) & 0xFFull))
            int mn = 1 << 20;
            bool outside = false;
#pragma unroll
            for (int a2 = -1; a2 <= 1; ++a2) {
#pragma unroll
              for (int b2 = -1; b2 <= 1; ++b2) {
                const int rq = rp + a2, cq = cp + b2;
                if (rq < 0 || rq >= nr || cq < 0 || cq >= ncl) {
                  outside = true;
                  continue;
                }
                const int R = 2 + a2, C = 2 + b2;
                int dl = SP_L(R, C);
                dl = max(dl, SP_L(R - 1, C));
                dl = max(dl, SP_L(R + 1, C));
                dl = max(dl, SP_L(R, C - 1));
                dl = max(dl, SP_L(R, C + 1));
                mn = min(mn, dl);
              }
            }
#undef SP_L
            if (outside && !P.erosion_border) mn = 0;
            if (mn >= (1 << 20)) mn = 0;
            cel[c2] = (uint8_t)mn;
            emax_local = max(emax_local, mn);
          }
          __builtin_amdgcn_wave_barrier();  // (the block is rewritten next round)
        }
        if (emax_local > 0) atomicMax(&ctr[S_EMAX], emax_local);
        __syncthreads();
        SP_STAMP(9);
        // (iii) Kruskal over eL (levels descending), union-find over candidate indices
        double sum_c = 0.0;
        const int emax_all = ctr[S_EMAX];
        if (emax_all > 0 && ncand <= WAVE) {
          // few candidates (most noise images): wave 0 alone, one candidate per lane; no barrier (only wave 0 needs
          // the result)
          if (wid == 0) {
            uint32_t* upar = reinterpret_cast<uint32_t*>(red);  // 64 entries (red is free until the record)
            const bool act = lane < ncand;
            const int p = act ? (int)clist[lane] : -1;
            const int e = act ? (int)cel[lane] : 0;
            int rp = 0, cp = 0;
            rowcol(p < 0 ? 0 : p, P, rp, cp);
            int nb[4] = {-1, -1, -1, -1};
            // forward neighbours through a 128-slot pixel -> lane hash over the survivor lists (the other waves clear
            // F and the counters meanwhile; the lists are rewritten only after the ion's last barrier)
            uint32_t* kt = reinterpret_cast<uint32_t*>(smem + SpLay::o_wsurv);
            kt[lane] = SP_EMPTY;
            kt[lane + WAVE] = SP_EMPTY;
            __builtin_amdgcn_wave_barrier();
            auto kslot = [](uint32_t q) { return (q * 2654435761u) >> 25; };
            if (act && e >= 1) {
              uint32_t h = kslot((uint32_t)p);
              while (atomicCAS(&kt[h], SP_EMPTY, ((uint32_t)p << 6) | (uint32_t)lane) != SP_EMPTY) h = (h + 1) & 127u;
            }
            __builtin_amdgcn_wave_barrier();
            auto kfind = [&](int q) -> int {
              uint32_t h = kslot((uint32_t)q);
              while (true) {
                const uint32_t k = kt[h];
                if (k == SP_EMPTY) return -1;
                if ((k >> 6) == (uint32_t)q) return (int)(k & 63u);
                h = (h + 1) & 127u;
              }
            };
            if (act && e >= 1) {
              if (cp + 1 < ncl) nb[0] = kfind(p + 1);
              if (rp + 1 < nr) {
                nb[1] = kfind(p + ncl);
                if (P.connectivity == 8 && cp > 0) nb[2] = kfind(p + ncl - 1);
                if (P.connectivity == 8 && cp + 1 < ncl) nb[3] = kfind(p + ncl + 1);
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
          // a candidate hash (pixel -> index) and the union-find in the values' space
          for (int i = tid; i < SP_HSZ; i += BLOCK) htab[i] = SP_EMPTY;
          __syncthreads();
          double esum = 0.0;
          auto hslot = [](uint32_t p) { return (p * 2654435761u) >> (32 - 11); };
          static_assert(SP_HSZ == 2048 && SP_CCAP <= 1024, "hash geometry");
          for (int c = tid; c < ncand; c += BLOCK) {
            par[c] = (uint32_t)c;
            const int e = cel[c];
            if (e == 0) continue;
            esum += (double)e;
            const uint32_t p = clist[c];
            uint32_t h = hslot(p);
            while (atomicCAS(&htab[h], SP_EMPTY, (p << 10) | (uint32_t)c) != SP_EMPTY) h = (h + 1) & (SP_HSZ - 1);
          }
          __syncthreads();
          auto find_c = [&](uint32_t q) -> int {
            uint32_t h = hslot(q);
            while (true) {
              const uint32_t k = htab[h];
              if (k == SP_EMPTY) return -1;
              if ((k >> 10) == q) return (int)(k & 1023u);
              h = (h + 1) & (SP_HSZ - 1);
            }
          };
          double wsum = 0.0;
          for (int t = emax_all; t >= 1; --t) {
            for (int c = tid; c < ncand; c += BLOCK) {
              const int e = cel[c];
              if (e < t) continue;
              const int p = (int)clist[c];
              int rp, cp;
              rowcol(p, P, rp, cp);
              auto edge = [&](int q) {
                const int j = find_c((uint32_t)q);
                if (j < 0) return;
                const int eq2 = cel[j];
                if ((e < eq2 ? e : eq2) == t && uf_unite(par, (uint32_t)c, (uint32_t)j)) wsum += (double)t;
              };
              if (cp + 1 < ncl) edge(p + 1);
              if (rp + 1 < nr) {
                edge(p + ncl);
                if (P.connectivity == 8) {
                  if (cp > 0) edge(p + ncl - 1);
                  if (cp + 1 < ncl) edge(p + ncl + 1);
                }
              }
            }
            __syncthreads();
          }
          double a2[2] = {esum, wsum};
          block_sum<BLOCK, 2, true>(a2, red);
          sum_c = a2[0] - a2[1];
        }
        chaos_raw = 1.0 - sum_c / (double)P.nlevels / npx_pos;
        SP_STAMP(10);
      }
    } else if (!skip) {
      flags |= SMG_ION_CHAOS_NAN;
    }

    // ---- the ion's sums -> its record (ion_finalize_kernel computes the scores); wave 0, lane k = window k
    if (!skip && wid == 0) {
      IonRec* R = reinterpret_cast<IonRec*>(desc + pos);
      const int k = lane;
      if (k < K) {
        double sk = 0.0, syy = D->syy[k], sxy = 0.0;
        if (k == 0) {
          sk = s0;
        } else {
#pragma unroll
          for (int w = 0; w < NW; ++w) {
            const double* pk = part + ((size_t)k * NW + w) * 4;
            sk += pk[0];
            syy += pk[2];
            sxy += pk[3];
          }
        }
        R->s[k] = sk;
        R->sxy[k] = sxy;
        R->syy[k] = syy;
      }
      if (lane == 0) {
        R->sx = sx;
        R->sxx = sxx;
        R->chaos = chaos_raw;
        R->flags = flags | SMG_ION_SPARSE | (uint32_t)D->hits;
        R->state = 1u;
      }
    }
    if (npos < 0) break;
    if (began && wid != 0) clear_fc(tid - WAVE, BLOCK - WAVE);  // (the chaos phase is done with both)
    pos = npos;
    npos = n2pos;
    cur ^= 1;
    __syncthreads();  // the next ion starts on cleared structures
    SP_STAMP(11);
  }
  SP_STAMP_FLUSH();
  // no load of this wave outlives it
  vm_wait<0>(pa);
  vm_wait<0>(pb);
  vm_wait<0>(pc);
  vm_wait<0>(pd);
  vm_wait<0>(pe);
}

SpGeo sparse_geo(const Params& P) {
  SpGeo G;
  int lg = 0;
  while ((1ll << lg) < (long long)P.npx) ++lg;
  G.bs = lg > 10 ? lg - 10 : 0;  // <= 1024 buckets
  // a band's bitmap holds its rows [rb, re): rows * ncols bits plus a partial bucket in front (and the uint4 rounding
  // of its zeroing)
  const long long rows = ((long long)SpLay::band_bits - 2ll * (1ll << G.bs) - 128) / P.ncols;
  G.band_rows = (int)(rows - 6 > 0x7FFFFFFF ? 0x7FFFFFFF : rows - 6);
  return G;
}

}  // namespace

bool sparse_main_fits(const Params& P) {
  if (P.clip || P.npx <= 0 || P.npx > NPX_LDS_MAX) return false;
  return P.npx <= SP_FWORDS * 32 || sparse_geo(P).band_rows >= 8;
}

int launch_sparse_main(Hits<SMG_HITS_PACKED_F32> hits, IonDesc* desc, Sched S, const Params& P, double* oc,
                       double* osp, double* osc, double* omsm, uint32_t* oflags, uint32_t* rej_list,
                       uint32_t* rej_count, int cus, hipStream_t st, const ChkCtx& ck) {
  (void)ck;
  const SpGeo G = sparse_geo(P);
  auto k = &ion_sparse_kernel<SP_BLOCK, SP_RMAX, SP_RC, SP_WPE>;

  // SP_WGPCU resident workgroups per CU, a multiple of the XCD count
  int64_t nwg = (int64_t)cus * SP_WGPCU;
  if (nwg > S.n) nwg = ((S.n + XCDS - 1) / XCDS) * XCDS;
  hipLaunchKernelGGL(k, dim3((unsigned)nwg), dim3(SP_BLOCK), 0, st, hits, desc, S, P, G, oc, osp, osc, omsm,
                     oflags, rej_list, rej_count SMG_CHK_ARG(ck));
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

int sparse_read_stamps(unsigned long long* host_out, int n) {
#ifdef SMG_STAMPS
  SMG_HIP(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_sp_stamps), sizeof(unsigned long long) * (n < 16 ? n : 16)));
  unsigned long long z[16] = {0};
  SMG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sp_stamps), z, sizeof(z)));
  return SMG_OK;
#else
  (void)host_out;
  (void)n;
  set_error("library built without -DSMG_STAMPS");
  return SMG_ERR_UNSUPPORTED;
#endif
}

}  // namespace smg
