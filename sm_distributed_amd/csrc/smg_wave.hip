// Main pass of the fused ion imaging + MSM scoring on gfx950: one wave per ion.
//
// Replaces, in frulo/SM_distributed (the same computation as ion_pipe_kernel in smg_metrics.hip):
//   formula_imager_segm.py:84-92   per-window COO construction   (_gen_iso_images)
//   formula_img_validator.py:72-84 compute(): spectral / spatial / chaos
//   pyImagingMSpec 0.1.1 isotope_pattern_match / isotope_image_correlation,
//   cpyImagingMSpec 0.0.4 measure_of_chaos   (restated, see oracle/msm_oracle.py)
//
// Why one wave per ion.  The 512-thread LDS kernel spends most of an ion's ~49k cycles in barriers and dependent
// LDS round trips, and its image-sized presence bitmap + rank prefix (39 KB at 500x500 px) caps a CU
// at two ions in flight.  Here a wave scores an ion alone: no barrier anywhere, and the principal image is kept as
// a *segment directory* whose size does not depend on the image: the image is cut into nseg <= 2046 runs of 2^S
// pixels, dir[s] .. dir[s+1] is the range of segment s's entries, and an entry is (index of the point in the
// principal window << 16 | dup flag << 15 | pixel offset in the segment).  That is 4 KB + 4 B per principal
// point (~17 KB per wave for 2560 points), so a CU holds nine ions in flight instead of two, and the four SIMDs
// interleave their dependent chains.
//
// Per ion (all in one wave, software-pipelined: the next ion's principal window and first four tail chunks are
// loaded while this ion finishes):
//   1. principal window (<= CAP points, CAP/64 registers per lane): flagged points (duplicate candidates) are
//      summed per pixel in a 64-entry LDS table; statistics sum x, sum x^2, sum x[x>0], #(x>0), max over the
//      distinct pixels; directory by counting sort (packed u16 LDS atomics, a DPP scan, a returning-atomic
//      scatter);
//   2. measure_of_chaos by threshold decomposition (as ion_pipe_kernel): candidates from the 7x7 neighbourhood of
//      each principal pixel (row queries on the directory), exact eL = erode_box(dilate_cross(L)) of each
//      candidate from the levels of its 5x5 neighbourhood, Kruskal over <= 64 candidates in registers + LDS;
//   3. tail windows 1..K-1 as one stream of 64-point groups (ion descriptors, smg_metrics.hip): every point is
//      looked up in the directory; a principal hit (~0.5% of the points) is parked in registers and its x
//      gathered after the stream; flagged points are listed and summed per pixel when the stream leaves their
//      window;
//   4. finalize (lane k = window k).
// Ions beyond its capacities (K > 8, principal window > CAP points, > 64 distinct duplicate pixels, > 128 flagged
// points in one tail window, > 64 chaos candidates) are handed to the big-ion LDS pass as positions, like the main pass's.
#include "smg_common.hpp"
#include "smg_ion.hpp"

namespace smg {

template <int CAP>
struct WaveLay {
  static constexpr int NDIR = 2048;  // directory: dir[0] = 0, dir[s + 1] = end of segment s (s < nseg <= 2046)
  static constexpr int DT = 64;      // distinct principal pixels with flagged points
  static constexpr int TL = 128;     // flagged tail points
  static constexpr int NC = 64;      // chaos candidates
  static constexpr uint32_t o_dir = 0;
  static constexpr uint32_t o_ent = o_dir + NDIR * 2;
  static constexpr uint32_t o_desc = o_ent + (uint32_t)CAP * 4;  // two descriptors (current, next)
  static constexpr uint32_t o_dtk = o_desc + 2 * 384;
  static constexpr uint32_t o_dtv = o_dtk + DT * 4;
  static constexpr uint32_t o_tlk = o_dtv + DT * 8;
  static constexpr uint32_t o_tlv = o_tlk + TL * 4;
  static constexpr uint32_t o_cand = o_tlv + TL * 4;
  static constexpr uint32_t o_uf = o_cand + NC * 4;
  static constexpr uint32_t o_part = o_uf + NC * 4;  // f64 [3][MAXK]: sum y[x>0], sum xy, flagged (sum y)^2
  static constexpr uint32_t bytes = o_part + 3 * MAXK * 8;
  static_assert(CAP % 64 == 0 && CAP <= 32768, "principal capacity");
  static_assert(o_dtv % 8 == 0 && o_part % 8 == 0 && o_desc % 16 == 0, "LDS alignment");
};

constexpr uint32_t WV_EMPTY = 0xFFFFFFFFu;
constexpr int WAVE_CAP = 2560;  // principal points per ion in the wave pass
constexpr int WAVE_RC = 2;      // tail groups (64 points) per ring buffer; four buffers in flight
constexpr int WAVE_PC = 8;      // principal slots per lane and chunk (512 points)

// one element of a row query: the pixel at directory entry t of segment range [a, b) (m: end of the first
// segment s0, the second is s0 + 1)
struct RowQ {
  int a, m, b, s0, q0, qa, qb;
};

__device__ __forceinline__ RowQ rowq_setup(int r, int c_lo, int W, const Params& P, const uint16_t* dir, int SH) {
  RowQ q;
  q.a = q.m = q.b = 0;
  q.s0 = 0;
  q.q0 = q.qa = 0;
  q.qb = -1;
  if (r < 0 || r >= P.nrows) return q;
  const int ca = c_lo > 0 ? c_lo : 0, cb = c_lo + W - 1 < P.ncols - 1 ? c_lo + W - 1 : P.ncols - 1;
  if (ca > cb) return q;
  const int rb = r * P.ncols;
  q.q0 = rb + c_lo;
  q.qa = rb + ca;
  q.qb = rb + cb;
  const int s0 = q.qa >> SH, s1 = q.qb >> SH;  // s1 <= s0 + 1 (W <= 8 <= 2^SH)
  q.s0 = s0;
  q.a = dir[s0];
  q.m = dir[s0 + 1];
  q.b = (s1 > s0) ? dir[s1 + 1] : q.m;
  return q;
}

// pixel of entry t in a row query's range
__device__ __forceinline__ int rowq_pix(const RowQ& q, int t, uint32_t e, int SH, uint32_t OM) {
  return ((t < q.m ? q.s0 : q.s0 + 1) << SH) | (int)(e & OM);
}

// Diagnostic build only (-DSMG_WAVE_CHECK): index checks on the wave pass's global accesses and directory
// positions; a failed check records (code, value, position) of its first occurrence and a count
// (smg_debug_wave_check) and the access is clamped, so a bad index is reported instead of faulting.
#ifdef SMG_WAVE_CHECK
__device__ unsigned long long g_wvchk[8];  // [0] code, [1] value, [2] failures, [3] position, [4] ions scored
__device__ __forceinline__ bool wvchk(bool ok, int code, long long v, long long pos) {
  if (!ok && atomicAdd(&g_wvchk[2], 1ull) == 0ull) {
    g_wvchk[0] = (unsigned long long)code;
    g_wvchk[1] = (unsigned long long)v;
    g_wvchk[3] = (unsigned long long)pos;
  }
  return ok;
}
#define WVCK(ok, code, v) wvchk((ok), (code), (long long)(v), (long long)pos)
#define WVIX(ix, code) (WVCK((ix) >= 0 && (ix) < (1ll << 36), code, ix) ? (ix) : 0)
#else
#define WVCK(ok, code, v) true
#define WVIX(ix, code) (ix)
#endif

// Diagnostic build only (-DSMG_WAVE_STAMPS): wall cycles per phase summed over waves (smg_debug_wave_stamps):
// 0 principal image + directory, 1 chaos screen, 2 exact eL + Kruskal, 3 next descriptor / ticket, 4 tail stream,
// 5 parked hits + flagged points, 6 issue + finalize, 7 skipped ions
#ifdef SMG_WAVE_STAMPS
__device__ unsigned long long g_wstamps[8];
#define WV_STAMP(i)                                    \
  do {                                                 \
    const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    wst[i] += _t - wst_t0;                             \
    wst_t0 = _t;                                       \
  } while (0)
#else
#define WV_STAMP(i)
#endif

#ifdef SMG_WAVE_TRACE
// diagnostic build only: per scored position (pos, ion, K, n0, ngroups, fits, rej, flagged tail points)
__device__ long long g_wtrace[8192][8];
#endif

template <int CAP, int RC>
__global__ void __attribute__((amdgpu_flat_work_group_size(64, 64), amdgpu_waves_per_eu(3)))
ion_wave_kernel(Hits<SMG_HITS_PACKED_F32> hits, const IonDesc* __restrict__ desc, Sched S, Params P, int SH,
                double* __restrict__ oc, double* __restrict__ osp, double* __restrict__ osc,
                double* __restrict__ omsm, uint32_t* __restrict__ oflags, uint32_t* __restrict__ rej_list,
                uint32_t* __restrict__ rej_count) {
  using LY = WaveLay<CAP>;
  using H = Hits<SMG_HITS_PACKED_F32>;
  constexpr int PC = WAVE_PC;
  constexpr int CH = 64 * PC;  // principal points per chunk
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* dir = reinterpret_cast<uint16_t*>(smem + LY::o_dir);
  uint32_t* dir32 = reinterpret_cast<uint32_t*>(smem + LY::o_dir);
  uint32_t* ent = reinterpret_cast<uint32_t*>(smem + LY::o_ent);
  IonDesc* dsl = reinterpret_cast<IonDesc*>(smem + LY::o_desc);
  uint32_t* dtk = reinterpret_cast<uint32_t*>(smem + LY::o_dtk);
  double* dtv = reinterpret_cast<double*>(smem + LY::o_dtv);
  uint32_t* tlk = reinterpret_cast<uint32_t*>(smem + LY::o_tlk);
  float* tlv = reinterpret_cast<float*>(smem + LY::o_tlv);
  uint32_t* cand = reinterpret_cast<uint32_t*>(smem + LY::o_cand);
  uint32_t* ufp = reinterpret_cast<uint32_t*>(smem + LY::o_uf);
  double* part = reinterpret_cast<double*>(smem + LY::o_part);
  const int lane = threadIdx.x;
  const uint32_t OM = (1u << SH) - 1u;
  const uint64_t* hb = hits.h;
  int64_t pos = -1, npos = -1;  // see the scheduling comment below

  // register buffers: the principal window's first chunk (PC slots, prefetched) and a ring of four tail buffers
  // (RC groups each).  The rest of the principal window is loaded chunk by chunk when it is processed (the
  // window is read twice, the second time from L2: registers for a whole 2560-point window would halve the waves)
  uint64_t hq[PC], ra[RC], rb[RC], rc[RC], rd[RC];
#pragma unroll
  for (int j = 0; j < PC; ++j) hq[j] = 0ull;
#pragma unroll
  for (int j = 0; j < RC; ++j) ra[j] = rb[j] = rc[j] = rd[j] = 0ull;
  // exactly PC loads (clamped to the window's last point, or hit 0 for an empty window)
  auto issue_principal = [&](const IonDesc* D, bool valid) {
    const int n0 = valid ? D->end[0] : 0;
    const int64_t a = valid ? D->base[0] : 0;
#pragma unroll
    for (int j = 0; j < PC; ++j) {
      const int i = lane + 64 * j;
      hq[j] = hb[WVIX(n0 > 0 ? a + (i < n0 ? i : n0 - 1) : 0, 1)];
    }
  };
  // tail chunk c = groups [c*RC, (c+1)*RC); exactly RC loads (lanes past their window's end load its last point,
  // groups past the tail hit 0: consumers mask both)
  auto issue_chunk = [&](const IonDesc* D, int c, uint64_t (&buf)[RC], bool valid = true) {
    const int ng = valid ? D->ngroups : 0;
    int gsv[MAXK];
#pragma unroll
    for (int kk = 2; kk < MAXK; ++kk) gsv[kk] = D->gs[kk];
#pragma unroll
    for (int j = 0; j < RC; ++j) {
      const int G = c * RC + j;
      int k = 1;
#pragma unroll
      for (int kk = 2; kk < MAXK; ++kk) k += (G >= gsv[kk]) ? 1 : 0;
      const int64_t bk = D->base[k];
      const int ek = D->end[k];
      const int64_t idx = (G < ng && ng > 0) ? bk + (int64_t)G * 64 + min(lane, ek - G * 64 - 1) : 0;
      buf[j] = hb[WVIX(idx, 2)];
    }
  };
  auto issue_ion = [&](const IonDesc* D, bool valid) {  // !valid: the same loads of hit 0 (no next ion)
    issue_principal(D, valid);
    issue_chunk(D, 0, ra, valid);
    issue_chunk(D, 1, rb, valid);
    issue_chunk(D, 2, rc, valid);
    issue_chunk(D, 3, rd, valid);
  };

  // pos: the ion scored in this iteration (-1: none -- the first iteration only loads); npos: the next one, whose
  // descriptor this iteration fetches and whose loads it issues at its single issue site (one definition of the
  // asynchronous registers per iteration: no copies of them in flight)
  {
    int64_t t = -1;
    if (lane == 0) t = sched_resolve<SRC_RANGES>(S, sched_issue<SRC_RANGES>(S));
    npos = uni64(__shfl(t, 0));
  }
  int cur = 1;
#ifdef SMG_WAVE_STAMPS
  unsigned long long wst[8] = {0, 0, 0, 0, 0, 0, 0, 0}, wst_t0 = __builtin_amdgcn_s_memtime();
#endif
  while (true) {
    const IonDesc* D = &dsl[cur];
    IonDesc* DN = &dsl[cur ^ 1];
    // npos's descriptor (one word per lane) and the ticket of the ion after it, both asynchronous
    const uint64_t dword =
        reinterpret_cast<const uint64_t*>(desc + (npos >= 0 ? npos : 0))[lane < DESC_QWORDS ? lane : 0];
    uint32_t ticket = 0u;
    if (lane == 0) ticket = sched_issue<SRC_RANGES>(S);
    // resolves the ticket and stores npos's descriptor (waits for every load of this wave)
    int64_t n2pos = -1;
    auto advance = [&]() {
      int64_t t = -1;
      if (lane == 0 && npos >= 0) t = sched_resolve<SRC_RANGES>(S, ticket);
      n2pos = uni64(__shfl(t, 0));
      if (npos >= 0 && lane < DESC_QWORDS) reinterpret_cast<uint64_t*>(DN)[lane] = dword;
      // the descriptor is stored as words and read as fields: no reordering across this point (the LDS itself
      // serves one wave's accesses in order; the file is also built with -fno-strict-aliasing)
      asm volatile("" ::: "memory");
    };

    const bool live = pos >= 0;
    const int K = live ? uni(D->K) : 0, ion = live ? uni(D->ion) : 0, n0 = live ? uni(D->end[0]) : 0,
              ng = live ? uni(D->ngroups) : 0;
    const int64_t base0 = live ? uni64(D->base[0]) : 0;
    const bool fits = live && K >= 1 && K <= MAXK && n0 <= CAP && ng >= 0;
#ifdef SMG_WAVE_CHECK
    if (live && lane == 0) atomicAdd(&g_wvchk[4], 1ull);
    if (live && !WVCK(ion >= 0 && ion < S.n && K >= 0 && K <= MAXK_DENSE && n0 >= 0 && base0 >= 0, 6, ion)) {
      advance();
      issue_ion(DN, npos >= 0);
      if (npos < 0) break;
      pos = npos;
      npos = n2pos;
      cur ^= 1;
      continue;
    }
#endif
    bool rej = live && K != 0 && !fits;
    double sx = 0.0, sxx = 0.0, spos = 0.0, npos_px = 0.0, vmax = 0.0;
    double chaos_raw = NAN;
    uint32_t flags = 0;
    int nd = 0;  // flagged tail points listed (uniform)
    int ncand_tr = -1;  // chaos candidates (trace builds)
    if (!fits) {
      advance();
    } else {
    // ---- 1. principal image ----------------------------------------------------------------------------------
    {
      uint4* z = reinterpret_cast<uint4*>(dir32);
#pragma unroll
      for (int q = 0; q < LY::NDIR * 2 / 16 / 64; ++q) z[lane + 64 * q] = make_uint4(0u, 0u, 0u, 0u);
      dtk[lane] = WV_EMPTY;
      dtv[lane] = 0.0;
      if (lane < 3 * MAXK) part[lane] = 0.0;
    }
    const int nch = (n0 + CH - 1) / CH;
    auto load_chunk = [&](int c, uint64_t (&h)[PC]) {  // compiler-tracked loads (L2: the window was read before)
#pragma unroll
      for (int j = 0; j < PC; ++j) {
        const int i = c * CH + lane + 64 * j;
        h[j] = hb[WVIX(base0 + (i < n0 ? i : n0 - 1), 3)];
      }
    };
    // pass 1: flagged points (duplicate candidates) summed per pixel in the table (coo.toarray() sums duplicates);
    // the statistics and segment counts of the unflagged points, each the only point of its pixel
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, mx = -INFINITY;
    auto acc = [&](double v) {
      a0 += v;
      a1 += v * v;
      if (v > 0.0) {
        a2 += v;
        a3 += 1.0;
      }
      mx = v > mx ? v : mx;
    };
    auto count = [&](uint32_t p) {  // dir[s + 1] counts segment s (packed u16 atomics)
      const uint32_t s1 = (p >> SH) + 1u;
      atomicAdd(&dir32[s1 >> 1], 1u << ((s1 & 1u) * 16u));
    };
    auto pass1 = [&](const uint64_t (&h)[PC], int c) {
      uint32_t flg = 0u;
#pragma unroll
      for (int j = 0; j < PC; ++j) {
        const bool in = c * CH + lane + 64 * j < n0;
        if (in && H::dup(h[j])) {
          flg |= 1u << j;
        } else if (in) {
          acc(H::val(h[j]));
          count(H::pix(h[j]));
        }
      }
      if (__ballot(flg != 0u)) {
#pragma unroll
        for (int j = 0; j < PC; ++j) {
          if (!__ballot((flg >> j) & 1u)) continue;
          if ((flg >> j) & 1u) {
            const uint32_t key = H::pix(h[j]);
            uint32_t hh = (key * 2654435761u) >> 26;  // 64 slots
            bool done = false;
            for (int t = 0; t < LY::DT; ++t) {
              const uint32_t old = atomicCAS(&dtk[hh], WV_EMPTY, key);
              if (old == WV_EMPTY || old == key) {
                atomicAdd(&dtv[hh], H::val(h[j]));
                done = true;
                break;
              }
              hh = (hh + 1) & (LY::DT - 1);
            }
            if (!done) rej = true;
          }
        }
      }
    };
    pass1(hq, 0);
#pragma unroll
    for (int j = 0; j < PC; ++j) hq[j] = 0ull;  // consumed: frees the registers until the next ion's loads
#pragma unroll 1
    for (int c = 1; c < nch; ++c) {
      uint64_t h[PC];
      load_chunk(c, h);
      pass1(h, c);
    }
    // the summed pixels (the table's entries): statistics and counts
    const uint32_t tk = dtk[lane];
    if (tk != WV_EMPTY) {
      acc(dtv[lane]);
      count(tk);
    }
    sx = wave_sum_dpp(a0);
    sxx = wave_sum_dpp(a1);
    spos = wave_sum_dpp(a2);
    npos_px = wave_sum_dpp(a3);
    vmax = wave_max_dpp(mx);
    // directory: exclusive scan of the counts (lane l owns dir[32 l .. 32 l + 31]: local sums, wave scan), then
    // the scatter; afterwards dir[s + 1] = end of segment s, dir[s] = its start
    {
      uint4* d4 = reinterpret_cast<uint4*>(dir32) + lane * 4;
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = d4[q];
        w[4 * q] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
      }
      uint32_t tot = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) tot += (w[q] & 0xFFFFu) + (w[q] >> 16);
      uint32_t run = (uint32_t)(wave_incl_scan_dpp((int)tot) - (int)tot);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint32_t lo = w[q] & 0xFFFFu, hi = w[q] >> 16;
        w[q] = run | ((run + lo) << 16);
        run += lo + hi;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) d4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    }
    auto place = [&](uint32_t p, uint32_t payload) {  // entry of pixel p at the next position of its segment
      const uint32_t s1 = (p >> SH) + 1u, sh = (s1 & 1u) * 16u;
      const uint32_t old = atomicAdd(&dir32[s1 >> 1], 1u << sh);
      const uint32_t at = (old >> sh) & 0xFFFFu;
      if (WVCK(at < (uint32_t)CAP, 4, at)) ent[at] = payload | (p & OM);
    };
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {  // pass 2: the unflagged points (the window again, from L2)
      uint64_t h[PC];
      load_chunk(c, h);
#pragma unroll
      for (int j = 0; j < PC; ++j) {
        const int i = c * CH + lane + 64 * j;
        if (i < n0 && !H::dup(h[j])) place(H::pix(h[j]), (uint32_t)i << 16);
      }
    }
    if (tk != WV_EMPTY) place(tk, ((uint32_t)lane << 16) | 0x8000u);
    // entry t -> x (f64): a summed pixel's from the table, else the point's f32 value in the principal window
    auto ent_x_issue = [&](uint32_t e, uint64_t& raw) {  // async gather (waited by the caller)
      if (!(e & 0x8000u)) raw = hb[WVIX(base0 + (e >> 16), 5)];
    };
    auto ent_x = [&](uint32_t e, uint64_t raw) -> double {
      return (e & 0x8000u) ? dtv[e >> 16] : H::val(raw);
    };

    WV_STAMP(0);
    // ---- 2. measure_of_chaos ----------------------------------------------------------------------------------
    const bool chaos_ok = (sx > 0.0) && (npos_px >= 4.0);
    if (chaos_ok && !rej) {
      int ncand = 0;  // uniform
      // (i) screen: candidate pixels in the 4-cross of each principal pixel s whose 3x3 box is covered by the
      // cross-dilated principal set; each listed once, by the first principal pixel on its cross (as
      // ion_pipe_kernel's screen)
      // the distinct principal pixels are the directory's entries: lane l walks entries [nent*l/64, nent*(l+1)/64)
      // with its segment pointer (first segment by binary search), so no register array is indexed at run time
      const int nseg = (int)(((uint32_t)P.npx + OM) >> SH);
      const int nent = dir[nseg];
      const int e_lo = (nent * lane) >> 6, e_hi = (nent * (lane + 1)) >> 6;
      int sg = 0;
      {
        int lo_s = 0, hi_s = nseg;  // first segment s with dir[s + 1] > e_lo
        while (lo_s < hi_s) {
          const int mid = (lo_s + hi_s) >> 1;
          if ((int)dir[mid + 1] > e_lo) hi_s = mid;
          else lo_s = mid + 1;
        }
        sg = lo_s;
      }
      const int iters = (nent + 63) >> 6;
#pragma unroll 1
      for (int it = 0; it < iters; ++it) {
        const int te = e_lo + it;
        const bool act = te < e_hi;
        if (act) {
          while ((int)dir[sg + 1] <= te) ++sg;
        }
        const int s = act ? ((sg << SH) | (int)(ent[te] & OM)) : 0;
        int rs, cs;
        rowcol(s, P, rs, cs);
        uint32_t H7[7];
        {
          RowQ q[7];
#pragma unroll
          for (int d = 0; d < 7; ++d) {
            q[d] = rowq_setup(rs - 3 + d, cs - 3, 7, P, dir, SH);
            H7[d] = 0u;
          }
          int t = 0;
          while (true) {
            bool any = false;
#pragma unroll
            for (int d = 0; d < 7; ++d) {
              if (act && q[d].a + t < q[d].b) {
                const int tt = q[d].a + t;
                const int px = rowq_pix(q[d], tt, ent[tt], SH, OM);
                if (px >= q[d].qa && px <= q[d].qb) H7[d] |= 1u << (px - q[d].q0);
                any = true;
              }
            }
            if (!__ballot(any)) break;
            ++t;
          }
        }
        const int clo = 3 - cs > 0 ? 3 - cs : 0, chi = P.ncols - cs + 3 < 7 ? P.ncols - cs + 3 : 7;
        const uint32_t cv = ((1u << chi) - 1u) & ~((1u << clo) - 1u);
        const bool sparse = !P.erosion_border && (__popc(H7[0]) + __popc(H7[1]) + __popc(H7[2]) + __popc(H7[3]) +
                                                  __popc(H7[4]) + __popc(H7[5]) + __popc(H7[6])) < 3;
        uint32_t pass = 0;
        if (act && !sparse) {
          uint32_t Dl[7];
          Dl[0] = Dl[6] = 0;
#pragma unroll
          for (int d = 1; d <= 5; ++d) {
            const int row = rs - 3 + d;
            const bool rv = row >= 0 && row < P.nrows;
            uint32_t x = (H7[d] | (H7[d] << 1) | (H7[d] >> 1) | H7[d - 1] | H7[d + 1]) & cv;
            if (!rv) x = 0;
            if (P.erosion_border) x |= rv ? (~cv & 0x7Fu) : 0x7Fu;
            Dl[d] = x & 0x7Fu;
          }
#define WV_HB(dr, dc) ((H7[3 + (dr)] >> (3 + (dc))) & 1u)
#define WV_BOX(dr, dc) ((((Dl[2 + (dr)] >> (2 + (dc))) & 7u) == 7u) && (((Dl[3 + (dr)] >> (2 + (dc))) & 7u) == 7u) && \
                        (((Dl[4 + (dr)] >> (2 + (dc))) & 7u) == 7u))
          const bool in_l = cs > 0, in_r = cs + 1 < P.ncols, in_u = rs > 0, in_d = rs + 1 < P.nrows;
          if (WV_BOX(0, 0) && !WV_HB(-1, 0) && !WV_HB(0, -1)) pass |= 1u;
          if (in_r && WV_BOX(0, 1) && !WV_HB(-1, 1)) pass |= 2u;
          if (in_l && WV_BOX(0, -1) && !WV_HB(-1, -1) && !WV_HB(0, -2) && !WV_HB(0, -1)) pass |= 4u;
          if (in_u && WV_BOX(-1, 0) && !WV_HB(-2, 0) && !WV_HB(-1, -1) && !WV_HB(-1, 0) && !WV_HB(-1, 1)) pass |= 8u;
          if (in_d && WV_BOX(1, 0)) pass |= 16u;
#undef WV_BOX
#undef WV_HB
        }
        const int cnt = __popc(pass);
        const int inc = wave_incl_scan_dpp(cnt);
        const int wtot = __builtin_amdgcn_readlane(inc, 63);
        if (wtot > 0) {
          int idx = ncand + inc - cnt;
          while (pass) {
            const int ci = __ffs(pass) - 1;
            pass &= pass - 1;
            const int p = s + (ci == 1 ? 1 : ci == 2 ? -1 : ci == 3 ? -P.ncols : ci == 4 ? P.ncols : 0);
            if (idx < LY::NC) cand[idx] = (uint32_t)p;
            ++idx;
          }
          ncand += wtot;
        }
      }
      ncand_tr = ncand;
      if (ncand > LY::NC) {
        rej = true;
      } else {
        WV_STAMP(1);
        // (ii) exact eL(p) = min_{q in box(p)} max_{q' in cross[q], in image} L(q'), from the levels of the principal
        // pixels in p's 5x5 neighbourhood (bytes of Lrow[d]: columns cp-2 .. cp+2 of row rp-2+d)
        const bool act = lane < ncand;
        const int p = act ? (int)cand[lane] : 0;
        int rp, cp;
        rowcol(p, P, rp, cp);
        uint64_t Lrow[5];
#pragma unroll 1
        for (int d = 0; d < 5; ++d) {
          const RowQ q = rowq_setup(rp - 2 + d, cp - 2, 5, P, dir, SH);
          int tcol[5] = {-1, -1, -1, -1, -1};
          for (int t = 0;; ++t) {
            const bool more = act && q.a + t < q.b;
            if (!__ballot(more)) break;
            if (more) {
              const int tt = q.a + t;
              const int px = rowq_pix(q, tt, ent[tt], SH, OM);
              if (px >= q.qa && px <= q.qb) {
                const int c = px - q.q0;
#pragma unroll
                for (int cc = 0; cc < 5; ++cc)
                  if (c == cc) tcol[cc] = tt;
              }
            }
          }
          uint32_t e5[5];
          uint64_t raw[5];
#pragma unroll
          for (int cc = 0; cc < 5; ++cc) {
            e5[cc] = tcol[cc] >= 0 ? ent[tcol[cc]] : 0x8000u;
            raw[cc] = 0ull;
          }
#pragma unroll
          for (int cc = 0; cc < 5; ++cc)
            if (tcol[cc] >= 0) ent_x_issue(e5[cc], raw[cc]);
          uint64_t packed = 0ull;
#pragma unroll
          for (int cc = 0; cc < 5; ++cc)
            if (tcol[cc] >= 0) packed |= (uint64_t)level_fast(ent_x(e5[cc], raw[cc]), vmax, P) << (8 * cc);
          Lrow[d] = packed;
        }
        int e = 0;
        if (act) {
#define WV_L(r, c) ((int)((Lrow[r] >> (8 * (c))) & 0xFFull))
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
              const int Rr = 2 + a2, Cc = 2 + b2;
              int dl = WV_L(Rr, Cc);
              dl = max(dl, WV_L(Rr - 1, Cc));
              dl = max(dl, WV_L(Rr + 1, Cc));
              dl = max(dl, WV_L(Rr, Cc - 1));
              dl = max(dl, WV_L(Rr, Cc + 1));
              mn = min(mn, dl);
            }
          }
#undef WV_L
          if (outside && !P.erosion_border) mn = 0;
          if (mn >= (1 << 20)) mn = 0;
          e = mn;
        }
        // (iii) Kruskal over eL (levels descending): forward neighbours found across lanes, LDS union-find
        double sum_c = 0.0;
        int emax = e;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) emax = max(emax, __shfl_xor(emax, o, 64));
        if (emax > 0) {
          int nb[4] = {-1, -1, -1, -1};
          for (int jj = 0; jj < ncand; ++jj) {
            const int pj = __shfl(p, jj, 64), ej = __shfl(e, jj, 64);
            if (act && e >= 1 && ej >= 1) {
              if (cp + 1 < P.ncols && pj == p + 1) nb[0] = jj;
              if (rp + 1 < P.nrows) {
                if (pj == p + P.ncols) nb[1] = jj;
                if (P.connectivity == 8 && cp > 0 && pj == p + P.ncols - 1) nb[2] = jj;
                if (P.connectivity == 8 && cp + 1 < P.ncols && pj == p + P.ncols + 1) nb[3] = jj;
              }
            }
          }
          int eq[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int v = __shfl(e, nb[q] < 0 ? 0 : nb[q], 64);
            eq[q] = nb[q] < 0 ? 0 : (e < v ? e : v);  // edge weight min(eL)
          }
          ufp[lane] = (uint32_t)lane;
          double wsum = 0.0;
          for (int t = emax; t >= 1; --t) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (eq[q] == t && uf_unite(ufp, (uint32_t)lane, (uint32_t)nb[q])) wsum += (double)t;
          }
          sum_c = wave_sum_dpp(e >= 1 ? (double)e : 0.0) - wave_sum_dpp(wsum);
        }
        chaos_raw = 1.0 - sum_c / (double)P.nlevels / npos_px;
      }
    } else if (!chaos_ok) {
      flags |= SMG_ION_CHAOS_NAN;
    }

    // ---- 3. tail windows: one stream of window-aligned 64-point groups ------------------------------------------
    WV_STAMP(2);
    advance();  // npos's descriptor into the LDS, the next ticket resolved (the tail buffers have landed)
    WV_STAMP(3);
    // flagged tail points are listed one window at a time (at most TL of them) and summed per pixel when the stream
    // leaves the window; each sum's square joins the window's sum y^2 (the prefix sums cover the unflagged points)
    int ndk = 0;  // window of the listed points (uniform)
    auto resolve_dups = [&]() {  // uniform
      if (nd > LY::TL) {
        rej = true;
      } else if (nd > 0) {
        const uint32_t k0 = lane < nd ? tlk[lane] : WV_EMPTY, k1 = lane + 64 < nd ? tlk[lane + 64] : WV_EMPTY;
        const float v0 = lane < nd ? tlv[lane] : 0.0f, v1 = lane + 64 < nd ? tlv[lane + 64] : 0.0f;
        double s0 = 0.0, s1 = 0.0;
        bool f0 = true, f1 = true;
        for (int jj = 0; jj < nd; ++jj) {
          const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)(jj < 64 ? k0 : k1), jj & 63);
          const float vj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(jj < 64 ? v0 : v1), jj & 63));
          if (kj == k0) {
            s0 += (double)vj;
            if (jj < lane) f0 = false;
          }
          if (kj == k1) {
            s1 += (double)vj;
            if (jj < lane + 64) f1 = false;
          }
        }
        if (lane < nd && f0) atomicAdd(&part[2 * MAXK + ndk], s0 * s0);
        if (lane + 64 < nd && f1) atomicAdd(&part[2 * MAXK + ndk], s1 * s1);
      }
      nd = 0;
    };
    uint64_t ev0 = 0ull, ev1 = 0ull;
    int evt0 = 0, evt1 = 0, evk0 = 0, evk1 = 0, nev = 0;
    {
      int curk = 1;
      int gnext = uni(D->gs[2]);
      int wend = uni(D->end[1]);
      auto hit_now = [&](uint64_t h, int t, int k) {  // a lane's third and later principal hits (rare)
        const uint32_t e = ent[t];
        uint64_t raw = 0ull;
        ent_x_issue(e, raw);
        const double x = ent_x(e, raw), y = H::val(h);
        atomicAdd(&part[MAXK + k], x * y);
        if (x > 0.0) atomicAdd(&part[k], y);
      };
      auto process = [&](int c, uint64_t (&buf)[RC]) {
        int a[RC], b[RC], kk[RC], hit[RC];
        uint32_t o[RC];
        bool valid[RC];
#pragma unroll
        for (int j = 0; j < RC; ++j) {
          const int G = c * RC + j;
          valid[j] = false;
          kk[j] = curk;
          if (G < ng) {
            while (G >= gnext) {  // the stream moves on to a later window (uniform)
              ++curk;
              gnext = curk + 1 < MAXK ? uni(D->gs[curk + 1]) : 0x7FFFFFFF;
              wend = uni(D->end[curk]);
            }
            kk[j] = curk;
            valid[j] = lane < wend - G * 64;
          }
          const uint32_t p = H::pix(buf[j]);
          const uint32_t s = valid[j] ? (p >> SH) : 0u;
          o[j] = p & OM;
          a[j] = valid[j] ? (int)dir[s] : 0;
          b[j] = valid[j] ? (int)dir[s + 1] : 0;
          hit[j] = -1;
        }
        for (int t = 0;; ++t) {
          bool any = false;
#pragma unroll
          for (int j = 0; j < RC; ++j) {
            if (a[j] + t < b[j]) {
              const int tt = a[j] + t;
              if ((ent[tt] & 0x7FFFu) == o[j]) hit[j] = tt;
              any = true;
            }
          }
          if (!__ballot(any)) break;
        }
#pragma unroll
        for (int j = 0; j < RC; ++j) {
          const bool h = hit[j] >= 0;
          const bool s0 = h && nev == 0, s1 = h && nev == 1;
          ev0 = s0 ? buf[j] : ev0;
          evt0 = s0 ? hit[j] : evt0;
          evk0 = s0 ? kk[j] : evk0;
          ev1 = s1 ? buf[j] : ev1;
          evt1 = s1 ? hit[j] : evt1;
          evk1 = s1 ? kk[j] : evk1;
          const bool ovf = h && nev >= 2;
          nev += h ? 1 : 0;
          if (__ballot(ovf))
            if (ovf) hit_now(buf[j], hit[j], kk[j]);
          // flagged points: listed for the per-(pixel, window) sums (ballot compaction)
          const bool f = valid[j] && H::dup(buf[j]);
          const uint64_t fm = __ballot(f);
          if (fm) {
            if (kk[j] != ndk) {  // the stream left the listed window
              resolve_dups();
              ndk = kk[j];
            }
            const int idx = nd + (int)__popcll(fm & ((1ull << lane) - 1ull));
            if (f && idx < LY::TL) {
              tlk[idx] = H::pix(buf[j]);
              tlv[idx] = __uint_as_float((uint32_t)(buf[j] >> 32));
            }
            nd += (int)__popcll(fm);
          }
        }
      };
      // buffers hold chunks 0..3; each is refilled four chunks ahead once processed (exactly 3*RC loads younger
      // than the one waited for)
      // every round waits for and refills all four buffers (processing only those inside the tail), so the loop
      // has one exit and the ring registers one definition each
#pragma unroll 1
      for (int c = 0; c * RC < ng; c += 4) {
        process(c, ra);
        issue_chunk(D, c + 4, ra);
        if ((c + 1) * RC < ng) process(c + 1, rb);
        issue_chunk(D, c + 5, rb);
        if ((c + 2) * RC < ng) process(c + 2, rc);
        issue_chunk(D, c + 6, rc);
        if ((c + 3) * RC < ng) process(c + 3, rd);
        issue_chunk(D, c + 7, rd);
      }
    }
    WV_STAMP(4);
    resolve_dups();
    // parked principal hits: both x gathers in flight together, then the window partials
    if (__ballot(nev > 0)) {
      const uint32_t e0 = nev > 0 ? ent[evt0] : 0x8000u, e1 = nev > 1 ? ent[evt1] : 0x8000u;
      uint64_t r0 = 0ull, r1 = 0ull;
      if (nev > 0) ent_x_issue(e0, r0);
      if (nev > 1) ent_x_issue(e1, r1);
      if (nev > 0) {
        const double x = ent_x(e0, r0), y = H::val(ev0);
        atomicAdd(&part[MAXK + evk0], x * y);
        if (x > 0.0) atomicAdd(&part[evk0], y);
      }
      if (nev > 1) {
        const double x = ent_x(e1, r1), y = H::val(ev1);
        atomicAdd(&part[MAXK + evk1], x * y);
        if (x > 0.0) atomicAdd(&part[evk1], y);
      }
    }
    }
    // ---- the registers of this ion are dead: npos's principal window and first four tail chunks go in flight
    WV_STAMP(fits ? 5 : 7);
    issue_ion(DN, npos >= 0);  // unconditional: one definition of the asynchronous registers
#ifdef SMG_WAVE_TRACE
    if (live && lane == 0) {
      long long* tr = g_wtrace[pos & 8191];
      tr[0] = pos; tr[1] = ion; tr[2] = K; tr[3] = n0; tr[4] = ng; tr[5] = fits; tr[6] = rej; tr[7] = ncand_tr;
    }
#endif
    // ---- 4. finalize (formula_img_validator.py:78-84 + the restated pyImagingMSpec functions): lane k = window k
    if (!live) {
    } else if (K == 0) {
      if (lane == 0) {
        oc[ion] = osp[ion] = osc[ion] = omsm[ion] = 0.0;
        oflags[ion] = 0;
      }
    } else if (rej) {
      if (lane == 0) rej_list[atomicAdd(rej_count, 1u)] = (uint32_t)pos;
    } else {
      const int k = lane;
      double t = 0.0, s = 0.0, sy = 0.0, syy = 0.0, sxy = 0.0;
      if (k < K) {
        t = D->theor[k];
        if (k == 0) {
          s = spos;
        } else {
          s = part[k];
          sy = D->sy[k];
          syy = D->syy[k] + part[2 * MAXK + k];
          sxy = part[MAXK + k];
        }
      }
      // isotope_pattern_match
      const double nt = sqrt(wave_sum_dpp(t * t)), ns = sqrt(wave_sum_dpp(s * s));
      double spectral = 1.0 - wave_sum_dpp(k < K ? fabs(t / nt - s / ns) : 0.0) / (double)K;
      if (spectral == 1.0) spectral = 0.0;
      // isotope_image_correlation: np.corrcoef rows, weights = theor[1:]
      double spatial = 0.0;
      if (K >= 2) {
        const double npx = (double)P.npx, n1 = npx - 1.0;
        const double sd0 = sqrt((sxx - sx * sx / npx) / n1);
        double rt = 0.0, tw = 0.0;
        if (k >= 1 && k < K) {
          const double syy_c = (syy - sy * sy / npx) / n1;
          const double sxy_c = (sxy - sx * sy / npx) / n1;
          double r = sxy_c / sqrt(syy_c) / sd0;
          if (!isnan(r)) r = r > 1.0 ? 1.0 : (r < -1.0 ? -1.0 : r);
          if (isinf(r)) r = 0.0;
          rt = r * t;
          tw = t;
        }
        spatial = wave_sum_dpp(rt) / wave_sum_dpp(tw);
      }
      if (lane == 0) {
        double chaos = chaos_raw;
        if (!isnan(chaos) && fabs(chaos - 1.0) <= 1e-8 + 1e-5) chaos = 0.0;  // np.isclose(moc, 1.0)
        chaos = clean(chaos);
        spatial = clean(spatial);
        spectral = clean(spectral);
        oc[ion] = chaos;
        osp[ion] = spatial;
        osc[ion] = spectral;
        omsm[ion] = chaos * spatial * spectral;
        oflags[ion] = flags | (uint32_t)D->hits;
      }
    }
    WV_STAMP(6);
    if (npos < 0) break;
    pos = npos;
    npos = n2pos;
    cur ^= 1;
  }
#ifdef SMG_WAVE_STAMPS
  if (lane == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&g_wstamps[i], wst[i]);
#endif
}

#ifdef SMG_WAVE_CHECK
extern "C" int smg_debug_wave_check(unsigned long long* host_out) {
  SMG_HIP(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wvchk), sizeof(unsigned long long) * 8));
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  SMG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wvchk), z, sizeof(z)));
  return SMG_OK;
}
#endif

#ifdef SMG_WAVE_STAMPS
extern "C" int smg_debug_wave_stamps(unsigned long long* host_out) {
  SMG_HIP(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wstamps), sizeof(unsigned long long) * 8));
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  SMG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wstamps), z, sizeof(z)));
  return SMG_OK;
}
#endif

#ifdef SMG_WAVE_TRACE
extern "C" int smg_debug_wave_trace(long long* host_out, int n) {
  SMG_HIP(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wtrace), sizeof(long long) * 8 * (n < 8192 ? n : 8192)));
  return SMG_OK;
}
#endif

// segment shift of the directory: the smallest S >= 3 with ceil(npx / 2^S) <= 2046 (0 if the image is too large)
static int wave_seg_shift(int npx) {
  for (int S = 3; S <= 15; ++S)
    if ((((int64_t)npx + (1ll << S) - 1) >> S) <= WaveLay<WAVE_CAP>::NDIR - 2) return S;
  return 0;
}

size_t wave_pass_lds_bytes() { return WaveLay<WAVE_CAP>::bytes; }

bool wave_pass_supports(int npx) { return npx < (1 << 24) && wave_seg_shift(npx) > 0; }

// main pass over every position of the processing order: one wave per workgroup, as many per CU as the LDS
// holds; rejects (positions) to rej_list for the big-ion LDS pass
int launch_wave_pass(const uint64_t* hits, const IonDesc* desc, int64_t n_ions, const Params& P, uint32_t* xcd_ctr,
                     double* oc, double* osp, double* osc, double* omsm, uint32_t* oflags, uint32_t* rej_list,
                     uint32_t* rej_count, int cus, hipStream_t st) {
  const int SH = wave_seg_shift(P.npx);
  if (SH == 0) {
    set_error("image too large for the wave pass");
    return SMG_ERR_INVALID;
  }
  auto k = &ion_wave_kernel<WAVE_CAP, WAVE_RC>;
  const size_t lds = WaveLay<WAVE_CAP>::bytes;
  SMG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = (int)((160 * 1024) / lds);
  if (per_cu > 12) per_cu = 12;
  int64_t nwg = (int64_t)cus * per_cu;
  if (nwg > n_ions) nwg = ((n_ions + XCDS - 1) / XCDS) * XCDS;
  Sched SA{n_ions, xcd_ctr, nullptr, nullptr};
  Hits<SMG_HITS_PACKED_F32> h{hits, nullptr};
  hipLaunchKernelGGL(k, dim3((unsigned)nwg), dim3(64), lds, st, h, desc, SA, P, SH, oc, osp, osc, omsm, oflags,
                     rej_list, rej_count);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // namespace smg
