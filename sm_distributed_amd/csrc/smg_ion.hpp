// Device-side definitions shared by the ion kernels of libsmg (smg_metrics.hip: the LDS, wide and
// pixel-indexed passes): kernel parameters, the two hit formats, asynchronous load helpers, level index, ion
// descriptors, persistent scheduling, LDS union-find.
#pragma once

#include "smg_common.hpp"

namespace smg {

constexpr int MAXK = 8;              // windows per ion on the LDS path
constexpr int MAXK_DENSE = 32;       // windows per ion supported at all
constexpr int NPX_LDS_MAX = 1 << 18; // images up to 262144 pixels use the LDS path

enum { C_NE = 0, C_EMAX, C_ABORT, C_PDUP, C_NEXT, C_NS, C_NCTR = 8 };

struct Params {
  int32_t nrows, ncols, npx;
  int32_t nlevels;
  int32_t connectivity;
  int32_t erosion_border;
  double step;      // np.linspace(0, 1, nlevels) step
  float inv_ncols;  // 1/ncols for the LDS path's row/column split (npx < 2^24)
  int32_t w32;      // LDS path: bitmap words (Lay::w32)
  uint32_t o_pf;    // LDS path: byte offset of the rank prefix (Lay::o_pf)
  double q;         // hot-spot clip percentile (dense path, when clip != 0)
  int32_t clip;     // image_generation.do_preprocessing
};

// row and column of pixel p < 2^24 from a float reciprocal: the estimate is off by at most one row
// (branch-free: the correction is two compares and selects)
__device__ __forceinline__ void rowcol(int p, const Params& P, int& r, int& c) {
  r = (int)((float)p * P.inv_ncols);
  c = p - r * P.ncols;
  const int adj = c < 0 ? -1 : (c >= P.ncols ? 1 : 0);
  r += adj;
  c -= adj * P.ncols;
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
  static __device__ __forceinline__ Reg zero() { return 0ull; }  // pixel 0, value 0, no flag
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

// Asynchronous 8-byte loads for the software pipeline of the LDS kernel.  The compiler's wait-count pass
// serialises any use of a register loaded before a loop or a branch behind s_waitcnt vmcnt(0), i.e. behind
// every load issued since, which would expose the latency of each prefetched chunk; these loads are
// invisible to it and are waited for with counted waits (vm_wait<N>: all but the N youngest vector-memory
// operations of this wave done).  Vector-memory operations complete in issue order, so operations the
// compiler issues in between only make a counted wait stricter.  The destination registers are neither
// read nor copied between issue and wait (the wait takes them as in/out operands).
// The destination is an in/out operand: its previous value counts as used by the next load into it, so
// a register with a load in flight is never reallocated to another value, even when that load's data end
// up unused (a refill past the tail, or an ion that is handed to another pass).
#ifdef SMG_CHECK
// The check build's extra code spills registers (the compiler cannot know that a register with one of these loads
// in flight must not be read -- a spill reads it), so there every asynchronous load is a compiler-tracked one and the
// counted waits are empty: slower, and immune to that hazard, which only scripts/check_async_regs.py rules out in
// the shipped ISA.
__device__ __forceinline__ void ld8_async(uint64_t& r, const void* sbase, uint32_t voff) {
  r = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(sbase) + voff);
}
__device__ __forceinline__ void ld8_async_v(uint64_t& r, const void* addr) { r = *reinterpret_cast<const uint64_t*>(addr); }
__device__ __forceinline__ void ld4_async_v(uint32_t& r, const void* addr) { r = *reinterpret_cast<const uint32_t*>(addr); }
template <int N>
__device__ __forceinline__ void vm_wait1(uint64_t&) {}
template <int N>
__device__ __forceinline__ void vm_wait1(uint32_t&) {}
#else
__device__ __forceinline__ void ld8_async(uint64_t& r, const void* sbase, uint32_t voff) {
  asm volatile("global_load_dwordx2 %0, %1, %2" : "+v"(r) : "v"(voff), "s"(sbase) : "memory");
}
__device__ __forceinline__ void ld8_async_v(uint64_t& r, const void* addr) {  // 64-bit vector address
  asm volatile("global_load_dwordx2 %0, %1, off" : "+v"(r) : "v"(addr) : "memory");
}
__device__ __forceinline__ void ld4_async_v(uint32_t& r, const void* addr) {
  asm volatile("global_load_dword %0, %1, off" : "+v"(r) : "v"(addr) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait1(uint64_t& r) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  asm volatile("" : "+v"(r));
}
template <int N>
__device__ __forceinline__ void vm_wait1(uint32_t& r) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  asm volatile("" : "+v"(r));
}
#endif
// Returning atomic add issued like the async loads: the compiler would wait for its result with
// s_waitcnt vmcnt(0) right away -- i.e. for every prefetch load of the wave in flight -- so it is waited
// for with a counted vm_wait1 where the ticket is consumed.
// Tagged "smg:wave0" in the ISA: issued by wave 0 only and waited by wave 0 only (scripts/check_async_regs.py
// accepts a path that skips its wait only through an exec-zero branch, i.e. in another wave).
#ifdef SMG_CHECK
__device__ __forceinline__ void atomic_add_rtn_async(uint32_t& r, uint32_t* addr, uint32_t v) { r = atomicAdd(addr, v); }
__device__ __forceinline__ void ld8_async_wave0(uint64_t& r, const void* addr) {
  r = *reinterpret_cast<const uint64_t*>(addr);
}
template <int N, int M>
__device__ __forceinline__ void vm_wait(uint64_t (&)[M]) {}
#else
__device__ __forceinline__ void atomic_add_rtn_async(uint32_t& r, uint32_t* addr, uint32_t v) {
  asm volatile("global_atomic_add %0, %1, %2, off sc0 ; smg:wave0" : "+v"(r) : "v"(addr), "v"(v) : "memory");
}
// an 8-byte load issued and waited by wave 0 only (the ion descriptor), tagged like the ticket
__device__ __forceinline__ void ld8_async_wave0(uint64_t& r, const void* addr) {
  asm volatile("global_load_dwordx2 %0, %1, off ; smg:wave0" : "+v"(r) : "v"(addr) : "memory");
}
template <int N, int M>
__device__ __forceinline__ void vm_wait(uint64_t (&r)[M]) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
  for (int j = 0; j < M; ++j) asm volatile("" : "+v"(r[j]));
}
#endif
template <int N, int M>
__device__ __forceinline__ void vm_wait(PixVal (&)[M]) {}  // split-format hits use compiler-tracked loads

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
  static __device__ __forceinline__ Reg zero() { return PixVal{0u, 0.0}; }
  __device__ __forceinline__ void get(int64_t i, uint32_t& p, double& v) const {
    p = pa[i] & 0x7FFFFFFFu;
    v = va[i];
  }
};

// level index L = #{i : linspace(0,1,n)[i] < v/vmax}  (measure_of_chaos: bw = im_clean > level)
// The levels are nondecreasing in i, so L is the lower bound of norm among them (binary search).
__device__ __forceinline__ int level_of(double v, double vmax, const Params& P) {
  const double norm = v / vmax;
  int lo = 0, len = P.nlevels;
  while (len > 0) {
    const int half = len >> 1, mid = lo + half;
    const double lev = (P.nlevels > 1 && mid == P.nlevels - 1) ? 1.0 : (double)mid * P.step;
    if (lev < norm) {
      lo = mid + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return lo;
}

__device__ __forceinline__ double clean(double v) {  // ImgMeasures._replace_nan
  return (v == 0.0 || isnan(v) || isinf(v)) ? 0.0 : v;
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

// the level index's f32 test: 1 (round 6) a margin of (n-1) * 1e-6 and the top interval included, 0 a margin of 1e-3
// with the top interval sent to the f64 test (the lanes of a wave with an entry in the top interval all waited for it;
// ion stage 25.97 -> 25.82 ms at config 3, profiles/round6/r6var4_variants.txt).  Used by ion_sparse_kernel and the
// join wide pass's eL (ion_wide_join_kernel)
#ifndef SMG_SP_LVM
#define SMG_SP_LVM 1
#endif

// the exact level index (divisions, loops), kept out of line so that the loops calling sp_level stay small
static __device__ __noinline__ int sp_level_exact(double v, double vmax, const Params& P) { return level_fast(v, vmax, P); }

// level_fast(v, vmax, P) = #{i <= n-2 : i*step < v/vmax} (+ [1 < v/vmax], 0 here: v <= vmax) with the division
// replaced by v * (1/vmax) where that cannot change the answer.  With x = (v/vmax)(n-1) non-integer, the count is
// floor(x) + 1 (capped at n-1); the two comparisons that decide it are checked against na = v*rcp with a margin above
// na's error (<= 2 ulp), and anything closer (or v ~ vmax) takes the exact path.  Straight-line: no loops.
__device__ __forceinline__ int sp_level(double v, double vmax, double rcp, const Params& P) {
  const int n = P.nlevels;
  if (!(v > 0.0)) return 0;  // (vmax > 0 whenever levels are needed)
  if (n == 1) return 1;
  if (n <= 2048) {  // f32 first: x = v/vmax (n-1) to ~2.4e-7 relative, i.e. (n-1) * 2.4e-7 absolute; farther than
                    // SMG_SP_LVM = (n-1) * 1e-6 from an integer and from n-1 itself (the top interval (n-2, n-1) is
                    // the count n-1 like any other) it decides alone
#if SMG_SP_LVM
    const float xf = (float)v * (float)rcp * (float)(n - 1);
    const float jf = floorf(xf), fr = xf - jf;
    const float mg = (float)(n - 1) * 1e-6f;
    if (fr > mg && fr < 1.0f - mg && xf < (float)(n - 1) - mg) return (int)jf + 1;
#else
    const float xf = (float)v * (float)rcp * (float)(n - 1);
    const float jf = floorf(xf), fr = xf - jf;
    if (fr > 1e-3f && fr < 1.0f - 1e-3f && xf < (float)(n - 1) - 1.0f) return (int)jf + 1;
#endif
  }
  const double na = v * rcp;
  const double tol = na * 1e-15;
  int j = (int)(na * (double)(n - 1)) + 1;
  j = j > n - 1 ? n - 1 : j;
  const bool lo_ok = (double)(j - 1) * P.step < na - tol;
  const bool hi_ok = j == n - 1 || (double)j * P.step >= na + tol;
  return (na < 1.0 - 1e-12 && lo_ok && hi_ok) ? j : sp_level_exact(v, vmax, P);
}


// ---------------------------------------------------------------------------------------------
// Ion descriptors: one 256-B record per position of the processing order (ion_desc_kernel), so that a
// workgroup reaches an ion's windows with one coalesced read instead of the ion_order -> ion_off -> lo/hi
// chain.  The tail windows 1..K-1 form one stream of 64-point groups, each window padded to whole groups,
// so that every group (one wave's share of a chunk slot) lies in a single window.
// ---------------------------------------------------------------------------------------------
struct IonDesc {
  int64_t base[MAXK];  // [0]: lo of the principal window; [k>=1]: lo[k] - 64*gs[k] (padded tail position -> hit)
  int32_t end[MAXK];   // [0]: principal points; [k>=1]: 64*gs[k] + n[k] (end of window k in the padded tail)
  int32_t gs[MAXK];    // [k>=1]: first group of window k; INT_MAX for k >= K
  double theor[MAXK];  // theoretical intensities
  double sy[MAXK];     // window sums of intensities (prefix-sum differences, smg_hit_prefix_sums)
  double syy[MAXK];    // window sums of squared intensities over points without the duplicate flag
  int32_t ion, K, ngroups, hits;  // ngroups < 0: tail too long for 32-bit positions (dense path)
  int32_t pad[12];
};
static_assert(sizeof(IonDesc) == 384, "IonDesc is 384 B");
constexpr int DESC_QWORDS = (int)(sizeof(IonDesc) / 8);  // 48: one 8-byte load per lane of wave 0

// The same 384 B once an LDS pass has scored the position: the consumed window fields (base, end, gs, pad) hold the
// ion's sums, and ion_finalize_kernel computes the scores from them (state == 1) after the pass.
struct IonRec {
  double s[MAXK];      // over base[]: s[0] = Σx[x>0] of the principal image, s[k>=1] = Σy_k[x>0]
  double sxy[MAXK];    // over end[], gs[]: Σ x·y_k
  double theor[MAXK];  // unchanged
  double sy[MAXK];     // unchanged: Σy_k
  double syy[MAXK];    // Σy_k² + the squared per-pixel sums of duplicate candidates
  int32_t ion, K, ngroups, hits;
  double sx, sxx, chaos;  // over pad[]: Σx, Σx², raw measure_of_chaos
  uint32_t flags, state;
  int32_t pad[4];
};
static_assert(sizeof(IonRec) == sizeof(IonDesc) && offsetof(IonRec, theor) == offsetof(IonDesc, theor) &&
                  offsetof(IonRec, syy) == offsetof(IonDesc, syy) && offsetof(IonRec, ion) == offsetof(IonDesc, ion) &&
                  offsetof(IonRec, sx) == offsetof(IonDesc, pad),
              "IonRec overlays IonDesc");

// Work sources of the persistent LDS kernel.
//  SRC_RANGES: positions [0, n) split into 8 contiguous ranges, one per XCD (workgroup w runs on XCD w % 8),
//    so concurrently scored ions of one XCD are m/z neighbours and share windows in that XCD's L2; a
//    workgroup whose range is exhausted steals from the other ranges.
//  SRC_LIST: a device list of positions (the rejects of the previous pass) with a global cursor.
enum { SRC_RANGES = 0, SRC_LIST = 1 };
#ifndef SMG_SCREEN2P
#define SMG_SCREEN2P 1  // chaos screen in two passes (pre-filtered survivors, then the full screen over them)
#endif
#ifndef SMG_NOB3
#define SMG_NOB3 1      // no barrier after the duplicate-table reduce when the two-pass screen follows
#endif
constexpr int CTR_STRIDE = 32;  // u32 words between counters (one 128-B line each)

struct Sched {
  int64_t n;              // SRC_RANGES: positions
  uint32_t* ctr;          // SRC_RANGES: XCDS counters; SRC_LIST: cursor
  const uint32_t* list;   // SRC_LIST
  const uint32_t* count;  // SRC_LIST
  uint32_t rej_cap;       // entries the pass's reject list holds (n_ions): a reject beyond it is dropped and counted
};

// ---- SMG_CHECK: the diagnostic build `make check` (-> libsmg_check.so, never the product) --------------------------
// Every ion pass checks, per position it scores: that no other workgroup took the same position in this pass (a
// claimed bit per position, set with atomicOr); that the 384-B descriptor it read equals what lo / hi / ion_off /
// ion_order say for that position (so a record or stale bytes read as a descriptor are caught); that every global
// index it loads lies inside its window and inside [0, n_points); and that no reject overflows its list.  Failures are
// counted (smg_debug_check_read) and the first few printed with their position.
// counters: positions claimed, descriptor mismatches, loads out of their window, double hand-outs, records read as
// descriptors, reject-list overflows, windows outside [0, n_points], descriptors checked
enum { CHK_IONS = 0, CHK_DESC, CHK_INDEX, CHK_DOUBLE, CHK_STATE, CHK_REJ, CHK_WINDOW, CHK_DESCS, CHK_N = 8 };
struct ChkCtx {
  const int64_t* lo;         // the scored windows (lo2 / hi2 of smg_ion_metrics)
  const int64_t* hi;
  const int64_t* ion_off;    // windows per ion (theoretical peaks)
  const int64_t* ion_order;  // position -> ion
  uint32_t* claim;           // bit per position and pass (zeroed per launch), pass p at claim + p * words
  int64_t words;
  int64_t n_points;          // resident hits (smg_debug_check_points)
  unsigned long long* cnt;   // CHK_N counters (persistent, read and reset by smg_debug_check_read)
};
#ifdef SMG_CHECK
#define SMG_CHK_PARAM , ::smg::ChkCtx CK
#define SMG_CHK_ARG(c) , (c)
__device__ __forceinline__ bool chk(const ChkCtx& C, bool ok, int code, int64_t a, int64_t b) {
  if (!ok) {
    const unsigned long long k = atomicAdd(&C.cnt[code], 1ull);
    if (k < 4) printf("SMG_CHECK failure %d: %lld %lld (wg %d, tid %d)\n", code, (long long)a, (long long)b,
                      (int)blockIdx.x, (int)threadIdx.x);
  }
  return ok;
}
// a load of hit `idx` for window k of ion `ion` (idx 0 stands for a group past the tail: a stand-in load)
__device__ __forceinline__ void chk_load(const ChkCtx& C, int64_t ion, int k, int64_t idx, bool standin) {
  if (standin) {
    chk(C, idx == 0, CHK_INDEX, ion, idx);
    return;
  }
  const int64_t w = C.ion_off[ion] + k;
  chk(C, idx >= C.lo[w] && idx < C.hi[w] && idx >= 0 && idx < C.n_points, CHK_INDEX, ion * 64 + k, idx);
}
// claims position `pos` for pass `pass`; wave-uniform call, lane 0 acts
__device__ __forceinline__ void chk_claim(const ChkCtx& C, int pass, int64_t pos) {
  if ((threadIdx.x & 63) == 0) {
    const uint32_t b = 1u << (pos & 31);
    chk(C, !(atomicOr(&C.claim[pass * C.words + (pos >> 5)], b) & b), CHK_DOUBLE, pass, pos);
    atomicAdd(&C.cnt[CHK_IONS], 1ull);
  }
}
// the descriptor D (LDS copy) of position pos against the arrays it was made from; wave-uniform call, lane k checks
// window k
__device__ __forceinline__ void chk_desc(const ChkCtx& C, int64_t pos, const IonDesc* D) {
  const int lane = threadIdx.x & 63;
  const int64_t ion = C.ion_order ? C.ion_order[pos] : pos;
  const int64_t w0 = C.ion_off[ion];
  const int K = (int)(C.ion_off[ion + 1] - w0);
  if (lane == 0) {
    chk(C, D->ion == ion && D->K == K, CHK_DESC, pos, ((int64_t)D->ion << 8) | (D->K & 255));
    atomicAdd(&C.cnt[CHK_DESCS], 1ull);
  }
  if (lane < K && lane < MAXK) {
    const int64_t a = C.lo[w0 + lane], b = C.hi[w0 + lane];
    chk(C, a >= 0 && b >= a && b <= C.n_points, CHK_WINDOW, pos * 64 + lane, a);
    const int64_t g = lane == 0 ? 0 : (int64_t)D->gs[lane] * 64;
    chk(C, D->base[lane] + g == a && (int64_t)D->end[lane] - g == b - a, CHK_DESC, pos * 64 + lane,
        D->base[lane] + g - a);
  }
}
#else
#define SMG_CHK_PARAM
#define SMG_CHK_ARG(c)
#endif

// A ticket is resolved against the counter it was drawn from (``home``, recorded at issue): a workgroup may move to
// another XCD between the two -- a queue eviction saves and restores its waves, possibly elsewhere -- and a ticket of
// one XCD's counter read against another XCD's range names a position that counter never handed out.  Two workgroups
// then score the same position, and one of them may read the other's IonRec (written over the descriptor) as a
// descriptor: window bases made of sums, a load from a wild address (round 5: a memory-aperture fault in a bench run
// that coincided with a KFD eviction of the process's queues).
template <int SRC>
__device__ __forceinline__ uint32_t sched_issue(const Sched& S, int& home) {
  home = home_xcd();
  if constexpr (SRC == SRC_RANGES) return atomicAdd(&S.ctr[home * CTR_STRIDE], 1u);
  else return atomicAdd(S.ctr, 1u);
}
// the same ticket, asynchronously (see atomic_add_rtn_async); valid after the counted wait
template <int SRC>
__device__ __forceinline__ void sched_issue_async(const Sched& S, uint32_t& t, int& home) {
  home = home_xcd();
  if constexpr (SRC == SRC_RANGES) atomic_add_rtn_async(t, &S.ctr[home * CTR_STRIDE], 1u);
  else atomic_add_rtn_async(t, S.ctr, 1u);
}

// resolves a ticket of sched_issue, drawn from XCD ``home``'s counter, into a position (-1: no work left); further
// tickets come from the next XCDs' counters in turn
template <int SRC>
__device__ __forceinline__ int64_t sched_resolve(const Sched& S, uint32_t t, int home) {
  if constexpr (SRC == SRC_RANGES) {
    for (int i = 0; i < XCDS; ++i) {
      const int x = (home + i) % XCDS;
      const int64_t a = (int64_t)((uint64_t)(S.n * x) / XCDS), b = (int64_t)((uint64_t)(S.n * (x + 1)) / XCDS);
      if (i > 0) t = atomicAdd(&S.ctr[x * CTR_STRIDE], 1u);
      if ((int64_t)t < b - a) return a + (int64_t)t;
    }
    return -1;
  } else {
    const uint32_t c = *S.count;
    return t < c ? (int64_t)S.list[t] : -1;
  }
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const int lo = __builtin_amdgcn_readfirstlane((int)v), hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
  return ((int64_t)hi << 32) | (uint32_t)lo;
}

// (a position some pass already scored holds an IonRec, state 1 -- pad[7] of a descriptor is 0: never read its
// sums as window bases, whatever hands such a position out twice)
__device__ __forceinline__ bool desc_lds_ok(const IonDesc* D, int capc) {
  const int K = D->K;
  return K >= 1 && K <= MAXK && D->end[0] <= capc && D->ngroups >= 0 &&
         reinterpret_cast<const IonRec*>(D)->state == 0u;
}
static_assert(offsetof(IonRec, state) == offsetof(IonDesc, pad) + 7 * sizeof(int32_t), "IonRec::state over pad[7]");

// (key, f64 sum) open-addressing table in LDS (empty key 0xFFFFFFFF): adds v to key's sum; false when full
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

// ---- the sparse main pass (smg_sparse.hip) ----------------------------------------------------------------
// true when the 256-thread sparse-set main pass takes this image (packed hits, no clip, <= 2^18 pixels);
// launch_sparse_main launches it with the main pass's interface (positions it cannot
// score go to rej_list / rej_count for the big-ion pass)
bool sparse_main_fits(const Params& P);
int launch_sparse_main(Hits<SMG_HITS_PACKED_F32> hits, IonDesc* desc, Sched S, const Params& P, double* oc,
                       double* osp, double* osc, double* omsm, uint32_t* oflags, uint32_t* rej_list,
                       uint32_t* rej_count, int cus, hipStream_t st, const ChkCtx& ck);
int sparse_read_stamps(unsigned long long* host_out, int n);

}  // namespace smg
