// Result rows of the ion images on gfx950 (search_results.py:88-97, SearchResults.store_sf_iso_images'
// iso_img_row_gen): per (ion, peak) image, the pixels whose summed intensity is > 0.001 in flattened-index order,
// their intensities, and the min / max over the whole nrows*ncols image -- without densifying any image.
//
// A window's image is the run [lo, hi) of the m/z-sorted hits; duplicate pixels are summed (coo.toarray()).
// Pipeline over the listed windows (all device, one stream):
//   1. exclusive scan of the run lengths -> each window's slice of a contiguous gather buffer
//   2. gather_rows_kernel: key = window << 31 | pixel (u64), value = f64 intensity, window-major
//   3. rocPRIM radix sort by key (stable: a pixel's duplicates keep their m/z order, so the f64 sums are
//      deterministic)
//   4. run_sums_kernel: each run of equal keys summed by its head; heads over the threshold flagged; per-window
//      distinct-pixel count, kept count, max and min of the sums (u64 atomics on order-preserving f64 bits)
//   5. exclusive scan of the flags -> compacted (pixel, value) rows, window-major, pixels ascending
//   6. window_stats_kernel: min / max over the full image (uncovered pixels are 0)
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "smg_common.hpp"

namespace smg {

// f64 -> u64 with the same order (so u64 atomicMax / atomicMin order the sums), and back
__device__ __forceinline__ unsigned long long ord_bits(double x) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double ord_value(unsigned long long u) {
  const unsigned long long b = (u >> 63) ? (u & 0x7FFFFFFFFFFFFFFFull) : ~u;
  return __longlong_as_double((long long)b);
}

__global__ void __launch_bounds__(256) gather_rows_kernel(const uint64_t* __restrict__ hits,
                                                          const int64_t* __restrict__ lo,
                                                          const int64_t* __restrict__ hi,
                                                          const int64_t* __restrict__ seg_off, int64_t n_windows,
                                                          uint64_t* __restrict__ keys, double* __restrict__ vals) {
  // one workgroup per window (grid-stride): the run is read coalesced
  for (int64_t w = blockIdx.x; w < n_windows; w += gridDim.x) {
    const int64_t a = lo[w], n = hi[w] - a, o = seg_off[w];
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
      const uint64_t h = hits[a + i];
      keys[o + i] = ((uint64_t)w << 31) | (h & 0x7FFFFFFFull);
      vals[o + i] = (double)__uint_as_float((uint32_t)(h >> 32));
    }
  }
}

__global__ void __launch_bounds__(256) run_sums_kernel(const uint64_t* __restrict__ keys,
                                                       const double* __restrict__ vals, int64_t total,
                                                       double threshold, double* __restrict__ sums,
                                                       int64_t* __restrict__ flag,
                                                       unsigned long long* __restrict__ wstat) {
  // wstat[4*w + {0,1,2,3}] = distinct pixels, kept pixels, max and min of the sums (ord_bits)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    const bool head = i == 0 || keys[i - 1] != k;
    int64_t f = 0;
    if (head) {
      double s = vals[i];
      for (int64_t j = i + 1; j < total && keys[j] == k; ++j) s += vals[j];  // duplicates, in m/z order
      sums[i] = s;
      const int64_t w = (int64_t)(k >> 31);
      unsigned long long* st = wstat + 4 * w;
      atomicAdd(&st[0], 1ull);
      const unsigned long long bits = ord_bits(s);
      atomicMax(&st[2], bits);
      atomicMin(&st[3], bits);
      if (s > threshold) {
        f = 1;
        atomicAdd(&st[1], 1ull);
      }
    }
    flag[i] = f;
  }
}

__global__ void __launch_bounds__(256) compact_rows_kernel(const uint64_t* __restrict__ keys,
                                                           const double* __restrict__ sums,
                                                           const int64_t* __restrict__ flag,
                                                           const int64_t* __restrict__ pos, int64_t total,
                                                           int32_t* __restrict__ out_pix,
                                                           double* __restrict__ out_val) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    if (flag[i]) {
      const int64_t p = pos[i];
      out_pix[p] = (int32_t)(keys[i] & 0x7FFFFFFFull);
      out_val[p] = sums[i];
    }
  }
}

__global__ void __launch_bounds__(256) window_stats_kernel(const unsigned long long* __restrict__ wstat,
                                                           int64_t n_windows, int64_t npx,
                                                           int64_t* __restrict__ out_count,
                                                           double* __restrict__ out_min,
                                                           double* __restrict__ out_max) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n_windows) return;
  const unsigned long long* st = wstat + 4 * w;
  const int64_t distinct = (int64_t)st[0];
  out_count[w] = (int64_t)st[1];
  // np.zeros(npx) + the coo sums: a pixel without a point is 0 (a None image is all zeros)
  const double mx = distinct > 0 ? ord_value(st[2]) : 0.0;
  const double mn = distinct > 0 ? ord_value(st[3]) : 0.0;
  const bool full = distinct >= npx;
  out_max[w] = full ? mx : (mx > 0.0 ? mx : 0.0);
  out_min[w] = full ? mn : (mn < 0.0 ? mn : 0.0);
}

__global__ void init_wstat_kernel(unsigned long long* __restrict__ wstat, int64_t n_windows) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n_windows) return;
  wstat[4 * w + 0] = 0ull;
  wstat[4 * w + 1] = 0ull;
  wstat[4 * w + 2] = 0ull;
  wstat[4 * w + 3] = ~0ull;
}

__global__ void run_lengths_kernel(const int64_t* __restrict__ lo, const int64_t* __restrict__ hi, int64_t n,
                                   int64_t* __restrict__ len) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < n) len[w] = hi[w] - lo[w];
  if (w == n) len[w] = 0;
}

// workspace carve (16-B aligned pieces)
struct RowsWs {
  int64_t* len;        // [n+1]
  int64_t* seg_off;    // [n+1]
  uint64_t* k0;        // [total]
  uint64_t* k1;
  double* v0;
  double* v1;
  double* sums;        // [total]
  int64_t* flag;       // [total]
  int64_t* pos;        // [total]
  unsigned long long* wstat;  // [4n]
  void* tmp;
  size_t tmp_bytes;
};

static inline size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

static int rows_tmp_bytes(int64_t total, int64_t n_windows, int end_bit, size_t* bytes) {
  size_t s1 = 0, s2 = 0, s3 = 0;
  rocprim::double_buffer<uint64_t> kb(nullptr, nullptr);
  rocprim::double_buffer<double> vb(nullptr, nullptr);
  SMG_HIP(rocprim::radix_sort_pairs(nullptr, s1, kb, vb, (size_t)(total > 0 ? total : 1), 0, end_bit));
  SMG_HIP(rocprim::exclusive_scan(nullptr, s2, (const int64_t*)nullptr, (int64_t*)nullptr, (int64_t)0,
                                  (size_t)(n_windows + 1), rocprim::plus<int64_t>()));
  SMG_HIP(rocprim::exclusive_scan(nullptr, s3, (const int64_t*)nullptr, (int64_t*)nullptr, (int64_t)0,
                                  (size_t)(total > 0 ? total : 1), rocprim::plus<int64_t>()));
  size_t m = s1 > s2 ? s1 : s2;
  *bytes = m > s3 ? m : s3;
  return SMG_OK;
}

static int end_bit_for(int64_t n_windows) {
  int b = 1;
  while (b < 33 && ((int64_t)1 << b) < n_windows) ++b;
  return 31 + b;
}

static int rows_carve(void* ws, int64_t total, int64_t n, int end_bit, RowsWs& R, size_t* need) {
  size_t tmp = 0;
  int rc = rows_tmp_bytes(total, n, end_bit, &tmp);
  if (rc != SMG_OK) return rc;
  const size_t t = (size_t)(total > 0 ? total : 1);
  size_t o = 0;
  auto take = [&](size_t b) {
    const size_t at = o;
    o += a16(b);
    return at;
  };
  const size_t o_len = take(8 * (size_t)(n + 1)), o_seg = take(8 * (size_t)(n + 1)), o_k0 = take(8 * t),
               o_k1 = take(8 * t), o_v0 = take(8 * t), o_v1 = take(8 * t), o_s = take(8 * t), o_f = take(8 * t),
               o_p = take(8 * t), o_w = take(32 * (size_t)(n > 0 ? n : 1)), o_tmp = take(tmp);
  *need = o;
  if (ws) {
    unsigned char* b = reinterpret_cast<unsigned char*>(ws);
    R.len = reinterpret_cast<int64_t*>(b + o_len);
    R.seg_off = reinterpret_cast<int64_t*>(b + o_seg);
    R.k0 = reinterpret_cast<uint64_t*>(b + o_k0);
    R.k1 = reinterpret_cast<uint64_t*>(b + o_k1);
    R.v0 = reinterpret_cast<double*>(b + o_v0);
    R.v1 = reinterpret_cast<double*>(b + o_v1);
    R.sums = reinterpret_cast<double*>(b + o_s);
    R.flag = reinterpret_cast<int64_t*>(b + o_f);
    R.pos = reinterpret_cast<int64_t*>(b + o_p);
    R.wstat = reinterpret_cast<unsigned long long*>(b + o_w);
    R.tmp = b + o_tmp;
    R.tmp_bytes = tmp;
  }
  return SMG_OK;
}

}  // namespace smg

using namespace smg;

extern "C" {

int smg_iso_image_rows_workspace_size(int64_t n_windows, int64_t total_points, size_t* bytes) {
  SMG_CHECK_ARG(bytes && n_windows >= 0 && total_points >= 0, "bad arguments");
  SMG_CHECK_ARG(n_windows < (1ll << 32), "too many windows");
  RowsWs R;
  return rows_carve(nullptr, total_points, n_windows, end_bit_for(n_windows), R, bytes);
}

int smg_iso_image_rows(const uint64_t* hits, const int64_t* lo, const int64_t* hi, int64_t n_windows,
                       int64_t total_points, int64_t npx, double threshold, int64_t* out_count, double* out_min,
                       double* out_max, int32_t* out_pix, double* out_val, void* workspace, size_t workspace_bytes,
                       void* stream) {
  SMG_CHECK_ARG(n_windows >= 0 && total_points >= 0 && npx > 0, "bad arguments");
  SMG_CHECK_ARG(n_windows < (1ll << 32), "too many windows");
  if (n_windows == 0) return SMG_OK;
  SMG_CHECK_ARG(hits && lo && hi && out_count && out_min && out_max && workspace, "null pointer");
  SMG_CHECK_ARG(total_points == 0 || (out_pix && out_val), "null output rows");
  const int end_bit = end_bit_for(n_windows);
  RowsWs R;
  size_t need = 0;
  int rc = rows_carve(workspace, total_points, n_windows, end_bit, R, &need);
  if (rc != SMG_OK) return rc;
  if (workspace_bytes < need) {
    set_error("iso_image_rows workspace too small: %zu < %zu", workspace_bytes, need);
    return SMG_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const unsigned nb = (unsigned)((n_windows + 1 + 255) / 256);
  hipLaunchKernelGGL(run_lengths_kernel, dim3(nb), dim3(256), 0, st, lo, hi, n_windows, R.len);
  SMG_LAUNCH_CHECK();
  size_t tb = R.tmp_bytes;
  SMG_HIP(rocprim::exclusive_scan(R.tmp, tb, R.len, R.seg_off, (int64_t)0, (size_t)(n_windows + 1),
                                  rocprim::plus<int64_t>(), st));
  hipLaunchKernelGGL(init_wstat_kernel, dim3((unsigned)((n_windows + 255) / 256)), dim3(256), 0, st, R.wstat,
                     n_windows);
  SMG_LAUNCH_CHECK();
  if (total_points > 0) {
    // the caller sized total_points = sum(hi - lo) (seg_off[n]); the gather writes exactly that many entries
    const unsigned gw = (unsigned)(n_windows < 65536 ? n_windows : 65536);
    hipLaunchKernelGGL(gather_rows_kernel, dim3(gw), dim3(256), 0, st, hits, lo, hi, R.seg_off, n_windows, R.k0,
                       R.v0);
    SMG_LAUNCH_CHECK();
    rocprim::double_buffer<uint64_t> kb(R.k0, R.k1);
    rocprim::double_buffer<double> vb(R.v0, R.v1);
    tb = R.tmp_bytes;
    SMG_HIP(rocprim::radix_sort_pairs(R.tmp, tb, kb, vb, (size_t)total_points, 0, end_bit, st));
    const int64_t g = (total_points + 255) / 256;
    const unsigned ge = (unsigned)(g < 65536 ? g : 65536);
    hipLaunchKernelGGL(run_sums_kernel, dim3(ge), dim3(256), 0, st, kb.current(), vb.current(), total_points,
                       threshold, R.sums, R.flag, R.wstat);
    SMG_LAUNCH_CHECK();
    tb = R.tmp_bytes;
    SMG_HIP(rocprim::exclusive_scan(R.tmp, tb, R.flag, R.pos, (int64_t)0, (size_t)total_points,
                                    rocprim::plus<int64_t>(), st));
    hipLaunchKernelGGL(compact_rows_kernel, dim3(ge), dim3(256), 0, st, kb.current(), R.sums, R.flag, R.pos,
                       total_points, out_pix, out_val);
    SMG_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(window_stats_kernel, dim3((unsigned)((n_windows + 255) / 256)), dim3(256), 0, st, R.wstat,
                     n_windows, npx, out_count, out_min, out_max);
  SMG_LAUNCH_CHECK();
  return SMG_OK;
}

}  // extern "C"
