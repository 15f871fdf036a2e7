/*
 * smg.h -- C-ABI of libsmg.so, the MI355X (gfx950) kernels of the SM_distributed molecule-annotation
 * hot path: ion-image generation (formula_imager_segm.compute_sf_images) and MSM scoring
 * (formula_img_validator.sf_image_metrics).
 *
 * Conventions
 *  - every entry point returns an int status (SMG_OK = 0, < 0 on error); the message of the last
 *    error on the calling thread is returned by smg_last_error();
 *  - the caller owns every buffer; pointers marked "device" are HBM pointers (e.g. torch
 *    tensor.data_ptr()), sizes are int64_t, `stream` is a hipStream_t passed as void* (NULL = the
 *    null stream).  Hot entry points never allocate: size the workspace with the matching
 *    *_workspace_size() call first;
 *  - all calls are asynchronous on `stream` and re-entrant.  The only global mutable state is the
 *    thread-local error string and the process-wide diagnostic switches smg_debug_force_two_level /
 *    smg_debug_force_dense / smg_debug_time_main_pass (off by default; a test or benchmark that sets one must
 *    not run concurrently with other callers of smg_ion_metrics in the same process).
 *
 * Each entry point cites the reference interface it replaces (paths under frulo/SM_distributed).
 */
#ifndef SMG_H
#define SMG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMG_OK 0
#define SMG_ERR_INVALID (-1)     /* bad argument / shape */
#define SMG_ERR_HIP (-2)         /* HIP runtime error */
#define SMG_ERR_WORKSPACE (-3)   /* workspace too small */
#define SMG_ERR_UNSUPPORTED (-4) /* configuration not implemented */

/* per-ion flags written by smg_ion_metrics */
#define SMG_ION_HAS_HITS 0x1u    /* >= 1 window with >= 1 point: the ion gets a row (formula_img_validator.py:115-118) */
#define SMG_ION_DENSE 0x2u       /* scored by the dense (global-scratch) path instead of the LDS path */
#define SMG_ION_CHAOS_NAN 0x4u   /* raw measure_of_chaos was NaN (empty / < 4 positive pixels) */
#define SMG_ION_BIG 0x8u         /* scored by the big-ion LDS pass (1024-thread workgroup, whole LDS) */
#define SMG_ION_TWO_LEVEL 0x10u  /* LDS pass with the two-level pixel set (images > 2^18 pixels) */
#define SMG_ION_WIDE 0x20u       /* dense path, rank-indexed wide pass (LDS presence bitmap + rank prefix) */
#define SMG_ION_SPARSE 0x40u     /* main pass with the sparse principal set (ion_sparse_kernel, 256-thread workgroups) */

/* hit formats accepted by smg_ion_metrics */
#define SMG_HITS_PACKED_F32 0    /* uint64: low 32 bits pixel index, high 32 bits float32 intensity */
#define SMG_HITS_SPLIT_F64 1     /* uint32 pixel[] + double intensity[] */

/* "smg <version> (gfx950) git <source revision>[-dirty]": the tree the library was built from */
const char* smg_version(void);
const char* smg_last_error(void);

/* Pack one dataset into the resident hit layout: hit[i] = pixel_map[spectrum(i)] | f32bits(ints[i]) << 32.
 * Replaces the (sp_id -> pixel) join of formula_imager_segm.py:60-63 (_sp_df_gen) /
 * dataset.py:68-75 (get_norm_img_pixel_inds).  sp_off: device int64[n_spectra+1];
 * pixel_map: device int32[n_spectra]; ints: device float[n_points]; hits: device uint64[n_points]. */
int smg_pack_hits(const int64_t* sp_off, const int32_t* pixel_map, int64_t n_spectra,
                  const float* ints, int64_t n_points, uint64_t* hits, void* stream);

/* Duplicate-candidate flags (bit 31 of the packed pixel field).  Two points of one theoretical window can
 * only fall on the same pixel (and must then be summed, coo.toarray() in formula_img_validator.py:73-75) if
 * they come from the same spectrum and lie within one window width of each other, i.e. they are neighbours
 * in the m/z-sorted spectrum with gap <= 2*ppm*1e-6*mz/(1-ppm*1e-6).  This pass sets the flag on exactly
 * those points (and on every point of a spectrum that is not m/z-sorted, or whose pixel is shared with
 * another spectrum: force[s] != 0), clears it elsewhere, and writes only hits whose flag changes.
 * flag_state (optional, device uint8[n_points]) mirrors the flag each hit carries (initialise it from the hits:
 * (hit >> 31) & 1); with it, hits are read only where the flag changes.
 * Run it on the dataset-order hits before smg_sort_points; consumers mask pixels with 0x7FFFFFFF. */
int smg_flag_duplicates(const int64_t* sp_off, int64_t n_spectra, const float* mz, uint64_t* hits,
                        int64_t n_points, double ppm, const uint8_t* force, uint8_t* flag_state, void* stream);

/* Global m/z sort of the packed points (the pandas sort_values('mz') of formula_imager_segm.py:73-74,
 * done once over the whole dataset instead of per m/z segment).  Keys are positive float32 m/z; only their
 * low key_bits bits are sorted on (all keys must agree above them: key_bits = 32 - clz(bits(min) ^ bits(max));
 * 0 = all 31 bits).  Stable (equal m/z keep dataset order); not in place.  A hand-written LSD radix sort
 * (smg_sort.hip: ceil(key_bits / 9) passes, each one kernel with a look-back over earlier tiles). */
int smg_sort_points_workspace_size(int64_t n_points, size_t* bytes);
int smg_sort_points(const float* mz, const uint64_t* hits, int64_t n_points, int32_t key_bits,
                    float* mz_sorted, uint64_t* hits_sorted, void* workspace, size_t workspace_bytes,
                    void* stream);
/* smg_flag_duplicates + smg_sort_points in one: the sort's first pass sets bit 31 of every output hit by the
 * flag pass's rule (a spectrum neighbour within one window width; spectra from sp_off[0..n_spectra]).  The same
 * flags as smg_flag_duplicates when every spectrum is m/z-sorted and no pixel is shared (force all zero) -- the
 * caller checks both and otherwise runs the two calls.  The input hits are not written (their flag bits are
 * ignored). */
int smg_sort_points_flag(const int64_t* sp_off, int64_t n_spectra, const float* mz, const uint64_t* hits,
                         int64_t n_points, int32_t key_bits, double ppm, float* mz_sorted, uint64_t* hits_sorted,
                         void* workspace, size_t workspace_bytes, void* stream);

/* m/z slice of the resident dataset for one rank of a multi-GPU search (the formula list is sharded by m/z,
 * SURVEY.md §8e; the reference instead shuffles every point into m/z segments, formula_imager_segm.py:45-49,
 * 112-121, 152-155): the points with lo <= mz <= hi (compared in float64, as smg_window_bounds compares), in
 * dataset order.  Spectra must be m/z-sorted.  Two calls: smg_slice_mz_count writes the slice's spectrum
 * offsets out_sp_off (device int64[n_spectra+1]; out_sp_off[n_spectra] = slice size) and keeps each spectrum's
 * first selected point in the workspace; smg_slice_mz_copy (same workspace, unchanged) copies the points and
 * sets bit 31 of each copied hit to its duplicate-candidate flag for `ppm` (smg_flag_duplicates semantics;
 * force: optional uint8[n_spectra]), so the slice needs no separate flag pass. */
int smg_slice_mz_workspace_size(int64_t n_spectra, size_t* bytes);
int smg_slice_mz_count(const int64_t* sp_off, int64_t n_spectra, const float* mz, double lo, double hi,
                       int64_t* out_sp_off, void* workspace, size_t workspace_bytes, void* stream);
int smg_slice_mz_copy(const int64_t* sp_off, int64_t n_spectra, const float* mz, const uint64_t* hits,
                      const int64_t* out_sp_off, double ppm, const uint8_t* force, float* out_mz,
                      uint64_t* out_hits, const void* workspace, void* stream);

/* Window search (formula_imager_segm.py:79-82): lower = mz - mz*ppm*1e-6, upper = mz + mz*ppm*1e-6
 * in float64, lo = searchsorted(mz_sorted, lower, 'left'), hi = searchsorted(mz_sorted, upper, 'right'),
 * compared in float64.  If `order` is non-NULL, thread t handles window order[t] (pass windows in
 * m/z order for cache locality); results are written at the window's own index. */
int smg_window_bounds(const double* peak_mz, const int64_t* order, int64_t n_windows, double ppm,
                      const float* mz_sorted, int64_t n_points, int64_t* lo, int64_t* hi, void* stream);

/* Window alignment for scoring (formula_img_validator.py:73-75 and 115-118): ion i has the layout windows
 * [win_off[i], win_off[i+1]) (one per peak_i of sf_peak_df) and kt_off[i+1] - kt_off[i] theoretical
 * intensities (len(sf_peak_ints[(sf_id, adduct)])); compute() pads the image list with empty images up to that
 * length and ignores images beyond it.  Writes, for every theoretical slot j = kt_off[i] + k, the window run
 * lo2[j], hi2[j] (layout window k, or the empty run 0, 0 when k is past the layout windows), and keep[i] = 1 if
 * the ion has a row in the metrics table: some layout window is non-empty, some scored window among the first
 * 32 is non-empty (the SMG_ION_HAS_HITS of smg_ion_metrics) and sel[i] != 0 (sel optional, NULL = all). */
int smg_align_windows(const int64_t* lo, const int64_t* hi, const int64_t* win_off, const int64_t* kt_off,
                      const uint8_t* sel, int64_t n_ions, int64_t* lo2, int64_t* hi2, uint8_t* keep, void* stream);

/* Prefix sums over the m/z-sorted hits at 64-point granularity (exclusive, 4 doubles per entry,
 * ceil(n_points/64)+1 entries): cum64[b] = (sum of intensities of points < 64*b, sum of squared intensities
 * of those points without the duplicate-candidate flag), each as a double-double (hi, lo) pair, so that a
 * window's sums do not lose precision to the total intensity preceding it in m/z order.  Window sums of the images of
 * formula_imager_segm.py:84-92 become block-prefix differences plus at most 63 points at either end
 * (smg_ion_metrics reads them).  hit_format/hits/hit_vals as smg_ion_metrics. */
int smg_hit_prefix_sums_workspace_size(int64_t n_points, size_t* bytes);
int smg_hit_prefix_sums(int32_t hit_format, const void* hits, const double* hit_vals, int64_t n_points,
                        double* cum64, void* workspace, size_t workspace_bytes, void* stream);

/* Fused ion imaging + MSM scoring (replaces formula_imager_segm.py:84-109 _gen_iso_images COO
 * construction + _img_pairs_to_list, and formula_img_validator.py:72-84,93-122 compute/sf_image_metrics).
 * Ion i owns windows [ion_win_off[i], ion_win_off[i+1]) in peak_i order; window w's image is the set
 * of points [lo[w], hi[w]) of the m/z-sorted hit array (duplicate pixels summed, as coo.toarray()).
 * hit_cum: smg_hit_prefix_sums (cum64) of the same hits.
 * theor_int[w] is the theoretical intensity of window w (FormulasSegm.get_sf_peak_ints).
 * Outputs (device, [n_ion]): cleaned chaos / spatial / spectral (ImgMeasures.to_tuple semantics),
 * msm = chaos*spatial*spectral, and SMG_ION_* flags.
 * connectivity (4 or 8) and erosion_border (0 or 1) select the measure_of_chaos variant (default 4, 0).
 * ion_order (optional, int64[n_ions]) is the processing order (pass ions sorted by principal m/z so
 * concurrently scored ions share cached windows); outputs are always written at the ion's own index.
 * do_preprocessing != 0 applies the q-th-percentile hot-spot clip (dense path). */
int smg_ion_metrics_workspace_size(int64_t n_ions, int32_t nrows, int32_t ncols, size_t* bytes);
int smg_ion_metrics(int32_t hit_format, const void* hits, const double* hit_vals, const double* hit_cum,
                    const int64_t* lo, const int64_t* hi, const int64_t* ion_win_off,
                    const double* theor_int, const int64_t* ion_order, int64_t n_ions, int32_t nrows, int32_t ncols,
                    int32_t nlevels, double q, int32_t do_preprocessing,
                    int32_t connectivity, int32_t erosion_border,
                    double* out_chaos, double* out_spatial, double* out_spectral, double* out_msm,
                    uint32_t* out_flags, void* workspace, size_t workspace_bytes, void* stream);

/* Result rows of ion images (search_results.py:88-97, iso_img_row_gen of SearchResults.store_sf_iso_images):
 * for each window w of the list (the run [lo[w], hi[w]) of the m/z-sorted packed hits = one (ion, peak) image,
 * duplicate pixels summed as coo.toarray() does), the pixels whose summed intensity is > threshold (the
 * reference's 0.001), in ascending flattened-pixel order (row * ncols + col), with their intensities, window-major
 * in out_pix / out_val (window w's rows start at the exclusive prefix sum of out_count), and the min / max over the
 * whole npx-pixel image (pixels without a point are 0).  total_points = sum(hi - lo) sizes the workspace and is
 * the capacity out_pix / out_val must have.  Nothing is densified: O(window points) work and memory. */
int smg_iso_image_rows_workspace_size(int64_t n_windows, int64_t total_points, size_t* bytes);
int smg_iso_image_rows(const uint64_t* hits, const int64_t* lo, const int64_t* hi, int64_t n_windows,
                       int64_t total_points, int64_t npx, double threshold, int64_t* out_count, double* out_min,
                       double* out_max, int32_t* out_pix, double* out_val, void* workspace, size_t workspace_bytes,
                       void* stream);

/* Legacy imager (formula_imager.py:9-38 _get_nonzero_ints / _sample_spectrum): for every spectrum s and
 * window j, v = cum_ints[searchsorted(mzs, upper_j, 'right')] - cum_ints[searchsorted(mzs, lower_j, 'left')],
 * emitted as (j, s, v) when v > 0.001.  sp_off: int64[n_spectra+1] into mzs; cum_ints has one extra
 * leading element per spectrum (offset sp_off[s] + s).  Writes up to `capacity` triples (unordered) and
 * the total count to *count (device int64). */
int smg_sample_spectra(const int64_t* sp_off, const double* mzs, const double* cum_ints, int64_t n_spectra,
                       const double* lower, const double* upper, int64_t n_windows,
                       int64_t* out_window, int64_t* out_spectrum, double* out_value, int64_t capacity,
                       int64_t* count, void* stream);

/* Theoretical isotope centroids (host code, no GPU): replaces the calculator behind
 * isocalc_wrapper.py:37-70 (complete_isodist(parseSumFormula(sf + adduct), sigma, charge, pts_per_mz,
 * centroid_kwargs={'weighted_bins': 5}) -> first centroids) as restated in oracle/isocalc_oracle.py: isotopic
 * fine structure, Gaussian profile of FWHM sigma/2.35482 on the grid j/pts_per_mz, gradient centroids weighted
 * over +-weighted_bins points, intensities scaled to max 100, ascending m/z.  sf_adduct is a sum formula with
 * '+'/'-' sub-formulas ("C6H12O6+H"); charge z shifts by z electron masses and divides by |z|.  Writes the first
 * min(cap, #centroids) centroids and their count; SMG_ERR_INVALID for an invalid formula (pyMSpec
 * InvalidFormulaError).  The batch form runs n formulas (bytes formulas[offsets[i]:offsets[i+1]]) on n_threads
 * host threads (<= 0: all cores; theor_peaks_gen.py:113-134's Spark fan-out), writing row i of the [n][cap]
 * outputs and n_out[i] (-1: invalid formula). */
int smg_isotope_centroids(const char* sf_adduct, int32_t charge, double sigma, int32_t pts_per_mz,
                          int32_t weighted_bins, int32_t cap, double* mzs, double* ints, int32_t* n_out);
int smg_isotope_centroids_batch(const char* formulas, const int64_t* offsets, int64_t n, int32_t charge,
                                double sigma, int32_t pts_per_mz, int32_t weighted_bins, int32_t cap,
                                double* mzs, double* ints, int32_t* n_out, int32_t n_threads);

/* Diagnostics.  Calibration stream for the rocprofv3 HBM-traffic counters: reads n_words 8-byte words with
 * the ion kernel's access width (one coalesced 8-byte load per lane) and XOR-folds them into out[n_blocks]
 * (device), so that FETCH_SIZE can be converted to bytes for this access pattern (bench.py `traffic`). */
int smg_debug_stream_read(const uint64_t* data, int64_t n_words, uint64_t* out, int32_t n_blocks, void* stream);
/* Test switch: on != 0 makes smg_ion_metrics score every image size with the two-level LDS passes (normally only
 * images above 2^18 pixels), so that the parity suite covers them on small images.  Process-wide; returns 0. */
int smg_debug_force_two_level(int32_t on);
/* Test switch: on = 1 makes smg_ion_metrics score every ion with the dense (global-scratch) path -- the
 * rank-indexed wide pass where the image fits it, the pixel-indexed slot kernel for the rest; on = 2 sends every
 * ion to the pixel-indexed slot kernel; so that the parity suite covers both on every case.  Process-wide;
 * returns 0. */
int smg_debug_force_dense(int32_t on);
/* smg_sort_points' implementation: 1 = the hand-written sort (default), 0 = rocPRIM's onesweep radix sort (kept for
 * A/B timing; smg_sort_points_flag always uses the hand-written one).  Process-wide; returns 0. */
int smg_debug_sort_impl(int32_t which);
/* The main LDS pass: 1 = ion_sparse_kernel where it applies (default: packed f32 hits, no hot-spot clip, images up
 * to 2^18 pixels), 0 = ion_pipe_kernel<512> for every image (kept for A/B timing and
 * so that the parity suite covers both).  Process-wide; returns 0. */
int smg_debug_main_kernel(int32_t which);
/* The rank-indexed wide pass: 1 = ion_wide_join_kernel where it applies (default: packed f32 hits, no hot-spot clip;
 * no per-pixel arrays in global memory), 0 = ion_wide_kernel for every image (kept for A/B timing and so that the
 * parity suite covers both).  Process-wide; returns 0, -1 for another value. */
int smg_debug_wide_impl(int32_t which);
/* Diagnostic builds only (-DSMG_STAMPS, libsmg_stamps.so): per-phase cycles of the main passes summed over their
 * workgroups since the last call (ion_pipe_kernel: smg_debug_stamps; ion_sparse_kernel: smg_debug_sparse_stamps),
 * reset on read; SMG_ERR_UNSUPPORTED in the shipped build. */
int smg_debug_stamps(unsigned long long* host_out, int n);
int smg_debug_sparse_stamps(unsigned long long* host_out, int n);
/* Diagnostic build only (-DSMG_CHECK, `make check` -> libsmg_check.so): every ion pass checks each position it scores
 * -- claimed once per pass, its descriptor equal to what lo / hi / ion_win_off / ion_order give, every hit index it
 * loads inside its window and inside [0, n_points), every reject inside its list -- and counts failures (printing the
 * first few).  smg_debug_check_points sets the resident hit count the next smg_ion_metrics calls are checked
 * against (every build accepts it; only the check build uses it).  smg_debug_check_read waits for the device, writes
 * up to n counters (positions claimed, descriptor mismatches, loads outside their window, double hand-outs, records
 * read as descriptors, reject-list overflows, windows outside [0, n_points], descriptors checked) and resets them;
 * SMG_ERR_UNSUPPORTED in the shipped build. */
int smg_debug_check_points(int64_t n_points);
int smg_debug_check_read(unsigned long long* host_out, int32_t n);

/* passes of smg_ion_metrics, as reported by smg_debug_pass_times */
#define SMG_PASS_DESC 0   /* ion descriptors (ion_desc8_kernel) */
#define SMG_PASS_MAIN 1   /* main LDS pass: ion_sparse_kernel (four 256-thread workgroups per CU, SMG_ION_SPARSE)
                             or, where it does not apply / smg_debug_main_kernel(0), ion_pipe_kernel<512> */
#define SMG_PASS_BIG 2    /* big-ion LDS pass over the main pass's rejects (ion_pipe_kernel<1024>): SMG_ION_BIG */
#define SMG_PASS_WIDE 3   /* rank-indexed wide pass (ion_wide_kernel): SMG_ION_WIDE */
#define SMG_PASS_DENSE 4  /* pixel-indexed pass (ion_dense_kernel): SMG_ION_DENSE without SMG_ION_WIDE */
#define SMG_PASS_FINALIZE 5 /* scores of the ions the LDS passes scored, from their recorded sums (ion_finalize_kernel) */

/* Diagnostics: on != 0 records HIP events on the launch stream around every pass launch of smg_ion_metrics.
 * smg_debug_pass_times waits for the recorded launches, writes up to `cap` (pass id, elapsed ms) pairs in launch
 * order, the number recorded to *n, and forgets them; smg_debug_main_pass_times does the same for the main-pass
 * launches only (the other passes' records are dropped).  Process-wide. */
int smg_debug_time_main_pass(int32_t on);
int smg_debug_main_pass_times(double* ms, int32_t cap, int32_t* n);
int smg_debug_pass_times(int32_t* pass, double* ms, int32_t cap, int32_t* n);

#ifdef __cplusplus
}
#endif

#endif /* SMG_H */
