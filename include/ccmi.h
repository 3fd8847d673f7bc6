/*
 * ccmi.h — C ABI of the MI355X-native consensus-clustering engine (libccmi.so).
 *
 * Plain C: pointers, sizes and a hipStream_t passed as void*.  No C++ or torch
 * types cross this boundary.  Every entry point returns 0 on success and a
 * negative code on error; the message is available from cc_last_error() on the
 * calling thread.  Device pointers are caller-owned (the Python host passes
 * torch-ROCm tensors' data_ptr()); the library allocates nothing on the device.
 * Launches are asynchronous on the given stream and safe to capture in a graph.
 *
 * Each entry point replaces a piece of the reference's hot path
 * (/root/reference/consensus_clustering_parallelised.py, "CC.py" below):
 *
 *   cc_resample_indices   CC.py:216-241  _get_subsampling_indices (numpy RandomState replay)
 *   cc_resample_device    the same on the device (n <= 65536), straight into HBM
 *   cc_resample_device_wide  the same for any n, without simulating the shuffle
 *   cc_scatter_labels     CC.py:260-262, :284-285  indicator / one-hot row placement
 *   cc_copy_label_columns CC.py:185-195 (the parallel paths' shared M) -> multi-GPU label exchange
 *   cc_cosample           CC.py:264  I = S^T S            (int8 MFMA, upper-triangle tiles)
 *   cc_coassoc            CC.py:287-290 + :338-344  M += L^T L fused with the 20-bin histogram
 *   cc_consensus          CC.py:372-373  C = f32(M) / f32(I + 1e-6), diag 1
 *   cc_kmeans_plan        packing of the (K, init) problems of one resample into units
 *   cc_split_f16          f16 hi/lo operand image of the rows for the k-means MFMAs
 *   cc_kmeans_batched     CC.py:282 clusterer.fit_predict for every (h, K) at once
 *   cc_kmeans_wide        the same for wide rows (d > 128), as distance/centre GEMM rounds
 *                         (sklearn KMeans: k-means++ init, Lloyd, best of n_init)
 *   cc_kmeans_f64         the same at float64 for float64 input
 *   cc_kmeans_fit         CC.py:282 in one call (plans and launches one of the three above)
 */
#ifndef CCMI_H
#define CCMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CC_OK 0
#define CC_ERR_ARG (-1)
#define CC_ERR_HIP (-2)
#define CC_ERR_UNSUPPORTED (-3)

/* Tile edge of the upper-triangle tiling used by cc_cosample / cc_coassoc. */
#define CC_TILE 256
/* Number of consensus-histogram bins (CC.py:316 bins=20). */
#define CC_NBINS 20

const char* cc_version(void);
const char* cc_last_error(void);
/* SHA-256 prefix (16 hex digits) of the sources and flags this library was built from
 * (the .hip, .cpp and .h files of csrc, include/ccmi.h and the csrc Makefile); the Python host
 * refuses a library whose id does not match the sources next to it. */
const char* cc_build_id(void);

/* ---- host-side helpers (native, no device) ------------------------------ */

/* Resample indices of CC.py:231-239 for h in [h_begin, h_end):
 * out[(h-h_begin)*m + r] = numpy.random.RandomState(seed + h).permutation(n)[r], r < m
 * (RandomState.choice(n, m, replace=False) == permutation(n)[:m]).  MT19937
 * init_genrand + legacy random_interval rejection sampling, bit-identical to
 * numpy 1.17+ legacy RandomState.  Runs on n_threads host threads (<=0: all). */
int cc_resample_indices(uint32_t seed, int h_begin, int h_end, int n, int m, int32_t* out,
                        int n_threads);

/* Raw doubles of numpy.random.RandomState(seed).random_sample(count). */
int cc_random_sample(uint32_t seed, int64_t count, double* out);

/* Number of tiles of the CC_TILE upper-triangle tiling for n samples. */
int64_t cc_num_tiles(int n);

/* ---- device kernels ----------------------------------------------------- */

/* cc_resample_indices on the device (CC.py:231-239): out [h_end-h_begin][m] int32 in device
 * memory, bit-identical to numpy.random.RandomState(seed + h).permutation(n)[:m].  One
 * workgroup per resample (Fisher-Yates over a uint16 array in LDS), so 1 <= n <=
 * cc_resample_device_max_n() (65536); larger n stays on the host replay. */
int cc_resample_device_max_n(void);
int cc_resample_device(uint32_t seed, int h_begin, int h_end, int n, int m, int32_t* out,
                       void* stream);

/* The same draws for any n (no 65536 limit): RandomState(seed + h).permutation(n)[:m] resolved
 * from the shuffle's swap partners (the draws on one lane per resample, a counting sort of the
 * steps by partner, then each output value as the end of a short chain of later writers), so no
 * step of the shuffle is simulated.  workspace: device, ws_bytes >= the bytes for one resample;
 * resamples run in batches that fit (cc_resample_device_wide_workspace_bytes(n, nh) for nh at
 * once).  Asynchronous on `stream`; out as cc_resample_device. */
int cc_resample_device_wide(uint32_t seed, int h_begin, int h_end, int n, int m, int32_t* out,
                            void* workspace, size_t ws_bytes, void* stream);
size_t cc_resample_device_wide_workspace_bytes(int n, int nh);

/* labels_nh[idx[h][r] * ldl + h] = labels_hm ? labels_hm[h*m + r] : 0 for h < H, r < m.
 * labels_nh must be pre-filled with 0xFF (= not sampled).  (CC.py:260-262, :284-285) */
int cc_scatter_labels(const int32_t* idx_hm, const int32_t* labels_hm, int H, int m, int n,
                      int8_t* labels_nh, int ldl, void* stream);

/* dst[r*ld_dst + col_dst + j] = src[r*ld_src + col_src + j] for r < rows, j < width (bytes).
 * Moves a window of resample columns between sample-major label matrices ([rows][ld] uint8):
 * the multi-GPU exchange packs a rank's own columns [h0, h1) into a contiguous block before an
 * all-gather and places each rank's block at its columns afterwards.  It replaces the
 * reference's shared in-place M of its parallel paths (CC.py:185-195): labels, not n x n
 * counts, cross the links.  Asynchronous on `stream`. */
int cc_copy_label_columns(const uint8_t* src, int64_t ld_src, int col_src, uint8_t* dst,
                          int64_t ld_dst, int col_dst, int64_t rows, int width, void* stream);

/* Co-sampling counts I_ij = #{h : i and j both sampled} for the tiles
 * [tile_begin, tile_end) of the upper-triangle tiling (CC.py:264).
 * labels_nh: [n][ldl] int8, 0xFF = not sampled; Hpad (multiple of 128, <= ldl) columns used;
 *            16-B aligned, like I_tiles and bin_table below (device allocations are).
 * I_tiles:   [tile_end - tile_begin][CC_TILE*CC_TILE] uint16, accumulator order (device-private).
 * I_full:    optional [n][n] int32 (both triangles), may be NULL. */
int cc_cosample(const int8_t* labels_nh, int n, int ldl, int Hpad, int64_t tile_begin,
                int64_t tile_end, uint16_t* I_tiles, int32_t* I_full, void* stream);

/* Co-association counts M_ij = #{h : label_h(i) == label_h(j) >= 0} for the same
 * tiles, fused with the numpy-exact 20-bin histogram of C = f32(M)/f32(I+1e-6)
 * over the strict upper triangle i < j (CC.py:287-290, :338-344).
 * edges: 21 float32 bin edges (numpy's), device.  bin_counts: [20] uint64, device,
 * accumulated into (not cleared).  M_full: optional [n][n] int32, may be NULL.
 * bin_table: optional cc_bin_table output with table_rows >= Hpad + 1 rows (binning without
 * a division; identical bins), NULL for the division path.  K <= 127. */
int cc_coassoc(const int8_t* labels_nh, int n, int ldl, int Hpad, int K, int64_t tile_begin,
               int64_t tile_end, const uint16_t* I_tiles, const float* edges,
               unsigned long long* bin_counts, int32_t* M_full, const uint16_t* bin_table,
               int table_rows, void* stream);

/* Bin thresholds per co-sampling count i in [0, rows): row i = 21 uint16 T[b] =
 * min{m : bin(f32(m) / f32(i + 1e-6)) >= b} (T[0] = 0, T[20] = 0xFFFF; i + 1 if no m <= i
 * reaches b), so bin = #{b in 1..19 : m >= T[b]} (numpy.histogram semantics, CC.py:338-344).
 * table: device, table_bytes >= cc_bin_table_bytes(rows).  After the rows * 21 uint16 (padded
 * to 16 B) it holds, when rows is small enough for cc_coassoc to stage them on chip, the
 * threshold pairs T[g] | T[g+1] << 16 (rows * 20 uint32) and the bins themselves for every
 * (m <= i) pair (one byte at i (i + 1) / 2 + m, padded to 16 B). */
int cc_bin_table(int rows, const float* edges, uint16_t* table, size_t table_bytes, void* stream);

/* Bytes of the cc_bin_table buffer for `rows` rows (0 when rows is out of range). */
size_t cc_bin_table_bytes(int rows);

/* Largest table (rows) cc_coassoc can stage on chip. */
int cc_bin_table_max_rows(void);

/* Largest row count for each staged form: 0 = uint16 thresholds (= cc_bin_table_max_rows),
 * 1 = threshold pairs, 2 = the bin triangle.  cc_coassoc stages the most compact form that fits. */
int cc_bin_table_form_rows(int form);

/* Self-test of the division-free binning: for EVERY pair of counts (m <= i < rows), compare
 * the table forms cc_coassoc uses (threshold table + reciprocal estimate computed per
 * element, and with the staged per-row reciprocal; the threshold pairs and the bin triangle
 * when the table holds them) against the direct numpy-exact bin of f32(m) / f32(i + 1e-6).
 * mismatches: device [4] uint64, accumulated into. */
int cc_bin_selftest(int rows, const float* edges, const uint16_t* table,
                    unsigned long long* mismatches, void* stream);

/* C = f32(M) / f32(f64(I) + 1e-6) with C_ii = 1 (CC.py:372-373), [n][n]. */
int cc_consensus(const int32_t* M, const int32_t* I, int n, float* C, void* stream);

/* Manhattan distances between the rows of C [n][d] float32: D [n][n] float64,
 * D_ij = sum_k |f64(C_ik) - f64(C_jk)| summed sequentially over k (scipy pdist 'cityblock'
 * order), for the consensus labels of CC.py:292-314 (AgglomerativeClustering on the rows of C
 * under the manhattan metric). */
int cc_manhattan(const float* C, int n, int d, double* D, void* stream);

/* Agglomerative linkage of the consensus labels (CC.py:306-312: AgglomerativeClustering ->
 * sklearn linkage_tree -> scipy.cluster.hierarchy.linkage -> _hierarchy.nn_chain) on the device:
 * D [n][n] float64 symmetric (e.g. from cc_manhattan) is overwritten; Z [n-1][4] float64 receives
 * (x, y, distance, size) per merge in nn_chain's merge order, before linkage()'s stable sort by
 * distance and relabelling (done by the caller).  Runs on G co-resident workgroups joined by
 * grid barriers (G from n; CCMI_LINK_G overrides, 0 = one workgroup); workspace of
 * cc_linkage_workspace_bytes(n) bytes; call cc_linkage_check after it. */
#define CC_LINK_AVERAGE 0
#define CC_LINK_COMPLETE 1
#define CC_LINK_WEIGHTED 2
size_t cc_linkage_workspace_bytes(int n);
int cc_linkage_nnchain(double* D, int n, int method, double* Z, void* workspace, size_t ws_bytes,
                       void* stream);

/* Single linkage of the consensus labels: sklearn's path for linkage='single' with the
 * reference's 'manhattan' affinity (CC.py:306-312 -> linkage_tree ->
 * _hierarchical_fast.mst_linkage_core, Prim's MST-LINKAGE-CORE) on the device, over the rows of
 * D [n][n] float64 (read only; cc_manhattan's values are DistanceMetric64 cityblock's).
 * out [n-1][3] float64 = (current node, new node, distance) per Prim step; the caller sorts the
 * edges by distance (stable) and labels them (_single_linkage_label).  G co-resident workgroups
 * as cc_linkage_nnchain; workspace of cc_linkage_mst_workspace_bytes(n) bytes; call
 * cc_linkage_check after it. */
size_t cc_linkage_mst_workspace_bytes(int n);
int cc_linkage_mst(const double* D, int n, double* out, void* workspace, size_t ws_bytes, void* stream);

/* After cc_linkage_nnchain / cc_linkage_mst on `stream` with this workspace: synchronises the
 * stream and returns CC_ERR_HIP if a grid barrier of the linkage timed out (its output is then
 * invalid), else CC_OK. */
int cc_linkage_check(const void* workspace, size_t ws_bytes, void* stream);

/* Batched k-means for every (resample h, K, init) problem, replacing the per-(K, h)
 * clusterer.fit_predict(X[indices]) of CC.py:282 for the default clusterer
 * (sklearn KMeans: k-means++ init with 2+floor(ln K) local trials, Lloyd with strict
 * and tol convergence, empty-cluster relocation, best of n_init;
 * sklearn/cluster/_kmeans.py:174-262, :624-752, :1427-1556).
 *
 * Work is split into UNITS = (resample, subset of the (K, init) problems); a persistent
 * grid of workgroups pulls units from an atomic counter and runs each unit's fits as one
 * problem engine (every sweep streams the resample's rows once for up to 256 centroid
 * slots, packed round-robin from the unit's seeding and Lloyd problems).
 * Unit descriptor u (int32, CC_KM_USTRIDE entries): [0] = P (<= CC_KM_PMAX, the n_init
 * runs of one K consecutive), then per problem p: [1+4p] = K, [2+4p] = kidx (index into
 * Ks), [3+4p] = init, [4+4p] = local trials. */
#define CC_KM_PMAX 64
#define CC_KM_USTRIDE (1 + 4 * CC_KM_PMAX)

/* Pack the (K, n_init) groups of Ks[0..nK) into at least n_sub units (balanced by a K^2
 * cost proxy, largest K first); returns the unit count (> 0) or a negative error.
 * units must hold max_units * CC_KM_USTRIDE int32. */
int cc_kmeans_plan(const int32_t* Ks, int nK, int n_init, int n_sub, int32_t* units, int max_units);

/* Workspace bytes of a cc_kmeans_batched launch with `grid` workgroups. */
size_t cc_kmeans_workspace_bytes(int m, int dpad, const int32_t* units_host, int nU, int seedmax,
                                 int grid);

/* f16 hi/lo image of the rows for the MFMA operands: Xhl[r][0][d] = f16(X[r][d] * 2^e),
 * Xhl[r][1][d] = f16(X[r][d] * 2^e - hi), e in [-62, 62] (host-chosen so that
 * max|X| * 2^e <= 2^14).  X [n][dpad] f32, Xhl [n][2][dpad] uint16. */
int cc_split_f16(const float* X, int n, int dpad, int scale_exp, uint16_t* Xhl, void* stream);

/*  X         [n][dpad] float32, mean-centred, zero-padded from dreal to dpad in {32,64,128}
 *  Xhl       cc_split_f16 image of X with the same scale_exp
 *  xnorm     [n] float32 squared row norms of X
 *  idx_hm    [H][m] int32 resample rows; this launch runs resamples [h_begin, h_end)
 *  units     device copy of the plan; units_host the same array on the host
 *  kpp_u     [nK][n_init][kpp_stride] float64: the RandomState(seed) doubles of each
 *            (K, init) k-means++ run (entry 0: the first-centre draw, consumed on the host)
 *  kpp_pos   [nK][n_init] int32 first-centre positions in resample order
 *  labels_nh [nK][n][ldl] uint8 output (pre-filled 0xFF); labels_nh[k][idx[h][r]][h]
 *  inertia   optional [nK][H] float32; n_iter optional [nK][H] int32
 *  stats     optional [8] uint64 accumulated: {Lloyd row x centroid distance products,
 *            seeding row x candidate distance products, Lloyd M-step row updates
 *            (rows x running problems), empty-cluster relocations, sweeps,
 *            32-slot column tiles x row tiles swept}
 *  grid      workgroups (<= units; one per CU is the intended size)
 *  seedmax   problems of a unit seeding concurrently (1..32)
 *  All pointers except units_host are device pointers; X, Xhl and workspace 16-B aligned
 *  (device allocations are; CC_ERR_ARG otherwise). */
int cc_kmeans_batched(const float* X, const uint16_t* Xhl, const float* xnorm, int n, int dreal,
                      int dpad, int scale_exp, const int32_t* idx_hm, int H, int m, int h_begin,
                      int h_end, const int32_t* units, const int32_t* units_host, int nU,
                      int n_init, int max_iter, double tol_rel, const double* kpp_u,
                      int kpp_stride, const int32_t* kpp_pos, uint8_t* labels_nh, int ldl,
                      float* inertia, int32_t* n_iter, unsigned long long* stats,
                      void* workspace, size_t ws_bytes, int grid, int seedmax, void* stream);

/* Wide rows (d > 128; BASELINE config 4, n = 5k x d = 20k): the same fits, decisions and
 * outputs as cc_kmeans_batched (CC.py:282 for the default clusterer), organised as ROUNDS
 * over a batch of `batch` resamples: per round a distance-GEMM launch fused with the
 * E-step, a centre-sum GEMM launch and a per-resample bookkeeping launch, until every
 * problem is done.  The call is synchronous with respect to the host (it reads one counter
 * per round to stop).  Ks [nK] host array (nK * n_init <= CC_KM_PMAX per call); dpad any
 * multiple of 32 >= dreal; other arguments as cc_kmeans_batched; stats[4] counts
 * resample-rounds and stats[5] 256-slot column tiles x rounds. */
size_t cc_kmeans_wide_workspace_bytes(int m, int dpad, const int32_t* Ks, int nK, int n_init,
                                      int batch);

int cc_kmeans_wide(const float* X, const uint16_t* Xhl, const float* xnorm, int n, int dreal,
                   int dpad, int scale_exp, const int32_t* idx_hm, int H, int m, int h_begin,
                   int h_end, const int32_t* Ks, int nK, int n_init, int max_iter,
                   double tol_rel, const double* kpp_u, int kpp_stride, const int32_t* kpp_pos,
                   uint8_t* labels_nh, int ldl, float* inertia, int32_t* n_iter,
                   unsigned long long* stats, void* workspace, size_t ws_bytes, int batch,
                   void* stream);

/* Float64 k-means for float64 input (the reference's clusterer at the reference's precision,
 * CC.py:282 with float64 X; sklearn/cluster/_kmeans.py restated in float64, see
 * csrc/kmeans_f64.hip).  Same fits, outputs and k-means++ tables as cc_kmeans_batched; X is
 * the raw [n][d] float64 input (the kernel centres each resample by its own mean, as
 * KMeans.fit does).  Ks [nK] is a host array (nK <= 64); one persistent workgroup per
 * (resample, K) unit (or pair of K's); inertia is float64 here.  Workspace from
 * cc_kmeans_f64_workspace_bytes(m, d, Ks, nK, grid, nh): grid workgroup areas and min(grid, nh)
 * per-resample slots for nh = h_end - h_begin (resamples beyond grid run in further launches on
 * the same stream).  X 8-B and workspace 16-B aligned. */
size_t cc_kmeans_f64_workspace_bytes(int m, int d, const int32_t* Ks, int nK, int grid, int nh);

int cc_kmeans_f64(const double* X, int n, int d, const int32_t* idx_hm, int H, int m, int h_begin,
                  int h_end, const int32_t* Ks, int nK, int n_init, int max_iter, double tol_rel,
                  const double* kpp_u, int kpp_stride, const int32_t* kpp_pos, uint8_t* labels_nh,
                  int ldl, double* inertia, int32_t* n_iter, void* workspace, size_t ws_bytes,
                  int grid, void* stream);

/* ---- one-call k-means (the advanced entry points above, planned internally) ----------- */

#define CC_KM_FAST 0 /* float32 input: f16 hi/lo MFMA engines (cc_kmeans_batched / _wide) */
#define CC_KM_F64 1  /* float64 input: cc_kmeans_f64 */

/* k-means++ tables of cc_kmeans_batched for Ks[0..nK) (host): sklearn KMeans(random_state=seed)
 * replays RandomState(seed) for every K; per init it draws the first centre with
 * choice(m, p=w/sum(w)) (_kmeans.py:225; unit weights, float32 unless weight_f64) and then
 * (K-1)*(2+floor(ln K)) uniforms (:243).  kpp_u [nK][n_init][kpp_stride], kpp_pos [nK][n_init]. */
int cc_kpp_tables(const int32_t* Ks, int nK, int n_init, uint32_t seed, int m, int weight_f64,
                  double* kpp_u, int kpp_stride, int32_t* kpp_pos);

/* Row image of the float32 engines from raw rows X [n][d] float32 (device): column means
 * (float64, fixed order), centred rows zero-padded to dpad (Xd [n][dpad]), squared norms
 * (xnorm [n]), the scale exponent (returned in *scale_exp; synchronises the stream) and the
 * cc_split_f16 image (Xhl [n][2][dpad]).  scratch: device, cc_prepare_rows_scratch_bytes. */
size_t cc_prepare_rows_scratch_bytes(int n, int d);
int cc_prepare_rows(const float* X, int n, int d, int dpad, float* Xd, float* xnorm, uint16_t* Xhl,
                    int* scale_exp, void* scratch, size_t scratch_bytes, void* stream);

/* Every (resample h in [h_begin, h_end), K, init) k-means fit of a consensus fit in one call:
 * the loop of clusterer.fit_predict(X[indices]) at CC.py:282 for the default KMeans(n_init)
 * clusterer.  Plans units, grid and seedmax, builds the k-means++ tables and the row image, and
 * runs cc_kmeans_batched (d <= 128), cc_kmeans_wide (d > 128) or cc_kmeans_f64.
 *  X        device [n][d] raw rows: float32 (CC_KM_FAST) or float64 (CC_KM_F64)
 *  idx_hm   device [H][m] int32 resample rows (rows outside [h_begin, h_end) are not read)
 *  Ks       host [nK], 1 <= K <= min(127, m)
 *  labels_nh device [nK][n][ldl] uint8, pre-filled 0xFF; labels_nh[k][idx[h][r]][h]
 *  inertia  optional device [nK][H] (float32 for CC_KM_FAST, float64 for CC_KM_F64)
 *  n_iter   optional device [nK][H] int32
 *  workspace device, ws_bytes >= cc_kmeans_fit_workspace_bytes(...) (less is fine for the
 *           persistent grid, which shrinks to fit; too little for one workgroup is an error)
 * Synchronous with respect to the host (it reads max|X| and, for wide rows, a counter per
 * round).  Results are identical to driving the advanced entry points with the same inputs. */
size_t cc_kmeans_fit_workspace_bytes(int n, int d, int m, int nh, const int32_t* Ks, int nK,
                                     int n_init, int precision);
int cc_kmeans_fit(const void* X, int n, int d, const int32_t* idx_hm, int H, int m, int h_begin,
                  int h_end, const int32_t* Ks, int nK, int n_init, int max_iter, double tol_rel,
                  uint32_t seed, int precision, uint8_t* labels_nh, int ldl, void* inertia,
                  int32_t* n_iter, void* workspace, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* CCMI_H */
