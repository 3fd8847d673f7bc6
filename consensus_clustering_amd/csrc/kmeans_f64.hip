// Float64 k-means for float64 input: the reference's clusterer at the reference's precision.
//
// The reference clusters whatever dtype X has (CC.py:282; its notebook and BASELINE config 1
// pass float64 `.values`), and scikit-learn's KMeans then runs in float64.  The f16 hi/lo MFMA
// engine (kmeans.hip) is float32-class; this kernel is the float64 path.  It restates
// scikit-learn 1.7 (sklearn/cluster/_kmeans.py, _k_means_lloyd.pyx, _k_means_common.pyx)
// operation by operation in float64, with its reduction orders where they are sequential:
//   * X_sub centred by its own column means (KMeans.fit, :1479-1481; rows summed in order);
//   * tol = mean(var(X_sub, axis=0)) * tol_rel (_tolerance; numpy pairwise mean over features);
//   * k-means++ (_kmeans_plusplus): squared distances ((-2 x.c) + |c|^2) + |x|^2 clipped at 0
//     (_euclidean_distances), candidates by searchsorted over the float64 cumsum, the
//     candidate with the lowest potential kept, the potentials in OpenBLAS's ddot / dgemv_t
//     orders (single-threaded; above numpy's BLAS threading threshold the order depends on
//     the host's thread count and is not reproduced);
//   * squared norms of rows and centres in numpy einsum's order (row_norms);
//   * Lloyd (_kmeans_single_lloyd / lloyd_iter_chunked_dense): distances |c|^2 - 2 x.c,
//     argmin with strict < (lowest index on ties), centre sums in row order, empty clusters
//     relocated to the farthest points, averaging with 1/weight, shifts by the 4-way unrolled
//     _euclidean_dense_dense, strict convergence else sum(shift^2) <= tol, a final E-step when
//     not strictly converged, inertia summed in row order;
//   * best of n_init: lower inertia and a different clustering (_is_same_clustering).
// Dot products are sequential fused multiply-adds over the features (the BLAS micro-kernel
// order); float contraction is otherwise off, as in the reference's compiled Cython.
//
// Mapping: a persistent grid; one 256-thread workgroup runs one (resample, K) unit at a time,
// units dealt in decreasing K, with per-workgroup float64 scratch in the caller's workspace.
// Each resample's centred rows, their fragment image, row norms and tol are built once, by two
// setup kernels before the units' launch, into per-resample slots of the workspace (up to grid
// resamples per launch); a unit of two adjacent K's (where units are plentiful) runs both K's
// problems in one lockstep group.
// Round 5: a unit's inits run in lockstep groups of up to GMAX (each pass over the rows - the
// k-means++ distances, the E-step, the centre sums, the inertia - serves every running init of
// the group; an init that converges leaves the group), and the centre sums accumulate in LDS
// where they fit; every init's values and orders are those of a run on its own.
// Round 4: the unit's centred rows are materialised once ([m][d] float64, the same subtraction;
// round 5: once per resample),
// every dot product runs as one of G (or ntr) independent sequential FMA chains per thread (a
// thread's row against G centres at once: the same chain per value, G times the ILP), and the
// centre sums walk per-cluster row lists built in row order (a ballot compaction), one thread
// per (cluster, feature) with coalesced row reads instead of one thread per feature
// read-modify-writing global sums row after row.  Every value keeps its sequential order, so
// the results are bit-identical to the previous kernel (and to sklearn where it was).
// The E-step and the k-means++ distances run on the float64 matrix cores (v_mfma_f64_16x16x4_f64,
// whose per-output accumulation is the sequential FMA chain: see mfma_dots), 16 rows x 16 centres
// per instruction; the rows enter as B operands from a fragment-ordered copy of the centred rows
// (one contiguous 512-B load per k-step and row tile), the centres straight from their rows.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>
#include <type_traits>

#include "ccmi_internal.h"

#pragma clang fp contract(off)

namespace {

constexpr int NT = 256;
constexpr int KMAX = 127;
constexpr int TMAX = 6;
constexpr int NKMAX = 64;
// problems of a unit run in lockstep groups of up to GM (in unit order): the kernel is built for
// GM = 4 (one K per unit, up to 4 inits) and GM = GMAX (two K's of 3 inits), see cc_kmeans_f64
constexpr int GMAX = 6;
constexpr int F64_KPACK = 2;        // K's per unit (at most GMAX / n_init)
constexpr int F64_KPAIR_MAX = 127;  // only K's up to this are grouped
constexpr int F64_UNITS_PER_WG = 2;  // ... and only with at least this many units per workgroup

struct F64Args {
  const double* X;  // [n][d] (not centred)
  int n, d;
  const int32_t* idx;  // [H][m]
  int H, m, h_begin, nh;
  int nK;
  int Ks[NKMAX];
  int korder[NKMAX];  // K indices by decreasing K: units are dealt heaviest first
  int ukfirst[NKMAX + 1];  // unit kind u: the K's korder[ukfirst[u] .. ukfirst[u + 1])
  int nuk;
  int n_init, max_iter;
  double tol_rel;
  const double* kpp_u;  // [nK][n_init][stride]
  int kpp_stride;
  const int32_t* kpp_pos;  // [nK][n_init]
  uint8_t* labels;         // [nK][n][ldl]
  int ldl;
  double* inertia_out;  // [nK][H] or null
  int32_t* niter_out;   // [nK][H] or null
  unsigned* counter;
  char* ws;
  size_t per_wg;
  size_t o_cl, o_dc, o_sq, o_cen, o_cnew, o_lab, o_lold, o_lbest, o_cf;
  size_t kd, cfs;  // per-init strides (doubles) of the centres and of their operand images
  // per-resample images (slot hb of this launch's resamples), built once by the setup kernels
  char* rs;
  size_t per_res, r_mean, r_var, r_tol, r_xsq, r_xc, r_xf;
};

// numpy pairwise_sum (numpy/_core/src/umath/loops_utils.h.src) of a contiguous double array:
// sequential below 8, eight interleaved partial sums up to 128, else split at
// floor(n / 2) rounded down to a multiple of 8 and recurse.
__device__ double np_pairwise(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
}

// sklearn row_norms(X, squared=True) = np.einsum('ij,ij->i', X, X): numpy's contiguous
// sum-of-products kernel (einsum_sumprod.c.src) on the x86-64 baseline: 2 double lanes, blocks
// of 8 accumulated as lane += a0 b0 + (a1 b1 + (a2 b2 + (a3 b3 + lane)))) (separate multiply and
// add), a zero-filled tail in lane steps, then lane 0 + lane 1.
template <class F>
__device__ __forceinline__ double einsum_sq(F x, int d) {
  double l0 = 0.0, l1 = 0.0;
  int i = 0;
  for (; d - i >= 8; i += 8) {
    const double a0 = x(i), a1 = x(i + 1), a2 = x(i + 2), a3 = x(i + 3);
    const double a4 = x(i + 4), a5 = x(i + 5), a6 = x(i + 6), a7 = x(i + 7);
    l0 = a0 * a0 + (a2 * a2 + (a4 * a4 + (a6 * a6 + l0)));
    l1 = a1 * a1 + (a3 * a3 + (a5 * a5 + (a7 * a7 + l1)));
  }
  for (; i < d; i += 2) {
    const double a = x(i), b = (i + 1 < d) ? x(i + 1) : 0.0;
    l0 = a * a + l0;
    l1 = b * b + l1;
  }
  return l0 + l1;
}

// _euclidean_dense_dense (squared): 4-way unrolled, left to right
__device__ __forceinline__ double euclid4(const double* a, const double* b, int d) {
  double res = 0.0;
  const int n4 = d / 4, rem = d % 4;
  for (int i = 0; i < n4; ++i) {
    const double d0 = a[4 * i] - b[4 * i], d1 = a[4 * i + 1] - b[4 * i + 1];
    const double d2 = a[4 * i + 2] - b[4 * i + 2], d3 = a[4 * i + 3] - b[4 * i + 3];
    res += ((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3;
  }
  for (int i = 0; i < rem; ++i) {
    const double t = a[4 * n4 + i] - b[4 * n4 + i];
    res += t * t;
  }
  return res;
}

// The k-means++ potentials are BLAS reductions of the closest distances with unit weights.
// Their orders were measured against the scipy-openblas build (OpenBLAS 0.3.29, DYNAMIC_ARCH,
// SkylakeX/Haswell kernels, one thread) that numpy uses in this image; with unit weights the
// products are exact, so each reduction is a fixed tree of additions.
//
// current_pot = closest_dist_sq @ sample_weight (a (1, m) @ (m,) product, numpy -> ddot):
// 16-element blocks; the first multiple of 32 in four 8-lane accumulators (each folded to 4 lanes,
// low half + high half), a 16-element remainder into four 4-lane accumulators, the accumulators
// summed ((a0 + a1) + a2) + a3, the lanes (q0 + q2) + (q1 + q3), then the tail sequentially.
__device__ double blas_ddot_ones(const double* x, int n) {
  const int n1 = n & -16, n32 = n1 & ~31;
  double A[4][4];
  {
    double Z[4][8];
    for (int a = 0; a < 4; ++a)
      for (int q = 0; q < 8; ++q) Z[a][q] = 0.0;
    for (int i = 0; i < n32; i += 32)
      for (int a = 0; a < 4; ++a)
        for (int q = 0; q < 8; ++q) Z[a][q] += x[i + 8 * a + q];
    for (int a = 0; a < 4; ++a)
      for (int q = 0; q < 4; ++q) A[a][q] = Z[a][q] + Z[a][q + 4];
  }
  for (int i = n32; i < n1; i += 16)
    for (int a = 0; a < 4; ++a)
      for (int q = 0; q < 4; ++q) A[a][q] += x[i + 4 * a + q];
  double L[4];
  for (int q = 0; q < 4; ++q) L[q] = ((A[0][q] + A[1][q]) + A[2][q]) + A[3][q];
  double dot = (L[0] + L[2]) + (L[1] + L[3]);
  for (int i = n1; i < n; ++i) dot += x[i];
  return dot;
}

// candidates_pot = distance_to_candidates @ sample_weight.reshape(-1, 1) ((ntr, m) @ (m, 1),
// numpy -> dgemv_t over ntr columns of length m).  Rows m & ~3 in blocks of 2048, each block's
// column sum added to y; columns in groups of 4 use 4-lane accumulators (lanes (q0 + q2) +
// (q1 + q3)), a pair of remaining columns 2 lanes (l0 + l1), a last odd column 4 lanes; the
// m & 3 tail rows are summed left to right and added last.
__device__ double blas_gemv_t_ones(const double* x, int m, int col, int ncol) {
  const int n4 = ncol & ~3, rem = ncol - n4;
  const bool two = rem >= 2 && col >= n4 && col < n4 + 2;
  const int m1 = m & ~3;
  double y = 0.0;
  for (int b = 0; b < m1; b += 2048) {
    const int e = b + 2048 < m1 ? b + 2048 : m1;
    double s;
    if (two) {
      double l0 = 0.0, l1 = 0.0;
      for (int i = b; i < e; i += 2) {
        l0 += x[i];
        l1 += x[i + 1];
      }
      s = l0 + l1;
    } else {
      double l[4] = {0.0, 0.0, 0.0, 0.0};
      for (int i = b; i < e; i += 4)
        for (int q = 0; q < 4; ++q) l[q] += x[i + q];
      s = (l[0] + l[2]) + (l[1] + l[3]);
    }
    y += s;
  }
  if (m1 < m) {
    double t = x[m1];
    for (int i = m1 + 1; i < m; ++i) t += x[i];
    y += t;
  }
  return y;
}

// Diagnostic build only (-DCC_F64_STAMPS, tools/f64_stamps.py): thread 0's wall-clock split of
// the units' phases.
#ifdef CC_F64_STAMPS
__device__ unsigned long long cc_f64_stamps[16];
constexpr int F64_UT = 16384;                        // units with recorded times
__device__ unsigned long long cc_f64_utimes[F64_UT][3];  // per unit: start, end, workgroup
#define F64_STAMP(ph)                               \
  do {                                              \
    if (tid == 0) {                                 \
      const unsigned long long t_ = wall_clock64(); \
      st_acc[ph] += t_ - st_acc[13];                \
      st_acc[13] = t_;                              \
    }                                               \
  } while (0)
#else
#define F64_STAMP(ph)
#endif

// Per-init arrays are GMAX consecutive copies: cl / lab / lold [GMAX][m], dc [GMAX][TMAX][m],
// cen / cnew [GMAX][kmax][d], cf [GMAX][cfs] (centre operand images).
struct WG {
  double *mean, *xsq, *cl, *dc, *sq, *cen, *cnew, *xc, *xf, *cf;
  int32_t *lab, *lold;
  uint8_t* lbest;
  int m;
  size_t kd, cfs;
  __device__ double* cl_of(int g) const { return cl + static_cast<size_t>(g) * m; }
  __device__ double* dc_of(int g) const { return dc + static_cast<size_t>(g) * TMAX * m; }
  __device__ int32_t* lab_of(int g) const { return lab + static_cast<size_t>(g) * m; }
  __device__ int32_t* lold_of(int g) const { return lold + static_cast<size_t>(g) * m; }
  __device__ double* cen_of(int g, int buf) const { return (buf ? cnew : cen) + static_cast<size_t>(g) * kd; }
  __device__ double* cf_of(int g) const { return cf + static_cast<size_t>(g) * cfs; }
};


// The unit's centred row r (materialised: X[idx[r]][k] - mean[k], rounded once).
__device__ __forceinline__ const double* xrow(const WG& w, int d, int r) { return w.xc + static_cast<size_t>(r) * d; }

// Feature k of row r read from the fragment image (the same value as xrow(w, d, r)[k]): where a
// thread walks its own row, the 16 rows of a tile sit in 128 contiguous bytes per feature, so a
// wave's load touches 4 segments instead of 64 rows.
struct XfRow {
  const double* p;  // row r's lane in its tile
  __device__ XfRow(const WG& w, int d, int r)
      : p(w.xf + static_cast<size_t>(r >> 4) * ((d + 3) >> 2) * 64 + (r & 15)) {}
  __device__ double operator[](int k) const { return p[(k >> 2) * 64 + 16 * (k & 3)]; }
};

// ---- float64 dot products on the matrix cores -------------------------------------------------
// v_mfma_f64_16x16x4_f64 accumulates each of its outputs as the sequential fused multiply-add
// chain over its 4 k values, starting from C: measured bit-identical to the VALU chain
// fma(a3, b3, fma(a2, b2, fma(a1, b1, fma(a0, b0, c)))) on 2^20 mixed-exponent results
// (tools/mfma_f64_probe.hip, profiles/r04/mfma_f64_probe.txt).  A chain of them over k-steps
// 0 .. d/4-1 is therefore the same sequential FMA dot product (the small-matrix dgemm order) the
// VALU loops computed, 1024 FMAs per instruction (lane l: row l & 15, feature 4s + (l >> 4)).
// The A operands (centres, candidates) are read from their row-major rows (consecutive steps reuse
// the same cache lines); the B operands (the unit's rows) from the fragment image o_xf, built once
// per unit, at step stride BS = 64: 16 scattered 32-B pieces per load became one 512-B piece
// (E-step 1.3-1.6x per iteration, profiles/r04/f64_budget_r4ak.txt).
// Orientation: A = 16 "centres", B = 16 rows; D's lane l holds row l & 15 against centres
// (l >> 4) + 4i, i = 0..3.  Features past d (d % 4 != 0) enter as exact zeros in both operands:
// fma(0, 0, acc) = acc for the accumulators here (never -0: they start at +0).
using f64x4 = __attribute__((ext_vector_type(4))) double;
constexpr int MG = 4;  // k-steps per operand load group; two groups in flight

template <int RT, int CT, int BS = 4, int AS = 4>
__device__ __forceinline__ void mfma_dots(const double* const (&pa)[CT], const double* const (&pb)[RT], int d,
                                          int q, f64x4 (&acc)[RT][CT]) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = f64x4{0.0, 0.0, 0.0, 0.0};
  const int S = d >> 2;
  double a0[MG][CT], b0[MG][RT], a1[MG][CT], b1[MG][RT];
  auto ld = [&](double (&a)[MG][CT], double (&b)[MG][RT], int s0) __attribute__((always_inline)) {
    if (s0 >= S) return;
#pragma unroll
    for (int i = 0; i < MG; ++i) {
      const int s = s0 + i < S ? s0 + i : S - 1;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) a[i][ct] = pa[ct][AS * s];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) b[i][rt] = pb[rt][BS * s];
    }
  };
  auto mm = [&](const double (&a)[MG][CT], const double (&b)[MG][RT], int s0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MG; ++i)
      if (s0 + i < S)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
            acc[rt][ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i][ct], b[i][rt], acc[rt][ct], 0, 0, 0);
  };
  ld(a0, b0, 0);
  for (int s0 = 0; s0 < S; s0 += 2 * MG) {
    ld(a1, b1, s0 + MG);
    mm(a0, b0, s0);
    ld(a0, b0, s0 + 2 * MG);
    mm(a1, b1, s0 + MG);
  }
  if (d & 3) {  // the last, partial k-step
    const bool in = 4 * S + q < d;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const double bv = in ? pb[rt][BS * S] : 0.0;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        acc[rt][ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(in ? pa[ct][AS * S] : 0.0, bv, acc[rt][ct], 0, 0, 0);
    }
  }
}

// (value, index) lexicographic minimum: with the centres visited in increasing index it is the
// sequential scan's strict-< argmin (lowest index on ties)
__device__ __forceinline__ void lexmin(double& v, int& j, double v2, int j2) {
  if (v2 < v || (v2 == v && j2 < j)) {
    v = v2;
    j = j2;
  }
}

// the A-operand fragment image of nrow rows (row j: src[j], nullptr = zeros; rows up to a
// multiple of 32): tile t, k-step s, lane l holds row 16t + (l & 15), feature 4s + (l >> 4)
template <class Row>
__device__ __forceinline__ void build_afrag(double* dst, Row row, int nrow, int d, int tid) {
  const int S4 = (d + 3) >> 2;
  const int ntl = ((nrow + 31) >> 5) * 2;
  for (int e = tid; e < ntl * S4 * 64; e += NT) {
    const int l = e & 63, ts = e >> 6;
    const int t = ts / S4, sk = ts - t * S4;
    const int j = 16 * t + (l & 15), k = 4 * sk + (l >> 4);
    const double* src = j < nrow ? row(j) : nullptr;
    dst[e] = (src && k < d) ? src[k] : 0.0;
  }
}

// par: bit g = which buffer holds init g's current centres (0: cen, 1: cnew)
// The E-step argmin of every row over the K centres: |c_j|^2 - 2 x.c_j (one rounding, as
// sklearn's dgemm with beta = 1 on the centre norms), strict < over increasing j (a (value, index)
// lexicographic minimum: lowest index on ties).  Each wave takes RT row tiles of 16 at a time.  The
// running problems of the lockstep group (inits, and the K's of a multi-K unit) share the pass:
// their centres are packed into one operand image (slot a = the a-th running problem, its K_a
// centres at rows off_a .. off_a + K_a; no per-problem padding to 16 rows), each pass of 16 CT
// rows feeds every problem's own running (distance, label) per row (jm[J] = a << 8 | j, gof[a]:
// the problem of slot a), and a row tile's B operands are read once for all of them.
// The passes over the rows (estep_packed, msum_packed, kpp_mfma_multi, kpp_search_multi,
// kpp_pots_multi) are out of line (round 6): each gets its own register allocation instead of
// sharing the kernel body's, whose VGPR spills fell from 91 / 162 to 51 / 64 (GM = 4 / 6); a call
// per pass costs nothing measurable.  C2 H = 500 1.08x, C5 H = 64 1.15x, C3 H = 128 0.99x, results
// identical (profiles/r06/f64_noinline_ab.txt).
template <int RT, int CT, int NA>
__device__ __attribute__((noinline)) void estep_packed(const WG& w, int na, const int* gof, const int* jm, const double* cnp, int nJ, int d,
                             int m, int tid) {
  const int l = tid & 63, q = l >> 4, c16 = l & 15;
  const int ntile = (m + 15) >> 4;
  for (int t0 = (tid >> 6) * RT; t0 < ntile; t0 += (NT / 64) * RT) {
    const double* pb[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      pb[rt] = w.xf + static_cast<size_t>(t0 + rt < ntile ? t0 + rt : ntile - 1) * ((d + 3) >> 2) * 64 + l;
    double bv[RT][NA];
    int bj[RT][NA];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        bv[rt][a] = __builtin_inf();
        bj[rt][a] = 0x7fffffff;
      }
    for (int J0 = 0; J0 < nJ; J0 += 16 * CT) {
      const double* pa[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) pa[ct] = w.cf + static_cast<size_t>((J0 >> 4) + ct) * ((d + 3) >> 2) * 64 + l;
      // the slots this tile of centres touches (wave-uniform: the others are skipped)
      const int a0 = __builtin_amdgcn_readfirstlane(jm[J0] >> 8);
      const int a1 = __builtin_amdgcn_readfirstlane(jm[(J0 + 16 * CT < nJ ? J0 + 16 * CT : nJ) - 1] >> 8);
      f64x4 acc[RT][CT];
      mfma_dots<RT, CT, 64, 64>(pa, pb, d, q, acc);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int J = J0 + 16 * ct + q + 4 * i;
          if (J >= nJ) continue;
          const int e = jm[J], a = e >> 8, j = e & 255;
          const double c2 = cnp[J];
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            const double v = __fma_rn(-2.0, acc[rt][ct][i], c2);
#pragma unroll
            for (int aa = 0; aa < NA; ++aa)
              if (aa >= a0 && aa <= a1 && aa == a) lexmin(bv[rt][aa], bj[rt][aa], v, j);
          }
        }
    }
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      if (a >= na) break;
      int32_t* lab = w.lab_of(gof[a]);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        double v = bv[rt][a];
        int jj = bj[rt][a];
        lexmin(v, jj, __shfl_xor(v, 16), __shfl_xor(jj, 16));
        lexmin(v, jj, __shfl_xor(v, 32), __shfl_xor(jj, 32));
        const int r = (t0 + rt) * 16 + c16;
        if (q == 0 && r < m) lab[r] = jj;
      }
    }
  }
}

// The slot map of the running problems act (in problem order): gof[a] = the a-th running
// problem, jm[J] = a << 8 | j for its centre j at packed row J, cnp[J] its |c|^2 (from cn, when
// given).  Returns the number of rows; the maps are read after the caller's next barrier.
__device__ __forceinline__ int slot_map(unsigned act, int G, const int* Kg, int* gof, int* jm, const double* cn,
                                        double* cnp, int tid) {
  int nJ = 0;
  for (int g = 0; g < G; ++g)
    if ((act >> g) & 1u) nJ += Kg[g];
  for (int J = tid; J < nJ; J += NT) {
    int a = 0, off = 0;
    for (int g = 0; g < G; ++g)
      if ((act >> g) & 1u) {
        if (J < off + Kg[g]) {
          jm[J] = (a << 8) | (J - off);
          if (cn) cnp[J] = cn[g * (KMAX + 1) + J - off];
          break;
        }
        off += Kg[g];
        ++a;
      }
  }
  if (tid == 0) {
    int a = 0;
    for (int g = 0; g < G; ++g)
      if ((act >> g) & 1u) gof[a++] = g;
  }
  return nJ;
}

// par: bit g = which buffer holds problem g's current centres (0: cen, 1: cnew)
template <int GM>
__device__ __forceinline__ int estep_multi(const WG& w, unsigned act, unsigned par, int G, const int* Kg,
                                           const double* cn, double* cnp, int d, int m, int* gof, int* jm, int tid) {
  const int nJ = slot_map(act, G, Kg, gof, jm, cn, cnp, tid);
  __syncthreads();
  int na = 0;
  for (int g = 0; g < G; ++g) na += (act >> g) & 1u;
  // the running problems' centres, packed
  build_afrag(w.cf, [&](int J) {
    const int e = jm[J], g = gof[e >> 8];
    return w.cen_of(g, (par >> g) & 1u) + static_cast<size_t>(e & 255) * d;
  }, nJ, d, tid);
  __syncthreads();
  // per-slot running minima for as many slots as run (registers: 3 * RT per slot)
  if (GM > 4 && na <= GM / 2) {
    if (nJ <= 16) estep_packed<2, 1, GM / 2>(w, na, gof, jm, cnp, nJ, d, m, tid);
    else estep_packed<2, 2, GM / 2>(w, na, gof, jm, cnp, nJ, d, m, tid);
  } else {
    if (nJ <= 16) estep_packed<2, 1, GM>(w, na, gof, jm, cnp, nJ, d, m, tid);
    else estep_packed<2, 2, GM>(w, na, gof, jm, cnp, nJ, d, m, tid);
  }
  __syncthreads();
  return nJ;
}

// k-means++ distances of a lockstep group: column jj < nc is candidate t of problem g (col[jj] =
// g << 8 | t, the candidate row cand[g * TMAX + t]; first centre: one column per problem), all
// nc <= GMAX * TMAX of them as the centres of one pass over the rows; each value is kpp_mfma's
// ((-2 x.c) + |c|^2) + |x|^2 clipped at 0, min with problem g's closest.
__device__ __attribute__((noinline)) void kpp_mfma_multi(const WG& w, int d, int m, const int* cand, const int* col, int nc,
                                               bool first, int tid) {
  const int l = tid & 63, q = l >> 4, c16 = l & 15;
  const int ntile = (m + 15) >> 4;
  build_afrag(w.cf, [&](int j) {
    const int e = col[j];
    return w.xc + static_cast<size_t>(cand[(e >> 8) * TMAX + (e & 255)]) * d;
  }, nc, d, tid);
  __syncthreads();
  // one candidate tile: four row tiles per wave (four independent MFMA chains, more rows in flight)
  auto body = [&](auto ctc) __attribute__((always_inline)) {
    constexpr int CT = decltype(ctc)::value;
    constexpr int RT = CT == 1 ? 4 : 2;
    const double* pa[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) pa[ct] = w.cf + static_cast<size_t>(ct) * ((d + 3) >> 2) * 64 + l;
    for (int t0 = (tid >> 6) * RT; t0 < ntile; t0 += (NT / 64) * RT) {
      const double* pb[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        pb[rt] = w.xf + static_cast<size_t>(t0 + rt < ntile ? t0 + rt : ntile - 1) * ((d + 3) >> 2) * 64 + l;
      f64x4 acc[RT][CT];
      mfma_dots<RT, CT, 64, 64>(pa, pb, d, q, acc);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = (t0 + rt) * 16 + c16;
        if (r >= m) continue;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int jj = 16 * ct + q + 4 * i;
            if (jj >= nc) continue;
            const int g = col[jj] >> 8, t = col[jj] & 255;
            double dd = -2.0 * acc[rt][ct][i];
            dd += w.xsq[cand[g * TMAX + t]];
            dd += w.xsq[r];
            dd = dd > 0.0 ? dd : 0.0;
            double* cl = w.cl_of(g);
            if (first) cl[r] = dd;
            else w.dc_of(g)[static_cast<size_t>(t) * m + r] = cl[r] < dd ? cl[r] : dd;
          }
      }
    }
  };
  if (nc <= 16) body(std::integral_constant<int, 1>{});
  else if (nc <= 32) body(std::integral_constant<int, 2>{});
  else body(std::integral_constant<int, 3>{});
  __syncthreads();
}

// The centre sums on the matrix cores: cnew[j][k] = sum over the rows r, in row order, of
// [lab[r] == j] * x[r][k], one sequential FMA chain per output over k-steps of 4 rows (A = the
// one-hot labels: lane l cluster l & 15, row 4s + (l >> 4); B = the rows: lane l feature l & 15).
// fma(1, x, acc) = acc + x is sklearn's addition (centers_new[j] += x * 1.0); fma(0, x, acc) =
// acc + (+-0) = acc exactly for finite x, the accumulators starting at +0 and never -0 - so each
// output is the row-order sum of its cluster's rows.  A wave owns CTP cluster tiles x FTP
// 16-feature tiles per pass over the rows.  The running problems of the lockstep group share the
// pass: their clusters are packed as in the E-step (jm, gof: one tile may hold clusters of two
// problems; lane l's A operand reads the labels of its own cluster's problem), and the B operands
// (the rows) are loaded once per k-step for all of them.
template <int CTP, int FTP>
__device__ __attribute__((noinline)) void msum_packed(const WG& w, unsigned par, const int* gof, const int* jm, int nJ, int d, int m, int tid) {
  const int l = tid & 63, q = l >> 4, c16 = l & 15;
  const int nct = (nJ + 15) >> 4, nft = (d + 15) >> 4;
  const int nfg = (nft + FTP - 1) / FTP;
  const int ncg = (nct + CTP - 1) / CTP;
  const int S = (m + 3) >> 2;
  for (int item = tid >> 6; item < ncg * nfg; item += NT / 64) {
    const int cg = item / nfg, fg = item - cg * nfg;
    int f[FTP];
    const double* pb[FTP];
#pragma unroll
    for (int u = 0; u < FTP; ++u) {
      f[u] = (fg * FTP + u) * 16 + c16;
      pb[u] = w.xc + (f[u] < d ? f[u] : d - 1) + static_cast<size_t>(q) * d;
    }
    // lane's A-operand cluster of each tile: packed row J -> (init, cluster); past nJ: none
    int jl[CTP];
    const int32_t* pl[CTP];
#pragma unroll
    for (int ct = 0; ct < CTP; ++ct) {
      const int J = (cg * CTP + ct) * 16 + c16;
      const int e = J < nJ ? jm[J] : 0;
      jl[ct] = J < nJ ? (e & 255) : -2;
      pl[ct] = w.lab_of(gof[e >> 8]) + q;
    }
    f64x4 acc[CTP][FTP];
#pragma unroll
    for (int ct = 0; ct < CTP; ++ct)
#pragma unroll
      for (int u = 0; u < FTP; ++u) acc[ct][u] = f64x4{0.0, 0.0, 0.0, 0.0};
    int lb0[MG][CTP], lb1[MG][CTP];
    double b0[MG][FTP], b1[MG][FTP];
    auto ld = [&](int (&lv)[MG][CTP], double (&bv)[MG][FTP], int s0) __attribute__((always_inline)) {
      if (s0 >= S) return;
#pragma unroll
      for (int i = 0; i < MG; ++i) {
        const int r = 4 * (s0 + i) + q;
        const bool in = s0 + i < S && r < m;
#pragma unroll
        for (int ct = 0; ct < CTP; ++ct) lv[i][ct] = in ? pl[ct][4 * (s0 + i)] : -1;
#pragma unroll
        for (int u = 0; u < FTP; ++u) bv[i][u] = in ? pb[u][static_cast<size_t>(4 * (s0 + i)) * d] : 0.0;
      }
    };
    auto mm = [&](const int (&lv)[MG][CTP], const double (&bv)[MG][FTP], int s0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < MG; ++i)
        if (s0 + i < S)
#pragma unroll
          for (int ct = 0; ct < CTP; ++ct) {
            const double av = lv[i][ct] == jl[ct] ? 1.0 : 0.0;
#pragma unroll
            for (int u = 0; u < FTP; ++u)
              acc[ct][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv[i][u], acc[ct][u], 0, 0, 0);
          }
    };
    ld(lb0, b0, 0);
    for (int s0 = 0; s0 < S; s0 += 2 * MG) {
      ld(lb1, b1, s0 + MG);
      mm(lb0, b0, s0);
      ld(lb0, b0, s0 + 2 * MG);
      mm(lb1, b1, s0 + MG);
    }
#pragma unroll
    for (int u = 0; u < FTP; ++u)
      if (f[u] < d)
#pragma unroll
        for (int ct = 0; ct < CTP; ++ct)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int J = (cg * CTP + ct) * 16 + q + 4 * i;
            if (J >= nJ) continue;
            const int e = jm[J], g = gof[e >> 8];
            double* cnew = w.cen_of(g, ((par >> g) & 1u) ^ 1u);
            cnew[static_cast<size_t>(e & 255) * d + f[u]] = acc[ct][u][i];
          }
  }
}

// the packed E-step's slot map must be current (estep_multi wrote gof / jm for the same act)
__device__ __forceinline__ void msum_multi(const WG& w, unsigned par, const int* gof, const int* jm, int nJ, int d,
                                           int m, int tid) {
  const int nct = (nJ + 15) >> 4, nft = (d + 15) >> 4;
  // as many cluster tiles per wave as keep every wave busy: each cluster-tile group re-reads the
  // rows, and the passes over the rows are what the sums wait on
  if (nct >= 3 && ((nct + 3) / 4) * nft >= NT / 64) msum_packed<4, 1>(w, par, gof, jm, nJ, d, m, tid);
  else if (nct >= 2 && ((nct + 1) / 2) * nft >= NT / 64) msum_packed<2, 1>(w, par, gof, jm, nJ, d, m, tid);
  else msum_packed<1, 1>(w, par, gof, jm, nJ, d, m, tid);
  __syncthreads();
}

// ---- k-means++ reductions over the closest distances ---------------------------------------------
// The candidate search and the potentials are sequential reductions over m values; each was one
// thread walking global memory (a load latency per few rows).  Now the same additions, in the
// same order, run over LDS-staged blocks (the search) or as independent chains spread over the
// workgroup (the BLAS potentials, whose accumulators are independent until their final folds).
constexpr int CB = 1024;  // search staging block (doubles); the LDS area holds 2 * CB

// The group's per-problem facts, in LDS: K, candidates per step (2 + ln K), K index, init.
struct GroupInfo {
  const int *K, *ntr, *kk, *ini;
};

// the walker thread of slot s (< GMAX): lanes 0 and 32 of wave s mod 4
__device__ __forceinline__ int walker_slot(int tid) {
  return (tid & 31) == 0 ? (tid >> 6) + (NT / 64) * ((tid >> 5) & 1) : GMAX;
}

// kpp_search for every seeding problem of a lockstep group at once (slot s: problem sg[s], s <
// ns): each walk runs on its own walker thread (the walks overlap), over its own staged blocks of
// CBM values (sb: [GMAX][2][CBM]).  Problem g at step c: cand[g TMAX + t] =
// searchsorted(cumsum(cl_g), u_g[c][t] pot[g]) clipped to m - 1, t < ntr_g: the float64
// cumulative sum in row order, 8 partial sums then one comparison with the next of the sorted
// thresholds (the sums do not decrease, so the thresholds are crossed in order).
constexpr int CBM = 512;
__device__ __attribute__((noinline)) void kpp_search_multi(const F64Args& a, const WG& w, const GroupInfo& gi, const int* sg, int ns, int c,
                                 const double* pot, int* cand, double* sb, int* sflag, double* s_thr, int* s_tix,
                                 int tid) {
  const int m = w.m;
  const int ws = walker_slot(tid);
  const bool walker = ws < ns;
  const int gw = walker ? sg[ws] : 0;
  const int ntr = walker ? gi.ntr[gw] : 0;
  if (walker) {
    const double* u = a.kpp_u + (static_cast<size_t>(gi.kk[gw]) * a.n_init + gi.ini[gw]) * a.kpp_stride + 1 +
                      static_cast<size_t>(c - 1) * ntr;
    double* thr = s_thr + ws * TMAX;
    int* tix = s_tix + ws * TMAX;
    for (int t = 0; t < ntr; ++t) {
      thr[t] = u[t] * pot[gw];
      tix[t] = t;
    }
    for (int t = 1; t < ntr; ++t)  // insertion sort of the thresholds (ties: either order)
      for (int v = t; v > 0 && thr[v] < thr[v - 1]; --v) {
        const double x = thr[v];
        thr[v] = thr[v - 1];
        thr[v - 1] = x;
        const int y = tix[v];
        tix[v] = tix[v - 1];
        tix[v - 1] = y;
      }
    for (int t = 0; t < ntr; ++t) cand[gw * TMAX + t] = m - 1;  // not crossed: clipped to m - 1
    sflag[ws] = 0;
  }
  for (int e = tid; e < ns * CBM; e += NT) {
    const int s = e / CBM, i = e - s * CBM;
    if (i < m) sb[s * 2 * CBM + i] = w.cl_of(sg[s])[i];
  }
  __syncthreads();
  double cum = 0.0, tn = walker ? s_thr[ws * TMAX] : 0.0;
  int next = 0;
  int buf = 0;
  for (int b0 = 0; b0 < m; b0 += CBM) {
    const int nb = b0 + CBM;
    for (int e = tid; e < ns * CBM; e += NT) {
      const int s = e / CBM, i = e - s * CBM;
      if (nb + i < m) sb[(s * 2 + (buf ^ 1)) * CBM + i] = w.cl_of(sg[s])[nb + i];
    }
    if (walker && !sflag[ws]) {
      const double* cur = sb + (ws * 2 + buf) * CBM;
      const double* thr = s_thr + ws * TMAX;
      const int* tix = s_tix + ws * TMAX;
      const int n = m - b0 < CBM ? m - b0 : CBM;
      for (int i0 = 0; i0 < n && next < ntr; i0 += 8) {
        // 8 partial sums, then one comparison with the next threshold (the sums do not decrease)
        double cs[8];
        const int g8 = n - i0 < 8 ? n - i0 : 8;
        double cc = cum;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (i < g8) cc += cur[i0 + i];
          cs[i] = cc;
        }
        if (!(cc < tn)) {
#pragma unroll
          for (int i = 0; i < 8; ++i)
            while (i < g8 && next < ntr && !(cs[i] < tn)) {
              const int p = b0 + i0 + i;
              cand[gw * TMAX + tix[next]] = p < m - 1 ? p : m - 1;
              ++next;
              tn = next < ntr ? thr[next] : 0.0;
            }
        }
        cum = cc;
      }
      if (next >= ntr) sflag[ws] = 1;
    }
    __syncthreads();
    int all = 1;
    for (int q = 0; q < ns; ++q) all &= sflag[q];
    if (all) break;
    buf ^= 1;
  }
  __syncthreads();
}

// a chain x[i0], x[i0 + L], ... (i < e) summed left to right from 0.0, loads 16 ahead
__device__ __forceinline__ double chain_sum(const double* x, int i0, int e, int L) {
  double acc = 0.0;
  for (int i = i0; i < e; i += 16 * L) {
    double v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = i + k * L < e ? x[i + k * L] : 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (i + k * L < e) acc += v[k];
  }
  return acc;
}

// The candidates' potentials for every column of a lockstep group at once (col[c] = g << 8 | t):
// pot[g TMAX + t] = blas_gemv_t_ones(column t of w.dc_of(g), m, t, ntr_g), its (column,
// 2048-row block, lane) accumulator chains one per thread, the folds by thread c.
__device__ __attribute__((noinline)) void kpp_pots_multi(const WG& w, const int* ntrg, const int* col, int nc, double* part, double* pot,
                               int tid) {
  const int m = w.m;
  const int m1 = m & ~3;
  const int nb = (m1 + 2047) / 2048;
  const int GB = (2 * CB) / (nc * 4);  // blocks per round
  // the lane count of column c's 4-lane / 2-lane grouping
  auto lanes = [&](int c) {
    const int t = col[c] & 255, ntr = ntrg[col[c] >> 8];
    const int n4 = ntr & ~3;
    return (ntr - n4 >= 2 && t >= n4 && t < n4 + 2) ? 2 : 4;
  };
  double y = 0.0;
  for (int bb = 0; bb < nb; bb += GB) {
    const int gb = nb - bb < GB ? nb - bb : GB;
    for (int ch = tid; ch < nc * gb * 4; ch += NT) {
      const int c = ch / (gb * 4), g = (ch >> 2) % gb, q = ch & 3;
      const int L = lanes(c);
      if (q >= L) continue;
      const int b = (bb + g) * 2048, e = b + 2048 < m1 ? b + 2048 : m1;
      part[(c * GB + g) * 4 + q] = chain_sum(w.dc_of(col[c] >> 8) + static_cast<size_t>(col[c] & 255) * m, b + q, e, L);
    }
    __syncthreads();
    if (tid < nc) {
      const bool two = lanes(tid) == 2;
      for (int g = 0; g < gb; ++g) {
        const double* pp = part + (tid * GB + g) * 4;
        y += two ? pp[0] + pp[1] : (pp[0] + pp[2]) + (pp[1] + pp[3]);
      }
    }
    __syncthreads();
  }
  if (tid < nc) {
    const int g = col[tid] >> 8, t = col[tid] & 255;
    if (m1 < m) {
      const double* x = w.dc_of(g) + static_cast<size_t>(t) * m;
      double tt = x[m1];
      for (int i = m1 + 1; i < m; ++i) tt += x[i];
      y += tt;
    }
    pot[g * TMAX + t] = y;
  }
  __syncthreads();
}

// *out = blas_ddot_ones(cl, m), its 32 accumulator chains one per thread, the folds by thread 0
__device__ void kpp_pot0(const double* cl, int m, double* part, double* out, int tid) {
  const int n1 = m & -16, n32 = n1 & ~31;
  if (tid < 32) part[tid] = chain_sum(cl, tid, n32, 32);  // Z[a][q] = chain of x[i + 8a + q]
  __syncthreads();
  if (tid == 0) {
    double A[4][4];
    for (int a = 0; a < 4; ++a)
      for (int q = 0; q < 4; ++q) A[a][q] = part[8 * a + q] + part[8 * a + q + 4];
    for (int i = n32; i < n1; i += 16)
      for (int a = 0; a < 4; ++a)
        for (int q = 0; q < 4; ++q) A[a][q] += cl[i + 4 * a + q];
    double L[4];
    for (int q = 0; q < 4; ++q) L[q] = ((A[0][q] + A[1][q]) + A[2][q]) + A[3][q];
    double dot = (L[0] + L[2]) + (L[1] + L[3]);
    for (int i = n1; i < m; ++i) dot += cl[i];
    *out = dot;
  }
  __syncthreads();
}

// centred feature k of resample row r
__device__ __forceinline__ double xc(const F64Args& a, const int32_t* idx, const double* mean, int r, int k) {
  return a.X[static_cast<size_t>(idx[r]) * a.d + k] - mean[k];
}

// ---- per-resample setup (KMeans.fit's centring and _tolerance, once per resample) -----------
// Thread (slot, feature k): the column mean of the resample's rows (rows in order), then the
// variance of the centred column, the loads of 16 rows in flight ahead of the adds.
__global__ __launch_bounds__(NT) void f64_setup_stats(const F64Args* __restrict__ pa) {
  const F64Args& a = *pa;
  const int d = a.d, m = a.m;
  const long long e = static_cast<long long>(blockIdx.x) * NT + threadIdx.x;
  if (e >= static_cast<long long>(a.nh) * d) return;
  const int hb = static_cast<int>(e / d), k = static_cast<int>(e - static_cast<long long>(hb) * d);
  const int32_t* idx = a.idx + static_cast<size_t>(a.h_begin + hb) * m;
  char* rb = a.rs + static_cast<size_t>(hb) * a.per_res;
  double s = 0.0;
  int r = 0;
  for (; r + 16 <= m; r += 16) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = a.X[static_cast<size_t>(idx[r + u]) * d + k];
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
  for (; r < m; ++r) s += a.X[static_cast<size_t>(idx[r]) * d + k];
  const double mu = s / m;
  double q = 0.0;
  for (r = 0; r + 16 <= m; r += 16) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = a.X[static_cast<size_t>(idx[r + u]) * d + k] - mu;
#pragma unroll
    for (int u = 0; u < 16; ++u) q += v[u] * v[u];
  }
  for (; r < m; ++r) {
    const double t = a.X[static_cast<size_t>(idx[r]) * d + k] - mu;
    q += t * t;
  }
  reinterpret_cast<double*>(rb + a.r_mean)[k] = mu;
  reinterpret_cast<double*>(rb + a.r_var)[k] = q / m;
}

constexpr int SRT = 4;  // row tiles of 16 per setup workgroup

// Workgroup (slot, block of SRT row tiles): the centred rows X[idx[r]][k] - mean[k] (rounded
// once), the same values as the matrix cores' B operand image (row tile t, k-step s, lane l
// holds row 16t + (l & 15), feature 4s + (l >> 4); exact zeros past m and d, so every operand
// load of a k-step is one contiguous 512-B piece), the rows' squared norms (einsum order); block 0
// also tol = mean(var) * tol_rel (_tolerance: numpy pairwise mean over the features).
__global__ __launch_bounds__(NT) void f64_setup_rows(const F64Args* __restrict__ pa, int nrb) {
  const F64Args& a = *pa;
  const int d = a.d, m = a.m, tid = threadIdx.x;
  const int hb = blockIdx.x / nrb, rbk = blockIdx.x - hb * nrb;
  const int32_t* idx = a.idx + static_cast<size_t>(a.h_begin + hb) * m;
  char* rb = a.rs + static_cast<size_t>(hb) * a.per_res;
  const double* mean = reinterpret_cast<const double*>(rb + a.r_mean);
  double* xcp = reinterpret_cast<double*>(rb + a.r_xc);
  double* xf = reinterpret_cast<double*>(rb + a.r_xf);
  double* xsq = reinterpret_cast<double*>(rb + a.r_xsq);
  if (rbk == 0 && tid == 0) {
    const double* var = reinterpret_cast<const double*>(rb + a.r_var);
    *reinterpret_cast<double*>(rb + a.r_tol) = (np_pairwise(var, d) / d) * a.tol_rel;
  }
  const int r0 = rbk * SRT * 16, r1 = r0 + SRT * 16 < m ? r0 + SRT * 16 : m;
  for (int r = r0; r < r1; ++r) {
    const double* xr = a.X + static_cast<size_t>(idx[r]) * d;
    for (int k = tid; k < d; k += NT) xcp[static_cast<size_t>(r) * d + k] = xr[k] - mean[k];
  }
  __syncthreads();
  const int S4 = (d + 3) >> 2;
  const int ntl = (m + 15) >> 4;
  const int l = tid & 63, wv = tid >> 6;
  const int rl = l & 15, kl = l >> 4;
  for (int t = rbk * SRT; t < ntl && t < (rbk + 1) * SRT; ++t) {
    const int r = 16 * t + rl;
    for (int sk = wv; sk < S4; sk += NT / 64) {
      const int k = 4 * sk + kl;
      xf[(static_cast<size_t>(t) * S4 + sk) * 64 + l] = (r < m && k < d) ? xcp[static_cast<size_t>(r) * d + k] : 0.0;
    }
  }
  __syncthreads();
  WG w;
  w.xf = xf;
  for (int r = r0 + tid; r < r1; r += NT) {
    const XfRow x(w, d, r);
    xsq[r] = einsum_sq([&](int k) { return x[k]; }, d);
  }
}

template <int GM>
__global__ __launch_bounds__(NT, 2) void kmeans_f64_kernel(const F64Args* __restrict__ pa) {
  // arguments read from the workspace header (as in kmeans.hip): re-loaded where used rather
  // than pinned in SGPRs for the whole kernel
  const F64Args& a = *pa;
  __shared__ int s_unit, s_flag, s_best[TMAX + 1], s_cand[GM * TMAX], s_map[KMAX + 1];
  __shared__ double s_tol;
  __shared__ double s_stage[2 * CB > GM * 2 * CBM ? 2 * CB : GM * 2 * CBM];  // search blocks / potential partials
  __shared__ double s_potg[GM], s_potc[GM];
  __shared__ double s_cn[GM][KMAX + 1], s_sh[GM][KMAX + 1];  // per problem: |c|^2, shift^2
  __shared__ int s_cnt[GM][KMAX + 1];                          // per problem: cluster counts
  __shared__ int s_gof[GM], s_jm[GM * KMAX];                 // packed E-step: slot / row maps
  __shared__ double s_cnp[GM * KMAX];                          // packed E-step: |c|^2 by row
  __shared__ double s_thrg[GM * TMAX], s_potm[GM * TMAX];   // k-means++ of the group
  __shared__ int s_tixg[GM * TMAX], s_sflag[GM], s_col[GM * TMAX], s_sg[GM];
  __shared__ int s_K[GM], s_ntr[GM], s_kk[GM], s_ini[GM];  // the group's problems
  GroupInfo gi;
  gi.K = s_K;
  gi.ntr = s_ntr;
  gi.kk = s_kk;
  gi.ini = s_ini;
  const int tid = threadIdx.x;
  char* base = a.ws + static_cast<size_t>(blockIdx.x) * a.per_wg;
  WG w;
  w.cl = reinterpret_cast<double*>(base + a.o_cl);
  w.dc = reinterpret_cast<double*>(base + a.o_dc);
  w.sq = reinterpret_cast<double*>(base + a.o_sq);
  w.cen = reinterpret_cast<double*>(base + a.o_cen);
  w.cnew = reinterpret_cast<double*>(base + a.o_cnew);
  w.lab = reinterpret_cast<int32_t*>(base + a.o_lab);
  w.lold = reinterpret_cast<int32_t*>(base + a.o_lold);
  w.lbest = reinterpret_cast<uint8_t*>(base + a.o_lbest);
  w.cf = reinterpret_cast<double*>(base + a.o_cf);
  const int m = a.m, d = a.d;
  w.m = m;
  w.kd = a.kd;
  w.cfs = a.cfs;
#ifdef CC_F64_STAMPS
  // the accumulators in LDS (thread 0's registers would move the kernel's allocation)
  __shared__ unsigned long long st_acc[14];
  if (tid == 0) {
    for (int q = 0; q < 13; ++q) st_acc[q] = 0;
    st_acc[13] = wall_clock64();
  }
#endif
  for (;;) {
    __syncthreads();
    if (tid == 0) s_unit = static_cast<int>(atomicAdd(a.counter, 1u));
    __syncthreads();
    const int unit = s_unit;
    if (unit >= a.nh * a.nuk) break;
    F64_STAMP(7);
#ifdef CC_F64_STAMPS
    if (tid == 0 && unit < F64_UT) {
      cc_f64_utimes[unit][0] = wall_clock64();
      cc_f64_utimes[unit][2] = blockIdx.x;
    }
#endif
    // unit kinds in decreasing K, every resample's unit of the heaviest kind first: the longest
    // units start first and the short ones fill the tail (longest-processing-time order).  A kind
    // is one K or a run of adjacent K's (korder[kf .. kf + P)) whose problems share the passes.
    const int ui = unit / a.nh, hb = unit - ui * a.nh;
    const int kf = a.ukfirst[ui], nprob = (a.ukfirst[ui + 1] - kf) * a.n_init;
    const int h = a.h_begin + hb;
    const int32_t* idx = a.idx + static_cast<size_t>(h) * m;

    // the resample's centred rows, their fragment image and norms, and tol: built once per
    // resample by the setup kernels
    {
      char* rb = a.rs + static_cast<size_t>(hb) * a.per_res;
      w.mean = reinterpret_cast<double*>(rb + a.r_mean);
      w.xsq = reinterpret_cast<double*>(rb + a.r_xsq);
      w.xc = reinterpret_cast<double*>(rb + a.r_xc);
      w.xf = reinterpret_cast<double*>(rb + a.r_xf);
      if (tid == 0) s_tol = *reinterpret_cast<const double*>(rb + a.r_tol);
    }
    __syncthreads();
    F64_STAMP(0);
    const double tol = s_tol;

    double best_inertia = 0.0;
    int best_iter = 0;
    // the unit's problems (K-major: every init of its first K, then of the next) in lockstep
    // groups of up to GM: every pass over the rows (the k-means++ distances, the E-step, the
    // centre sums) serves all of the group's running problems; each problem's values and their
    // order are those of a run on its own
    for (int g0 = 0; g0 < nprob; g0 += GM) {
      const int G = nprob - g0 < GM ? nprob - g0 : GM;
      __syncthreads();
      if (tid < G) {
        const int e = g0 + tid, q = e / a.n_init;
        const int kk = a.korder[kf + q];
        s_kk[tid] = kk;
        s_ini[tid] = e - q * a.n_init;
        s_K[tid] = a.Ks[kk];
        s_ntr[tid] = 2 + static_cast<int>(log(static_cast<double>(a.Ks[kk])));
      }
      __syncthreads();
      int KM = 0;
      for (int g = 0; g < G; ++g) KM = s_K[g] > KM ? s_K[g] : KM;
      // ---- k-means++ -------------------------------------------------------------
      for (int g = 0; g < G; ++g) {
        const int cp = a.kpp_pos[s_kk[g] * a.n_init + s_ini[g]];
        double* cen = w.cen_of(g, 0);
        for (int k = tid; k < d; k += NT) cen[k] = xrow(w, d, cp)[k];
        if (tid == 0) {
          s_cand[g * TMAX] = cp;
          s_col[g] = g << 8;
        }
      }
      __syncthreads();
      kpp_mfma_multi(w, d, m, s_cand, s_col, G, true, tid);
      for (int g = 0; g < G; ++g) {
        kpp_pot0(w.cl_of(g), m, s_stage, &s_potc[g], tid);
      }
      for (int c = 1; c < KM; ++c) {
        // the problems still seeding (c < K_g), their candidate columns
        int ns = 0, nc = 0;
        for (int g = 0; g < G; ++g)
          if (c < s_K[g]) {
            if (tid == 0) s_sg[ns] = g;
            if (tid < s_ntr[g]) s_col[nc + tid] = (g << 8) | tid;
            ++ns;
            nc += s_ntr[g];
          }
        __syncthreads();
        // candidates: searchsorted(cumsum(closest), u * pot), clipped to m - 1
        F64_STAMP(1);
        kpp_search_multi(a, w, gi, s_sg, ns, c, s_potc, s_cand, s_stage, s_sflag, s_thrg, s_tixg, tid);
        F64_STAMP(10);
        kpp_mfma_multi(w, d, m, s_cand, s_col, nc, false, tid);
        F64_STAMP(11);
        kpp_pots_multi(w, s_ntr, s_col, nc, s_stage, s_potm, tid);
        F64_STAMP(12);
        for (int q = 0; q < ns; ++q) {
          const int g = s_sg[q];
          const double* sp = s_potm + g * TMAX;
          int bt = 0;
          for (int t = 1; t < s_ntr[g]; ++t)
            if (sp[t] < sp[bt]) bt = t;
          const int cp = s_cand[g * TMAX + bt];
          double* cl = w.cl_of(g);
          const double* dcb = w.dc_of(g) + static_cast<size_t>(bt) * m;
          for (int r = tid; r < m; r += NT) cl[r] = dcb[r];
          double* cen = w.cen_of(g, 0);
          for (int k = tid; k < d; k += NT) cen[static_cast<size_t>(c) * d + k] = xrow(w, d, cp)[k];
          __syncthreads();
          if (tid == 0) s_potc[g] = sp[bt];
        }
        __syncthreads();
      }
      F64_STAMP(1);
      // ---- Lloyd -------------------------------------------------------------------
      for (int g = 0; g < G; ++g) {
        int32_t* lold = w.lold_of(g);
        for (int r = tid; r < m; r += NT) lold[r] = -1;
      }
      unsigned act = (1u << G) - 1u;  // running problems
      unsigned par = 0;                // bit g: problem g's current centres are in cnew
      unsigned strict = 0;
      int nit[GM];
#pragma unroll
      for (int g = 0; g < GM; ++g) nit[g] = a.max_iter;
      for (int it = 0; it < a.max_iter && act; ++it) {
        // |c|^2 into s_cn[g][0..K_g), the counts to zero
        __syncthreads();
        for (int g = 0; g < G; ++g)
          for (int j = tid; j < s_K[g]; j += NT) {
            s_cnt[g][j] = 0;
            if (!((act >> g) & 1u)) continue;
            const double* cj = w.cen_of(g, (par >> g) & 1u) + static_cast<size_t>(j) * d;
            s_cn[g][j] = einsum_sq([&](int k) { return cj[k]; }, d);
          }
        __syncthreads();
        const int nJ = estep_multi<GM>(w, act, par, G, s_K, &s_cn[0][0], s_cnp, d, m, s_gof, s_jm, tid);
        F64_STAMP(2);
#ifdef CC_F64_STAMPS
        if (tid == 0) st_acc[8] += 1;
#endif
        unsigned chg = 0;
        for (int g = 0; g < G; ++g) {
          if (!((act >> g) & 1u)) continue;
          const int32_t* lab = w.lab_of(g);
          const int32_t* lold = w.lold_of(g);
          int c1 = 0;
          for (int r = tid; r < m; r += NT) {
            const int lb = lab[r];
            c1 |= (lb != lold[r]);
            atomicAdd(&s_cnt[g][lb], 1);  // counts (integers: order-free)
          }
          if (__syncthreads_or(c1)) chg |= 1u << g;
        }
        F64_STAMP(3);
        msum_multi(w, par, s_gof, s_jm, nJ, d, m, tid);
        F64_STAMP(4);
        for (int g = 0; g < G; ++g) {
          if (!((act >> g) & 1u)) continue;
          const int K = s_K[g];
          const double* cen = w.cen_of(g, (par >> g) & 1u);
          double* cnew = w.cen_of(g, ((par >> g) & 1u) ^ 1u);
          const int32_t* lab = w.lab_of(g);
          int* cnt = s_cnt[g];
          if (tid == 0) {
            int ne = 0;
            for (int j = 0; j < K; ++j) ne += (cnt[j] == 0);
            s_flag = ne;
          }
          __syncthreads();
          if (s_flag > 0) {
            // _relocate_empty_clusters_dense: the empty clusters are fixed first (np.where), then
            // each takes the farthest remaining row from its old centre (lowest index on ties)
            for (int r = tid; r < m; r += NT) {
              // ((X - centers_old[labels]) ** 2).sum(axis=1): numpy pairwise over the features
              // (exact for d <= 128: one 8-accumulator block)
              const double* c = cen + static_cast<size_t>(lab[r]) * d;
              double sacc = 0.0;
              if (d < 8) {
                for (int k = 0; k < d; ++k) {
                  const double e = xrow(w, d, r)[k] - c[k];
                  sacc += e * e;
                }
              } else {
                double v[8];
                for (int q = 0; q < 8; ++q) {
                  const double e = xrow(w, d, r)[q] - c[q];
                  v[q] = e * e;
                }
                int k = 8;
                for (; k < d - (d % 8); k += 8)
                  for (int q = 0; q < 8; ++q) {
                    const double e = xrow(w, d, r)[k + q] - c[k + q];
                    v[q] += e * e;
                  }
                sacc = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
                for (; k < d; ++k) {
                  const double e = xrow(w, d, r)[k] - c[k];
                  sacc += e * e;
                }
              }
              w.sq[r] = sacc;
            }
            __syncthreads();
            if (tid == 0) {
              double mx = 0.0;
              for (int r = 0; r < m; ++r) mx = w.sq[r] > mx ? w.sq[r] : mx;
              int ne = 0;
              for (int j = 0; j < K; ++j)
                if (cnt[j] == 0) s_map[ne++] = j;
              s_flag = (mx == 0.0) ? 0 : ne;
            }
            __syncthreads();
            // Parity gap (documented): sklearn takes the n_empty farthest rows from
            // np.argpartition(distances, -n_empty)[:-n_empty-1:-1], whose order among those rows
            // (and whose tie-break) is introselect's; here empty cluster e takes the e-th farthest
            // remaining row, lowest index on ties.  The two agree for one empty cluster without
            // tied distances; with n_empty >= 2 or ties, bit-parity with sklearn is not claimed.
            const int ne = s_flag;
            for (int e = 0; e < ne; ++e) {
              if (tid == 0) {
                int far = 0;
                for (int r = 1; r < m; ++r)
                  if (w.sq[r] > w.sq[far]) far = r;
                s_best[0] = far;
              }
              __syncthreads();
              const int far = s_best[0], j = s_map[e], old = lab[far];
              for (int k = tid; k < d; k += NT) {
                const double x = xrow(w, d, far)[k];
                cnew[static_cast<size_t>(old) * d + k] -= x;
                cnew[static_cast<size_t>(j) * d + k] = x;
              }
              __syncthreads();
              if (tid == 0) {
                cnt[j] = 1;
                cnt[old] -= 1;
                w.sq[far] = -1.0;
              }
              __syncthreads();
            }
          }
          // _average_centers: in cluster order; an empty cluster copies argmax(weight)'s row as it
          // stands (still a raw sum when the argmax comes later)
          if (tid == 0) {
            int am = 0;
            for (int j = 1; j < K; ++j)
              if (cnt[j] > cnt[am]) am = j;
            s_best[1] = am;
          }
          __syncthreads();
          const int am = s_best[1];
          for (int k = tid; k < d; k += NT)
            for (int j = 0; j < K; ++j) {
              double* cj = cnew + static_cast<size_t>(j) * d;
              if (cnt[j] > 0) cj[k] *= 1.0 / static_cast<double>(cnt[j]);
              else cj[k] = cnew[static_cast<size_t>(am) * d + k];
            }
          __syncthreads();
          // shifts and convergence
          if (tid < K) {
            const double sh = sqrt(euclid4(cnew + static_cast<size_t>(tid) * d, cen + static_cast<size_t>(tid) * d, d));
            s_sh[g][tid] = sh * sh;
          }
          __syncthreads();
        }
        F64_STAMP(5);
        for (int g = 0; g < G; ++g) {
          if (!((act >> g) & 1u)) continue;
          par ^= 1u << g;  // the new centres are current
          if (!((chg >> g) & 1u)) {
            strict |= 1u << g;
            act &= ~(1u << g);
            nit[g] = it + 1;
            continue;
          }
          const double tot = np_pairwise(s_sh[g], s_K[g]);
          const int32_t* lab = w.lab_of(g);
          int32_t* lold = w.lold_of(g);
          for (int r = tid; r < m; r += NT) lold[r] = lab[r];
          if (tot <= tol) {
            act &= ~(1u << g);
            nit[g] = it + 1;
          }
        }
      }
      __syncthreads();
      const unsigned fin = ((1u << G) - 1u) & ~strict;  // final E-step against the last centres
      if (fin) {
        for (int g = 0; g < G; ++g) {
          if (!((fin >> g) & 1u)) continue;
          for (int j = tid; j < s_K[g]; j += NT) {
            const double* cj = w.cen_of(g, (par >> g) & 1u) + static_cast<size_t>(j) * d;
            s_cn[g][j] = einsum_sq([&](int k) { return cj[k]; }, d);
          }
        }
        __syncthreads();
        estep_multi<GM>(w, fin, par, G, s_K, &s_cn[0][0], s_cnp, d, m, s_gof, s_jm, tid);
      }
      // inertia of every problem of the group in one pass over the rows: per-row squared distance
      // to its centre (into the problem's free k-means++ buffer), then each problem's row-order
      // sum on its own walker thread
      for (int r = tid; r < m; r += NT) {
        const XfRow x(w, d, r);
        for (int g = 0; g < G; ++g) {
          const double* c = w.cen_of(g, (par >> g) & 1u) + static_cast<size_t>(w.lab_of(g)[r]) * d;
          double res = 0.0;
          const int n4 = d / 4, rem = d % 4;
          for (int i = 0; i < n4; ++i) {
            const double d0 = x[4 * i] - c[4 * i];
            const double d1 = x[4 * i + 1] - c[4 * i + 1];
            const double d2 = x[4 * i + 2] - c[4 * i + 2];
            const double d3 = x[4 * i + 3] - c[4 * i + 3];
            res += ((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3;
          }
          for (int i = 0; i < rem; ++i) {
            const double t = x[4 * n4 + i] - c[4 * n4 + i];
            res += t * t;
          }
          w.dc_of(g)[r] = res;
        }
      }
      __syncthreads();
      {
        const int gw = walker_slot(tid);
        if (gw < G) {
          // the row-order sum, its loads 16 rows ahead of the adds (one thread walking global
          // memory otherwise waits a round trip per row)
          const double* sq = w.dc_of(gw);
          double sacc = 0.0;
          int r = 0;
          for (; r + 16 <= m; r += 16) {
            double v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = sq[r + u];
#pragma unroll
            for (int u = 0; u < 16; ++u) sacc += v[u];
          }
          for (; r < m; ++r) sacc += sq[r];
          s_potg[gw] = sacc;
        }
      }
      __syncthreads();
      for (int g = 0; g < G; ++g) {
        const int32_t* lab = w.lab_of(g);
        const double inertia = s_potg[g];
        const int n_iter = nit[g];
        const int ini = s_ini[g];
        // best of n_init (per K, in init order): lower inertia AND a different clustering
        bool take = (ini == 0);
        if (!take && inertia < best_inertia) {
          for (int j = tid; j <= KMAX; j += NT) s_map[j] = -1;
          __syncthreads();
          if (tid == 0) {
            // _is_same_clustering in row order, the labels loaded 16 rows ahead
            int same = 1;
            for (int r0 = 0; r0 < m && same; r0 += 16) {
              int l1v[16], l2v[16];
#pragma unroll
              for (int u = 0; u < 16; ++u) {
                l1v[u] = r0 + u < m ? lab[r0 + u] : 0;
                l2v[u] = r0 + u < m ? static_cast<int>(w.lbest[r0 + u]) : 0;
              }
              for (int u = 0; u < 16 && r0 + u < m && same; ++u) {
                const int l1 = l1v[u], l2 = l2v[u];
                if (s_map[l1] == -1) s_map[l1] = l2;
                else if (s_map[l1] != l2) same = 0;
              }
            }
            s_flag = same;
          }
          __syncthreads();
          take = !s_flag;
        }
        if (take) {
          for (int r = tid; r < m; r += NT) w.lbest[r] = static_cast<uint8_t>(lab[r]);
          best_inertia = inertia;
          best_iter = n_iter;
        }
        __syncthreads();
        if (ini == a.n_init - 1) {  // this K's last init: its best clustering is final
          const int kk = s_kk[g];
          uint8_t* out = a.labels + static_cast<size_t>(kk) * a.n * a.ldl + h;
          for (int r = tid; r < m; r += NT) out[static_cast<size_t>(idx[r]) * a.ldl] = w.lbest[r];
          if (tid == 0) {
            if (a.inertia_out) a.inertia_out[static_cast<size_t>(kk) * a.H + h] = best_inertia;
            if (a.niter_out) a.niter_out[static_cast<size_t>(kk) * a.H + h] = best_iter;
          }
          __syncthreads();
        }
      }
      F64_STAMP(6);
    }
#ifdef CC_F64_STAMPS
    if (tid == 0 && unit < F64_UT) cc_f64_utimes[unit][1] = wall_clock64();
#endif
  }
#ifdef CC_F64_STAMPS
  if (tid == 0) {
    st_acc[9] = 1;
    for (int q = 0; q < 13; ++q) atomicAdd(&cc_f64_stamps[q], st_acc[q]);
  }
#endif
}

// The workspace after its header: grid per-workgroup areas, then grid per-resample slots (a
// launch takes up to grid resamples at a time).
struct F64Layout {
  size_t o_cl, o_dc, o_sq, o_cen, o_cnew, o_lab, o_lold, o_lbest, o_cf, per_wg;
  size_t cfs;
  size_t r_mean, r_var, r_tol, r_xsq, r_xc, r_xf, per_res;
};

F64Layout f64_layout(int m, int d, int kmax) {
  auto al = [](size_t x) { return (x + 255) & ~static_cast<size_t>(255); };
  F64Layout L{};
  size_t o = 0;
  L.o_cl = o;    o += al(sizeof(double) * m * GMAX);
  L.o_dc = o;    o += al(sizeof(double) * m * TMAX * GMAX);
  L.o_sq = o;    o += al(sizeof(double) * std::max(m, d));
  L.o_cen = o;   o += al(sizeof(double) * kmax * d * GMAX);
  L.o_cnew = o;  o += al(sizeof(double) * kmax * d * GMAX);
  L.o_lab = o;   o += al(sizeof(int32_t) * m * GMAX);
  L.o_lold = o;  o += al(sizeof(int32_t) * m * GMAX);
  L.o_lbest = o; o += al(m);
  L.cfs = static_cast<size_t>(std::max((kmax + 31) / 32, 1)) * 32 * ((d + 3) / 4) * 4;  // >= GMAX * TMAX rows
  L.o_cf = o;    o += al(sizeof(double) * L.cfs * GMAX);
  L.per_wg = o;
  o = 0;
  L.r_mean = o;  o += al(sizeof(double) * d);
  L.r_var = o;   o += al(sizeof(double) * d);
  L.r_tol = o;   o += al(sizeof(double));
  L.r_xsq = o;   o += al(sizeof(double) * m);
  L.r_xc = o;    o += al(sizeof(double) * static_cast<size_t>(m) * d);
  L.r_xf = o;    o += al(sizeof(double) * static_cast<size_t>((m + 15) / 16) * 16 * ((d + 3) / 4) * 4);
  L.per_res = o;
  return L;
}

constexpr size_t WS_ARGS = 64;  // the work counter at 0, the kernel's F64Args at WS_ARGS
constexpr size_t WS_HEADER = (WS_ARGS + sizeof(F64Args) + 255) / 256 * 256;

}  // namespace

#ifdef CC_F64_STAMPS
// the accumulated stamps (then zeroed): [0..7] phase clocks, [8] Lloyd iterations, [9] workgroups
// per-unit wall clocks of the last launch (start, end, workgroup), units < n
extern "C" int cc_kmeans_f64_unit_times(unsigned long long* out, int n) {
  n = std::min(n, F64_UT);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(cc_f64_utimes), static_cast<size_t>(n) * 3 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -1;
}

extern "C" int cc_kmeans_f64_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cc_f64_stamps), 16 * sizeof(unsigned long long)) != hipSuccess) return -1;
  const unsigned long long z[16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(cc_f64_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

// A launch takes min(grid, nh) resamples (their per-resample slots) and runs them on the grid.
static size_t f64_ws_bytes(const F64Layout& L, int grid, int nh) {
  return WS_HEADER + L.per_wg * static_cast<size_t>(grid) + L.per_res * static_cast<size_t>(std::min(grid, nh));
}

extern "C" size_t cc_kmeans_f64_workspace_bytes(int m, int d, const int32_t* Ks, int nK, int grid, int nh) {
  if (m <= 0 || d <= 0 || !Ks || nK <= 0 || grid <= 0 || nh <= 0) return 0;
  int kmax = 1;
  for (int i = 0; i < nK; ++i) kmax = std::max(kmax, Ks[i]);
  return f64_ws_bytes(f64_layout(m, d, kmax), grid, nh);
}

extern "C" int cc_kmeans_f64(const double* X, int n, int d, const int32_t* idx_hm, int H, int m,
                             int h_begin, int h_end, const int32_t* Ks, int nK, int n_init,
                             int max_iter, double tol_rel, const double* kpp_u, int kpp_stride,
                             const int32_t* kpp_pos, uint8_t* labels_nh, int ldl, double* inertia,
                             int32_t* n_iter, void* workspace, size_t ws_bytes, int grid,
                             void* stream) {
  if (!X || !idx_hm || !Ks || !kpp_u || !kpp_pos || !labels_nh || n <= 0 || d <= 0 || m <= 0 ||
      m > n || H <= 0 || h_begin < 0 || h_end > H || h_end < h_begin || nK <= 0 || nK > NKMAX ||
      n_init <= 0 || max_iter <= 0 || ldl < H || grid <= 0) {
    cc::set_error("cc_kmeans_f64: bad arguments");
    return CC_ERR_ARG;
  }
  if ((reinterpret_cast<uintptr_t>(X) & 7) != 0 || (reinterpret_cast<uintptr_t>(workspace) & 15) != 0) {
    cc::set_error("cc_kmeans_f64: X must be 8-B and the workspace 16-B aligned");
    return CC_ERR_ARG;
  }
  int kmax = 1, tmax = 0;
  for (int i = 0; i < nK; ++i) {
    if (Ks[i] < 1 || Ks[i] > KMAX || Ks[i] > m) {
      cc::set_error("cc_kmeans_f64: need 1 <= K <= min(127, m)");
      return CC_ERR_ARG;
    }
    kmax = std::max(kmax, Ks[i]);
    tmax = std::max(tmax, 2 + static_cast<int>(std::log(static_cast<double>(Ks[i]))));
  }
  if (kpp_stride < 1 + (kmax - 1) * tmax) {
    cc::set_error("cc_kmeans_f64: kpp_stride too small");
    return CC_ERR_ARG;
  }
  const int nh = h_end - h_begin;
  if (nh == 0) return CC_OK;
  const F64Layout L = f64_layout(m, d, kmax);
  if (!workspace || ws_bytes < f64_ws_bytes(L, grid, nh)) {
    cc::set_error("cc_kmeans_f64: workspace too small");
    return CC_ERR_ARG;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  F64Args a{};
  a.X = X;
  a.n = n;
  a.d = d;
  a.idx = idx_hm;
  a.H = H;
  a.m = m;
  a.h_begin = h_begin;
  a.nh = nh;
  a.nK = nK;
  for (int i = 0; i < nK; ++i) a.Ks[i] = Ks[i];
  for (int i = 0; i < nK; ++i) a.korder[i] = i;
  std::stable_sort(a.korder, a.korder + nK, [&](int x, int y) { return Ks[x] > Ks[y]; });
  // unit kinds: runs of up to P adjacent K's (in decreasing K) whose P * n_init problems fit one
  // lockstep group, so each pass over a resample's rows serves several K's.  Only K <= kpair_max
  // are grouped (the light units: their centre tiles are mostly empty and the per-unit setup
  // dominates); the kinds are then dealt in decreasing total K (longest-processing-time order).
  int P = std::max(1, std::min(F64_KPACK, GMAX / n_init));
  // grouped K's make heavier units, and the launch's tail is about one unit long: group only where
  // every workgroup gets a few units (with the per-resample setup, against one K per unit: C2
  // H = 500 1.13x, C3 H = 512 1.12x, C3 H = 128 at ~2.5 units per workgroup 1.03x)
  if (P > 1) {
    int dev = 0, cus = 0;  // resident workgroups: two per CU (the kernel's occupancy)
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = grid;
    const long long resident = std::min<long long>(grid, 2LL * cus);
    if (static_cast<long long>(std::min(nh, grid)) * ((nK + P - 1) / P) < F64_UNITS_PER_WG * resident) P = 1;
  }
  if (const char* ev = std::getenv("CCMI_F64_KPACK")) P = std::max(1, std::min(std::atoi(ev), GMAX / std::max(n_init, 1)));
  int kpair_max = F64_KPAIR_MAX;
  if (const char* ev = std::getenv("CCMI_F64_KPAIR_MAX")) kpair_max = std::atoi(ev);
  {
    int kinds[NKMAX][2], nk = 0;  // (first position in the sorted K order, count)
    for (int i = 0; i < nK;) {
      int c = 1;
      if (Ks[a.korder[i]] <= kpair_max)
        while (c < P && i + c < nK) ++c;
      kinds[nk][0] = i;
      kinds[nk][1] = c;
      ++nk;
      i += c;
    }
    auto wt = [&](int u) {
      int s = 0;
      for (int q = 0; q < kinds[u][1]; ++q) s += Ks[a.korder[kinds[u][0] + q]];
      return s;
    };
    int ord[NKMAX];
    for (int u = 0; u < nk; ++u) ord[u] = u;
    std::stable_sort(ord, ord + nk, [&](int x, int y) { return wt(x) > wt(y); });
    int ko[NKMAX], pos = 0;
    a.nuk = nk;
    for (int u = 0; u < nk; ++u) {
      a.ukfirst[u] = pos;
      for (int q = 0; q < kinds[ord[u]][1]; ++q) ko[pos++] = a.korder[kinds[ord[u]][0] + q];
    }
    a.ukfirst[nk] = pos;
    for (int i = 0; i < nK; ++i) a.korder[i] = ko[i];
  }
  a.n_init = n_init;
  a.max_iter = max_iter;
  a.tol_rel = tol_rel;
  a.kpp_u = kpp_u;
  a.kpp_stride = kpp_stride;
  a.kpp_pos = kpp_pos;
  a.labels = labels_nh;
  a.ldl = ldl;
  a.inertia_out = inertia;
  a.niter_out = n_iter;
  a.counter = static_cast<unsigned*>(workspace);
  a.ws = static_cast<char*>(workspace) + WS_HEADER;
  a.per_wg = L.per_wg;
  a.o_cl = L.o_cl;
  a.o_dc = L.o_dc;
  a.o_sq = L.o_sq;
  a.o_cen = L.o_cen;
  a.o_cnew = L.o_cnew;
  a.o_lab = L.o_lab;
  a.o_lold = L.o_lold;
  a.o_lbest = L.o_lbest;
  a.o_cf = L.o_cf;
  a.kd = static_cast<size_t>(kmax) * d;
  a.cfs = L.cfs;
  a.rs = a.ws + L.per_wg * static_cast<size_t>(grid);
  a.per_res = L.per_res;
  a.r_mean = L.r_mean;
  a.r_var = L.r_var;
  a.r_tol = L.r_tol;
  a.r_xsq = L.r_xsq;
  a.r_xc = L.r_xc;
  a.r_xf = L.r_xf;
  const F64Args* pa = reinterpret_cast<const F64Args*>(static_cast<char*>(workspace) + WS_ARGS);
  const int nrb = ((m + 15) / 16 + SRT - 1) / SRT;
  // up to grid resamples per launch (the per-resample slots): their setup, then their units
  const int chunk = std::min(nh, grid);
  for (int c0 = 0; c0 < nh; c0 += chunk) {
    const int cn = std::min(chunk, nh - c0);
    a.h_begin = h_begin + c0;
    a.nh = cn;
    // one upload: the zeroed counter and the arguments (a pageable source is consumed before
    // hipMemcpyAsync returns; the previous launches read theirs first, in stream order)
    alignas(16) unsigned char header[WS_ARGS + sizeof(F64Args)] = {};
    std::memcpy(header + WS_ARGS, &a, sizeof(F64Args));
    hipError_t e = hipMemcpyAsync(workspace, header, sizeof(header), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
      const long long nst = (static_cast<long long>(cn) * d + NT - 1) / NT;
      hipLaunchKernelGGL(f64_setup_stats, dim3(static_cast<unsigned>(nst)), dim3(NT), 0, st, pa);
      hipLaunchKernelGGL(f64_setup_rows, dim3(static_cast<unsigned>(cn) * nrb), dim3(NT), 0, st, pa, nrb);
      const unsigned blocks = static_cast<unsigned>(std::min<long long>(grid, static_cast<long long>(cn) * a.nuk));
      if (P * n_init > 4) hipLaunchKernelGGL(kmeans_f64_kernel<GMAX>, dim3(blocks), dim3(NT), 0, st, pa);
      else hipLaunchKernelGGL(kmeans_f64_kernel<4>, dim3(blocks), dim3(NT), 0, st, pa);
      e = hipGetLastError();
    }
    if (e != hipSuccess) {
      cc::set_error(std::string("cc_kmeans_f64: ") + hipGetErrorString(e));
      return CC_ERR_HIP;
    }
  }
  return CC_OK;
}
