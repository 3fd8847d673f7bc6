// Batched k-means for every (resample, K, init) problem of a consensus fit, on gfx950.
//
// Replaces the per-(K, h) `clusterer.fit_predict(X[indices])` of the reference
// (consensus_clustering_parallelised.py:282, default clusterer KMeans(), CC.py:88-90,
// with set_params(random_state=seed, n_init=3), CC.py:212-214) by ONE launch over all
// problems.  The algorithm is scikit-learn's KMeans (sklearn/cluster/_kmeans.py):
//   * k-means++ seeding (:174-262): first centre from RandomState(seed).choice with
//     uniform p (resolved on the host), then per centre 2+floor(ln K) candidates drawn
//     by searchsorted(cumsum(closest d^2), u * pot), the candidate minimising the
//     potential kept;  every fit of one K replays the same RandomState(seed) stream;
//   * Lloyd (:624-752, _k_means_lloyd.pyx:23-212): labels = argmin_c |c|^2 - 2 x.c
//     (strict <, lowest index on ties), centres = sums * f32(1/count), empty clusters
//     relocated to the farthest points (_k_means_common.pyx:167-212), strict
//     convergence on unchanged labels else sum(shift^2) <= tol, tol = 1e-4 * mean var,
//     a final E-step when not strictly converged;
//   * best of n_init: lower inertia AND a different clustering (:1525-1531).
//
// Mapping.  A workgroup (512 threads, 8 waves, ~142 KiB LDS) owns one resample h and
// one GROUP of problems (<= 128 centroid columns, <= 64 problems; all n_init runs of a
// K in one group).  It runs the whole fit of every problem of the group on-chip: the
// resample's rows stream through LDS in 64-row tiles, once per sweep for ALL the
// group's centroids, so X is read once per sweep per group instead of once per
// problem.  Per tile:
//   distances   D = cnorm - 2 * C.X^T on v_mfma_f32_32x32x2_f32 (exact f32 fma
//               chain), centroids and rows from LDS by ds_read_b128; the 8 waves own
//               (row-half, 32-column tile) work items;
//   argmin      one wave per problem, one lane per row, counts by wave ballots;
//   M-step sums S += onehot(labels)^T . X on the same f32 MFMA (0/1 operand: exact
//               products, deterministic order), accumulators resident in registers for
//               the whole sweep.
// Nothing crosses workgroups, so the result is independent of scheduling and of how
// resamples are sharded over launches or GPUs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "ccmi_internal.h"

namespace {

typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int NT = 512;
constexpr int NW = 8;
constexpr int RT = 64;              // rows per tile
constexpr int CMAX = CC_KM_CMAX;    // 128 centroid / candidate columns
constexpr int PMAX = CC_KM_PMAX;    // 64 problems per group
constexpr int TMAX = 6;             // max local trials: 2 + floor(ln 127)
constexpr int DSD = CMAX + 1;       // distance-tile row stride (floats)
constexpr int GS = CC_KM_GSTRIDE;
constexpr int KMAX = 127;

enum { ST_IDLE = 0, ST_RUN = 1, ST_FINAL = 2, ST_DONE = 3 };

struct KArgs {
  const float* X;
  const float* xnorm;
  int ldx, dreal;
  const int32_t* idx;
  int m, h_begin, nh;
  const int32_t* groups;
  int nG;
  int max_iter;
  double tol_rel;
  const double* kpp_u;
  int kpp_stride, n_init;
  const int32_t* kpp_pos;
  uint8_t* labels_out;
  int n, ldl, H;
  float* inertia_out;
  int32_t* niter_out;
  unsigned long long* stats;
  uint8_t* ws;
  size_t ws_per_wg, off_dbuf, off_cpos;
  int Pws, Tws, Kws;
};

// Small per-workgroup state (LDS).
struct State {
  int K[PMAX], kidx[PMAX], init[PMAX], ntr[PMAX], off[PMAX], st[PMAX], iter[PMAX], cs[PMAX];
  int colbase[PMAX], amax[PMAX], nempty[PMAX];
  unsigned changed[PMAX];
  float pot32[PMAX], inert[PMAX];
  double sweep_inert[PMAX];
  int cand[PMAX][TMAX];
  short colprob[CMAX], coltr[CMAX];
  unsigned cnt[CMAX];
  float cnorm[CMAX], shift[CMAX];
  double potc[CMAX];
  float xn[RT];
  int map[KMAX + 1];
  double red_v[NT / 64];
  int red_i[NT / 64];
  int P, ncols, colmask, any, flag, Kg;
  float tol;
  unsigned long long n_lloyd, n_seed, n_mrows, n_reloc;
};

template <int DP>
struct Lay {
  static constexpr int DS = DP + 4;  // LDS row stride of centroid / row / sum tiles (floats)
  static constexpr int CS_BYTES = CMAX * DS * 4;
  static constexpr int XS_BYTES = RT * DS * 4;
  static constexpr int DD_BYTES = RT * DSD * 4;
  static constexpr int U_BYTES = (XS_BYTES + DD_BYTES > CS_BYTES) ? XS_BYTES + DD_BYTES : CS_BYTES;
  static constexpr int OFF_U = CS_BYTES;
  static constexpr int OFF_LS = OFF_U + U_BYTES;
  static constexpr int OFF_ST = OFF_LS + PMAX * RT;
  static constexpr int TOTAL = OFF_ST + ((sizeof(State) + 15) / 16) * 16;
  static constexpr int NDT = DP / 32;  // 32-wide dim tiles of the M-step GEMM
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// 64 resample rows [r0, r0+64) -> Xs (zero-padded past m) and their squared norms.
template <int DP>
__device__ __forceinline__ void load_tile(const KArgs& a, const int32_t* idx, int r0, float* Xs,
                                          State& S, int tid) {
  using LY = Lay<DP>;
  constexpr int NV = DP / 4;
  constexpr int PER = RT * NV / NT;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = tid + NT * i;
    const int row = e / NV, c4 = e - (e / NV) * NV;
    const int r = r0 + row;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < a.m) v = *reinterpret_cast<const float4*>(a.X + static_cast<size_t>(idx[r]) * a.ldx + 4 * c4);
    *reinterpret_cast<float4*>(Xs + row * LY::DS + 4 * c4) = v;
  }
  if (tid < RT) {
    const int r = r0 + tid;
    S.xn[tid] = r < a.m ? a.xnorm[idx[r]] : 0.f;
  }
}

// Ds[row][col] = cnorm[col] - 2 * <C[col], X[row]> for the 32-column tiles set in mask.
// Work item of wave w: rows (w & 1) * 32 .. +32, columns (w >> 1) * 32 .. +32.
template <int DP>
__device__ __forceinline__ void dist_phase(const float* Cs, const float* Xs, const State& S,
                                           float* Ds, unsigned mask, int wave, int lane) {
  using LY = Lay<DP>;
  const int rs = wave & 1, ct = wave >> 1;
  if (!((mask >> ct) & 1u)) return;
  const float* ap = Cs + (ct * 32 + (lane & 31)) * LY::DS + 4 * (lane >> 5);
  const float* bp = Xs + (rs * 32 + (lane & 31)) * LY::DS + 4 * (lane >> 5);
  v16f acc = {};
#pragma unroll
  for (int s = 0; s < DP / 8; ++s) {
    const float4 av = *reinterpret_cast<const float4*>(ap + 8 * s);
    const float4 bv = *reinterpret_cast<const float4*>(bp + 8 * s);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv.w, acc, 0, 0, 0);
  }
  float* drow = Ds + (rs * 32 + (lane & 31)) * DSD + ct * 32 + 4 * (lane >> 5);
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int i = (v & 3) + 8 * (v >> 2);
    drow[i] = S.cnorm[ct * 32 + 4 * (lane >> 5) + i] - 2.0f * acc[v];
  }
}

// sum of squares of a centroid row (sklearn row_norms: f32, sequential).
template <int DP>
__device__ __forceinline__ float row_sq(const float* c, int dreal) {
  float s = 0.f;
  for (int d = 0; d < dreal; ++d) s = fmaf(c[d], c[d], s);
  return s;
}

// numpy pairwise_sum of a short contiguous float32 array (n <= 128), as
// `(center_shift ** 2).sum()` evaluates it (numpy/_core/src/umath/loops_utils.h).
__device__ __forceinline__ float np_pairwise_sum(const float* a, int n) {
  if (n < 8) {
    float res = 0.f;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

// Empty-cluster relocation for problem p (rare path; _k_means_common.pyx:167-212).
// Sn holds the un-averaged sums, Cs the centres the labels were computed with.
template <int DP>
__device__ void relocate(const KArgs& a, const int32_t* idx, int p, float* Cs, float* Sn,
                         State& S, uint8_t* glab, float* dist, int tid) {
  using LY = Lay<DP>;
  const int m = a.m, off = S.off[p], K = S.K[p];
  // distances of every row to its (old) centre, f32 like ((X - C[labels])**2).sum(1)
  float mymax = 0.f;
  for (int r = tid; r < m; r += NT) {
    const float* x = a.X + static_cast<size_t>(idx[r]) * a.ldx;
    const float* c = Cs + (off + glab[static_cast<size_t>(p) * m + r]) * LY::DS;
    float s = 0.f;
    for (int d = 0; d < a.dreal; ++d) {
      const float t = x[d] - c[d];
      s = fmaf(t, t, s);
    }
    dist[r] = s;
    mymax = fmaxf(mymax, s);
  }
  // block max: 0 => nothing to relocate (sklearn returns early)
  for (int o = 32; o > 0; o >>= 1) mymax = fmaxf(mymax, __shfl_xor(mymax, o));
  if ((tid & 63) == 0) S.red_v[tid >> 6] = mymax;
  __syncthreads();
  double gmax = 0.0;
  for (int w = 0; w < NW; ++w) gmax = fmax(gmax, S.red_v[w]);
  __syncthreads();
  if (gmax == 0.0) return;
  // the empty clusters are fixed before any relocation (np.where(weight == 0))
  if (tid == 0) {
    int ne = 0;
    for (int c = 0; c < K; ++c)
      if (S.cnt[off + c] == 0) S.map[ne++] = c;
    S.flag = ne;
  }
  __syncthreads();
  const int ne = S.flag;
  for (int e = 0; e < ne; ++e) {
    const int c = S.map[e];
    // far = argmax dist (ties -> lowest row)
    float bv = -1.f;
    int bi = 0x7fffffff;
    for (int r = tid; r < m; r += NT) {
      const float v = dist[r];
      if (v > bv) {
        bv = v;
        bi = r;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o);
      const int oi = __shfl_xor(bi, o);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if ((tid & 63) == 0) {
      S.red_v[tid >> 6] = bv;
      S.red_i[tid >> 6] = bi;
    }
    __syncthreads();
    double gv = -2.0;
    int gi = 0x7fffffff;
    for (int w = 0; w < NW; ++w)
      if (S.red_v[w] > gv || (S.red_v[w] == gv && S.red_i[w] < gi)) {
        gv = S.red_v[w];
        gi = S.red_i[w];
      }
    const int old = glab[static_cast<size_t>(p) * m + gi];
    const float* x = a.X + static_cast<size_t>(idx[gi]) * a.ldx;
    for (int d = tid; d < DP; d += NT) {
      Sn[(off + old) * LY::DS + d] -= x[d];
      Sn[(off + c) * LY::DS + d] = x[d];
    }
    __syncthreads();
    if (tid == 0) {
      S.cnt[off + c] = 1;
      S.cnt[off + old] -= 1;
      dist[gi] = -1.f;
      S.n_reloc += 1;
    }
    __syncthreads();
  }
}

template <int DP>
__global__ __launch_bounds__(NT, 1) void kmeans_kernel(KArgs a) {
  using LY = Lay<DP>;
  constexpr int DS = LY::DS;
  constexpr int NDT = LY::NDT;
  __shared__ __attribute__((aligned(16))) char smem[LY::TOTAL];
  float* Cs = reinterpret_cast<float*>(smem);
  float* Xs = reinterpret_cast<float*>(smem + LY::OFF_U);
  float* Ds = reinterpret_cast<float*>(smem + LY::OFF_U + LY::XS_BYTES);
  float* Sn = reinterpret_cast<float*>(smem + LY::OFF_U);
  uint8_t* Ls = reinterpret_cast<uint8_t*>(smem + LY::OFF_LS);
  State& S = *reinterpret_cast<State*>(smem + LY::OFF_ST);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x / a.nh;  // heavy groups (planned first) dispatch first
  const int hb = blockIdx.x - g * a.nh;
  const int h = a.h_begin + hb;
  const int m = a.m;
  const int32_t* idx = a.idx + static_cast<size_t>(h) * m;
  const int32_t* gd = a.groups + g * GS;
  uint8_t* wsb = a.ws + static_cast<size_t>(blockIdx.x) * a.ws_per_wg;
  uint8_t* glab = wsb;                                                // [Pws][m]
  float* dbuf = reinterpret_cast<float*>(wsb + a.off_dbuf);           // [Pws][Tws+1][m]
  int32_t* cpos = reinterpret_cast<int32_t*>(wsb + a.off_cpos);       // [Pws][Kws]
  const int T1 = a.Tws + 1;

  // ---- problem table --------------------------------------------------------
  if (tid == 0) {
    const int P = gd[0];
    S.P = P;
    int kg = 0;
    for (int p = 0; p < P; ++p) {
      S.K[p] = gd[1 + 4 * p];
      S.kidx[p] = gd[2 + 4 * p];
      S.init[p] = gd[3 + 4 * p];
      S.ntr[p] = gd[4 + 4 * p];
      S.cs[p] = a.Tws;
      kg = max(kg, S.K[p]);
    }
    S.Kg = kg;
    S.n_lloyd = S.n_seed = S.n_mrows = S.n_reloc = 0;
  }
  __syncthreads();
  const int P = S.P;

  // ---- tol = tol_rel * mean(var(X_sub, axis=0)) (sklearn _tolerance, :270-278) --
  {
    double* red = reinterpret_cast<double*>(Xs);  // [NT/DP][DP]
    double* mean = reinterpret_cast<double*>(Xs) + NT;
    constexpr int NPH = NT / DP;
    const int d = tid % DP, ph = tid / DP;
    double s = 0.0;
    for (int r = ph; r < m; r += NPH) s += static_cast<double>(a.X[static_cast<size_t>(idx[r]) * a.ldx + d]);
    red[ph * DP + d] = s;
    __syncthreads();
    if (tid < DP) {
      double t = 0.0;
      for (int k = 0; k < NPH; ++k) t += red[k * DP + tid];
      mean[tid] = t / m;
    }
    __syncthreads();
    const double mu = mean[d];
    double q = 0.0;
    for (int r = ph; r < m; r += NPH) {
      const double v = static_cast<double>(a.X[static_cast<size_t>(idx[r]) * a.ldx + d]) - mu;
      q += v * v;
    }
    __syncthreads();
    red[ph * DP + d] = q;
    __syncthreads();
    if (tid == 0) {
      double tot = 0.0;
      for (int dd = 0; dd < a.dreal; ++dd) {
        double t = 0.0;
        for (int k = 0; k < NPH; ++k) t += red[k * DP + dd];
        tot += t / m;
      }
      S.tol = static_cast<float>(static_cast<float>(tot / a.dreal) * a.tol_rel);
    }
    __syncthreads();
  }

  // ---- k-means++ seeding (all problems of the group in lockstep over centres c) ----
  for (int c = 0; c < S.Kg; ++c) {
    if (c > 0) {
      // candidates: searchsorted(cumsum_f64(closest), u * pot) per problem, one wave each
      for (int p = wave; p < P; p += NW) {
        if (S.K[p] <= c) continue;
        const int ntr = S.ntr[p];
        const double* u = a.kpp_u +
                          (static_cast<size_t>(S.kidx[p]) * a.n_init + S.init[p]) * a.kpp_stride +
                          1 + static_cast<size_t>(c - 1) * ntr;
        const double pot = static_cast<double>(S.pot32[p]);
        double rv[TMAX];
        unsigned cntv[TMAX];
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
          rv[t] = (t < ntr) ? u[t] * pot : 0.0;
          cntv[t] = 0;
        }
        const float* cl = dbuf + (static_cast<size_t>(p) * T1 + S.cs[p]) * m;
        double run = 0.0;
        for (int r0 = 0; r0 < m; r0 += 64) {
          const int r = r0 + lane;
          const bool ok = r < m;
          double v = ok ? static_cast<double>(cl[r]) : 0.0;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const double y = __shfl_up(v, o);
            if (lane >= o) v += y;
          }
          const double cum = run + v;
#pragma unroll
          for (int t = 0; t < TMAX; ++t)
            if (t < ntr) cntv[t] += static_cast<unsigned>(__popcll(__ballot(ok && cum < rv[t])));
          run = __shfl(cum, 63);
        }
        if (lane == 0)
#pragma unroll
          for (int t = 0; t < TMAX; ++t)
            if (t < ntr) S.cand[p][t] = min(static_cast<int>(cntv[t]), m - 1);
      }
    } else if (tid < P) {
      S.cand[tid][0] = a.kpp_pos[S.kidx[tid] * a.n_init + S.init[tid]];
    }
    __syncthreads();
    if (tid == 0) {
      int j = 0;
      for (int p = 0; p < P; ++p) {
        if (S.K[p] <= c) continue;
        const int nt = (c == 0) ? 1 : S.ntr[p];
        S.colbase[p] = j;
        for (int t = 0; t < nt; ++t) {
          S.colprob[j] = static_cast<short>(p);
          S.coltr[j] = static_cast<short>(t);
          ++j;
        }
      }
      S.ncols = j;
      S.colmask = (1u << ((j + 31) / 32)) - 1u;
      S.n_seed += static_cast<unsigned long long>(j) * m;
    }
    __syncthreads();
    const int ncols = S.ncols;
    const unsigned mask = static_cast<unsigned>(S.colmask);
    // candidate rows -> Cs, cnorm
    for (int e = tid; e < CMAX * (DP / 4); e += NT) {
      const int col = e / (DP / 4), c4 = e - col * (DP / 4);
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (col < ncols) {
        const int p = S.colprob[col];
        const int row = idx[S.cand[p][S.coltr[col]]];
        v = *reinterpret_cast<const float4*>(a.X + static_cast<size_t>(row) * a.ldx + 4 * c4);
      }
      *reinterpret_cast<float4*>(Cs + col * DS + 4 * c4) = v;
    }
    if (tid < CMAX) {
      float cn = 0.f;
      if (tid < ncols) cn = a.xnorm[idx[S.cand[S.colprob[tid]][S.coltr[tid]]]];
      S.cnorm[tid] = cn;
    }
    __syncthreads();
    double pacc[CMAX / NW];
#pragma unroll
    for (int i = 0; i < CMAX / NW; ++i) pacc[i] = 0.0;
    for (int r0 = 0; r0 < m; r0 += RT) {
      load_tile<DP>(a, idx, r0, Xs, S, tid);
      __syncthreads();
      dist_phase<DP>(Cs, Xs, S, Ds, mask, wave, lane);
      __syncthreads();
      const int r = r0 + lane;
      if (r < m) {
        const float xnr = S.xn[lane];
#pragma unroll
        for (int i = 0; i < CMAX / NW; ++i) {
          const int j = wave + NW * i;
          if (j < ncols) {
            const int p = S.colprob[j], t = S.coltr[j];
            const float dist = fmaxf(xnr + Ds[lane * DSD + j], 0.f);
            const int cs = S.cs[p];
            const float dmin = (c == 0) ? dist : fminf(dbuf[(static_cast<size_t>(p) * T1 + cs) * m + r], dist);
            const int slot = (t < cs) ? t : t + 1;
            dbuf[(static_cast<size_t>(p) * T1 + slot) * m + r] = dmin;
            pacc[i] += static_cast<double>(dmin);
          }
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < CMAX / NW; ++i) {
      const int j = wave + NW * i;
      if (j < ncols) {
        const double v = wave_sum(pacc[i]);
        if (lane == 0) S.potc[j] = v;
      }
    }
    __syncthreads();
    if (tid < P && S.K[tid] > c) {
      const int p = tid, j0 = S.colbase[p];
      const int nt = (c == 0) ? 1 : S.ntr[p];
      int best = 0;
      float bv = static_cast<float>(S.potc[j0]);
      for (int t = 1; t < nt; ++t) {
        const float v = static_cast<float>(S.potc[j0 + t]);
        if (v < bv) {
          bv = v;
          best = t;
        }
      }
      S.pot32[p] = bv;
      S.cs[p] = (best < S.cs[p]) ? best : best + 1;
      cpos[p * a.Kws + c] = S.cand[p][best];
    }
    __syncthreads();
  }

  // ---- Lloyd ------------------------------------------------------------------
  if (tid == 0) {
    int o = 0;
    for (int p = 0; p < P; ++p) {
      S.off[p] = o;
      for (int c = 0; c < S.K[p]; ++c) S.colprob[o + c] = static_cast<short>(p);
      o += S.K[p];
      S.st[p] = ST_RUN;
      S.iter[p] = 0;
    }
    S.ncols = o;
  }
  __syncthreads();
  const int ncols = S.ncols;
  for (int e = tid; e < CMAX * (DP / 4); e += NT) {
    const int col = e / (DP / 4), c4 = e - col * (DP / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (col < ncols) {
      const int p = S.colprob[col];
      const int row = idx[cpos[p * a.Kws + (col - S.off[p])]];
      v = *reinterpret_cast<const float4*>(a.X + static_cast<size_t>(row) * a.ldx + 4 * c4);
    }
    *reinterpret_cast<float4*>(Cs + col * DS + 4 * c4) = v;
  }
  for (size_t e = tid; e < static_cast<size_t>(P) * m; e += NT) glab[e] = 0xFF;
  __syncthreads();
  if (tid < CMAX) S.cnorm[tid] = (tid < ncols) ? row_sq<DP>(Cs + tid * DS, a.dreal) : 0.f;
  __syncthreads();

  for (;;) {
    if (tid == 0) {
      unsigned msk = 0;
      int any = 0;
      unsigned long long work = 0, mrows = 0;
      for (int p = 0; p < P; ++p) {
        const int st = S.st[p];
        if (st == ST_RUN || st == ST_FINAL) {
          any = 1;
          for (int ct = S.off[p] / 32; ct <= (S.off[p] + S.K[p] - 1) / 32; ++ct) msk |= 1u << ct;
          work += static_cast<unsigned long long>(S.K[p]) * m;
          if (st == ST_RUN) mrows += m;
        }
      }
      S.colmask = static_cast<int>(msk);
      S.any = any;
      S.n_lloyd += work;
      S.n_mrows += mrows;
    }
    if (tid < CMAX) S.cnt[tid] = 0;
    if (tid < PMAX) S.changed[tid] = 0;
    __syncthreads();
    if (!S.any) break;
    const unsigned mask = static_cast<unsigned>(S.colmask);

    v16f sacc[2];
    sacc[0] = v16f{};
    sacc[1] = v16f{};
    double iacc[PMAX / NW];
#pragma unroll
    for (int i = 0; i < PMAX / NW; ++i) iacc[i] = 0.0;

    for (int r0 = 0; r0 < m; r0 += RT) {
      load_tile<DP>(a, idx, r0, Xs, S, tid);
      __syncthreads();
      dist_phase<DP>(Cs, Xs, S, Ds, mask, wave, lane);
      __syncthreads();
      // E-step: wave per problem, lane per row
      {
        const int r = r0 + lane;
        const bool ok = r < m;
#pragma unroll
        for (int i = 0; i < PMAX / NW; ++i) {
          const int p = wave + NW * i;
          if (p >= P) break;
          const int st = S.st[p];
          if (st != ST_RUN && st != ST_FINAL) continue;
          const int K = S.K[p], off = S.off[p];
          const float* drow = Ds + lane * DSD + off;
          float best = drow[0];
          int lab = 0;
          for (int c = 1; c < K; ++c) {
            const float v = drow[c];
            if (v < best) {
              best = v;
              lab = c;
            }
          }
          bool ch = false;
          if (ok) {
            uint8_t* gl = glab + static_cast<size_t>(p) * m + r;
            ch = (*gl != static_cast<uint8_t>(lab));
            *gl = static_cast<uint8_t>(lab);
            iacc[i] += static_cast<double>(S.xn[lane]) + static_cast<double>(best);
          }
          Ls[p * RT + lane] = ok ? static_cast<uint8_t>(lab) : 0xFF;
          if (st == ST_RUN) {
            if (__ballot(ch) != 0ull && lane == 0) S.changed[p] = 1;
            for (int c = 0; c < K; ++c) {
              const unsigned long long b = __ballot(ok && lab == c);
              if (lane == 0) S.cnt[off + c] += static_cast<unsigned>(__popcll(b));
            }
          }
        }
      }
      __syncthreads();
      // M-step sums: S[col][dim] += sum_row onehot[col][row] * X[row][dim]
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int tau = wave + NW * i;
        if (tau >= 4 * NDT) break;
        const int ct = tau / NDT, dt = tau - (tau / NDT) * NDT;
        if (!((mask >> ct) & 1u)) continue;
        const int col = ct * 32 + (lane & 31);
        int pc = -1, cl = -1;
        if (col < ncols) {
          pc = S.colprob[col];
          cl = col - S.off[pc];
          if (S.st[pc] != ST_RUN) cl = -1;
        }
        const uint32_t* lrow = reinterpret_cast<const uint32_t*>(Ls + (pc < 0 ? 0 : pc) * RT);
        const float* xb = Xs + dt * 32 + (lane & 31);
        const int g4 = 4 * (lane >> 5);
#pragma unroll
        for (int s = 0; s < RT / 8; ++s) {
          const uint32_t l4 = lrow[(8 * s + g4) >> 2];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int lb = static_cast<int>((l4 >> (8 * q)) & 0xFFu);
            const float av = (lb == cl) ? 1.0f : 0.0f;
            const float bv = xb[(8 * s + g4 + q) * DS];
            sacc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, sacc[i], 0, 0, 0);
          }
        }
      }
      __syncthreads();
    }

    // ---- end of sweep: inertia, sums -> Sn --------------------------------
#pragma unroll
    for (int i = 0; i < PMAX / NW; ++i) {
      const int p = wave + NW * i;
      if (p < P) {
        const double v = wave_sum(iacc[i]);
        if (lane == 0) S.sweep_inert[p] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int tau = wave + NW * i;
      if (tau >= 4 * NDT) break;
      const int ct = tau / NDT, dt = tau - (tau / NDT) * NDT;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int col = ct * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
        Sn[col * DS + dt * 32 + (lane & 31)] = sacc[i][v];
      }
    }
    if (tid == 0) {
      int f = 0;
      for (int p = 0; p < P; ++p) {
        S.nempty[p] = 0;
        if (S.st[p] != ST_RUN) continue;
        for (int c = 0; c < S.K[p]; ++c) S.nempty[p] += (S.cnt[S.off[p] + c] == 0);
        f |= (S.nempty[p] > 0);
      }
      S.flag = f;
    }
    __syncthreads();
    if (S.flag) {
      for (int p = 0; p < P; ++p) {
        if (S.nempty[p] == 0) continue;
        relocate<DP>(a, idx, p, Cs, Sn, S, glab,
                     dbuf + static_cast<size_t>(p) * T1 * m, tid);
        __syncthreads();
      }
    }
    // first argmax of counts per problem (for clusters still empty: _average_centers)
    if (tid < P && S.st[tid] == ST_RUN) {
      const int off = S.off[tid];
      int am = 0;
      for (int c = 1; c < S.K[tid]; ++c)
        if (S.cnt[off + c] > S.cnt[off + am]) am = c;
      S.amax[tid] = am;
    }
    __syncthreads();
    // _average_centers (_k_means_common.pyx:215-237) runs j in order: an empty cluster
    // j copies centre argmax(weight), which is still a raw sum when j < argmax.
    for (int e = tid; e < ncols * DP; e += NT) {
      const int col = e / DP, d = e - col * DP;
      const int p = S.colprob[col];
      if (S.st[p] != ST_RUN || S.cnt[col] != 0 || col - S.off[p] > S.amax[p]) continue;
      Sn[col * DS + d] = Sn[(S.off[p] + S.amax[p]) * DS + d];
    }
    __syncthreads();
    for (int e = tid; e < ncols * DP; e += NT) {
      const int col = e / DP, d = e - col * DP;
      const int p = S.colprob[col];
      if (S.st[p] != ST_RUN) continue;
      const unsigned cn = S.cnt[col];
      if (cn > 0) {
        const float alpha = static_cast<float>(1.0 / static_cast<double>(static_cast<float>(cn)));
        Sn[col * DS + d] *= alpha;
      }
    }
    __syncthreads();
    for (int e = tid; e < ncols * DP; e += NT) {
      const int col = e / DP, d = e - col * DP;
      const int p = S.colprob[col];
      if (S.st[p] != ST_RUN || S.cnt[col] != 0 || col - S.off[p] < S.amax[p]) continue;
      Sn[col * DS + d] = Sn[(S.off[p] + S.amax[p]) * DS + d];
    }
    __syncthreads();
    // centre shifts (sklearn _euclidean_dense_dense, 4-way unrolled f32)
    if (tid < ncols && S.st[S.colprob[tid]] == ST_RUN) {
      const float* cn = Sn + tid * DS;
      const float* co = Cs + tid * DS;
      float res = 0.f;
      const int n4 = a.dreal / 4, rem = a.dreal % 4;
      for (int i = 0; i < n4; ++i) {
        const float d0 = cn[4 * i] - co[4 * i], d1 = cn[4 * i + 1] - co[4 * i + 1];
        const float d2 = cn[4 * i + 2] - co[4 * i + 2], d3 = cn[4 * i + 3] - co[4 * i + 3];
        res += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
      }
      for (int i = 0; i < rem; ++i) {
        const float dd = cn[4 * n4 + i] - co[4 * n4 + i];
        res += dd * dd;
      }
      const float sh = sqrtf(res);
      S.shift[tid] = sh * sh;
    }
    __syncthreads();
    // convergence decisions (_kmeans_single_lloyd :697-736)
    if (tid < P) {
      const int p = tid;
      const int st = S.st[p];
      if (st == ST_RUN) {
        S.iter[p] += 1;
        if (!S.changed[p]) {
          S.st[p] = ST_DONE;  // strict convergence: final labels and centres are this sweep's
          S.inert[p] = static_cast<float>(S.sweep_inert[p]);
        } else {
          const float tot = np_pairwise_sum(S.shift + S.off[p], S.K[p]);
          S.st[p] = (tot <= S.tol || S.iter[p] >= a.max_iter) ? ST_FINAL : ST_RUN;
        }
      } else if (st == ST_FINAL) {
        S.st[p] = ST_DONE;
        S.inert[p] = static_cast<float>(S.sweep_inert[p]);
      }
    }
    __syncthreads();
    // commit the new centres of problems that sweep again
    for (int e = tid; e < ncols * (DP / 4); e += NT) {
      const int col = e / (DP / 4), c4 = e - col * (DP / 4);
      const int st = S.st[S.colprob[col]];
      if (st == ST_RUN || st == ST_FINAL)
        *reinterpret_cast<float4*>(Cs + col * DS + 4 * c4) =
            *reinterpret_cast<const float4*>(Sn + col * DS + 4 * c4);
    }
    __syncthreads();
    if (tid < ncols) {
      const int st = S.st[S.colprob[tid]];
      if (st == ST_RUN || st == ST_FINAL) S.cnorm[tid] = row_sq<DP>(Cs + tid * DS, a.dreal);
    }
    __syncthreads();
  }

  // ---- best of n_init per K, output (KMeans.fit :1495-1531) -------------------
  for (int p0 = 0; p0 < P; p0 += a.n_init) {
    int best = p0;
    for (int i = 1; i < a.n_init; ++i) {
      const int p = p0 + i;
      if (!(S.inert[p] < S.inert[best])) continue;
      // _is_same_clustering(labels_p, labels_best): labels_p -> labels_best must be a function
      if (tid <= KMAX) S.map[tid] = -1;
      if (tid == 0) S.flag = 0;
      __syncthreads();
      const uint8_t* l1 = glab + static_cast<size_t>(p) * m;
      const uint8_t* l2 = glab + static_cast<size_t>(best) * m;
      for (int r = tid; r < m; r += NT) S.map[l1[r]] = l2[r];
      __syncthreads();
      bool bad = false;
      for (int r = tid; r < m; r += NT) bad |= (S.map[l1[r]] != l2[r]);
      if (bad) S.flag = 1;
      __syncthreads();
      if (S.flag) best = p;
      __syncthreads();
    }
    const int kidx = S.kidx[p0];
    const uint8_t* lb = glab + static_cast<size_t>(best) * m;
    uint8_t* out = a.labels_out + static_cast<size_t>(kidx) * a.n * a.ldl + h;
    for (int r = tid; r < m; r += NT) out[static_cast<size_t>(idx[r]) * a.ldl] = lb[r];
    if (tid == 0) {
      if (a.inertia_out) a.inertia_out[static_cast<size_t>(kidx) * a.H + h] = S.inert[best];
      if (a.niter_out) a.niter_out[static_cast<size_t>(kidx) * a.H + h] = S.iter[best];
    }
  }
  if (tid == 0 && a.stats) {
    atomicAdd(&a.stats[0], S.n_lloyd);
    atomicAdd(&a.stats[1], S.n_seed);
    atomicAdd(&a.stats[2], S.n_mrows);
    atomicAdd(&a.stats[3], S.n_reloc);
  }
}

int local_trials(int K) { return 2 + static_cast<int>(std::log(static_cast<double>(K))); }

struct WsLayout {
  int Pws = 0, Tws = 0, Kws = 0;
  size_t off_dbuf = 0, off_cpos = 0, per_wg = 0;
};

WsLayout ws_layout(int m, const int32_t* groups, int nG) {
  WsLayout L;
  for (int g = 0; g < nG; ++g) {
    const int32_t* gd = groups + static_cast<size_t>(g) * GS;
    L.Pws = std::max(L.Pws, gd[0]);
    for (int p = 0; p < gd[0]; ++p) {
      L.Kws = std::max(L.Kws, gd[1 + 4 * p]);
      L.Tws = std::max(L.Tws, gd[4 + 4 * p]);
    }
  }
  auto al = [](size_t x) { return (x + 255) & ~static_cast<size_t>(255); };
  L.off_dbuf = al(static_cast<size_t>(L.Pws) * m);
  L.off_cpos = L.off_dbuf + al(static_cast<size_t>(L.Pws) * (L.Tws + 1) * m * sizeof(float));
  L.per_wg = L.off_cpos + al(static_cast<size_t>(L.Pws) * L.Kws * sizeof(int32_t));
  return L;
}

template <int DP>
void launch(const KArgs& a, unsigned blocks, hipStream_t st) {
  hipLaunchKernelGGL(kmeans_kernel<DP>, dim3(blocks), dim3(NT), 0, st, a);
}

}  // namespace

extern "C" int cc_kmeans_plan(const int32_t* Ks, int nK, int n_init, int32_t* groups,
                              int max_groups) {
  if (!Ks || nK <= 0 || n_init <= 0 || !groups || max_groups <= 0) {
    cc::set_error("cc_kmeans_plan: bad arguments");
    return CC_ERR_ARG;
  }
  std::vector<int> order(nK);
  for (int i = 0; i < nK; ++i) {
    if (Ks[i] < 1 || Ks[i] > KMAX || Ks[i] * n_init > CMAX || n_init > PMAX) {
      cc::set_error("cc_kmeans_plan: need 1 <= K <= 127 and K * n_init <= 128 (n_init <= 64)");
      return CC_ERR_UNSUPPORTED;
    }
    order[i] = i;
  }
  // first-fit decreasing by K: heavy groups first (they also dispatch first)
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return Ks[x] > Ks[y]; });
  std::vector<int> cols, probs;
  int nG = 0;
  for (int k : order) {
    const int need = Ks[k] * n_init;
    int g = 0;
    for (; g < nG; ++g)
      if (cols[g] + need <= CMAX && probs[g] + n_init <= PMAX) break;
    if (g == nG) {
      if (nG == max_groups) {
        cc::set_error("cc_kmeans_plan: max_groups too small");
        return CC_ERR_ARG;
      }
      cols.push_back(0);
      probs.push_back(0);
      int32_t* gd = groups + static_cast<size_t>(nG) * GS;
      std::fill(gd, gd + GS, 0);
      ++nG;
    }
    int32_t* gd = groups + static_cast<size_t>(g) * GS;
    for (int i = 0; i < n_init; ++i) {
      const int p = probs[g] + i;
      gd[1 + 4 * p] = Ks[k];
      gd[2 + 4 * p] = k;
      gd[3 + 4 * p] = i;
      gd[4 + 4 * p] = local_trials(Ks[k]);
    }
    probs[g] += n_init;
    cols[g] += need;
    gd[0] = probs[g];
  }
  return nG;
}

extern "C" size_t cc_kmeans_workspace_bytes(int m, const int32_t* groups_host, int nG, int nh) {
  if (m <= 0 || !groups_host || nG <= 0 || nh <= 0) return 0;
  return ws_layout(m, groups_host, nG).per_wg * static_cast<size_t>(nG) * nh;
}

extern "C" int cc_kmeans_batched(const float* X, const float* xnorm, int n, int dreal, int dpad,
                                 const int32_t* idx_hm, int H, int m, int h_begin, int h_end,
                                 const int32_t* groups, const int32_t* groups_host, int nG,
                                 int n_init, int max_iter, double tol_rel, const double* kpp_u,
                                 int kpp_stride, const int32_t* kpp_pos, uint8_t* labels_nh,
                                 int ldl, float* inertia, int32_t* n_iter,
                                 unsigned long long* stats, void* workspace, size_t ws_bytes,
                                 void* stream) {
  if (!X || !xnorm || !idx_hm || !groups || !groups_host || !kpp_u || !kpp_pos || !labels_nh ||
      n <= 0 || m <= 0 || m > n || H <= 0 || h_begin < 0 || h_end > H || h_end < h_begin ||
      nG <= 0 || n_init <= 0 || max_iter <= 0 || dreal <= 0 || dreal > dpad || ldl < H) {
    cc::set_error("cc_kmeans_batched: bad arguments");
    return CC_ERR_ARG;
  }
  if (dpad != 32 && dpad != 64 && dpad != 128) {
    cc::set_error("cc_kmeans_batched: dpad must be 32, 64 or 128 (d <= 128 in this build)");
    return CC_ERR_UNSUPPORTED;
  }
  int kmax = 0, tmax = 0;
  for (int g = 0; g < nG; ++g) {
    const int32_t* gd = groups_host + static_cast<size_t>(g) * GS;
    int cols = 0;
    if (gd[0] <= 0 || gd[0] > PMAX || gd[0] % n_init != 0) {
      cc::set_error("cc_kmeans_batched: malformed group descriptor");
      return CC_ERR_ARG;
    }
    for (int p = 0; p < gd[0]; ++p) {
      const int K = gd[1 + 4 * p];
      if (K < 1 || K > KMAX || K > m || gd[4 + 4 * p] != local_trials(K) || gd[4 + 4 * p] > TMAX) {
        cc::set_error("cc_kmeans_batched: bad K in group (1 <= K <= min(127, m))");
        return CC_ERR_ARG;
      }
      cols += K;
      kmax = std::max(kmax, K);
      tmax = std::max(tmax, gd[4 + 4 * p]);
    }
    if (cols > CMAX) {
      cc::set_error("cc_kmeans_batched: group exceeds 128 centroid columns");
      return CC_ERR_ARG;
    }
  }
  if (kpp_stride < 1 + (kmax - 1) * tmax) {
    cc::set_error("cc_kmeans_batched: kpp_stride too small");
    return CC_ERR_ARG;
  }
  const int nh = h_end - h_begin;
  if (nh == 0) return CC_OK;
  const WsLayout L = ws_layout(m, groups_host, nG);
  if (!workspace || ws_bytes < L.per_wg * static_cast<size_t>(nG) * nh) {
    cc::set_error("cc_kmeans_batched: workspace too small");
    return CC_ERR_ARG;
  }
  const size_t blocks = static_cast<size_t>(nG) * nh;
  if (blocks > 0x7fffffffu) {
    cc::set_error("cc_kmeans_batched: too many workgroups");
    return CC_ERR_ARG;
  }
  KArgs a{};
  a.X = X;
  a.xnorm = xnorm;
  a.ldx = dpad;
  a.dreal = dreal;
  a.idx = idx_hm;
  a.m = m;
  a.h_begin = h_begin;
  a.nh = nh;
  a.groups = groups;
  a.nG = nG;
  a.max_iter = max_iter;
  a.tol_rel = tol_rel;
  a.kpp_u = kpp_u;
  a.kpp_stride = kpp_stride;
  a.n_init = n_init;
  a.kpp_pos = kpp_pos;
  a.labels_out = labels_nh;
  a.n = n;
  a.ldl = ldl;
  a.H = H;
  a.inertia_out = inertia;
  a.niter_out = n_iter;
  a.stats = stats;
  a.ws = static_cast<uint8_t*>(workspace);
  a.ws_per_wg = L.per_wg;
  a.off_dbuf = L.off_dbuf;
  a.off_cpos = L.off_cpos;
  a.Pws = L.Pws;
  a.Tws = L.Tws;
  a.Kws = L.Kws;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  switch (dpad) {
    case 32: launch<32>(a, static_cast<unsigned>(blocks), st); break;
    case 64: launch<64>(a, static_cast<unsigned>(blocks), st); break;
    default: launch<128>(a, static_cast<unsigned>(blocks), st); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_kmeans_batched: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}
