// Batched k-means for every (resample, K, init) problem of a consensus fit, on gfx950.
//
// Replaces the per-(K, h) `clusterer.fit_predict(X[indices])` of the reference
// (consensus_clustering_parallelised.py:282, default clusterer KMeans(), CC.py:88-90,
// with set_params(random_state=seed, n_init=3), CC.py:212-214) by launches that run
// every problem at once.  The algorithm is scikit-learn's KMeans (sklearn/cluster/_kmeans.py):
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
// Mapping.  A workgroup (512 threads, ~145 KiB LDS, one per CU) owns one resample h and
// one GROUP of problems (<= 128 centroid columns, <= 32 problems; all n_init runs of a
// K in one group) and runs their whole fits on-chip.  The resample's rows stream
// through LDS in 32-row tiles, once per sweep for ALL the group's centroids.  The 8
// waves are specialised, one of each kind per SIMD:
//   MFMA waves (0-3)  wave w owns centroid columns 32w..32w+31 as register-resident
//                     A fragments and computes D = |c|^2 - 2 c.x for the tile on
//                     v_mfma_f32_32x32x2_f32 (exact f32 fma chain);
//   VALU waves (4-7)  gather the next tile's rows into LDS, run the E-step of the
//                     previous tile (argmin per row and problem: strict <, lowest
//                     index) and its M-step (per-(column, dim) owner threads add the
//                     rows into LDS sums with ds_add_f32: one owner per address, rows
//                     in order -> deterministic sums).
// The two kinds overlap through a 3-deep tile ring with two workgroup barriers per
// tile: tile t's distances (MFMA) run beside tile t-1's E/M-steps and tile t+1's gather.
// Nothing crosses workgroups, so results do not depend on scheduling or on how the
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
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 512;
constexpr int NW = 8;
constexpr int NVT = 256;            // VALU-role threads (waves 4..7)
constexpr int RT = 32;              // rows per tile (one MFMA row block)
constexpr int CMAX = CC_KM_CMAX;    // 128 centroid / candidate columns (4 MFMA waves x 32)
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
  int colrow[CMAX];  // source row of each MFMA column (seeding candidates / initial centres)
  unsigned cnt[CMAX];
  float cnorm[CMAX], shift[CMAX];
  double potc[CMAX], potc2[CMAX];
  float xn[3][RT];
  int map[KMAX + 1];
  double red_v[NW];
  int red_i[NW];
  int P, ncols, colmask, any, flag, Kg;
  float tol;
  unsigned long long n_lloyd, n_seed, n_mrows, n_reloc;
};

template <int DP>
struct Lay {
  static constexpr int XS = DP + 4;            // X tile row stride (floats): conflict-free b128 reads
  static constexpr int XBUF = RT * XS;         // floats per X ring slot
  static constexpr int OFF_D = 3 * XBUF * 4;   // distance tile [RT][DSD]
  static constexpr int U_END = OFF_D + RT * DSD * 4;
  static constexpr int S_BYTES = CMAX * DP * 4;      // sums / new centres, aliasing the ring
  static_assert(S_BYTES <= U_END, "centre sums must fit in the tile ring");
  static constexpr int OFF_CO = (U_END + 15) / 16 * 16;  // old centres [CMAX][DP]
  static constexpr int OFF_LS = OFF_CO + S_BYTES;        // tile labels [PMAX][RT]
  static constexpr int OFF_ST = OFF_LS + RT * PMAX;
  static constexpr int TOTAL = OFF_ST + ((sizeof(State) + 15) / 16) * 16;
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double half_sum(double v) {  // over the 32 lanes of a half-wave
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Diagnostic build only (-DCC_KM_STAMPS): per-wave cycle accounting of the Lloyd sweep
// phases of workgroup 0, added into stats[4 + 4*wave + k] (k: work1, wait1, work2, wait2).
#ifdef CC_KM_STAMPS
#define KM_STAMP(var) \
  __builtin_amdgcn_sched_barrier(0); \
  const unsigned long long var = __builtin_amdgcn_s_memtime(); \
  __builtin_amdgcn_sched_barrier(0)
#define KM_ACC(k, a, b) st_acc[k] += (b) - (a)
#else
#define KM_STAMP(var)
#define KM_ACC(k, a, b)
#endif

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

// sum of squares of a centre row (sklearn row_norms: f32, sequential).
__device__ __forceinline__ float row_sq(const float* c, int dreal) {
  float s = 0.f;
  for (int d = 0; d < dreal; ++d) s = fmaf(c[d], c[d], s);
  return s;
}

// ---- VALU-role tile gather: issue the global loads early, commit to LDS late ----
template <int DP>
struct TileRegs {
  static constexpr int PER = RT * (DP / 4) / NVT;  // float4 per VALU thread (1, 2 or 4)
  float4 v[PER];
  float xn;
};

template <int DP>
__device__ __forceinline__ void tile_issue(const KArgs& a, const int32_t* idx, int r0, int vt,
                                           TileRegs<DP>& R) {
  // Branch-free gather: all row indices first, then all rows (two dependent round trips).
  constexpr int NV = DP / 4;
  constexpr int PER = TileRegs<DP>::PER;
  int src[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int row = (vt + NVT * i) / NV;
    src[i] = idx[min(r0 + row, a.m - 1)];
  }
  const int xr = min(r0 + (vt & (RT - 1)), a.m - 1);
  const float xn = a.xnorm[idx[xr]];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = vt + NVT * i;
    const int row = e / NV, c4 = e - (e / NV) * NV;
    const float4 v = *reinterpret_cast<const float4*>(a.X + static_cast<size_t>(src[i]) * a.ldx + 4 * c4);
    const bool ok = r0 + row < a.m;
    R.v[i] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  R.xn = (r0 + (vt & (RT - 1)) < a.m) ? xn : 0.f;
}

template <int DP>
__device__ __forceinline__ void tile_commit(float* Xb, float* xn, int vt, const TileRegs<DP>& R) {
  using LY = Lay<DP>;
  constexpr int NV = DP / 4;
#pragma unroll
  for (int i = 0; i < TileRegs<DP>::PER; ++i) {
    const int e = vt + NVT * i;
    const int row = e / NV, c4 = e - (e / NV) * NV;
    *reinterpret_cast<float4*>(Xb + row * LY::XS + 4 * c4) = R.v[i];
  }
  if (vt < RT) xn[vt] = R.xn;
}

// ---- MFMA-role helpers -------------------------------------------------------
// Fragment of column (32*ct + lane%32): dims 8s + 4*(lane/32) .. +3 for s < DP/8.
template <int DP>
__device__ __forceinline__ void frag_load(float4 (&cf)[DP / 8], const float* src, bool valid, int lane) {
  const int g4 = 4 * (lane >> 5);
#pragma unroll
  for (int s = 0; s < DP / 8; ++s)
    cf[s] = valid ? *reinterpret_cast<const float4*>(src + 8 * s + g4) : make_float4(0.f, 0.f, 0.f, 0.f);
}

template <int DP, int S0, int S1>
__device__ __forceinline__ void mfma_dims(const float4 (&cf)[DP / 8], const float* Xb, v16f& acc, int lane) {
  using LY = Lay<DP>;
  const float* bp = Xb + (lane & 31) * LY::XS + 4 * (lane >> 5);
#pragma unroll
  for (int s = S0; s < S1; ++s) {
    const float4 bv = *reinterpret_cast<const float4*>(bp + 8 * s);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cf[s].x, bv.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cf[s].y, bv.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cf[s].z, bv.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cf[s].w, bv.w, acc, 0, 0, 0);
  }
}

// Ds[row][col] = cnorm[col] - 2 acc  (acc = D[col][row]: lane = row, regs = columns)
__device__ __forceinline__ void store_dist(const v16f& acc, const State& S, float* Ds, int ct, int lane) {
  float* drow = Ds + (lane & 31) * DSD + ct * 32 + 4 * (lane >> 5);
  const float* cn = S.cnorm + ct * 32 + 4 * (lane >> 5);
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int i = (v & 3) + 8 * (v >> 2);
    drow[i] = cn[i] - 2.0f * acc[v];
  }
}

// ---- M-step on bf16 MFMA: S[col][dim] += sum_rows onehot[col][row] * x[row][dim] ----
// x = x0 + x1 + x2 with bf16 x0 = RN(x), x1 = RN(x - x0), x2 = RN(x - x0 - x1): the one-hot
// products are exact and the three bf16 MFMAs add the row's value back to f32 precision.
__device__ __forceinline__ unsigned bf16_pack(float a, float b) {
  return static_cast<unsigned>(__builtin_bit_cast(unsigned short, static_cast<__bf16>(a))) |
         (static_cast<unsigned>(__builtin_bit_cast(unsigned short, static_cast<__bf16>(b))) << 16);
}
__device__ __forceinline__ float bf16_lo(unsigned p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float bf16_hi(unsigned p) { return __builtin_bit_cast(float, p & 0xFFFF0000u); }

// 8 f32 values -> 3 bf16x8 fragments (hi, mid, lo parts)
__device__ __forceinline__ void split3(const float (&x)[8], u32x4& f0, u32x4& f1, u32x4& f2) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = x[2 * i], b = x[2 * i + 1];
    const unsigned p0 = bf16_pack(a, b);
    const float ra = a - bf16_lo(p0), rb = b - bf16_hi(p0);
    const unsigned p1 = bf16_pack(ra, rb);
    const unsigned p2 = bf16_pack(ra - bf16_lo(p1), rb - bf16_hi(p1));
    f0[i] = p0;
    f1[i] = p1;
    f2[i] = p2;
  }
}

__device__ __forceinline__ v16f mfma_bf16(const u32x4& a, const u32x4& b, const v16f& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// Empty-cluster relocation for problem p (rare path; _k_means_common.pyx:167-212).
// Sm holds the un-averaged sums [CMAX][DP], Co the centres the labels came from.
template <int DP>
__device__ void relocate(const KArgs& a, const int32_t* idx, int p, const float* Co, float* Sm,
                         State& S, const uint8_t* glab, float* dist, int tid) {
  const int m = a.m, off = S.off[p], K = S.K[p];
  float mymax = 0.f;
  for (int r = tid; r < m; r += NT) {
    const float* x = a.X + static_cast<size_t>(idx[r]) * a.ldx;
    const float* c = Co + (off + glab[static_cast<size_t>(p) * m + r]) * DP;
    float s = 0.f;
    for (int d = 0; d < a.dreal; ++d) {
      const float t = x[d] - c[d];
      s = fmaf(t, t, s);
    }
    dist[r] = s;
    mymax = fmaxf(mymax, s);
  }
  for (int o = 32; o > 0; o >>= 1) mymax = fmaxf(mymax, __shfl_xor(mymax, o));
  if ((tid & 63) == 0) S.red_v[tid >> 6] = mymax;
  __syncthreads();
  double gmax = 0.0;
  for (int w = 0; w < NW; ++w) gmax = fmax(gmax, S.red_v[w]);
  // the empty clusters are fixed before any relocation (np.where(weight == 0))
  if (tid == 0) {
    int ne = 0;
    for (int c = 0; c < K; ++c)
      if (S.cnt[off + c] == 0) S.map[ne++] = c;
    S.flag = ne;
  }
  __syncthreads();
  if (gmax == 0.0) return;  // sklearn returns early when every point sits on its centre
  const int ne = S.flag;
  for (int e = 0; e < ne; ++e) {
    const int c = S.map[e];
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
      Sm[(off + old) * DP + d] -= x[d];
      Sm[(off + c) * DP + d] = x[d];
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
  __shared__ __attribute__((aligned(16))) char smem[LY::TOTAL];
  float* Xr = reinterpret_cast<float*>(smem);                 // 3-slot tile ring
  float* Ds = reinterpret_cast<float*>(smem + LY::OFF_D);     // distance tile
  float* Co = reinterpret_cast<float*>(smem + LY::OFF_CO);    // old centres (sweep end)
  float* Sm = reinterpret_cast<float*>(smem);                 // sums / new centres (aliases ring)
  uint8_t* Ls = reinterpret_cast<uint8_t*>(smem + LY::OFF_LS);
  State& S = *reinterpret_cast<State*>(smem + LY::OFF_ST);

  const int tid = threadIdx.x, lane = tid & 63;
  // wave index made provably uniform, so the role branches below are scalar branches
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool mrole = wave < 4;      // MFMA waves 0-3, VALU waves 4-7 (one of each per SIMD)
  const int ct = wave;              // MFMA role: centroid column tile
  const int vt = tid - NVT;         // VALU role: 0..255
  const int g = blockIdx.x / a.nh;  // heavy groups (planned first) dispatch first
  const int hb = blockIdx.x - g * a.nh;
  const int h = a.h_begin + hb;
  const int m = a.m;
  const int T = (m + RT - 1) / RT;
  const int32_t* idx = a.idx + static_cast<size_t>(h) * m;
  const int32_t* gd = a.groups + g * GS;
  uint8_t* wsb = a.ws + static_cast<size_t>(blockIdx.x) * a.ws_per_wg;
  uint8_t* glab = wsb;                                           // [Pws][m]
  float* dbuf = reinterpret_cast<float*>(wsb + a.off_dbuf);      // [Pws][Tws+1][m]
  int32_t* cpos = reinterpret_cast<int32_t*>(wsb + a.off_cpos);  // [Pws][Kws]
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
    double* red = reinterpret_cast<double*>(Xr);  // [NT/DP][DP]
    double* mean = reinterpret_cast<double*>(Xr) + NT;
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
          S.colrow[j] = idx[S.cand[p][t]];
          ++j;
        }
      }
      S.ncols = j;
      S.colmask = (1u << ((j + 31) / 32)) - 1u;
      S.n_seed += static_cast<unsigned long long>(j) * m;
    }
    __syncthreads();
    const int ncols = S.ncols;
    // Role-split pipeline (same barrier count on both sides): the MFMA waves keep the
    // candidate fragments live, the VALU waves keep the potential partial live.
    if (mrole) {
      float4 cf[DP / 8];
      const bool active = (S.colmask >> ct) & 1;
      const int col = ct * 32 + (lane & 31);
      const bool ok = col < ncols;
      frag_load<DP>(cf, a.X + static_cast<size_t>(ok ? S.colrow[col] : 0) * a.ldx, ok, lane);
      __syncthreads();
      for (int t = 0; t <= T; ++t) {
        v16f acc = {};
        if (active && t < T) mfma_dims<DP, 0, DP / 16>(cf, Xr + (t % 3) * LY::XBUF, acc, lane);
        __syncthreads();
        if (active && t < T) {
          mfma_dims<DP, DP / 16, DP / 8>(cf, Xr + (t % 3) * LY::XBUF, acc, lane);
          store_dist(acc, S, Ds, ct, lane);
        }
        __syncthreads();
      }
    } else {
      if (vt < CMAX) S.cnorm[vt] = (vt < ncols) ? a.xnorm[S.colrow[vt]] : 0.f;
      {
        TileRegs<DP> R;
        tile_issue<DP>(a, idx, 0, vt, R);
        tile_commit<DP>(Xr, S.xn[0], vt, R);
      }
      __syncthreads();
      // candidate potentials: thread = (column j, half tile of 16 rows)
      const int j = vt & (CMAX - 1), rh = vt >> 7;
      const bool jok = j < ncols;
      int p = 0, cs = 0, slot = 0;
      if (jok) {
        p = S.colprob[j];
        cs = S.cs[p];
        const int tr = S.coltr[j];
        slot = (tr < cs) ? tr : tr + 1;
      }
      const float* closest = dbuf + (static_cast<size_t>(p) * T1 + cs) * m;
      float* dout = dbuf + (static_cast<size_t>(p) * T1 + slot) * m;
      double pacc = 0.0;
      for (int t = 0; t <= T; ++t) {
        int vtl = vt;
        asm volatile("" : "+v"(vtl));
        TileRegs<DP> R;
        if (t + 1 < T) tile_issue<DP>(a, idx, (t + 1) * RT, vtl, R);
        if (t >= 1 && jok) {
          const float* xnr = S.xn[(t - 1) % 3];
          const int rb = (t - 1) * RT + rh * 16;
          float cl[16];  // branch-free: clamped rows, value unused when c == 0 or past m
#pragma unroll
          for (int q = 0; q < 16; ++q) cl[q] = closest[min(rb + q, m - 1)];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int rr = rh * 16 + q;
            if (rb + q < m) {
              const float dist = fmaxf(xnr[rr] + Ds[rr * DSD + j], 0.f);
              const float dmin = (c == 0) ? dist : fminf(cl[q], dist);
              dout[rb + q] = dmin;
              pacc += static_cast<double>(dmin);
            }
          }
        }
        if (t + 1 < T) tile_commit<DP>(Xr + ((t + 1) % 3) * LY::XBUF, S.xn[(t + 1) % 3], vtl, R);
        __syncthreads();
        __syncthreads();
      }
      if (jok) (rh ? S.potc2 : S.potc)[j] = pacc;
    }
    __syncthreads();
    if (tid < ncols) S.potc[tid] += S.potc2[tid];
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
      for (int c = 0; c < S.K[p]; ++c) {
        S.colprob[o + c] = static_cast<short>(p);
        S.colrow[o + c] = idx[cpos[p * a.Kws + c]];
      }
      o += S.K[p];
      S.st[p] = ST_RUN;
      S.iter[p] = 0;
    }
    S.ncols = o;
  }
  for (size_t e = tid; e < static_cast<size_t>(P) * m; e += NT) glab[e] = 0xFF;
  __syncthreads();
  const int ncols = S.ncols;
  // initial centres (the seeded rows) -> Sm, their norms
  for (int e = tid; e < CMAX * (DP / 4); e += NT) {
    const int col = e / (DP / 4), c4 = e - col * (DP / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (col < ncols) v = *reinterpret_cast<const float4*>(a.X + static_cast<size_t>(S.colrow[col]) * a.ldx + 4 * c4);
    *reinterpret_cast<float4*>(Sm + col * DP + 4 * c4) = v;
  }
  if (tid < CMAX) S.cnorm[tid] = (tid < ncols) ? row_sq(a.X + static_cast<size_t>(S.colrow[tid]) * a.ldx, a.dreal) : 0.f;
  if (tid < PMAX) S.changed[tid] = 0;
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
          for (int q = S.off[p] / 32; q <= (S.off[p] + S.K[p] - 1) / 32; ++q) msk |= 1u << q;
          work += static_cast<unsigned long long>(S.K[p]) * m;
          if (st == ST_RUN) mrows += m;
        }
      }
      S.colmask = static_cast<int>(msk);
      S.any = any;
      S.n_lloyd += work;
      S.n_mrows += mrows;
    }
    __syncthreads();
    if (!S.any) break;

    // Role-split sweep: both sides execute 2 + 2*(T+1) barriers.
    if (mrole) {
      float4 cf[DP / 8];  // register-resident centres of column tile ct
      const bool active = (S.colmask >> ct) & 1;
      const int col = ct * 32 + (lane & 31);
      frag_load<DP>(cf, Sm + col * DP, true, lane);
      __syncthreads();  // B0: fragments read, Sm may be cleared
      __syncthreads();  // B1: tile 0 in the ring
#ifdef CC_KM_STAMPS
      unsigned long long st_acc[4] = {0, 0, 0, 0};
#endif
      for (int t = 0; t <= T; ++t) {
        KM_STAMP(s0);
        v16f acc = {};
        if (active && t < T) mfma_dims<DP, 0, DP / 16>(cf, Xr + (t % 3) * LY::XBUF, acc, lane);
        KM_STAMP(s1);
        __syncthreads();
        KM_STAMP(s2);
        if (active && t < T) {
          mfma_dims<DP, DP / 16, DP / 8>(cf, Xr + (t % 3) * LY::XBUF, acc, lane);
          store_dist(acc, S, Ds, ct, lane);
        }
        KM_STAMP(s3);
        __syncthreads();
        KM_STAMP(s4);
        KM_ACC(0, s0, s1);
        KM_ACC(1, s1, s2);
        KM_ACC(2, s2, s3);
        KM_ACC(3, s3, s4);
      }
#ifdef CC_KM_STAMPS
      if (blockIdx.x == 0 && lane == 0 && a.stats)
        for (int k = 0; k < 4; ++k) atomicAdd(&a.stats[4 + 4 * wave + k], st_acc[k]);
#endif
      // old centres -> Co
      float* co = Co + col * DP + 4 * (lane >> 5);
#pragma unroll
      for (int s = 0; s < DP / 8; ++s) *reinterpret_cast<float4*>(co + 8 * s) = cf[s];
    } else {
      __syncthreads();  // B0
      {
        TileRegs<DP> R;
        tile_issue<DP>(a, idx, 0, vt, R);
        tile_commit<DP>(Xr, S.xn[0], vt, R);
      }
      __syncthreads();  // B1
      constexpr int NS = PMAX / NW;  // E-step slots per thread: problems ps + 8i
      double iacc[NS];
      unsigned chmask = 0;  // bit i: a label of problem ps + 8i changed in this sweep
      const int row0 = vt & 31, ps = vt >> 5;
      int sK[NS], soff[NS], sst[NS];
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        iacc[i] = 0.0;
        const int p = ps + NW * i;
        sst[i] = (p < P) ? S.st[p] : ST_IDLE;
        sK[i] = (p < P) ? S.K[p] : 0;
        soff[i] = (p < P) ? S.off[p] : 0;
      }
      // M-step role: this wave owns centroid column tile mct, all dims (NDT tiles), counts
      constexpr int NDT = DP / 32;
      const int mct = wave - 4;
      const int mcol = mct * 32 + (lane & 31);
      int mcl = -1, mpc = 0;
      if (mcol < ncols) {
        mpc = S.colprob[mcol];
        if (S.st[mpc] == ST_RUN) mcl = mcol - S.off[mpc];
      }
      const bool mact = __ballot(mcl >= 0) != 0ull;  // wave-uniform: any running column
      v16f sacc[NDT], cacc = {};
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) sacc[dt] = v16f{};
      const u32x4 ones = {0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
#ifdef CC_KM_STAMPS
      unsigned long long st_acc[4] = {0, 0, 0, 0};
#endif
      for (int t = 0; t <= T; ++t) {
        KM_STAMP(s0);
        // Opaque copies: keep the compiler from hoisting (and spilling) every per-slot and
        // per-element address out of the tile loop; they are cheap to recompute.
        int row = row0, vtl = vt;
        asm volatile("" : "+v"(row), "+v"(vtl));
        // phase 1: gather tile t+1 | E-step of tile t-1
        TileRegs<DP> R;
        if (t + 1 < T) tile_issue<DP>(a, idx, (t + 1) * RT, vtl, R);
        if (t >= 1) {
          const int r = (t - 1) * RT + row;
          const bool ok = r < m;
          const float xnr = S.xn[(t - 1) % 3][row];
          uint8_t old[NS];
#pragma unroll
          for (int i = 0; i < NS; ++i)
            old[i] = (ok && sst[i] == ST_RUN) ? glab[static_cast<size_t>(ps + NW * i) * m + r] : 0;
#pragma unroll
          for (int i = 0; i < NS; ++i) {
            if (sst[i] != ST_RUN && sst[i] != ST_FINAL) continue;
            const int p = ps + NW * i;
            const float* drow = Ds + row * DSD + soff[i];
            const int K = sK[i];
            float best = drow[0];
            int lab = 0;
            for (int c0 = 1; c0 < K; c0 += 8) {  // 8 loads in flight, then strict-< scan
              float v[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = drow[min(c0 + j, K - 1)];
#pragma unroll
              for (int j = 0; j < 8; ++j)
                if (c0 + j < K && v[j] < best) {
                  best = v[j];
                  lab = c0 + j;
                }
            }
            if (ok) {
              if (sst[i] == ST_RUN && old[i] != static_cast<uint8_t>(lab)) chmask |= 1u << i;
              glab[static_cast<size_t>(p) * m + r] = static_cast<uint8_t>(lab);
              iacc[i] += static_cast<double>(xnr) + static_cast<double>(best);
            }
            Ls[p * RT + row] = ok ? static_cast<uint8_t>(lab) : 0xFF;
          }
        }
        if (t + 1 < T) tile_commit<DP>(Xr + ((t + 1) % 3) * LY::XBUF, S.xn[(t + 1) % 3], vtl, R);
        KM_STAMP(s1);
        __syncthreads();
        KM_STAMP(s2);
        // phase 2: M-step of tile t-1 on bf16 MFMA (one-hot A, bf16x3 rows B, ones for counts)
        if (t >= 1 && mact) {
          const float* Xb = Xr + ((t - 1) % 3) * LY::XBUF + (lane & 31);
          const int g8 = 8 * (lane >> 5);
          constexpr int NQ = (RT / 16) * NDT;  // (k-step, dim tile) pairs
          float xc[8], xn8[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) xc[j] = Xb[(g8 + j) * LY::XS];
          u32x4 afr;
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int ks = q / NDT, dt = q - (q / NDT) * NDT;
            if (q + 1 < NQ) {  // prefetch the next (k-step, dim tile) rows
              const int ks1 = (q + 1) / NDT, dt1 = (q + 1) - ((q + 1) / NDT) * NDT;
#pragma unroll
              for (int j = 0; j < 8; ++j) xn8[j] = Xb[(16 * ks1 + g8 + j) * LY::XS + dt1 * 32];
            }
            if (dt == 0) {  // one-hot of this lane's column over its 8 rows of k-step ks
              const unsigned long long lab8 =
                  *reinterpret_cast<const unsigned long long*>(Ls + mpc * RT + 16 * ks + g8);
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int b0 = static_cast<int>((lab8 >> (16 * j)) & 0xFFu);
                const int b1 = static_cast<int>((lab8 >> (16 * j + 8)) & 0xFFu);
                afr[j] = ((b0 == mcl) ? 0x3F80u : 0u) | ((b1 == mcl) ? 0x3F800000u : 0u);
              }
              cacc = mfma_bf16(afr, ones, cacc);
            }
            u32x4 f0, f1, f2;
            split3(xc, f0, f1, f2);
            sacc[dt] = mfma_bf16(afr, f0, sacc[dt]);
            sacc[dt] = mfma_bf16(afr, f1, sacc[dt]);
            sacc[dt] = mfma_bf16(afr, f2, sacc[dt]);
            __builtin_amdgcn_sched_barrier(0);  // bound the live split fragments
#pragma unroll
            for (int j = 0; j < 8; ++j) xc[j] = xn8[j];
          }
        }
        KM_STAMP(s3);
        __syncthreads();
        KM_STAMP(s4);
        KM_ACC(0, s0, s1);
        KM_ACC(1, s1, s2);
        KM_ACC(2, s2, s3);
        KM_ACC(3, s3, s4);
      }
#ifdef CC_KM_STAMPS
      if (blockIdx.x == 0 && (vt & 63) == 0 && a.stats)
        for (int k = 0; k < 4; ++k) atomicAdd(&a.stats[4 + 4 * wave + k], st_acc[k]);
#endif
#pragma unroll
      for (int i = 0; i < PMAX / NW; ++i) {
        const int p = ps + NW * i;
        if (p < P) {
          const double v = half_sum(iacc[i]);
          if (row0 == 0) S.sweep_inert[p] = v;
          if ((chmask >> i) & 1u) S.changed[p] = 1;
        }
      }
      // sums -> Sm (aliases the ring: every ring reader passed the last barrier) ; counts
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int c = mct * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
          Sm[c * DP + dt * 32 + (lane & 31)] = sacc[dt][v];
        }
      if ((lane & 31) == 0)
#pragma unroll
        for (int v = 0; v < 16; ++v)
          S.cnt[mct * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5)] = static_cast<unsigned>(cacc[v]);
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
        relocate<DP>(a, idx, p, Co, Sm, S, glab, dbuf + static_cast<size_t>(p) * T1 * m, tid);
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
      Sm[col * DP + d] = Sm[(S.off[p] + S.amax[p]) * DP + d];
    }
    __syncthreads();
    for (int e = tid; e < ncols * DP; e += NT) {
      const int col = e / DP;
      const int p = S.colprob[col];
      if (S.st[p] != ST_RUN) continue;
      const unsigned cn = S.cnt[col];
      if (cn > 0) {
        const float alpha = static_cast<float>(1.0 / static_cast<double>(static_cast<float>(cn)));
        Sm[e] *= alpha;
      }
    }
    __syncthreads();
    for (int e = tid; e < ncols * DP; e += NT) {
      const int col = e / DP, d = e - col * DP;
      const int p = S.colprob[col];
      if (S.st[p] != ST_RUN || S.cnt[col] != 0 || col - S.off[p] < S.amax[p]) continue;
      Sm[col * DP + d] = Sm[(S.off[p] + S.amax[p]) * DP + d];
    }
    __syncthreads();
    // centre shifts (sklearn _euclidean_dense_dense, 4-way unrolled f32)
    if (tid < ncols && S.st[S.colprob[tid]] == ST_RUN) {
      const float* cn = Sm + tid * DP;
      const float* co = Co + tid * DP;
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
      S.changed[p] = 0;
    }
    __syncthreads();
    // norms of the centres of problems that sweep again (Sm keeps them for the fragments)
    if (tid < ncols) {
      const int st = S.st[S.colprob[tid]];
      if (st == ST_RUN || st == ST_FINAL) S.cnorm[tid] = row_sq(Sm + tid * DP, a.dreal);
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
      cc::set_error("cc_kmeans_plan: need 1 <= K <= 127 and K * n_init <= 128 (n_init <= 32)");
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
