// One-call k-means of a consensus fit (cc_kmeans_fit) and the shared row preparation
// (cc_prepare_rows).
//
// cc_kmeans_fit replaces the whole per-(K, h) `clusterer.fit_predict(X[indices])` loop of the
// reference (consensus_clustering_parallelised.py:282, KMeans(n_init=3) per CC.py:88-90 and
// :212-214) for resamples [h_begin, h_end): it prepares the MFMA row image, replays the
// k-means++ RandomState streams (cc_kpp_tables), plans the units and the persistent grid, sizes
// everything from the caller's workspace and launches the engine that fits the row width and
// precision (cc_kmeans_batched, cc_kmeans_wide or cc_kmeans_f64).  The separate entry points stay
// the advanced API; the Python host drives them directly and gives the same results.
//
// cc_prepare_rows: sklearn centres each resample by its own mean (_kmeans.py:1479-1481); the
// f32 engines centre once by the column means of all rows (distances are translation
// invariant), zero-pad to dpad, take squared row norms and the operand scale 2^e with
// max|X| 2^e <= 2^14, and split the rows into the f16 hi/lo image.  Every reduction has a fixed
// order, so the row image is reproducible run to run.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "ccmi_internal.h"

extern "C" int cc_kpp_tables(const int32_t* Ks, int nK, int n_init, uint32_t seed, int m,
                             int weight_f64, double* kpp_u, int kpp_stride, int32_t* kpp_pos);

namespace {

constexpr int RB = 256;  // rows per column-sum block

// partial column sums of rows [RB b, RB b + RB) in float64, rows in order
__global__ void colsum_kernel(const float* __restrict__ X, int n, int d, double* __restrict__ part) {
  const int b = blockIdx.x;
  for (int k = threadIdx.x; k < d; k += blockDim.x) {
    double s = 0.0;
    const int r1 = min(n, RB * (b + 1));
    for (int r = RB * b; r < r1; ++r) s += static_cast<double>(X[static_cast<size_t>(r) * d + k]);
    part[static_cast<size_t>(b) * d + k] = s;
  }
}

// column means: the block partials summed in block order
__global__ void colmean_kernel(const double* __restrict__ part, int nb, int n, int d, float* __restrict__ mean) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= d) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += part[static_cast<size_t>(b) * d + k];
  mean[k] = static_cast<float>(s / n);
}

// centred, zero-padded rows, squared norms (sequential fma over the features) and per-block
// max |x| (order-free)
__global__ void centre_kernel(const float* __restrict__ X, int n, int d, int dpad, const float* __restrict__ mean,
                              float* __restrict__ Xd, float* __restrict__ xnorm, float* __restrict__ amax_part) {
  __shared__ float red[256];
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  float am = 0.f;
  if (r < n) {
    float q = 0.f;
    for (int k = 0; k < dpad; ++k) {
      const float v = k < d ? X[static_cast<size_t>(r) * d + k] - mean[k] : 0.f;
      Xd[static_cast<size_t>(r) * dpad + k] = v;
      q = fmaf(v, v, q);
      am = fmaxf(am, fabsf(v));
    }
    xnorm[r] = q;
  }
  red[threadIdx.x] = am;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) amax_part[blockIdx.x] = red[0];
}

int hip_status(const char* fn) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cc::set_error(std::string(fn) + ": " + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}

int dpad_for(int d) {
  for (int p : {32, 64, 128})
    if (d <= p) return p;
  return (d + 31) / 32 * 32;
}

int scale_exponent(float amax) {
  if (!std::isfinite(amax)) return INT32_MIN;
  if (amax == 0.f) return 0;
  const int e = 14 - static_cast<int>(std::ceil(std::log2(static_cast<double>(amax))));
  return std::max(-62, std::min(62, e));
}

size_t align256(size_t b) { return (b + 255) & ~static_cast<size_t>(255); }

// scratch of cc_prepare_rows: column partials, means, per-block maxima
size_t prep_scratch_bytes(int n, int d) {
  const size_t nb = (static_cast<size_t>(n) + RB - 1) / RB, nr = (static_cast<size_t>(n) + 255) / 256;
  return align256(nb * d * 8) + align256(static_cast<size_t>(d) * 4) + align256(nr * 4);
}

int local_trials(int K) { return 2 + static_cast<int>(std::log(static_cast<double>(K))); }

// units per resample: enough to fill every CU of the persistent grid with a balanced last round,
// as few as possible (kmeans.choose_subsets)
int choose_subsets(int nh, int n_groups, int cus) {
  int best = 1;
  double best_eff = -1.0;
  for (int s = 1; s <= std::max(1, n_groups); ++s) {
    const long long units = static_cast<long long>(nh) * s;
    const long long rounds = (units + cus - 1) / cus;
    const double eff = units >= cus ? static_cast<double>(units) / (static_cast<double>(cus) * rounds)
                                    : static_cast<double>(units) / cus;
    if (eff >= 0.85) return s;
    if (eff > best_eff + 1e-9) {
      best = s;
      best_eff = eff;
    }
  }
  return best;
}

int default_seedmax(int m) { return std::max(2, std::min(24, 4000000 / std::max(m, 1))); }  // kmeans.py default_seedmax

int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return cus;
}

// Everything cc_kmeans_fit needs besides the engine workspace.
struct FitPlan {
  int dpad = 0, nU = 0, seedmax = 0, stride = 0, grid = 0, cus = 0;
  std::vector<int32_t> units;
  size_t rows_bytes = 0;    // Xd, xnorm, Xhl, prep scratch (f32 engines)
  size_t tables_bytes = 0;  // units, kpp_u, kpp_pos, stats
};

FitPlan make_plan(int d, int m, int nh, const int32_t* Ks, int nK, int n_init, int precision, int n) {
  FitPlan P;
  P.cus = device_cus();
  P.dpad = dpad_for(d);
  int stride = 1;
  for (int k = 0; k < nK; ++k) stride = std::max(stride, 1 + (Ks[k] - 1) * local_trials(Ks[k]));
  P.stride = stride;
  if (precision == CC_KM_FAST) {
    P.rows_bytes = align256(static_cast<size_t>(n) * P.dpad * 4) + align256(static_cast<size_t>(n) * 4) +
                   align256(static_cast<size_t>(n) * 2 * P.dpad * 2) + prep_scratch_bytes(n, d);
    if (P.dpad <= 128) {
      const int n_sub = choose_subsets(nh, nK, std::max(P.cus, 1));
      P.units.assign(static_cast<size_t>(std::max(n_sub, nK) + 1) * CC_KM_USTRIDE, 0);
      P.nU = cc_kmeans_plan(Ks, nK, n_init, n_sub, P.units.data(), std::max(n_sub, nK) + 1);
      if (P.nU > 0) {
        int pmax = 0;
        for (int u = 0; u < P.nU; ++u) pmax = std::max(pmax, static_cast<int>(P.units[static_cast<size_t>(u) * CC_KM_USTRIDE]));
        P.seedmax = std::max(1, std::min({default_seedmax(m), 32, pmax}));
      }
    }
  }
  P.tables_bytes = align256(static_cast<size_t>(std::max(P.nU, 1)) * CC_KM_USTRIDE * 4) +
                   align256(static_cast<size_t>(nK) * n_init * stride * 8) +
                   align256(static_cast<size_t>(nK) * n_init * 4) + align256(128 * 8);
  return P;
}

}  // namespace

extern "C" size_t cc_prepare_rows_scratch_bytes(int n, int d) {
  if (n <= 0 || d <= 0) return 0;
  return prep_scratch_bytes(n, d);
}

extern "C" int cc_prepare_rows(const float* X, int n, int d, int dpad, float* Xd, float* xnorm, uint16_t* Xhl,
                               int* scale_exp, void* scratch, size_t scratch_bytes, void* stream) {
  if (!X || !Xd || !xnorm || !Xhl || !scale_exp || !scratch || n <= 0 || d <= 0 || dpad < d ||
      scratch_bytes < prep_scratch_bytes(n, d)) {
    cc::set_error("cc_prepare_rows: bad arguments");
    return CC_ERR_ARG;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const int nb = (n + RB - 1) / RB, nr = (n + 255) / 256;
  char* s = static_cast<char*>(scratch);
  double* part = reinterpret_cast<double*>(s);
  float* mean = reinterpret_cast<float*>(s + align256(static_cast<size_t>(nb) * d * 8));
  float* amax = reinterpret_cast<float*>(s + align256(static_cast<size_t>(nb) * d * 8) + align256(static_cast<size_t>(d) * 4));
  hipLaunchKernelGGL(colsum_kernel, dim3(nb), dim3(std::min(256, (d + 63) / 64 * 64)), 0, st, X, n, d, part);
  hipLaunchKernelGGL(colmean_kernel, dim3((d + 255) / 256), dim3(256), 0, st, part, nb, n, d, mean);
  hipLaunchKernelGGL(centre_kernel, dim3(nr), dim3(256), 0, st, X, n, d, dpad, mean, Xd, xnorm, amax);
  int rc = hip_status("cc_prepare_rows");
  if (rc) return rc;
  std::vector<float> am(static_cast<size_t>(nr));
  if (hipMemcpyAsync(am.data(), amax, sizeof(float) * nr, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    cc::set_error("cc_prepare_rows: reading max|X| failed");
    return CC_ERR_HIP;
  }
  float mx = 0.f;
  for (float v : am) mx = (std::isnan(v) || std::isnan(mx)) ? NAN : std::max(mx, v);
  const int e = scale_exponent(mx);
  if (e == INT32_MIN) {
    cc::set_error("cc_prepare_rows: X contains non-finite values");
    return CC_ERR_ARG;
  }
  *scale_exp = e;
  return cc_split_f16(Xd, n, dpad, e, Xhl, stream);
}

extern "C" size_t cc_kmeans_fit_workspace_bytes(int n, int d, int m, int nh, const int32_t* Ks, int nK,
                                                int n_init, int precision) {
  if (n <= 0 || d <= 0 || m <= 0 || m > n || nh <= 0 || !Ks || nK <= 0 || n_init <= 0 ||
      (precision != CC_KM_FAST && precision != CC_KM_F64))
    return 0;
  FitPlan P = make_plan(d, m, nh, Ks, nK, n_init, precision, n);
  if (P.cus <= 0) return 0;
  size_t engine = 0;
  if (precision == CC_KM_F64) {
    for (int k0 = 0; k0 < nK; k0 += 64) {
      const int nk = std::min(64, nK - k0);
      const int g = std::min(4 * P.cus, nh * nk);
      engine = std::max(engine, cc_kmeans_f64_workspace_bytes(m, d, Ks + k0, nk, g, nh));
    }
  } else if (P.dpad <= 128) {
    if (P.nU <= 0) return 0;
    const int g = std::min(P.cus, nh * P.nU);
    engine = cc_kmeans_workspace_bytes(m, P.dpad, P.units.data(), P.nU, P.seedmax, g);
  } else {
    const int per_call = std::max(1, CC_KM_PMAX / n_init);
    for (int k0 = 0; k0 < nK; k0 += per_call) {
      const int nk = std::min(per_call, nK - k0);
      engine = std::max(engine, cc_kmeans_wide_workspace_bytes(m, P.dpad, Ks + k0, nk, n_init, std::min(nh, 128)));
    }
  }
  if (engine == 0) return 0;
  return P.rows_bytes + P.tables_bytes + align256(engine);
}

extern "C" int cc_kmeans_fit(const void* X, int n, int d, const int32_t* idx_hm, int H, int m, int h_begin,
                             int h_end, const int32_t* Ks, int nK, int n_init, int max_iter, double tol_rel,
                             uint32_t seed, int precision, uint8_t* labels_nh, int ldl, void* inertia,
                             int32_t* n_iter, void* workspace, size_t ws_bytes, void* stream) {
  if (!X || !idx_hm || !Ks || !labels_nh || !workspace || n <= 0 || d <= 0 || m <= 0 || m > n || H <= 0 ||
      h_begin < 0 || h_end > H || h_end < h_begin || nK <= 0 || n_init <= 0 || max_iter <= 0 ||
      ldl < H || (precision != CC_KM_FAST && precision != CC_KM_F64)) {
    cc::set_error("cc_kmeans_fit: bad arguments");
    return CC_ERR_ARG;
  }
  for (int k = 0; k < nK; ++k)
    if (Ks[k] < 1 || Ks[k] > 127 || Ks[k] > m) {
      cc::set_error("cc_kmeans_fit: every K must lie in [1, min(127, m)]");
      return CC_ERR_ARG;
    }
  const int nh = h_end - h_begin;
  if (nh == 0) return CC_OK;
  FitPlan P = make_plan(d, m, nh, Ks, nK, n_init, precision, n);
  if (P.cus <= 0) {
    cc::set_error("cc_kmeans_fit: no HIP device");
    return CC_ERR_HIP;
  }
  if (precision == CC_KM_FAST && P.dpad <= 128 && P.nU <= 0) return P.nU;
  // reject an undersized workspace before anything is carved from it or copied into it: the
  // tables, plus the row image on the float32 path (the engine's own share is checked below)
  const size_t need_pre = P.tables_bytes + (precision == CC_KM_FAST ? P.rows_bytes : 0);
  if (ws_bytes < need_pre) {
    cc::set_error("cc_kmeans_fit: workspace too small");
    return CC_ERR_ARG;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  char* w = static_cast<char*>(workspace);
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    char* p = w + off;
    off += align256(bytes);
    return p;
  };
  // host tables -> device (pageable copies, ordered on the stream)
  std::vector<double> u(static_cast<size_t>(nK) * n_init * P.stride);
  std::vector<int32_t> pos(static_cast<size_t>(nK) * n_init);
  int rc = cc_kpp_tables(Ks, nK, n_init, seed, m, precision == CC_KM_F64, u.data(), P.stride, pos.data());
  if (rc) return rc;
  int32_t* units_d = reinterpret_cast<int32_t*>(carve(static_cast<size_t>(std::max(P.nU, 1)) * CC_KM_USTRIDE * 4));
  double* u_d = reinterpret_cast<double*>(carve(u.size() * 8));
  int32_t* pos_d = reinterpret_cast<int32_t*>(carve(pos.size() * 4));
  unsigned long long* stats = reinterpret_cast<unsigned long long*>(carve(128 * 8));
  if (hipMemcpyAsync(u_d, u.data(), u.size() * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(pos_d, pos.data(), pos.size() * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemsetAsync(stats, 0, 128 * 8, st) != hipSuccess ||
      (P.nU > 0 && hipMemcpyAsync(units_d, P.units.data(), static_cast<size_t>(P.nU) * CC_KM_USTRIDE * 4,
                                  hipMemcpyHostToDevice, st) != hipSuccess)) {
    cc::set_error("cc_kmeans_fit: table upload failed");
    return CC_ERR_HIP;
  }
  if (precision == CC_KM_F64) {
    if (off > ws_bytes) {
      cc::set_error("cc_kmeans_fit: workspace too small");
      return CC_ERR_ARG;
    }
    for (int k0 = 0; k0 < nK; k0 += 64) {
      const int nk = std::min(64, nK - k0);
      int g = std::min(4 * P.cus, nh * nk);
      while (g > 1 && off + align256(cc_kmeans_f64_workspace_bytes(m, d, Ks + k0, nk, g, nh)) > ws_bytes) g /= 2;
      const size_t eb = cc_kmeans_f64_workspace_bytes(m, d, Ks + k0, nk, g, nh);
      if (eb == 0 || off + eb > ws_bytes) {
        cc::set_error("cc_kmeans_fit: workspace too small");
        return CC_ERR_ARG;
      }
      // the (K, init) tables of this chunk: rows k0.. of u / pos (same stride)
      rc = cc_kmeans_f64(static_cast<const double*>(X), n, d, idx_hm, H, m, h_begin, h_end, Ks + k0, nk,
                         n_init, max_iter, tol_rel, u_d + static_cast<size_t>(k0) * n_init * P.stride,
                         P.stride, pos_d + k0 * n_init, labels_nh + static_cast<size_t>(k0) * n * ldl, ldl,
                         inertia ? static_cast<double*>(inertia) + static_cast<size_t>(k0) * H : nullptr,
                         n_iter ? n_iter + static_cast<size_t>(k0) * H : nullptr, w + off, ws_bytes - off, g,
                         stream);
      if (rc) return rc;
    }
    return CC_OK;
  }
  // float32 engines: the row image
  float* Xd = reinterpret_cast<float*>(carve(static_cast<size_t>(n) * P.dpad * 4));
  float* xnorm = reinterpret_cast<float*>(carve(static_cast<size_t>(n) * 4));
  uint16_t* Xhl = reinterpret_cast<uint16_t*>(carve(static_cast<size_t>(n) * 2 * P.dpad * 2));
  void* scratch = carve(prep_scratch_bytes(n, d));
  if (off > ws_bytes) {
    cc::set_error("cc_kmeans_fit: workspace too small");
    return CC_ERR_ARG;
  }
  int e = 0;
  rc = cc_prepare_rows(static_cast<const float*>(X), n, d, P.dpad, Xd, xnorm, Xhl, &e, scratch,
                       prep_scratch_bytes(n, d), stream);
  if (rc) return rc;
  if (P.dpad <= 128) {
    int g = std::min(P.cus, nh * P.nU);
    while (g > 1 && off + cc_kmeans_workspace_bytes(m, P.dpad, P.units.data(), P.nU, P.seedmax, g) > ws_bytes) g /= 2;
    const size_t eb = cc_kmeans_workspace_bytes(m, P.dpad, P.units.data(), P.nU, P.seedmax, g);
    if (off + eb > ws_bytes) {
      cc::set_error("cc_kmeans_fit: workspace too small");
      return CC_ERR_ARG;
    }
    return cc_kmeans_batched(Xd, Xhl, xnorm, n, d, P.dpad, e, idx_hm, H, m, h_begin, h_end, units_d,
                             P.units.data(), P.nU, n_init, max_iter, tol_rel, u_d, P.stride, pos_d, labels_nh,
                             ldl, static_cast<float*>(inertia), n_iter, stats, w + off, ws_bytes - off, g,
                             P.seedmax, stream);
  }
  // wide rows: rounds over batches of resamples sized to the workspace, <= CC_KM_PMAX problems
  // per call
  const int per_call = std::max(1, CC_KM_PMAX / n_init);
  for (int k0 = 0; k0 < nK; k0 += per_call) {
    const int nk = std::min(per_call, nK - k0);
    const size_t w1 = cc_kmeans_wide_workspace_bytes(m, P.dpad, Ks + k0, nk, n_init, 1);
    const size_t w2 = cc_kmeans_wide_workspace_bytes(m, P.dpad, Ks + k0, nk, n_init, 2);
    if (w1 == 0 || off + w1 > ws_bytes) {
      cc::set_error("cc_kmeans_fit: workspace too small");
      return CC_ERR_ARG;
    }
    const size_t per = w2 - w1;
    const long long cap = std::max<long long>(1, std::min<long long>(nh, (ws_bytes - off - (w1 - per)) / per));
    const long long nb = (nh + cap - 1) / cap;
    const int batch = static_cast<int>((nh + nb - 1) / nb);
    rc = cc_kmeans_wide(Xd, Xhl, xnorm, n, d, P.dpad, e, idx_hm, H, m, h_begin, h_end, Ks + k0, nk, n_init,
                        max_iter, tol_rel, u_d + static_cast<size_t>(k0) * n_init * P.stride, P.stride,
                        pos_d + k0 * n_init, labels_nh + static_cast<size_t>(k0) * n * ldl, ldl,
                        inertia ? static_cast<float*>(inertia) + static_cast<size_t>(k0) * H : nullptr,
                        n_iter ? n_iter + static_cast<size_t>(k0) * H : nullptr, stats, w + off, ws_bytes - off,
                        batch, stream);
    if (rc) return rc;
  }
  return CC_OK;
}
