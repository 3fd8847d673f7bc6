// Manhattan distances between the rows of the consensus matrix, for the consensus labels.
//
// The reference's consensus labels (consensus_clustering_parallelised.py:292-314,
// `_get_consensus_labels`) run AgglomerativeClustering(affinity='manhattan') on the rows of C;
// sklearn hands that to scipy.cluster.hierarchy.linkage(C, metric='cityblock'), whose pdist
// sums |u_k - v_k| over k in float64, sequentially (scipy/spatial/src/distance_impl.h).  This
// kernel produces the same float64 values (same terms, same order), so the host linkage over
// them is the reference's linkage.
//
// Tiling: 64 x 64 output tiles of the upper triangle (the lower one is mirrored), 256 threads
// as 16 x 16, each thread 4 x 4 pairs; 32-wide k slabs of both row blocks staged in LDS as
// float32, [k][row] so that a thread reads its 4 rows and 4 columns with two 16-B reads.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "ccmi_internal.h"

namespace {

constexpr int TB = 64;   // output tile edge
constexpr int KS = 32;   // k slab

__global__ __launch_bounds__(256) void manhattan_kernel(const float* __restrict__ C, int n, int d,
                                                        double* __restrict__ D) {
  // blockIdx.x enumerates the upper-triangle tiles row-major
  const int nb = (n + TB - 1) / TB;
  int t = static_cast<int>(blockIdx.x), bi = 0;
  while (t >= nb - bi) {
    t -= nb - bi;
    ++bi;
  }
  const int bj = bi + t;
  __shared__ __attribute__((aligned(16))) float sa[KS][TB];
  __shared__ __attribute__((aligned(16))) float sb[KS][TB];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int i0 = bi * TB, j0 = bj * TB;
  double acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = 0.0;
  for (int k0 = 0; k0 < d; k0 += KS) {
    // stage: 64 rows x 32 k per side, one element per thread and pass (coalesced along k)
    for (int e = tid; e < TB * KS; e += 256) {
      const int r = e / KS, k = e % KS;
      const int gi = i0 + r, gj = j0 + r, gk = k0 + k;
      sa[k][r] = (gi < n && gk < d) ? C[static_cast<int64_t>(gi) * d + gk] : 0.f;
      sb[k][r] = (gj < n && gk < d) ? C[static_cast<int64_t>(gj) * d + gk] : 0.f;
    }
    __syncthreads();
    const int kn = min(KS, d - k0);
    for (int k = 0; k < kn; ++k) {
      const float4 a4 = *reinterpret_cast<const float4*>(&sa[k][4 * ty]);
      const float4 b4 = *reinterpret_cast<const float4*>(&sb[k][4 * tx]);
      const double a[4] = {a4.x, a4.y, a4.z, a4.w};
      const double b[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] += fabs(a[r] - b[c]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int i = i0 + 4 * ty + r, j = j0 + 4 * tx + c;
      if (i < n && j < n) {
        D[static_cast<int64_t>(i) * n + j] = acc[r][c];
        D[static_cast<int64_t>(j) * n + i] = acc[r][c];
      }
    }
}

}  // namespace

extern "C" int cc_manhattan(const float* C, int n, int d, double* D, void* stream) {
  if (!C || !D || n <= 0 || d <= 0) {
    cc::set_error("cc_manhattan: bad arguments");
    return CC_ERR_ARG;
  }
  const int64_t nb = (n + TB - 1) / TB;
  const int64_t tiles = nb * (nb + 1) / 2;
  if (tiles > 0x7fffffff) {
    cc::set_error("cc_manhattan: n too large");
    return CC_ERR_ARG;
  }
  hipLaunchKernelGGL(manhattan_kernel, dim3(static_cast<unsigned>(tiles)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), C, n, d, D);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_manhattan: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}
