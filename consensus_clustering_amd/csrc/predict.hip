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

// ---- Agglomerative linkage on the device: scipy.cluster.hierarchy.nn_chain
// (scipy/cluster/_hierarchy.pyx, the algorithm linkage() runs for 'complete', 'average' and
// 'weighted'), the tree AgglomerativeClustering cuts (CC.py:306-312 -> sklearn linkage_tree ->
// hierarchy.linkage).  The same sequence of decisions as scipy's loop: the chain grows from the
// first live cluster; a step's nearest neighbour of the chain top x is the first index (scan
// order) of the minimum over live i != x of D[x, i], taken only when strictly below D[x, prev]
// (so the previous chain element wins ties); mutual neighbours merge (x < y kept as in
// fastcluster), the merged cluster takes y's row and column, x dies; the Lance-Williams update is
// the float64 expression of _hierarchy_distance_update.pxi with no contraction.  One workgroup
// runs the whole chain (every step is a scan or an update over n entries; the full symmetric
// n x n float64 matrix stays in HBM: 20 GB at n = 50k).  Z is written in merge order, unsorted;
// the host sorts it by distance (stable) and relabels, as linkage() does after nn_chain.
//
// Round 4: the live set is a bitmask in LDS (n / 8 bytes), and every row pass issues its loads
// in batches of NB per thread before any compare (branch-free: dead and diagonal entries read
// as +inf), so a scan is a few HBM round trips instead of one per element and thread (8.3 s ->
// see DESIGN.md K7 at n = 50k).
//
// Single linkage: sklearn's own path (linkage_tree -> _hierarchical_fast.mst_linkage_core, Prim's
// MST-LINKAGE-CORE, for a non-precomputed metric such as the reference's 'manhattan'): from node 0,
// each step folds the current node's row into the running minimum distance of every node not in
// the tree (strict <) and takes the first node of the smallest, as mst_kernel does with D's rows
// (the cityblock values of DistanceMetric64 are cc_manhattan's, same terms and order).
namespace {

constexpr int LT = 1024;  // threads of the linkage workgroup
constexpr int NB = 8;     // loads per thread in flight per row pass

__device__ __forceinline__ double lw_update(int method, double dxi, double dyi, int nx, int ny) {
#pragma clang fp contract(off)  // scipy's products and sum rounded separately (no FMA)
  if (method == CC_LINK_COMPLETE) return dxi > dyi ? dxi : dyi;  // fmax(d_xi, d_yi)
  if (method == CC_LINK_WEIGHTED) return 0.5 * (dxi + dyi);
  // average: (size_x * d_xi + size_y * d_yi) / (size_x + size_y)
  const double a = static_cast<double>(nx) * dxi;
  const double b = static_cast<double>(ny) * dyi;
  return (a + b) / static_cast<double>(nx + ny);
}

// Block minimum of (v, i): the lower value, ties to the lower index.
__device__ __forceinline__ void block_argmin(double& v, int& i, double* rv, int* ri) {
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(v, o);
    const int oi = __shfl_xor(i, o);
    if (ov < v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    rv[w] = v;
    ri[w] = i;
  }
  __syncthreads();
  v = rv[0];
  i = ri[0];
  for (int k = 1; k < LT / 64; ++k)
    if (rv[k] < v || (rv[k] == v && ri[k] < i)) {
      v = rv[k];
      i = ri[k];
    }
}

__device__ __forceinline__ bool live(const unsigned* mask, int i) { return (mask[i >> 5] >> (i & 31)) & 1u; }

// First minimum over live i != x of row[i]: thread tid visits i = base + tid + LT u in increasing
// order, NB loads in flight per batch.
__device__ __forceinline__ void row_argmin(const double* row, int n, int x, const unsigned* mask, double& v,
                                           int& bi) {
  constexpr double INF = __builtin_huge_val();
  const int tid = threadIdx.x;
  v = INF;
  bi = 0x7fffffff;
  for (int base = 0; base < n; base += LT * NB) {
    double d[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int i = base + tid + LT * u;
      d[u] = i < n ? row[i] : INF;
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int i = base + tid + LT * u;
      const bool ok = i < n && i != x && live(mask, i);
      if (ok && d[u] < v) {
        v = d[u];
        bi = i;
      }
    }
  }
}

__global__ __launch_bounds__(LT) void nnchain_kernel(double* __restrict__ D, int n, int method,
                                                     double* __restrict__ Z, int* __restrict__ size,
                                                     int* __restrict__ chain) {
  extern __shared__ unsigned mask[];  // live clusters, one bit each
  __shared__ double rv[LT / 64];
  __shared__ int ri[LT / 64];
  const int tid = threadIdx.x;
  const size_t nn = static_cast<size_t>(n);
  const int nw = (n + 31) >> 5;
  constexpr double INF = __builtin_huge_val();
  for (int i = tid; i < n; i += LT) size[i] = 1;
  for (int w = tid; w < nw; w += LT) mask[w] = (w < nw - 1 || (n & 31) == 0) ? 0xFFFFFFFFu : ((1u << (n & 31)) - 1u);
  __syncthreads();
  int len = 0;  // uniform: every thread runs the same control flow
  for (int k = 0; k < n - 1; ++k) {
    if (len == 0) {  // the first live cluster
      double v = INF;
      int i0 = 0x7fffffff;
      for (int w = tid; w < nw; w += LT)
        if (mask[w]) {
          i0 = 32 * w + __builtin_ctz(mask[w]);
          v = 0.0;
          break;
        }
      block_argmin(v, i0, rv, ri);
      if (tid == 0) chain[0] = i0;
      __syncthreads();
      len = 1;
    }
    int x, y;
    double cur;
    for (;;) {
      x = chain[len - 1];
      y = -1;
      cur = INF;
      if (len > 1) {
        y = chain[len - 2];
        cur = D[x * nn + y];
      }
      double v;
      int bi;
      row_argmin(D + x * nn, n, x, mask, v, bi);
      block_argmin(v, bi, rv, ri);
      if (v < cur) {
        cur = v;
        y = bi;
      }
      if (len > 1 && y == chain[len - 2]) break;
      __syncthreads();  // every thread has read chain[len - 2] before it may be overwritten
      if (tid == 0) chain[len] = y;
      __syncthreads();
      ++len;
    }
    len -= 2;
    if (x > y) {
      const int t = x;
      x = y;
      y = t;
    }
    const int nx = size[x], ny = size[y];
    __syncthreads();  // every thread has read the sizes
    if (tid == 0) {
      Z[4 * static_cast<size_t>(k) + 0] = x;
      Z[4 * static_cast<size_t>(k) + 1] = y;
      Z[4 * static_cast<size_t>(k) + 2] = cur;
      Z[4 * static_cast<size_t>(k) + 3] = nx + ny;
      size[x] = 0;
      size[y] = nx + ny;
      mask[x >> 5] &= ~(1u << (x & 31));
    }
    __syncthreads();
    const double* rx = D + x * nn;
    double* ry = D + y * nn;
    for (int base = 0; base < n; base += LT * NB) {
      double dx[NB], dy[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int i = base + tid + LT * u;
        dx[u] = i < n ? rx[i] : 0.0;
        dy[u] = i < n ? ry[i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int i = base + tid + LT * u;
        if (i < n && i != y && live(mask, i)) {
          const double nd = lw_update(method, dx[u], dy[u], nx, ny);
          ry[i] = nd;
          D[i * nn + y] = nd;
        }
      }
    }
    __syncthreads();
  }
}

// sklearn mst_linkage_core (Prim) over the rows of the symmetric D: out [n-1][3] = (current
// node, new node, distance) per step; cur: the running minimum distance of every node ([n]
// float64 workspace).
__global__ __launch_bounds__(LT) void mst_kernel(const double* __restrict__ D, int n, double* __restrict__ out,
                                                 double* __restrict__ cur) {
  extern __shared__ unsigned tree[];  // in_tree, one bit per node
  __shared__ double rv[LT / 64];
  __shared__ int ri[LT / 64];
  const int tid = threadIdx.x;
  const int nw = (n + 31) >> 5;
  constexpr double INF = __builtin_huge_val();
  for (int i = tid; i < n; i += LT) cur[i] = INF;
  for (int w = tid; w < nw; w += LT) tree[w] = 0u;
  __syncthreads();
  int node = 0;
  for (int k = 0; k < n - 1; ++k) {
    if (tid == 0) tree[node >> 5] |= 1u << (node & 31);
    __syncthreads();
    const double* row = D + static_cast<size_t>(node) * n;
    double v = INF;
    int bi = 0x7fffffff;
    for (int base = 0; base < n; base += LT * NB) {
      double l[NB], r[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int j = base + tid + LT * u;
        l[u] = j < n ? row[j] : INF;
        r[u] = j < n ? cur[j] : INF;
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int j = base + tid + LT * u;
        if (j < n && !((tree[j >> 5] >> (j & 31)) & 1u)) {
          double c = r[u];
          if (l[u] < c) {  // left_value < right_value
            c = l[u];
            cur[j] = c;
          }
          if (c < v) {  // current_distances[j] < new_distance: the first minimum
            v = c;
            bi = j;
          }
        }
      }
    }
    block_argmin(v, bi, rv, ri);
    const int nxt = (v < INF) ? bi : 0;  // sklearn's new_node starts at 0
    if (tid == 0) {
      out[3 * static_cast<size_t>(k) + 0] = node;
      out[3 * static_cast<size_t>(k) + 1] = nxt;
      out[3 * static_cast<size_t>(k) + 2] = v;
    }
    node = nxt;
    __syncthreads();  // cur[] of this step is written before the next step reads it
  }
}

size_t mask_bytes(int n) { return static_cast<size_t>((n + 31) >> 5) * sizeof(unsigned); }

// the dynamic LDS of the bitmask (up to the 160 KiB of a CU, less the static part)
constexpr size_t MASK_LDS_MAX = 160 * 1024 - 1024;

}  // namespace

extern "C" size_t cc_linkage_workspace_bytes(int n) {
  return n > 0 ? 2 * static_cast<size_t>(n) * sizeof(int) : 0;
}

extern "C" int cc_linkage_nnchain(double* D, int n, int method, double* Z, void* workspace, size_t ws_bytes,
                                  void* stream) {
  if (!D || !Z || n < 2 || !workspace || ws_bytes < cc_linkage_workspace_bytes(n) ||
      (method != CC_LINK_AVERAGE && method != CC_LINK_COMPLETE && method != CC_LINK_WEIGHTED) ||
      mask_bytes(n) > MASK_LDS_MAX) {
    cc::set_error("cc_linkage_nnchain: bad arguments");
    return CC_ERR_ARG;
  }
  int* size = static_cast<int*>(workspace);
  hipLaunchKernelGGL(nnchain_kernel, dim3(1), dim3(LT), mask_bytes(n), static_cast<hipStream_t>(stream), D, n,
                     method, Z, size, size + n);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_linkage_nnchain: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}

extern "C" size_t cc_linkage_mst_workspace_bytes(int n) { return n > 0 ? static_cast<size_t>(n) * sizeof(double) : 0; }

extern "C" int cc_linkage_mst(const double* D, int n, double* out, void* workspace, size_t ws_bytes, void* stream) {
  if (!D || !out || n < 2 || !workspace || ws_bytes < cc_linkage_mst_workspace_bytes(n) ||
      mask_bytes(n) > MASK_LDS_MAX) {
    cc::set_error("cc_linkage_mst: bad arguments");
    return CC_ERR_ARG;
  }
  hipLaunchKernelGGL(mst_kernel, dim3(1), dim3(LT), mask_bytes(n), static_cast<hipStream_t>(stream), D, n, out,
                     static_cast<double*>(workspace));
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_linkage_mst: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}
