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
#include <tuple>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "ccmi_internal.h"

namespace {

// 128 x 128 output tiles of the upper triangle, 256 threads as 16 x 16, each thread an 8 x 8
// block of float64 accumulators (rows 8 ty + r, columns 8 tx + c); k slabs of 16 staged in LDS
// as float (two float4 reads per side and k serve 64 accumulators), the next slab's global loads
// in flight under the current slab's arithmetic.  Every output is still one sequential sum over
// k in increasing order, so the values are those of the scalar loop.
constexpr int TB = 128;  // output tile edge
constexpr int KS = 16;   // k slab
constexpr int RB = 8;    // accumulators per thread and side

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
  __shared__ __attribute__((aligned(16))) double sa[KS][TB];  // staged as float64: no conversions in the k loop
  __shared__ __attribute__((aligned(16))) double sb[KS][TB];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int i0 = bi * TB, j0 = bj * TB;
  double acc[RB][RB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < RB; ++c) acc[r][c] = 0.0;
  // staging: thread tid loads 4 consecutive k of row (tid >> 2) and of row (tid >> 2) + 64, per side
  const int sr = tid >> 2, sk = 4 * (tid & 3);
  float4 ga[2], gb[2];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = sr + 64 * h, gk = k0 + sk;
      const int gi = i0 + r, gj = j0 + r;
      float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
      if (gk + 3 < d) {
        if (gi < n) va = *reinterpret_cast<const float4*>(C + static_cast<int64_t>(gi) * d + gk);
        if (gj < n) vb = *reinterpret_cast<const float4*>(C + static_cast<int64_t>(gj) * d + gk);
      } else {  // the tail of k (or a row of d not a multiple of 4: scalar, unaligned-safe)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float a = (gi < n && gk + q < d) ? C[static_cast<int64_t>(gi) * d + gk + q] : 0.f;
          const float b = (gj < n && gk + q < d) ? C[static_cast<int64_t>(gj) * d + gk + q] : 0.f;
          (&va.x)[q] = a;
          (&vb.x)[q] = b;
        }
      }
      ga[h] = va;
      gb[h] = vb;
    }
  };
  const bool vec = (d & 3) == 0;  // 16-B aligned rows
  auto load_any = [&](int k0) __attribute__((always_inline)) {
    if (vec) {
      load(k0);
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = sr + 64 * h, gk = k0 + sk;
        const int gi = i0 + r, gj = j0 + r;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          (&ga[h].x)[q] = (gi < n && gk + q < d) ? C[static_cast<int64_t>(gi) * d + gk + q] : 0.f;
          (&gb[h].x)[q] = (gj < n && gk + q < d) ? C[static_cast<int64_t>(gj) * d + gk + q] : 0.f;
        }
      }
    }
  };
  load_any(0);
  for (int k0 = 0; k0 < d; k0 += KS) {
    __syncthreads();  // the previous slab's reads are done
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sa[sk + q][sr + 64 * h] = static_cast<double>((&ga[h].x)[q]);
        sb[sk + q][sr + 64 * h] = static_cast<double>((&gb[h].x)[q]);
      }
    __syncthreads();
    if (k0 + KS < d) load_any(k0 + KS);  // in flight under this slab
    const int kn = min(KS, d - k0);
    for (int k = 0; k < kn; ++k) {
      double a[RB], b[RB];
#pragma unroll
      for (int q = 0; q < RB; q += 2) {
        const double2 av = *reinterpret_cast<const double2*>(&sa[k][RB * ty + q]);
        const double2 bv = *reinterpret_cast<const double2*>(&sb[k][RB * tx + q]);
        a[q] = av.x;
        a[q + 1] = av.y;
        b[q] = bv.x;
        b[q + 1] = bv.y;
      }
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int c = 0; c < RB; ++c) acc[r][c] += fabs(a[r] - b[c]);
    }
  }
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < RB; ++c) {
      const int i = i0 + RB * ty + r, j = j0 + RB * tx + c;
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

// ---- Grid forms (round 4): the same decisions on G co-resident workgroups.  Workgroup g owns
// the index slice [n g / G, n (g + 1) / G): it scans its slice of a row, updates its slice of a
// merged row and its slice's entries of the merged column, and keeps the running minima of its
// slice (Prim).  Each workgroup keeps a replica of the whole live / in-tree bitmask in LDS and
// private copies of the chain and the cluster sizes, and every workgroup takes every decision
// itself from the same data, so the control flow is identical on all of them.  Per step the
// slices' (minimum, first index) pairs go through a grid barrier and every workgroup reduces
// them in slice order (strict <: the lowest index wins ties, as the one-workgroup scan does).
// nn_chain needs a second barrier after each Lance-Williams update (a later scan of another
// slice reads the merged column).  The barrier is a counter and a generation word in the
// workspace, with agent-scope release / acquire fences (buffer_wbl2 / buffer_inv on gfx950, so
// the D writes of one XCD are seen by the others); a workgroup that waits for more than ~2^27
// polls sets an error word and every workgroup leaves (cc_linkage_check reports it).  The
// workgroups are made co-resident, not assumed so: G is capped by the occupancy query of the
// kernel at its dynamic LDS, and the grid forms are started with hipLaunchCooperativeKernel,
// which the runtime starts only when all G workgroups can run at once; if it refuses, the
// one-workgroup kernel runs instead (nothing has been written by then).
constexpr int LG = 256;    // threads of a grid-form workgroup
constexpr int GMAX = 128;  // workgroups of a grid form (all co-resident: one per CU at most)
constexpr int NBG = 8;     // loads per thread in flight per slice pass
constexpr size_t GHDR = 256;  // workspace header: barrier count, generation, error

struct GridWs {
  unsigned* bar;    // [0] arrivals, [1] generation, [2] error
  double* pv;       // [2][GMAX] slice minima (double-buffered by barrier parity)
  int* pi;          // [2][GMAX] their indices
};

__device__ __forceinline__ GridWs grid_ws(void* ws) {
  char* b = static_cast<char*>(ws);
  GridWs g;
  g.bar = reinterpret_cast<unsigned*>(b);
  g.pv = reinterpret_cast<double*>(b + GHDR);
  g.pi = reinterpret_cast<int*>(b + GHDR + 2 * GMAX * sizeof(double));
  return g;
}
constexpr size_t grid_ws_bytes() { return GHDR + 2 * GMAX * (sizeof(double) + sizeof(int)); }

// Grid barrier.  FULL: every thread's global writes are complete and written back before the
// arrival and every thread reads after the acquire (agent-scope fences: the D updates of
// nn_chain cross XCDs).  Light (FULL = false): only the slice minima cross, and they are written
// and read with agent-scope atomics, so the arrival only has to follow their completion (no
// cache write-back or invalidation).  Returns false when the wait timed out or another workgroup
// reported an error (the caller returns at once).
template <bool FULL>
__device__ bool grid_sync(const GridWs& gw, unsigned& gen) {
  __shared__ int s_ok;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's stores and atomics have completed
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    const unsigned want = gen + 1;
    if constexpr (FULL) __threadfence();  // release (writes back this XCD's L2)
    // arrival and generation at agent scope (the slice minima of the light form are agent-scope
    // atomics; these order them against the arrival and the generation word).  The arrival is
    // acquire-release: the last arriver's fetch_add reads every earlier arrival (a release
    // sequence on bar[0]), so its generation store below carries their writes to the waiters.
    if (__hip_atomic_fetch_add(&gw.bar[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(&gw.bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // the reset is done before the release
      if constexpr (FULL) __threadfence();
      __hip_atomic_store(&gw.bar[1], want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned polls = 0;
      while (__hip_atomic_load(&gw.bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
        __builtin_amdgcn_s_sleep(2);
        if ((++polls & 1023u) == 0) {
          if (__hip_atomic_load(&gw.bar[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || polls > (1u << 27)) {
            __hip_atomic_store(&gw.bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = 0;
            break;
          }
        }
      }
      // acquire: nothing after this reads before the generation word was seen
      if (ok) (void)__hip_atomic_load(&gw.bar[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (FULL) __threadfence();  // acquire (invalidates this CU's L1 and this XCD's L2)
    s_ok = ok;
  }
  __syncthreads();
  ++gen;
  return s_ok != 0;
}

// Block minimum of (v, i) over LG threads: the lower value, ties to the lower index.
__device__ __forceinline__ void block_argmin_g(double& v, int& i, double* rv, int* ri) {
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
  for (int k = 1; k < LG / 64; ++k)
    if (rv[k] < v || (rv[k] == v && ri[k] < i)) {
      v = rv[k];
      i = ri[k];
    }
  __syncthreads();  // rv / ri may be rewritten by the next call
}

// Publish this workgroup's slice minimum, pass the barrier, and reduce every slice's in slice
// order (the same result on every workgroup).  Returns false on a barrier error.
__device__ bool grid_argmin(const GridWs& gw, unsigned& gen, double& v, int& i, double* rv, int* ri) {
  const int par = gen & 1;
  if (threadIdx.x == 0) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(gw.pv) + par * GMAX + blockIdx.x,
                       static_cast<unsigned long long>(__double_as_longlong(v)), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gw.pi + par * GMAX + blockIdx.x, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!grid_sync<false>(gw, gen)) return false;
  constexpr double INF = __builtin_huge_val();
  v = INF;
  i = 0x7fffffff;
  if (threadIdx.x < static_cast<int>(gridDim.x)) {  // slice order = index order
    v = __longlong_as_double(static_cast<long long>(__hip_atomic_load(
        reinterpret_cast<unsigned long long*>(gw.pv) + par * GMAX + threadIdx.x, __ATOMIC_RELAXED,
        __HIP_MEMORY_SCOPE_AGENT)));
    i = __hip_atomic_load(gw.pi + par * GMAX + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  block_argmin_g(v, i, rv, ri);
  return true;
}

__global__ __launch_bounds__(LG) void nnchain_grid_kernel(double* __restrict__ D, int n, int method,
                                                          double* __restrict__ Z, int* __restrict__ sizes,
                                                          int* __restrict__ chains, void* ws) {
  extern __shared__ unsigned mask[];  // live clusters, one bit each (a replica per workgroup)
  __shared__ double rv[LG / 64];
  __shared__ int ri[LG / 64];
  __shared__ int s_i0;
  const GridWs gw = grid_ws(ws);
  const int tid = threadIdx.x, G = gridDim.x, g = blockIdx.x;
  const int j0 = static_cast<int>(static_cast<int64_t>(n) * g / G);
  const int j1 = static_cast<int>(static_cast<int64_t>(n) * (g + 1) / G);
  const size_t nn = static_cast<size_t>(n);
  int* size = sizes + static_cast<size_t>(g) * nn;   // private copies: no sharing
  int* chain = chains + static_cast<size_t>(g) * nn;
  const int nw = (n + 31) >> 5;
  constexpr double INF = __builtin_huge_val();
  for (int i = tid; i < n; i += LG) size[i] = 1;
  for (int w = tid; w < nw; w += LG) mask[w] = (w < nw - 1 || (n & 31) == 0) ? 0xFFFFFFFFu : ((1u << (n & 31)) - 1u);
  __syncthreads();
  unsigned gen = 0;
  int len = 0;
  for (int k = 0; k < n - 1; ++k) {
    if (len == 0) {  // the first live cluster (from the replicated mask)
      double v = INF;
      int i0 = 0x7fffffff;
      for (int w = tid; w < nw; w += LG)
        if (mask[w]) {
          i0 = 32 * w + __builtin_ctz(mask[w]);
          v = 0.0;
          break;
        }
      block_argmin_g(v, i0, rv, ri);
      if (tid == 0) s_i0 = i0;
      __syncthreads();
      if (tid == 0) chain[0] = s_i0;
      len = 1;
    }
    int x, y;
    double cur;
    for (;;) {
      __syncthreads();  // chain[] writes of thread 0 are visible to the workgroup
      x = chain[len - 1];
      y = -1;
      cur = INF;
      if (len > 1) {
        y = chain[len - 2];
        cur = D[x * nn + y];
      }
      double v = INF;
      int bi = 0x7fffffff;
      const double* row = D + x * nn;
      for (int base = j0; base < j1; base += LG * NBG) {
        double d[NBG];
#pragma unroll
        for (int u = 0; u < NBG; ++u) {
          const int i = base + tid + LG * u;
          d[u] = i < j1 ? row[i] : INF;
        }
#pragma unroll
        for (int u = 0; u < NBG; ++u) {
          const int i = base + tid + LG * u;
          if (i < j1 && i != x && live(mask, i) && d[u] < v) {
            v = d[u];
            bi = i;
          }
        }
      }
      block_argmin_g(v, bi, rv, ri);
      if (!grid_argmin(gw, gen, v, bi, rv, ri)) return;
      if (v < cur) {
        cur = v;
        y = bi;
      }
      if (len > 1 && y == chain[len - 2]) break;
      __syncthreads();  // every thread has read chain[len - 2]
      if (tid == 0) chain[len] = y;
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
      if (g == 0) {
        Z[4 * static_cast<size_t>(k) + 0] = x;
        Z[4 * static_cast<size_t>(k) + 1] = y;
        Z[4 * static_cast<size_t>(k) + 2] = cur;
        Z[4 * static_cast<size_t>(k) + 3] = nx + ny;
      }
      size[x] = 0;
      size[y] = nx + ny;
      mask[x >> 5] &= ~(1u << (x & 31));
    }
    __syncthreads();
    const double* rx = D + x * nn;
    double* ry = D + y * nn;
    for (int base = j0; base < j1; base += LG * NBG) {
      double dx[NBG], dy[NBG];
#pragma unroll
      for (int u = 0; u < NBG; ++u) {
        const int i = base + tid + LG * u;
        dx[u] = i < j1 ? rx[i] : 0.0;
        dy[u] = i < j1 ? ry[i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < NBG; ++u) {
        const int i = base + tid + LG * u;
        if (i < j1 && i != y && live(mask, i)) {
          const double nd = lw_update(method, dx[u], dy[u], nx, ny);
          ry[i] = nd;
          D[i * nn + y] = nd;
        }
      }
    }
    if (!grid_sync<true>(gw, gen)) return;  // the merged row and column before any later scan
  }
}

// sklearn mst_linkage_core on G workgroups: each keeps the running minima of its slice.
__global__ __launch_bounds__(LG) void mst_grid_kernel(const double* __restrict__ D, int n, double* __restrict__ out,
                                                      double* __restrict__ cur, void* ws) {
  extern __shared__ unsigned tree[];  // in_tree, one bit per node (a replica per workgroup)
  __shared__ double rv[LG / 64];
  __shared__ int ri[LG / 64];
  const GridWs gw = grid_ws(ws);
  const int tid = threadIdx.x, G = gridDim.x, g = blockIdx.x;
  const int j0 = static_cast<int>(static_cast<int64_t>(n) * g / G);
  const int j1 = static_cast<int>(static_cast<int64_t>(n) * (g + 1) / G);
  const int nw = (n + 31) >> 5;
  constexpr double INF = __builtin_huge_val();
  for (int i = j0 + tid; i < j1; i += LG) cur[i] = INF;
  for (int w = tid; w < nw; w += LG) tree[w] = 0u;
  __syncthreads();
  unsigned gen = 0;
  int node = 0;
  for (int k = 0; k < n - 1; ++k) {
    if (tid == 0) tree[node >> 5] |= 1u << (node & 31);
    __syncthreads();
    const double* row = D + static_cast<size_t>(node) * n;
    double v = INF;
    int bi = 0x7fffffff;
    for (int base = j0; base < j1; base += LG * NBG) {
      double l[NBG], r[NBG];
#pragma unroll
      for (int u = 0; u < NBG; ++u) {
        const int j = base + tid + LG * u;
        l[u] = j < j1 ? row[j] : INF;
        r[u] = j < j1 ? cur[j] : INF;
      }
#pragma unroll
      for (int u = 0; u < NBG; ++u) {
        const int j = base + tid + LG * u;
        if (j < j1 && !((tree[j >> 5] >> (j & 31)) & 1u)) {
          double c = r[u];
          if (l[u] < c) {  // left_value < right_value
            c = l[u];
            cur[j] = c;
          }
          if (c < v) {  // the first minimum
            v = c;
            bi = j;
          }
        }
      }
    }
    block_argmin_g(v, bi, rv, ri);
    if (!grid_argmin(gw, gen, v, bi, rv, ri)) return;
    const int nxt = (v < INF) ? bi : 0;  // sklearn's new_node starts at 0
    if (g == 0 && tid == 0) {
      out[3 * static_cast<size_t>(k) + 0] = node;
      out[3 * static_cast<size_t>(k) + 1] = nxt;
      out[3 * static_cast<size_t>(k) + 2] = v;
    }
    node = nxt;
  }
}

size_t mask_bytes(int n) { return static_cast<size_t>((n + 31) >> 5) * sizeof(unsigned); }

// the dynamic LDS of the bitmask (up to the 160 KiB of a CU, less the static part)
constexpr size_t MASK_LDS_MAX = 160 * 1024 - 1024;

// Workgroups of the grid forms for n (CCMI_LINK_G overrides; 0 = the one-workgroup kernels):
// about 1536 entries per slice (six loads per thread), at most GMAX and at most what the kernel's
// occupancy at its dynamic LDS keeps resident on all CUs at once.
template <typename Kern>
int link_groups(int n, Kern kernel) {
  const char* e = std::getenv("CCMI_LINK_G");
  int cus = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 1;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kernel), LG,
                                                   mask_bytes(n)) != hipSuccess)
    per_cu = 0;
  (void)hipGetLastError();
  const int cap = std::min(GMAX, per_cu * cus);
  if (cap <= 0) return 0;
  if (e && e[0]) return std::min(std::max(0, std::atoi(e)), cap);
  return std::max(1, std::min(cap, n / 1536));
}

// Start a grid form cooperatively (all G workgroups co-resident, or the launch fails); without
// cooperative-launch support a plain launch of the occupancy-capped G.
template <typename... KArgs, typename... Args>
hipError_t launch_grid(void (*kernel)(KArgs...), int G, size_t lds, hipStream_t st, Args... args) {
  int dev = 0, coop = 0;
  if (hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev) == hipSuccess && coop) {
    std::tuple<KArgs...> a(args...);  // the kernel's own parameter types
    void* argv[sizeof...(KArgs)];
    std::apply([&argv](auto&... x) {
      int k = 0;
      ((argv[k++] = static_cast<void*>(&x)), ...);
    }, a);
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(kernel), dim3(G), dim3(LG), argv,
                                      static_cast<unsigned>(lds), st);
  }
  hipLaunchKernelGGL(kernel, dim3(G), dim3(LG), lds, st, static_cast<KArgs>(args)...);
  return hipGetLastError();
}

// Both forms: the barrier header (zeroed at every launch, so cc_linkage_check also reads a
// one-workgroup run's as clean), then the sizes and chains ([G][n] each, or [n] at G = 0) or the
// running minima.
size_t nnchain_ws(int n, int G) {
  return grid_ws_bytes() + 2 * static_cast<size_t>(G > 0 ? G : 1) * static_cast<size_t>(n) * sizeof(int);
}
size_t mst_ws(int n, int) { return grid_ws_bytes() + static_cast<size_t>(n) * sizeof(double); }

}  // namespace

extern "C" size_t cc_linkage_workspace_bytes(int n) {
  return n > 0 ? nnchain_ws(n, link_groups(n, nnchain_grid_kernel)) : 0;
}

extern "C" int cc_linkage_nnchain(double* D, int n, int method, double* Z, void* workspace, size_t ws_bytes,
                                  void* stream) {
  const int G = n > 0 ? link_groups(n, nnchain_grid_kernel) : 0;
  if (!D || !Z || n < 2 || !workspace || ws_bytes < nnchain_ws(n, G) ||
      (method != CC_LINK_AVERAGE && method != CC_LINK_COMPLETE && method != CC_LINK_WEIGHTED) ||
      mask_bytes(n) > MASK_LDS_MAX) {
    cc::set_error("cc_linkage_nnchain: bad arguments");
    return CC_ERR_ARG;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(workspace, 0, GHDR, st);
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_linkage_nnchain: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  int* sizes = reinterpret_cast<int*>(static_cast<char*>(workspace) + grid_ws_bytes());
  e = hipErrorNotReady;
  if (G > 0) {
    e = launch_grid(nnchain_grid_kernel, G, mask_bytes(n), st, D, n, method, Z, sizes,
                    sizes + static_cast<size_t>(G) * n, workspace);
    if (e != hipSuccess) (void)hipGetLastError();  // refused before any workgroup ran
  }
  if (e != hipSuccess) {
    hipLaunchKernelGGL(nnchain_kernel, dim3(1), dim3(LT), mask_bytes(n), st, D, n, method, Z, sizes, sizes + n);
    e = hipGetLastError();
  }
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_linkage_nnchain: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}

extern "C" size_t cc_linkage_mst_workspace_bytes(int n) { return n > 0 ? mst_ws(n, link_groups(n, mst_grid_kernel)) : 0; }

extern "C" int cc_linkage_mst(const double* D, int n, double* out, void* workspace, size_t ws_bytes, void* stream) {
  const int G = n > 0 ? link_groups(n, mst_grid_kernel) : 0;
  if (!D || !out || n < 2 || !workspace || ws_bytes < mst_ws(n, G) || mask_bytes(n) > MASK_LDS_MAX) {
    cc::set_error("cc_linkage_mst: bad arguments");
    return CC_ERR_ARG;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(workspace, 0, GHDR, st);
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_linkage_mst: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  double* cur = reinterpret_cast<double*>(static_cast<char*>(workspace) + grid_ws_bytes());
  e = hipErrorNotReady;
  if (G > 0) {
    e = launch_grid(mst_grid_kernel, G, mask_bytes(n), st, D, n, out, cur, workspace);
    if (e != hipSuccess) (void)hipGetLastError();  // refused before any workgroup ran
  }
  if (e != hipSuccess) {
    hipLaunchKernelGGL(mst_kernel, dim3(1), dim3(LT), mask_bytes(n), st, D, n, out, cur);
    e = hipGetLastError();
  }
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_linkage_mst: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}

extern "C" int cc_linkage_check(const void* workspace, size_t ws_bytes, void* stream) {
  if (!workspace || ws_bytes < GHDR) {
    cc::set_error("cc_linkage_check: bad arguments");
    return CC_ERR_ARG;
  }
  unsigned err = 0;
  hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
  if (e == hipSuccess) e = hipMemcpy(&err, static_cast<const char*>(workspace) + 2 * sizeof(unsigned), sizeof(err), hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_linkage_check: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  if (err) {
    cc::set_error("cc_linkage: a grid barrier timed out (workgroups not co-resident?)");
    return CC_ERR_HIP;
  }
  return CC_OK;
}
