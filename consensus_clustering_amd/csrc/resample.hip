// Resampling on the device: RandomState(seed + h).choice(n, m, replace=False) for every
// resample h, bit-identical to numpy (reference consensus_clustering_parallelised.py:231-239,
// `_get_subsampling_indices`).
//
// numpy's legacy choice without p is permutation(n)[:m]: a Fisher-Yates shuffle of arange(n)
// that draws j = random_interval(i) for i = n-1 .. 1 (mask-and-reject on 32-bit MT19937 outputs)
// and swaps x[i], x[j].  The shuffle walks from the end, so the first m entries are final only
// after the whole pass.  Position i is never touched again after step i, so its final value
// (the old x[j]) is written out at step i; position 0 is written at the end.
//
// Mapping: one 64-lane workgroup per resample, the array in LDS as uint16 (n <= 65536; dynamic
// LDS of 2n bytes, so several resamples share a CU at small n).
//   * the wave generates the MT19937 stream 624 words at a time (init_genrand on lane 0, the
//     twist in four dependency phases across the lanes, tempering) into an LDS draw buffer;
//   * lane 0 consumes the draws four at a time: mask-and-reject, then the swap (one LDS round
//     trip per accepted step: read x[i] and x[j], write x[j], store x[j]'s old value to
//     out[i] when i < m).
// Resamples are independent, so nothing crosses workgroups; each rank launches only its own
// h range.  Any n: cc_resample_device_wide (below) resolves the shuffle from its swap partners
// without simulating it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "ccmi_internal.h"

namespace {

constexpr int MT_N = 624, MT_M = 397;
constexpr int RS_MAXN = 65536;
constexpr int RS_NT = 64;

__device__ __forceinline__ uint32_t mt_twist_word(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// One twist of the 624-word state (in place in `mt`, through `nw`), then the tempered words
// into `draws`.  Phases follow the in-place recurrence: new[k] uses old[k], old[k+1] and
// old[k+397] for k < 227, new[k-227] for 227 <= k < 623, and new[0], new[396] for k = 623.
__device__ void mt_block(uint32_t* mt, uint32_t* nw, uint32_t* draws, int lane) {
  for (int k = lane; k < MT_N - MT_M; k += RS_NT) nw[k] = mt_twist_word(mt[k], mt[k + 1], mt[k + MT_M]);
  __syncthreads();
  for (int k = MT_N - MT_M + lane; k < 2 * (MT_N - MT_M); k += RS_NT)
    nw[k] = mt_twist_word(mt[k], mt[k + 1], nw[k - (MT_N - MT_M)]);
  __syncthreads();
  for (int k = 2 * (MT_N - MT_M) + lane; k < MT_N - 1; k += RS_NT)
    nw[k] = mt_twist_word(mt[k], mt[k + 1], nw[k - (MT_N - MT_M)]);
  __syncthreads();
  if (lane == 0) nw[MT_N - 1] = mt_twist_word(mt[MT_N - 1], nw[0], nw[MT_M - 1]);
  __syncthreads();
  for (int k = lane; k < MT_N; k += RS_NT) {
    const uint32_t v = nw[k];
    mt[k] = v;
    draws[k] = mt_temper(v);
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t interval_mask(uint32_t max) {
  uint32_t mask = max;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  return mask;
}

__global__ __launch_bounds__(RS_NT) void resample_kernel(uint32_t seed, int n, int m, int h_begin, int32_t* out) {
  __shared__ uint32_t mt[MT_N], nw[MT_N];
  __shared__ __attribute__((aligned(16))) uint32_t draws[MT_N];
  __shared__ int st_i;
  extern __shared__ uint16_t arr[];  // [n]
  const int lane = threadIdx.x;
  const int h = h_begin + blockIdx.x;
  int32_t* o = out + static_cast<size_t>(blockIdx.x) * m;
  for (int i = lane; i < n; i += RS_NT) arr[i] = static_cast<uint16_t>(i);
  if (lane == 0) {  // init_genrand(seed + h)
    uint32_t x = seed + static_cast<uint32_t>(h);
    mt[0] = x;
    for (int i = 1; i < MT_N; ++i) {
      x = 1812433253u * (x ^ (x >> 30)) + static_cast<uint32_t>(i);
      mt[i] = x;
    }
    st_i = n - 1;
  }
  __syncthreads();
  while (st_i >= 1) {  // wave-uniform (LDS broadcast of lane 0's position)
    mt_block(mt, nw, draws, lane);
    if (lane == 0) {
      int i = st_i;
      uint32_t mask = interval_mask(static_cast<uint32_t>(i));
      for (int p = 0; p < MT_N && i >= 1; p += 4) {
        const uint4 d4 = *reinterpret_cast<const uint4*>(draws + p);
        const uint32_t dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (i < 1) break;
          const uint32_t v = dv[u] & mask;
          if (v > static_cast<uint32_t>(i)) continue;  // rejected
          const uint16_t xi = arr[i], xj = arr[v];
          arr[v] = xi;  // x[i] <-> x[j]; x[i] is final from here on
          if (i < m) o[i] = xj;
          --i;
          if (static_cast<uint32_t>(i) <= (mask >> 1)) mask >>= 1;  // mask = interval_mask(i)
        }
      }
      st_i = i;
    }
    __syncthreads();
  }
  if (lane == 0 && m > 0) o[0] = arr[0];
}

// ---- any n: the shuffle resolved from its swap partners -----------------------------------
// Step i of the shuffle swaps positions i and J[i] (J[i] = the accepted random_interval(i) draw,
// J[i] <= i).  Let g(i) be the value at position i just before step i.  Position i was last
// written before that by the latest earlier step i' > i with J[i'] = i (the smallest such i'),
// which moved g(i') there; with no such step it still holds i.  So with the steps grouped by
// partner position (bucket p = {i : J[i] = p}, ascending):
//   succ(p) = the first step of bucket p greater than p;  g(i) = succ(i) ? g(succ(i)) : i;
//   out[k] (k >= 1) = the value at J[k] before step k = (next step after k in bucket J[k]) ?
//                     g(next) : J[k];   out[0] = (first step of bucket 0) ? g(first) : 0.
// Only the draws are sequential (lane 0 of one wave per resample, no memory round trip per
// step); buckets are a counting sort, and the g chains are short (mean ~1, max ~20 at n = 200k).
// Arrays per resample (workspace, uint32 [n] each): J, bucket offsets, cursors, the sorted
// steps, next-in-bucket, succ.
constexpr int RSW_ARRAYS = 6;

// The draws: 64 at a time, one per lane.  Within a block of 64 draws the step i_k of draw k lies
// in [i - k, i] (at most k acceptances before it), so draw k is accepted for sure when
// (v & mask) <= i - k and rejected for sure when (v & mask) > i.  When every lane is sure (and
// neither the mask nor the end can change inside the block) the accepted lanes take steps
// i - (accepted lanes before them) at once; otherwise (about 2000 / mask of the blocks, and the
// last few thousand steps) lane 0 walks the block as numpy does.
__global__ __launch_bounds__(RS_NT) void rsw_draw_kernel(uint32_t seed, int n, int h_begin, size_t stride,
                                                        uint32_t* J) {
  __shared__ uint32_t mt[MT_N], nw[MT_N];
  __shared__ __attribute__((aligned(16))) uint32_t draws[MT_N];
  const int lane = threadIdx.x;
  const int h = h_begin + blockIdx.x;
  uint32_t* Jh = J + static_cast<size_t>(blockIdx.x) * stride;
  if (lane == 0) {  // init_genrand(seed + h)
    uint32_t x = seed + static_cast<uint32_t>(h);
    mt[0] = x;
    for (int i = 1; i < MT_N; ++i) {
      x = 1812433253u * (x ^ (x >> 30)) + static_cast<uint32_t>(i);
      mt[i] = x;
    }
    Jh[0] = 0;
  }
  __syncthreads();
  int i = n - 1;  // wave-uniform
  uint32_t mask = interval_mask(static_cast<uint32_t>(i > 0 ? i : 0));
  while (i >= 1) {
    mt_block(mt, nw, draws, lane);
    for (int p = 0; p < MT_N && i >= 1; p += RS_NT) {
      const int nb = min(RS_NT, MT_N - p);
      const bool have = lane < nb;
      const uint32_t v = have ? (draws[p + lane] & mask) : 0xFFFFFFFFu;
      const bool acc = have && static_cast<int64_t>(v) <= static_cast<int64_t>(i) - lane;
      const bool rej = !have || v > static_cast<uint32_t>(i);
      const bool steady = i - RS_NT > static_cast<int>(mask >> 1) && i - RS_NT >= 1;  // mask and end fixed
      if (steady && __all(acc || rej)) {
        const unsigned long long bal = __ballot(acc);
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        if (acc) Jh[i - before] = v;
        i -= __popcll(bal);
      } else {
        if (lane == 0) {
          for (int q = 0; q < nb && i >= 1; ++q) {
            const uint32_t w = draws[p + q] & mask;
            if (w > static_cast<uint32_t>(i)) continue;  // rejected
            Jh[i] = w;
            --i;
            if (static_cast<uint32_t>(i) <= (mask >> 1)) mask >>= 1;  // mask = interval_mask(i)
          }
        }
        i = __shfl(i, 0);
        mask = __shfl(mask, 0);
      }
    }
  }
}

// bucket sizes, then (one workgroup per resample) their exclusive scan -> offsets, cursors zeroed
__global__ void rsw_count_kernel(int n, int nh, size_t stride, const uint32_t* __restrict__ J, uint32_t* cnt) {
  const int64_t total = static_cast<int64_t>(nh) * (n - 1);
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t h = e / (n - 1);
    const int i = static_cast<int>(e - h * (n - 1)) + 1;
    atomicAdd(&cnt[h * stride + J[h * stride + i]], 1u);
  }
}

__global__ __launch_bounds__(256) void rsw_scan_kernel(int n, size_t stride, uint32_t* cnt, uint32_t* cur) {
  // coalesced chunks of 1024 counts (16 B per thread), a block scan per chunk, a running carry;
  // the next chunk's loads are issued before this chunk's scan
  __shared__ uint32_t wsum[4];
  uint32_t* c = cnt + static_cast<size_t>(blockIdx.x) * stride;
  uint32_t* u = cur + static_cast<size_t>(blockIdx.x) * stride;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  auto load = [&](int base) -> uint4 {
    const int i = base + 4 * t;
    if (i + 3 < n) return *reinterpret_cast<const uint4*>(c + i);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (i < n) v.x = c[i];
    if (i + 1 < n) v.y = c[i + 1];
    if (i + 2 < n) v.z = c[i + 2];
    return v;
  };
  uint32_t carry = 0;
  uint4 v = load(0);
  for (int base = 0; base < n; base += 1024) {
    const uint4 vn = load(base + 1024 < n ? base + 1024 : base);
    const uint32_t s = v.x + v.y + v.z + v.w;
    uint32_t inc = s;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      wpre += (k < w) ? wsum[k] : 0u;
      tot += wsum[k];
    }
    const uint32_t e0 = carry + wpre + inc - s;  // exclusive offset of this thread's first count
    const int i = base + 4 * t;
    const uint32_t o[4] = {e0, e0 + v.x, e0 + v.x + v.y, e0 + v.x + v.y + v.z};
    if (i + 3 < n) {
      *reinterpret_cast<uint4*>(c + i) = make_uint4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<uint4*>(u + i) = make_uint4(0, 0, 0, 0);
    } else {
      for (int k = 0; k < 4; ++k)
        if (i + k < n) {
          c[i + k] = o[k];
          u[i + k] = 0;
        }
    }
    carry += tot;
    v = vn;
    __syncthreads();  // wsum is rewritten by the next chunk
  }
}

__global__ void rsw_scatter_kernel(int n, int nh, size_t stride, const uint32_t* __restrict__ J,
                                   const uint32_t* __restrict__ off, uint32_t* cur, uint32_t* sorted) {
  const int64_t total = static_cast<int64_t>(nh) * (n - 1);
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t h = e / (n - 1);
    const int i = static_cast<int>(e - h * (n - 1)) + 1;
    const uint32_t p = J[h * stride + i];
    const uint32_t k = atomicAdd(&cur[h * stride + p], 1u);
    sorted[h * stride + off[h * stride + p] + k] = static_cast<uint32_t>(i);
  }
}

// per bucket p: sort its steps ascending (insertion sort in place: buckets are small), then
// next-in-bucket for each step and succ(p) (0 = none: every step is >= 1)
__global__ void rsw_bucket_kernel(int n, int nh, size_t stride, const uint32_t* __restrict__ off,
                                  const uint32_t* __restrict__ cur, uint32_t* sorted, uint32_t* nxt,
                                  uint32_t* succ) {
  const int64_t total = static_cast<int64_t>(nh) * n;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t h = e / n;
    const uint32_t p = static_cast<uint32_t>(e - h * n);
    uint32_t* b = sorted + h * stride + off[h * stride + p];
    const int len = static_cast<int>(cur[h * stride + p]);
    for (int a = 1; a < len; ++a) {
      const uint32_t v = b[a];
      int q = a - 1;
      while (q >= 0 && b[q] > v) {
        b[q + 1] = b[q];
        --q;
      }
      b[q + 1] = v;
    }
    uint32_t first = 0;
    for (int a = 0; a < len; ++a) {
      nxt[h * stride + b[a]] = (a + 1 < len) ? b[a + 1] : 0u;
      if (first == 0 && b[a] > p) first = b[a];
    }
    succ[h * stride + p] = first;
  }
}

__global__ void rsw_out_kernel(int n, int m, int nh, size_t stride, const uint32_t* __restrict__ J,
                               const uint32_t* __restrict__ off, const uint32_t* __restrict__ cur,
                               const uint32_t* __restrict__ sorted, const uint32_t* __restrict__ nxt,
                               const uint32_t* __restrict__ succ, int32_t* __restrict__ out) {
  const int64_t total = static_cast<int64_t>(nh) * m;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t h = e / m;
    const int k = static_cast<int>(e - h * m);
    const size_t b = h * stride;
    uint32_t s, v;
    if (k == 0) {
      s = cur[b] ? sorted[b + off[b]] : 0u;
      v = 0u;
    } else {
      s = nxt[b + k];
      v = J[b + k];
    }
    if (s) {  // g(s): follow the chain of first later writers
      uint32_t x = s;
      for (uint32_t y = succ[b + x]; y; y = succ[b + x]) x = y;
      v = x;
    }
    out[e] = static_cast<int32_t>(v);
  }
}

}  // namespace

extern "C" int cc_resample_device_max_n(void) { return RS_MAXN; }

extern "C" size_t cc_resample_device_wide_workspace_bytes(int n, int nh) {
  if (n <= 0 || nh <= 0) return 0;
  return static_cast<size_t>(RSW_ARRAYS) * static_cast<size_t>(nh) * ((static_cast<size_t>(n) + 63) & ~static_cast<size_t>(63)) *
         sizeof(uint32_t);
}

extern "C" int cc_resample_device_wide(uint32_t seed, int h_begin, int h_end, int n, int m, int32_t* out,
                                       void* workspace, size_t ws_bytes, void* stream) {
  if (n <= 0 || m < 0 || m > n || h_begin < 0 || h_end < h_begin || (h_end > h_begin && m > 0 && !out)) {
    cc::set_error("cc_resample_device_wide: bad arguments (n >= 1, 0 <= m <= n)");
    return CC_ERR_ARG;
  }
  if (static_cast<uint64_t>(seed) + static_cast<uint64_t>(h_end) > 0xffffffffull + 1) {
    cc::set_error("cc_resample_device_wide: seed + h exceeds 2**32 - 1 (numpy raises ValueError)");
    return CC_ERR_ARG;
  }
  const int H = h_end - h_begin;
  if (H == 0 || m == 0) return CC_OK;
  const size_t per = cc_resample_device_wide_workspace_bytes(n, 1);
  if (!workspace || ws_bytes < per) {
    cc::set_error("cc_resample_device_wide: workspace too small (cc_resample_device_wide_workspace_bytes(n, 1) at least)");
    return CC_ERR_ARG;
  }
  const int batch = static_cast<int>(std::min<size_t>(static_cast<size_t>(H), ws_bytes / per));
  const size_t stride = (static_cast<size_t>(n) + 63) & ~static_cast<size_t>(63);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  for (int hb = 0; hb < H; hb += batch) {
    const int nh = std::min(batch, H - hb);
    uint32_t* base = static_cast<uint32_t*>(workspace);
    const size_t A = static_cast<size_t>(nh) * stride;
    uint32_t *J = base, *off = base + A, *cur = base + 2 * A, *sorted = base + 3 * A, *nxt = base + 4 * A,
             *succ = base + 5 * A;
    if (hipMemsetAsync(off, 0, A * sizeof(uint32_t), st) != hipSuccess) {
      cc::set_error("cc_resample_device_wide: memset failed");
      return CC_ERR_HIP;
    }
    hipLaunchKernelGGL(rsw_draw_kernel, dim3(nh), dim3(RS_NT), 0, st, seed, n, h_begin + hb, stride, J);
    const int64_t work = static_cast<int64_t>(nh) * n;
    const unsigned g = static_cast<unsigned>(std::min<int64_t>((work + 255) / 256, 65536));
    if (n > 1) hipLaunchKernelGGL(rsw_count_kernel, dim3(g), dim3(256), 0, st, n, nh, stride, J, off);
    hipLaunchKernelGGL(rsw_scan_kernel, dim3(nh), dim3(256), 0, st, n, stride, off, cur);
    if (n > 1) hipLaunchKernelGGL(rsw_scatter_kernel, dim3(g), dim3(256), 0, st, n, nh, stride, J, off, cur, sorted);
    hipLaunchKernelGGL(rsw_bucket_kernel, dim3(g), dim3(256), 0, st, n, nh, stride, off, cur, sorted, nxt, succ);
    const int64_t owork = static_cast<int64_t>(nh) * m;
    const unsigned go = static_cast<unsigned>(std::min<int64_t>((owork + 255) / 256, 65536));
    hipLaunchKernelGGL(rsw_out_kernel, dim3(go), dim3(256), 0, st, n, m, nh, stride, J, off, cur, sorted, nxt, succ,
                       out + static_cast<size_t>(hb) * m);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      cc::set_error(std::string("cc_resample_device_wide: ") + hipGetErrorString(e));
      return CC_ERR_HIP;
    }
  }
  return CC_OK;
}

extern "C" int cc_resample_device(uint32_t seed, int h_begin, int h_end, int n, int m, int32_t* out,
                                  void* stream) {
  if (n <= 0 || n > RS_MAXN || m < 0 || m > n || h_begin < 0 || h_end < h_begin ||
      (h_end > h_begin && m > 0 && !out)) {
    cc::set_error("cc_resample_device: bad arguments (1 <= n <= 65536, 0 <= m <= n)");
    return CC_ERR_ARG;
  }
  if (static_cast<uint64_t>(seed) + static_cast<uint64_t>(h_end) > 0xffffffffull + 1) {
    cc::set_error("cc_resample_device: seed + h exceeds 2**32 - 1 (numpy raises ValueError)");
    return CC_ERR_ARG;
  }
  const int H = h_end - h_begin;
  if (H == 0 || m == 0) return CC_OK;
  const size_t lds = (static_cast<size_t>(n) * sizeof(uint16_t) + 15) & ~static_cast<size_t>(15);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(resample_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_resample_device: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  hipLaunchKernelGGL(resample_kernel, dim3(H), dim3(RS_NT), lds, static_cast<hipStream_t>(stream), seed, n, m,
                     h_begin, out);
  e = hipGetLastError();
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_resample_device: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}
