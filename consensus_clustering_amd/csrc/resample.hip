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
// h range.  The host replay (host_rng.cpp) stays for n > 65536 (the uint16 array).
#include <hip/hip_runtime.h>

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

}  // namespace

extern "C" int cc_resample_device_max_n(void) { return RS_MAXN; }

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
