// Micro-benchmark of the slot-tile E-step (kmeans.hip ste_estep) variants: one 64-lane wave per
// workgroup (or two waves per SIMD with -DPAIR), a distance tile in LDS, R repetitions, cycles per
// repetition from s_memtime.  Build: hipcc -O3 --offload-arch=gfx950 ste_bench.hip -o ste_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int RT = 32, DSD = 260, R = 2000;

__device__ __forceinline__ void grp(const float4 v, int base, float& m, int& i) {
  float m0 = v.x, m1 = v.z;
  int i0 = base, i1 = base + 2;
  if (v.y < m0) { m0 = v.y; i0 = base + 1; }
  if (v.w < m1) { m1 = v.w; i1 = base + 3; }
  if (m1 < m0) { m0 = m1; i0 = i1; }
  m = m0;
  i = i0;
}

// VAR 0: the kernel's form (compare / select per pair)
// VAR 1: group minimum by v_min3 / v_min, index by equality (first match)
__device__ __forceinline__ void grp1(const float4 v, int base, float& m, int& i) {
  const float mn = fminf(fminf(v.x, v.y), fminf(v.z, v.w));
  int j = base + 3;
  j = (v.z == mn) ? base + 2 : j;
  j = (v.y == mn) ? base + 1 : j;
  j = (v.x == mn) ? base : j;
  m = mn;
  i = j;
}

__global__ __launch_bounds__(64 * NWAVE) void bench(const float* Dsrc, unsigned char* out, float* acc_out,
                                                    unsigned long long* cyc, unsigned smask, unsigned emask) {
  __shared__ float D[RT * DSD];
  for (int e = threadIdx.x; e < RT * DSD; e += blockDim.x) D[e] = Dsrc[e];
  __syncthreads();
  const int lane = threadIdx.x & 63, ler = lane & 31, hh = lane >> 5;
  const int q = (threadIdx.x >> 6) & 3;
  float iacc[16];
  for (int G = 0; G < 16; ++G) iacc[G] = 0.f;
  unsigned char* gl = out + blockIdx.x * 4096 + (threadIdx.x >> 6) * 512;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < R; ++r) {
    int lanel = lane;
    asm volatile("" : "+v"(lanel));
    const float* drow = D + (lanel & 31) * DSD + 64 * q + 4 * (lanel >> 5);
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(drow + 8 * u);
    float gm[8], om[8];
    int gi[8], oi[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (VAR == 1) grp1(v[u], 8 * u + 4 * hh, gm[u], gi[u]);
      else grp(v[u], 8 * u + 4 * hh, gm[u], gi[u]);
    }
#if STAGE == 1
    float sink = 0.f;
    for (int u = 0; u < 8; ++u) sink += gm[u] + gi[u];
    iacc[0] += sink;
    continue;
#endif
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const auto bs = __builtin_amdgcn_permlane32_swap(__float_as_uint(gm[u]), __float_as_uint(gm[u]), false, false);
      const auto is = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(gi[u]), static_cast<unsigned>(gi[u]), false, false);
      om[u] = __uint_as_float(bs[1]);
      oi[u] = static_cast<int>(is[1]);
    }
#if STAGE == 2
    float sink = 0.f;
    for (int u = 0; u < 8; ++u) sink += om[u] + oi[u];
    iacc[0] += sink;
    continue;
#endif
    constexpr float INF = __builtin_huge_valf();
    float run = INF;
    int ri = 0, sbase = 0;
#pragma unroll
    for (int G = 0; G < 16; ++G) {
      const float val = (G & 1) ? om[G >> 1] : gm[G >> 1];
      const int vi = (G & 1) ? oi[G >> 1] : gi[G >> 1];
      const bool st = (smask >> G) & 1u;
      run += st ? INF : 0.f;
      sbase = st ? 4 * G : sbase;
      const bool lt = val < run;
      run = lt ? val : run;
      ri = lt ? vi : ri;
      if (STAGE >= 4 && ((emask >> G) & 1u)) {
        if (hh == 0) {
          gl[G * 32 + ler] = static_cast<unsigned char>(ri - sbase);
          iacc[G] += run;
        }
      }
    }
#if STAGE == 3
    iacc[1] += run + ri;
#endif
#if NOBAR == 0
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
#endif
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int G = 0; G < 16; ++G) s += iacc[G];
  acc_out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  std::vector<float> h(RT * DSD);
  unsigned x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (x >> 8) * (1.0f / 16777216.0f) * 100.f - 50.f; }
  float *d, *acc;
  unsigned char* out;
  unsigned long long* cyc;
  const int B = 256;
  hipMalloc(&d, h.size() * 4);
  hipMalloc(&out, B * 4096);
  hipMalloc(&acc, B * 64 * NWAVE * 4);
  hipMalloc(&cyc, B * 8);
  hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  // problems of K = 12..20 (3-5 groups) packed: starts at 0, 4, 8, 12 (4 problems of 4 groups)
  const unsigned smask = 0x1111u, emask = 0x8888u;
  for (int it = 0; it < 3; ++it) {
    hipLaunchKernelGGL(bench, dim3(B), dim3(64 * NWAVE), 0, 0, d, out, acc, cyc, smask, emask);
    hipDeviceSynchronize();
  }
  std::vector<unsigned long long> c(B);
  hipMemcpy(c.data(), cyc, B * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (auto v : c) m += v;
  printf("VAR %d NWAVE %d NOBAR %d: %.1f cycles per repetition\n", VAR, NWAVE, NOBAR, m / B / R);
  return 0;
}
