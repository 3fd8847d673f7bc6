// Probe: does v_mfma_f64_16x16x4_f64 round like a sequential FMA chain over k?
// For random operands (mixed exponents, cancellations) each lane compares its 4 MFMA results
// with candidate orders computed by VALU:  fma chain k = 0..3 from C, fma chain k = 3..0,
// products rounded then summed in order, and exact-sum-then-one-rounding (via a double-double).
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_f64_probe.hip -o /tmp/mfma_f64_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#pragma clang fp contract(off)

using v4d = __attribute__((ext_vector_type(4))) double;

__device__ double two_sum(double a, double b, double& e) {
  const double s = a + b, bb = s - a;
  e = (a - (s - bb)) + (b - bb);
  return s;
}

// exact c + sum p_k rounded once (double-double accumulation is enough for 5 terms here)
__device__ double exact_round(double c, const double* a, const double* b) {
  double hi = c, lo = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double p = a[k] * b[k];
    const double pe = __fma_rn(a[k], b[k], -p);
    double e1, e2;
    hi = two_sum(hi, p, e1);
    lo += e1 + pe;
    (void)e2;
  }
  return hi + lo;
}

__global__ void probe(const double* A, const double* B, const double* C, int ntile,
                      unsigned long long* cnt) {
  // tile t: A[t][16][4], B[t][4][16], C[t][16][16]
  const int l = threadIdx.x;
  for (int t = blockIdx.x; t < ntile; t += gridDim.x) {
    const double* At = A + t * 64;
    const double* Bt = B + t * 64;
    const double* Ct = C + t * 256;
    const double a = At[(l & 15) * 4 + (l >> 4)];
    const double b = Bt[(l >> 4) * 16 + (l & 15)];
    v4d c;
    for (int i = 0; i < 4; ++i) c[i] = Ct[((l >> 4) + 4 * i) * 16 + (l & 15)];
    const v4d dres = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    unsigned long long m[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
      const int row = (l >> 4) + 4 * i, col = l & 15;
      double ar[4], br[4];
      for (int k = 0; k < 4; ++k) {
        ar[k] = At[row * 4 + k];
        br[k] = Bt[k * 16 + col];
      }
      const double c0 = Ct[row * 16 + col];
      double f = c0;
      for (int k = 0; k < 4; ++k) f = __fma_rn(ar[k], br[k], f);
      double g = c0;
      for (int k = 3; k >= 0; --k) g = __fma_rn(ar[k], br[k], g);
      double s = c0;
      for (int k = 0; k < 4; ++k) s = s + ar[k] * br[k];
      const double x = exact_round(c0, ar, br);
      const double dv = dres[i];
      m[0] += (dv == f);
      m[1] += (dv == g);
      m[2] += (dv == s);
      m[3] += (dv == x);
      m[4] += 1;
    }
    for (int q = 0; q < 5; ++q) atomicAdd(&cnt[q], m[q]);
  }
}

int main() {
  const int ntile = 4096;
  std::vector<double> A(ntile * 64), B(ntile * 64), C(ntile * 256);
  uint64_t s = 88172645463325252ull;
  auto rnd = [&]() {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    return s;
  };
  auto val = [&](int mode) {
    const double u = (rnd() >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
    if (mode == 0) return u;
    const int e = static_cast<int>(rnd() % 40) - 20;
    return std::ldexp(u, e);
  };
  for (int t = 0; t < ntile; ++t) {
    const int mode = t & 1;
    for (int i = 0; i < 64; ++i) A[t * 64 + i] = val(mode);
    for (int i = 0; i < 64; ++i) B[t * 64 + i] = val(mode);
    for (int i = 0; i < 256; ++i) C[t * 256 + i] = (t % 4 == 3) ? 0.0 : val(mode);
  }
  double *dA, *dB, *dC;
  unsigned long long* dn;
  hipMalloc(&dA, A.size() * 8);
  hipMalloc(&dB, B.size() * 8);
  hipMalloc(&dC, C.size() * 8);
  hipMalloc(&dn, 5 * 8);
  hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipMemset(dn, 0, 5 * 8);
  hipLaunchKernelGGL(probe, dim3(256), dim3(64), 0, 0, dA, dB, dC, ntile, dn);
  unsigned long long n[5];
  hipMemcpy(n, dn, 5 * 8, hipMemcpyDeviceToHost);
  hipError_t e = hipDeviceSynchronize();
  std::printf("status %s; of %llu results: fma k0..3 %llu, fma k3..0 %llu, rounded products %llu, "
              "exact-once %llu\n", hipGetErrorString(e), n[4], n[0], n[1], n[2], n[3]);
  return 0;
}
