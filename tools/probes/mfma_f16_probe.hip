// Probe: how does v_mfma_f32_32x32x16_f16 round?  Random f16 operands (K1's hi/lo operand
// range) and f32 accumulators; the GPU results are written next to the inputs for the host
// model check (tools/probes/mfma_f16_models.py): one rounding of C + the exact 16-term sum,
// sequential float32 additions, pairwise trees, ...
//   hipcc --offload-arch=gfx950 -O2 tools/probes/mfma_f16_probe.hip -o /tmp/mfma_f16_probe
//   /tmp/mfma_f16_probe OUT.bin
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

// tile t: A[t][32][16] (row-major, M x K), B[t][16][32] (K x N), C/D[t][32][32]
__global__ void probe(const _Float16* A, const _Float16* B, const float* C, float* D, int ntile) {
  const int l = threadIdx.x;
  for (int t = blockIdx.x; t < ntile; t += gridDim.x) {
    const _Float16* At = A + t * 512;
    const _Float16* Bt = B + t * 512;
    h8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = At[(l & 31) * 16 + 8 * (l >> 5) + j];
      b[j] = Bt[(8 * (l >> 5) + j) * 32 + (l & 31)];
    }
    v16f c;
    for (int v = 0; v < 16; ++v) c[v] = C[t * 1024 + ((v & 3) + 8 * (v >> 2) + 4 * (l >> 5)) * 32 + (l & 31)];
    const v16f d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    for (int v = 0; v < 16; ++v) D[t * 1024 + ((v & 3) + 8 * (v >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = d[v];
  }
}

static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return static_cast<uint32_t>(st >> 16);
}
static _Float16 rh(int emin, int emax) {  // random sign, exponent in [emin, emax], 10-bit mantissa
  const int e = emin + static_cast<int>(rnd() % static_cast<uint32_t>(emax - emin + 1));
  const float m = 1.0f + static_cast<float>(rnd() & 1023) / 1024.0f;
  const float v = ldexpf(m, e) * ((rnd() & 1) ? -1.0f : 1.0f);
  return static_cast<_Float16>(v);
}

int main(int argc, char** argv) {
  const int ntile = 256;
  std::vector<_Float16> A(ntile * 512), B(ntile * 512);
  std::vector<float> C(ntile * 1024), D(ntile * 1024);
  for (int t = 0; t < ntile; ++t) {
    // mixes: hi*hi-like (wide range), lo parts (small), cancellations via signs
    const int mode = t % 4;
    for (int i = 0; i < 512; ++i) {
      A[t * 512 + i] = mode == 1 ? rh(-14, -8) : rh(-6, 3);
      B[t * 512 + i] = mode == 2 ? rh(-14, -8) : rh(-6, 3);
    }
    for (int i = 0; i < 1024; ++i) {
      const float m = 1.0f + static_cast<float>(rnd() & 0x7FFFFF) / 8388608.0f;
      const int e = mode == 3 ? -20 + static_cast<int>(rnd() % 8) : -4 + static_cast<int>(rnd() % 10);
      C[t * 1024 + i] = ldexpf(m, e) * ((rnd() & 1) ? -1.0f : 1.0f);
    }
  }
  _Float16 *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, A.size() * 2);
  hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dC, C.size() * 4);
  hipMalloc(&dD, D.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(64), dim3(64), 0, 0, dA, dB, dC, dD, ntile);
  hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
  FILE* f = fopen(argc > 1 ? argv[1] : "mfma_f16_probe.bin", "wb");
  fwrite(&ntile, 4, 1, f);
  fwrite(A.data(), 2, A.size(), f);
  fwrite(B.data(), 2, B.size(), f);
  fwrite(C.data(), 4, C.size(), f);
  fwrite(D.data(), 4, D.size(), f);
  fclose(f);
  printf("wrote %d tiles\n", ntile);
  return 0;
}
