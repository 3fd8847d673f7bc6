// Host-native replay of numpy's legacy RandomState streams used on the hot path.
//
// * cc_resample_indices: RandomState(seed + h).choice(n, m, replace=False) for every
//   resample h (reference CC.py:231-239).  numpy's legacy choice without p is
//   permutation(n)[:m]; permutation is a Fisher-Yates shuffle of arange(n) drawing
//   j = random_interval(i) for i = n-1 .. 1 (mask-and-reject on 32-bit MT19937
//   outputs while i <= 0xffffffff).  Seeding an int is MT19937 init_genrand.
// * cc_random_sample: RandomState(seed).random_sample(count), the 53-bit double
//   (a >> 5, b >> 6) construction, used for the k-means++ uniform stream of
//   sklearn's KMeans (sklearn/cluster/_kmeans.py:225, :243).
//
// The shuffle walks from the END of the array, so the first m entries are final
// only after the whole pass: all n-1 draws are replayed.  Resamples are
// independent streams and run on host threads.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ccmi_internal.h"

namespace {

struct MT19937 {
  static constexpr int N = 624, M = 397;
  uint32_t mt[N];
  int pos;

  explicit MT19937(uint32_t seed) {
    mt[0] = seed;
    for (int i = 1; i < N; ++i)
      mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + static_cast<uint32_t>(i);
    pos = N;
  }

  void twist() {
    constexpr uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MATRIX_A = 0x9908b0dfu;
    int k = 0;
    for (; k < N - M; ++k) {
      uint32_t y = (mt[k] & UPPER) | (mt[k + 1] & LOWER);
      mt[k] = mt[k + M] ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
    }
    for (; k < N - 1; ++k) {
      uint32_t y = (mt[k] & UPPER) | (mt[k + 1] & LOWER);
      mt[k] = mt[k + (M - N)] ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
    }
    uint32_t y = (mt[N - 1] & UPPER) | (mt[0] & LOWER);
    mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
    pos = 0;
  }

  inline uint32_t next32() {
    if (pos == N) twist();
    uint32_t y = mt[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  inline double next_double() {
    int32_t a = static_cast<int32_t>(next32() >> 5), b = static_cast<int32_t>(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }

  // numpy random_interval for max <= 0xffffffff (n is an int here).
  inline uint32_t interval(uint32_t max) {
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32() & mask)) > max) {
    }
    return v;
  }
};

void permute_prefix(uint32_t seed, int n, int m, int32_t* out, std::vector<int32_t>& buf) {
  buf.resize(n);
  for (int i = 0; i < n; ++i) buf[i] = i;
  MT19937 g(seed);
  for (int i = n - 1; i >= 1; --i) {
    uint32_t j = g.interval(static_cast<uint32_t>(i));
    std::swap(buf[i], buf[j]);
  }
  std::memcpy(out, buf.data(), sizeof(int32_t) * static_cast<size_t>(m));
}

}  // namespace

extern "C" int cc_resample_indices(uint32_t seed, int h_begin, int h_end, int n, int m,
                                   int32_t* out, int n_threads) {
  if (n <= 0 || m < 0 || m > n || h_begin < 0 || h_end < h_begin || !out) {
    cc::set_error("cc_resample_indices: bad arguments");
    return CC_ERR_ARG;
  }
  if (static_cast<uint64_t>(seed) + static_cast<uint64_t>(h_end) > 0xffffffffull + 1) {
    cc::set_error("cc_resample_indices: seed + h exceeds 2**32 - 1 (numpy raises ValueError)");
    return CC_ERR_ARG;
  }
  int H = h_end - h_begin;
  int nt = n_threads > 0 ? n_threads : static_cast<int>(std::thread::hardware_concurrency());
  nt = std::max(1, std::min(nt, H));
  auto work = [&](int t) {
    std::vector<int32_t> buf;
    for (int h = h_begin + t; h < h_end; h += nt)
      permute_prefix(seed + static_cast<uint32_t>(h), n, m,
                     out + static_cast<size_t>(h - h_begin) * m, buf);
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(nt);
    for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  return CC_OK;
}

extern "C" int cc_random_sample(uint32_t seed, int64_t count, double* out) {
  if (count < 0 || (count > 0 && !out)) {
    cc::set_error("cc_random_sample: bad arguments");
    return CC_ERR_ARG;
  }
  MT19937 g(seed);
  for (int64_t i = 0; i < count; ++i) out[i] = g.next_double();
  return CC_OK;
}

// k-means++ streams of every (K, init) run: sklearn's KMeans(random_state=seed) fit draws, for
// each of its n_init runs, the first centre with RandomState.choice(m, p=sample_weight/sum)
// (_kmeans.py:225) and then (K-1) * (2 + floor(ln K)) uniforms, one block of local trials per
// centre (:243).  Every fit of one K replays RandomState(seed) from the start.  choice with p is
// numpy's legacy form: p as float64, cdf = cumsum(p) (sequential), cdf /= cdf[-1], one
// random_sample, searchsorted(side='right').  weight_f64 = 0: unit float32 weights, p = f32(1/m).
extern "C" int cc_kpp_tables(const int32_t* Ks, int nK, int n_init, uint32_t seed, int m,
                             int weight_f64, double* kpp_u, int kpp_stride, int32_t* kpp_pos) {
  if (!Ks || nK <= 0 || n_init <= 0 || m <= 0 || !kpp_u || !kpp_pos) {
    cc::set_error("cc_kpp_tables: bad arguments");
    return CC_ERR_ARG;
  }
  for (int k = 0; k < nK; ++k) {
    const int K = Ks[k];
    const int t = 2 + static_cast<int>(std::log(static_cast<double>(K)));
    if (K < 1 || 1 + (K - 1) * t > kpp_stride) {
      cc::set_error("cc_kpp_tables: K out of range or kpp_stride too small");
      return CC_ERR_ARG;
    }
  }
  const double p = weight_f64 ? 1.0 / static_cast<double>(m)
                              : static_cast<double>(1.0f / static_cast<float>(m));
  std::vector<double> cdf(static_cast<size_t>(m));
  double c = 0.0;
  for (int i = 0; i < m; ++i) {
    c += p;
    cdf[i] = c;
  }
  const double last = cdf[m - 1];
  for (int i = 0; i < m; ++i) cdf[i] /= last;
  for (int k = 0; k < nK; ++k) {
    const int K = Ks[k];
    const int t = 2 + static_cast<int>(std::log(static_cast<double>(K)));
    MT19937 g(seed);
    for (int i = 0; i < n_init; ++i) {
      double* u = kpp_u + (static_cast<size_t>(k) * n_init + i) * kpp_stride;
      const double r = g.next_double();
      kpp_pos[k * n_init + i] =
          static_cast<int32_t>(std::upper_bound(cdf.begin(), cdf.end(), r) - cdf.begin());
      u[0] = 0.0;
      for (int j = 0; j < (K - 1) * t; ++j) u[1 + j] = g.next_double();
      for (int j = 1 + (K - 1) * t; j < kpp_stride; ++j) u[j] = 0.0;
    }
  }
  return CC_OK;
}
