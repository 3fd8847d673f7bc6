// Co-sampling (I), co-association (M) and the fused consensus histogram on gfx950.
//
// Reference behaviour (consensus_clustering_parallelised.py, "CC.py"):
//   I = S^T S over the H x n sampled-indicator matrix            CC.py:259-264
//   M += L^T L over the K x n one-hot label matrix, per resample  CC.py:284-290
//   C = f32(M) / f32(I + 1e-6); histogram of triu(C, 1), 20 bins  CC.py:338-344, :372
//
// Formulation.  With the labels of every resample stored sample-major as bytes
// (labels_nh[i][h], 0xFF = not sampled), M_ij = sum over the virtual index
// v = (h, c) of onehot_i(v) * onehot_j(v) with onehot_i(h, c) = [label_h(i) == c],
// and I_ij the same sum over v = h with the sampled flag.  Both are int8 GEMMs
// A * A^T with a 0/1 operand, run on v_mfma_i32_32x32x32_i8 with int32 accumulators:
// exact integer counts.  The one-hot operand is never stored in HBM: each
// super-step, every thread of the 512-thread workgroup loads the label bytes of ONE
// row of the tile (A side or B side) for 128 virtual-k values, expands them to
// 128 one-hot bytes in registers and writes them to LDS already in MFMA fragment
// order (one ds_write_b128 per 16 bytes); the 8 waves then read fragments with
// ds_read_b128 and issue 32 MFMAs each.  Channels are padded to KP = next pow2 >= K
// so one virtual chunk of 32 holds 32/KP resamples (KP <= 32) or a channel slice.
//
// Tiling.  The n x n count matrix is covered by 256 x 256 tiles of the upper
// triangle (bi <= bj), numbered row-major; a launch handles tiles
// [tile_begin, tile_end), which is also how the triangle is row-band sharded over
// GPUs.  Waves are arranged 2 x 4, each owning 128 x 64 outputs (4 x 2 blocks of
// 32 x 32, 128 accumulator registers).
//
// Epilogue.  The I kernel stores its tile in accumulator order (uint16, coalesced)
// so the M kernel re-reads exactly the I value of each of its own accumulator
// elements.  The M kernel bins every strict-upper pair with numpy.histogram's
// uniform-bin arithmetic (numpy/lib/_histograms_impl.py:851-868): x = f32(m) /
// f32(f64(i) + 1e-6) correctly rounded, b = floor(f64(x) * 20), b == 20 -> 19,
// then the two edge corrections against the float32 edges.  Per-thread private
// LDS counters (ds_add, conflict-free [bin][thread] layout) are reduced per
// workgroup and added to 20 uint64 global counters (integer atomics: order-free).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cmath>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "ccmi_internal.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int T = CC_TILE;            // 256
constexpr int NT = 512;               // threads per workgroup (8 waves)
constexpr int KC = 4;                 // 32-wide k-chunks per super-step (128 virtual k)
constexpr int FRAG = 1024;            // one 32x32x32 i8 operand fragment: 64 lanes x 16 B
constexpr int SIDE = 8 * KC * FRAG;   // 8 row blocks x 4 chunks = 32 KiB
constexpr int BUF = 2 * SIDE;         // A side + B side
constexpr int LDS_BYTES = 2 * BUF;    // double buffered = 128 KiB
constexpr int NBINS = CC_NBINS;
constexpr int NW = NT / 64;
// epilogue LDS: hist [NBINS][NT] u32 | 32 edges f32 | wave sums [NBINS][NW] u32 | bin table
constexpr int BT_OFF = NBINS * NT * 4 + 32 * 4 + NBINS * NW * 4;
// The on-chip binning table, staged per tile in one of three forms (chosen by the row count,
// i.e. by H):
//   TRI  (rows <= BT_TRI_ROWS, H <= ~420): the bin itself, one byte per (m <= i) pair at
//        i (i + 1) / 2 + m: one LDS read per element;
//   PAIR (rows <= BT_PAIR_ROWS, H <= ~1060): per row 20 uint32 threshold pairs
//        T[g] | T[g + 1] << 16 and the reciprocal 20 / i: two LDS reads per element;
//   U16  (rows <= BT_MAX_ROWS): per row 21 uint16 thresholds and the reciprocal: three.
// cc_bin_table writes every form that fits into one global buffer (u16 part first, then the
// pair part, then the triangle), so each tile copies its form with 16-B loads.
constexpr int BT_AVAIL = LDS_BYTES - BT_OFF - 32;
constexpr int BT_MAX_ROWS = BT_AVAIL / ((NBINS + 1) * 2 + 4);
constexpr int BT_PAIR_ROWS = (BT_AVAIL - 16) / (NBINS * 4 + 4);
constexpr int bt_tri_rows() {
  int r = 1;
  while ((static_cast<int64_t>(r + 1) * (r + 2) / 2 + 15) / 16 * 16 <= BT_AVAIL) ++r;
  return r;
}
constexpr int BT_TRI_ROWS = bt_tri_rows();
static_assert(BT_OFF % 16 == 0, "table copies are 16-B");
enum { BT_U16 = 0, BT_PAIR = 1, BT_TRI = 2 };
__host__ __device__ constexpr int bt_form(int rows) {
  return rows <= BT_TRI_ROWS ? BT_TRI : (rows <= BT_PAIR_ROWS ? BT_PAIR : BT_U16);
}
__host__ __device__ constexpr int64_t bt_u16_bytes(int rows) { return (static_cast<int64_t>(rows) * (NBINS + 1) * 2 + 15) / 16 * 16; }
__host__ __device__ constexpr int64_t bt_pair_bytes(int rows) { return rows <= BT_PAIR_ROWS ? static_cast<int64_t>(rows) * NBINS * 4 : 0; }
__host__ __device__ constexpr int64_t bt_tri_bytes(int rows) {
  return rows <= BT_TRI_ROWS ? (static_cast<int64_t>(rows) * (rows + 1) / 2 + 15) / 16 * 16 : 0;
}

__device__ __forceinline__ void tile_coords(int64_t t, int nb, int& bi, int& bj) {
  auto start = [nb](int64_t b) -> int64_t { return b * nb - b * (b - 1) / 2; };
  double a = 2.0 * nb + 1.0;
  int r = static_cast<int>(floor((a - sqrt(a * a - 8.0 * static_cast<double>(t))) * 0.5));
  r = r < 0 ? 0 : (r > nb - 1 ? nb - 1 : r);
  while (r > 0 && start(r) > t) --r;
  while (r + 1 < nb && start(r + 1) <= t) ++r;
  bi = r;
  bj = static_cast<int>(r + (t - start(r)));
}

// Histogram bin of one pair, exactly as numpy.histogram(bins=20, range=(0, 1)) on the
// float32 consensus value (CC.py:339-344 -> _histograms_impl.py:851-868).
__device__ __forceinline__ int consensus_bin(uint32_t m, uint32_t i, const float* e) {
  const float fi = static_cast<float>(static_cast<double>(i) + 1e-6);
  const float x = static_cast<float>(m) / fi;  // IEEE RN (no fast-math in this build)
  int b = static_cast<int>(static_cast<double>(x) * 20.0);
  if (b >= NBINS) b = NBINS - 1;
  if (x < e[b]) b -= 1;
  if (b != NBINS - 1 && x >= e[b + 1]) b += 1;
  return b;
}

// The same bin from the per-co-sampling-count threshold table (cc_bin_table): row i holds
// T[b] = min{m : consensus_bin(m, i) >= b} for b = 0..20 (T[0] = 0, T[20] = 0xFFFF), so the bin
// is #{b in 1..19 : m >= T[b]}.  A reciprocal estimate of 20 m / i is within one bin of it and
// one compare on each side makes it exact: no division, no f64.
constexpr int BT_ROW = NBINS + 1;

__device__ __forceinline__ int table_bin(uint32_t m, uint32_t i, const uint16_t* tab) {
  int g = 0;
  if (i > 0) {
    g = static_cast<int>(static_cast<float>(m) * (20.0f * __builtin_amdgcn_rcpf(static_cast<float>(i))));
    g = g > NBINS - 1 ? NBINS - 1 : g;
  }
  const uint16_t* row = tab + i * BT_ROW;
  return g - (m < row[g] ? 1 : 0) + (m >= row[g + 1] ? 1 : 0);
}

// table_bin with the reciprocal estimate read from the staged per-row table rtab[i] =
// 20 * rcp(f32(i)) (rtab[0] = 0): the same g as table_bin, without the convert/rcp/select.
__device__ __forceinline__ int table_bin_r(uint32_t m, uint32_t i, const uint16_t* tab, const float* rtab) {
  int g = static_cast<int>(static_cast<float>(m) * rtab[i]);
  g = g > NBINS - 1 ? NBINS - 1 : g;
  const uint16_t* row = tab + i * BT_ROW;
  return g - (m < row[g] ? 1 : 0) + (m >= row[g + 1] ? 1 : 0);
}

__global__ void bin_table_kernel(int rows, const float* __restrict__ edges, uint16_t* __restrict__ table) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * BT_ROW) return;
  const int i = e / BT_ROW, b = e - i * BT_ROW;
  uint32_t t;
  if (b == 0) {
    t = 0;
  } else if (b == NBINS) {
    t = 0xFFFFu;
  } else {  // first m in [0, i] with bin >= b (monotone in m), i + 1 if none
    uint32_t lo = 0, hi = static_cast<uint32_t>(i) + 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (consensus_bin(mid, static_cast<uint32_t>(i), edges) >= b) hi = mid;
      else lo = mid + 1;
    }
    t = lo;
  }
  table[e] = static_cast<uint16_t>(t);
}

// The bin of (m, i) from the threshold-pair form: P[i][g] = T[g] | T[g + 1] << 16.
__device__ __forceinline__ int pair_bin(uint32_t m, uint32_t i, const uint32_t* pair, const float* rtab) {
  int g = static_cast<int>(static_cast<float>(m) * rtab[i]);
  g = g > NBINS - 1 ? NBINS - 1 : g;
  const uint32_t pr = pair[i * NBINS + g];
  return g - (m < (pr & 0xFFFFu) ? 1 : 0) + (m >= (pr >> 16) ? 1 : 0);
}

// The bin of (m <= i) from the triangle form.
__device__ __forceinline__ int tri_bin(uint32_t m, uint32_t i, const uint8_t* tri) {
  return tri[((i * (i + 1)) >> 1) + m];
}

// pair and triangle forms from the u16 thresholds (cc_bin_table, after bin_table_kernel)
__global__ void bin_table_pack_kernel(int rows, uint16_t* __restrict__ table) {
  const uint16_t* t16 = table;
  uint32_t* pair = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(table) + bt_u16_bytes(rows));
  uint8_t* tri = reinterpret_cast<uint8_t*>(table) + bt_u16_bytes(rows) + bt_pair_bytes(rows);
  const int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (bt_pair_bytes(rows) && e < static_cast<int64_t>(rows) * NBINS) {
    const int i = static_cast<int>(e / NBINS), g = static_cast<int>(e - static_cast<int64_t>(i) * NBINS);
    pair[e] = static_cast<uint32_t>(t16[i * BT_ROW + g]) | (static_cast<uint32_t>(t16[i * BT_ROW + g + 1]) << 16);
  }
  if (bt_tri_bytes(rows) && e < static_cast<int64_t>(rows) * (rows + 1) / 2) {
    int i = static_cast<int>((sqrt(8.0 * static_cast<double>(e) + 1.0) - 1.0) * 0.5);
    while (static_cast<int64_t>(i) * (i + 1) / 2 > e) --i;
    while (static_cast<int64_t>(i + 1) * (i + 2) / 2 <= e) ++i;
    const uint32_t m = static_cast<uint32_t>(e - static_cast<int64_t>(i) * (i + 1) / 2);
    int b = 0;
    for (int k = 1; k < NBINS; ++k) b += m >= t16[i * BT_ROW + k] ? 1 : 0;
    tri[e] = static_cast<uint8_t>(b);
  }
}

// Exhaustive check of the division-free binning: for every pair (m <= i < rows) compare
// table_bin and table_bin_r (with the epilogue's own reciprocal 20 * rcp(i)) and, where the
// table holds them, the pair and triangle forms, against the direct numpy-exact consensus_bin;
// mismatches[0..3] count the disagreements of the four forms.
__global__ void bin_selftest_kernel(int rows, const float* __restrict__ edges,
                                    const uint16_t* __restrict__ table,
                                    unsigned long long* __restrict__ mismatches) {
  const int i = blockIdx.x;
  const float rt = i > 0 ? 20.0f * __builtin_amdgcn_rcpf(static_cast<float>(i)) : 0.0f;
  __shared__ float rtab_i[1];
  if (threadIdx.x == 0) rtab_i[0] = rt;
  __syncthreads();
  const uint32_t* pair = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + bt_u16_bytes(rows));
  const uint8_t* tri = reinterpret_cast<const uint8_t*>(table) + bt_u16_bytes(rows) + bt_pair_bytes(rows);
  unsigned long long bad0 = 0, bad1 = 0, bad2 = 0, bad3 = 0;
  for (int m = threadIdx.x; m <= i; m += blockDim.x) {
    const int want = consensus_bin(static_cast<uint32_t>(m), static_cast<uint32_t>(i), edges);
    bad0 += table_bin(static_cast<uint32_t>(m), static_cast<uint32_t>(i), table) != want;
    // table_bin_r / pair_bin read rtab[i]: point it at a one-entry array holding row i's reciprocal
    bad1 += table_bin_r(static_cast<uint32_t>(m), static_cast<uint32_t>(i), table, rtab_i - i) != want;
    if (bt_pair_bytes(rows)) bad2 += pair_bin(static_cast<uint32_t>(m), static_cast<uint32_t>(i), pair, rtab_i - i) != want;
    if (bt_tri_bytes(rows)) bad3 += tri_bin(static_cast<uint32_t>(m), static_cast<uint32_t>(i), tri) != want;
  }
  if (bad0) atomicAdd(&mismatches[0], bad0);
  if (bad1) atomicAdd(&mismatches[1], bad1);
  if (bad2) atomicAdd(&mismatches[2], bad2);
  if (bad3) atomicAdd(&mismatches[3], bad3);
}

// Load the HS label bytes of one row for one super-step into w[] (HS = 128 / KP for the i8
// kernels, 256 / KP for the FP4 kernels).
// Branch-free: an out-of-range row reads row 0 and is masked to 0xFF (= not sampled).
template <int HS>
__device__ __forceinline__ void load_labels(const uint8_t* rowp, bool valid, uint32_t (&w)[32]) {
  static_assert(HS >= 1 && HS <= 128, "at most 128 label bytes per row and step");
  const uint32_t msk = valid ? 0u : 0xFFFFFFFFu;
  if constexpr (HS >= 16) {
#pragma unroll
    for (int q = 0; q < HS / 16; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(rowp)[q];
      w[4 * q + 0] = v.x | msk;
      w[4 * q + 1] = v.y | msk;
      w[4 * q + 2] = v.z | msk;
      w[4 * q + 3] = v.w | msk;
    }
  } else if constexpr (HS == 8) {
    const uint2 v = *reinterpret_cast<const uint2*>(rowp);
    w[0] = v.x | msk;
    w[1] = v.y | msk;
  } else if constexpr (HS == 4) {
    w[0] = *reinterpret_cast<const uint32_t*>(rowp) | msk;
  } else if constexpr (HS == 2) {
    w[0] = 0xFFFF0000u | *reinterpret_cast<const uint16_t*>(rowp) | msk;
  } else {
    w[0] = 0xFFFFFF00u | *rowp | msk;
  }
}

__device__ __forceinline__ uint32_t spread01(uint32_t v) {  // bits {0, 8} -> bits {0, 16}
  return (v | (v << 8)) & 0x00010001u;
}

// Expand label bytes into 128 one-hot bytes (32 dwords): dword q holds virtual
// k = 4q .. 4q+3 with k = h_local * KP + c (KP = 1: k = h_local, sampled flag).
template <int KP>
__device__ __forceinline__ void expand(const uint32_t (&w)[32], uint32_t (&o)[32]) {
  if constexpr (KP == 1) {
#pragma unroll
    for (int q = 0; q < 32; ++q) o[q] = (~w[q] >> 7) & 0x01010101u;  // byte != 0xFF
  } else if constexpr (KP == 2) {
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const uint32_t x = w[p];
      const uint32_t is0 = ~x & 0x01010101u;               // label == 0
      const uint32_t is1 = x & ~(x >> 1) & 0x01010101u;    // label == 1 (0xFF excluded)
      o[2 * p + 0] = spread01(is0 & 0x101u) | (spread01(is1 & 0x101u) << 8);
      o[2 * p + 1] = spread01((is0 >> 16) & 0x101u) | (spread01((is1 >> 16) & 0x101u) << 8);
    }
  } else {
    constexpr int LOG = (KP == 4) ? 2 : (KP == 8) ? 3 : (KP == 16) ? 4 : (KP == 32) ? 5
                      : (KP == 64) ? 6 : 7;
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int k0 = 4 * q;
      const int h = k0 >> LOG;
      const uint32_t cq = static_cast<uint32_t>((k0 & (KP - 1)) >> 2);
      const uint32_t lab = (w[h >> 2] >> (8 * (h & 3))) & 0xFFu;
      o[q] = ((lab >> 2) == cq) ? (1u << ((lab & 3u) << 3)) : 0u;
    }
  }
}

// Dwords 8 kc .. 8 kc + 7 of expand() (virtual k = 32 kc .. 32 kc + 31).
template <int KP>
__device__ __forceinline__ void expand_chunk(const uint32_t (&w)[32], int kc, uint32_t (&o)[8]) {
  if constexpr (KP == 1) {
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (~w[8 * kc + q] >> 7) & 0x01010101u;  // byte != 0xFF
  } else if constexpr (KP == 2) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint32_t x = w[4 * kc + p];
      const uint32_t is0 = ~x & 0x01010101u;               // label == 0
      const uint32_t is1 = x & ~(x >> 1) & 0x01010101u;    // label == 1 (0xFF excluded)
      o[2 * p + 0] = spread01(is0 & 0x101u) | (spread01(is1 & 0x101u) << 8);
      o[2 * p + 1] = spread01((is0 >> 16) & 0x101u) | (spread01((is1 >> 16) & 0x101u) << 8);
    }
  } else {
    constexpr int LOG = (KP == 4) ? 2 : (KP == 8) ? 3 : (KP == 16) ? 4 : (KP == 32) ? 5
                      : (KP == 64) ? 6 : 7;
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) {
      const int k0 = 4 * (8 * kc + qq);
      const int h = k0 >> LOG;
      const uint32_t cq = static_cast<uint32_t>((k0 & (KP - 1)) >> 2);
      const uint32_t lab = (w[h >> 2] >> (8 * (h & 3))) & 0xFFu;
      o[qq] = ((lab >> 2) == cq) ? (1u << ((lab & 3u) << 3)) : 0u;
    }
  }
}

// FP4 (e2m1) one-hot, power-of-two KP >= 4: dwords 8 kc .. 8 kc + 7 of a 256-channel super-step
// (virtual k = h_local * KP + c, chunk kc = virtual k 64 kc .. 64 kc + 63).  Each dword holds 8
// channels as nibbles, 0x2 = 1.0 where the label matches (products 1.0 x 1.0, f32 sums: exact
// counts).  Nibble order inside a dword: channel 8 q + i at nibble i.  Any fixed placement is
// valid, since the A and B operands are expanded by this same code.
template <int KP>
__device__ __forceinline__ void expand_chunk_f4(const uint32_t (&w)[32], int kc, uint32_t (&o)[8]) {
  static_assert(KP >= 4 && (KP & (KP - 1)) == 0, "power-of-two KP >= 4");
  constexpr int LOG = (KP == 4) ? 2 : (KP == 8) ? 3 : (KP == 16) ? 4 : (KP == 32) ? 5 : (KP == 64) ? 6 : 7;
#pragma unroll
  for (int qq = 0; qq < 8; ++qq) {
    const int k0 = 64 * kc + 8 * qq;
    if constexpr (KP == 4) {  // two resamples per dword (h even: same label dword)
      const int h = k0 >> 2;
      const uint32_t l0 = (w[h >> 2] >> (8 * (h & 3))) & 0xFFu;
      const uint32_t l1 = (w[h >> 2] >> (8 * (h & 3) + 8)) & 0xFFu;
      o[qq] = (l0 < 4u ? (2u << (l0 << 2)) : 0u) | (l1 < 4u ? (2u << (16u + (l1 << 2))) : 0u);
    } else {  // one resample, channels 8 cq .. 8 cq + 7
      const int h = k0 >> LOG;
      const uint32_t cq = static_cast<uint32_t>((k0 & (KP - 1)) >> 3);
      const uint32_t lab = (w[h >> 2] >> (8 * (h & 3))) & 0xFFu;
      o[qq] = ((lab >> 3) == cq) ? (2u << ((lab & 7u) << 2)) : 0u;
    }
  }
}

// ---- exact-K channel packing (K not a power of two, K <= 32) -------------------------------
// A super-step holds HS = floor(128 / K) whole resamples at virtual k = h_local * K + c, and
// the HS*K..127 tail is zero: channels are no longer padded to the next power of two (at C3,
// K = 2..20, 1720 super-steps per tile instead of 2384).  Step s starts at label byte s * HS,
// which is not 16-B aligned: each row loads the chunks covering it and shifts them into place
// by the wave-uniform offset (ExactK::DW).
// Diagnostic build only (-DCC_CO_STAMPS): per-phase cycles of the co-association workgroups
// (thread 0 of each), summed into cc_co_stamp_acc: prologue, main loop, epilogue setup,
// binning, reduction; read with cc_co_stamps().
#ifdef CC_CO_STAMPS
__device__ unsigned long long cc_co_stamp_acc[8];
#define CO_STAMP(var) \
  __builtin_amdgcn_sched_barrier(0); \
  const unsigned long long var = __builtin_amdgcn_s_memtime(); \
  __builtin_amdgcn_sched_barrier(0)
#define CO_ACC(k, a, b) \
  if (KP > 1 && threadIdx.x == 0) atomicAdd(&cc_co_stamp_acc[k], (b) - (a))
#else
#define CO_STAMP(var)
#define CO_ACC(k, a, b)
#endif

// Two load forms, chosen per K by measurement (C3, tools/gpu_co3.sh): for K < 10 aligned 16-B
// chunks and a dword shift by selects; for K >= 10 dword-aligned 16-B loads from the dword holding
// the first byte, so only the byte shift remains (fewer VALU where steps are many).
template <int K, int VK = 128>
struct ExactK {
  static constexpr int HS = VK / K;                 // resamples per super-step (VK virtual k)
  static constexpr int NWX = (HS + 3) / 4;          // aligned label dwords of a step
  static constexpr bool DW = K >= 10;               // dword-aligned loads
  static constexpr int NC16 = DW ? (NWX + 1 + 3) / 4 : (HS + 15 + 15) / 16;
  static constexpr int RAW = 4 * NC16;
  static_assert(RAW >= NWX + (DW ? 1 : 4), "chunk cover");
};

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

// Raw dwords of step s of one row, as loaded: nothing touches them until realign, so the load
// stays in flight for a whole super-step.  No load goes past the row (the 16-B form re-reads
// the row's last 16 bytes for a chunk at or past ldl, a multiple of 16; realign fills those
// with 0xFF and applies the invalid-row mask).
template <int K, int VK>
__device__ __forceinline__ void load_raw(const uint8_t* rowp, int s, int ldl, uint32_t (&raw)[ExactK<K, VK>::RAW]) {
  using E = ExactK<K, VK>;
  if constexpr (E::DW) {
    const int a4 = (s * E::HS) & ~3;
#pragma unroll
    for (int c = 0; c < E::NC16; ++c) {
      const int o = a4 + 16 * c;
      u32x4_a4 v;
      if (o + 16 <= ldl) {  // wave-uniform
        v = *reinterpret_cast<const u32x4_a4*>(rowp + o);
      } else {  // the row's end (last step only): dword by dword
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[q] = (o + 4 * q + 4 <= ldl) ? *reinterpret_cast<const uint32_t*>(rowp + o + 4 * q) : 0xFFFFFFFFu;
      }
      raw[4 * c + 0] = v.x;
      raw[4 * c + 1] = v.y;
      raw[4 * c + 2] = v.z;
      raw[4 * c + 3] = v.w;
    }
  } else {
    const int a16 = (s * E::HS) & ~15;
#pragma unroll
    for (int c = 0; c < E::NC16; ++c) {  // branch-free: clamped re-reads, masked
      const int o = a16 + 16 * c;
      const uint4 v = *reinterpret_cast<const uint4*>(rowp + (o < ldl ? o : ldl - 16));
      raw[4 * c + 0] = v.x;
      raw[4 * c + 1] = v.y;
      raw[4 * c + 2] = v.z;
      raw[4 * c + 3] = v.w;
    }
  }
}

// Label bytes of step s in place (byte h of w = resample s * HS + h); resamples at or past Hpad
// (the last step's tail) read as 0xFF = not sampled.  The dword shift (16-B form) is a select on
// the wave-uniform offset (a switch made the compiler spill), the byte shift v_alignbyte.
template <int K, int VK>
__device__ __forceinline__ void realign(const uint32_t (&raw_in)[ExactK<K, VK>::RAW], int s, int Hpad, int ldl,
                                        bool valid, uint32_t (&w)[32]) {
  using E = ExactK<K, VK>;
  // every raw dword counts as read here: a loaded dword that realign does not need would
  // otherwise be reused as a temporary, and that write-after-load stalls on the label load
  // (issued one step ago) at the top of the next super-step instead of here
#pragma unroll
  for (int j = 0; j < E::RAW; ++j) asm volatile("" ::"v"(raw_in[j]));
  uint32_t raw[E::RAW];
#pragma unroll
  for (int j = 0; j < E::RAW; ++j) raw[j] = raw_in[j];
  if constexpr (!E::DW) {  // chunks at or past ldl (clamped re-reads) read as 0xFF
    const int a16 = (s * E::HS) & ~15;
#pragma unroll
    for (int j = 0; j < E::RAW; ++j)
      if (a16 + 16 * (j / 4) >= ldl) raw[j] = 0xFFFFFFFFu;  // wave-uniform
  }
  const int off = (s * E::HS) & (E::DW ? 3 : 15);  // wave-uniform
  const int bsh = off & 3;
  if constexpr (E::DW) {
#pragma unroll
    for (int i = 0; i < E::NWX; ++i) w[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], bsh);
  } else {
    const int dsh = off >> 2;
    auto at = [&](int j) __attribute__((always_inline)) { return j < E::RAW ? raw[j] : 0xFFFFFFFFu; };
    uint32_t sh[E::NWX + 1];  // dwords dsh .. dsh + NWX of raw
#pragma unroll
    for (int i = 0; i <= E::NWX; ++i) {
      const uint32_t x01 = (dsh & 1) ? at(i + 1) : at(i);
      const uint32_t x23 = (dsh & 1) ? at(i + 3) : at(i + 2);
      sh[i] = (dsh & 2) ? x23 : x01;
    }
#pragma unroll
    for (int i = 0; i < E::NWX; ++i) w[i] = __builtin_amdgcn_alignbyte(sh[i + 1], sh[i], bsh);
  }
  if (!valid) {  // a row past n: not sampled in any resample
#pragma unroll
    for (int i = 0; i < E::NWX; ++i) w[i] = 0xFFFFFFFFu;
  }
  const int rem = Hpad - s * E::HS;
  if (rem < E::HS) {  // wave-uniform: the last step
#pragma unroll
    for (int i = 0; i < E::NWX; ++i) {
      const int k = rem - 4 * i;
      w[i] |= (k >= 4) ? 0u : (k <= 0 ? 0xFFFFFFFFu : (0xFFFFFFFFu << (8 * k)));
    }
  }
}

// Dwords 8 kc .. 8 kc + 7 of the exact-K one-hot: byte j = [label(j / K) == j % K] for
// j < HS * K, else 0.  Per dword: v_perm gathers the (at most two) label bytes its 4 channels
// belong to, XOR with the channel numbers, and a carry-free zero-byte test gives the 0/1 bytes.
template <int K>
__device__ __forceinline__ void expand_chunk_exact(const uint32_t (&w)[32], int kc, uint32_t (&o)[8]) {
  using E = ExactK<K>;
#pragma unroll
  for (int qq = 0; qq < 8; ++qq) {
    const int j0 = 4 * (8 * kc + qq);
    if (j0 >= E::HS * K) {
      o[qq] = 0u;
      continue;
    }
    const int dA = (j0 / K) >> 2;
    uint32_t sel = 0, cc = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int j = j0 + b;
      const bool ok = j < E::HS * K;
      sel |= static_cast<uint32_t>(ok ? (j / K - 4 * dA) : 0x0C) << (8 * b);
      cc |= static_cast<uint32_t>(ok ? (j % K) : 0xFE) << (8 * b);
    }
    const uint32_t s1 = w[dA];
    const uint32_t s0 = (dA + 1 < E::NWX) ? w[dA + 1] : s1;
    const uint32_t x = __builtin_amdgcn_perm(s0, s1, sel) ^ cc;
    const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    o[qq] = (~(t | x) & 0x80808080u) >> 7;
  }
}

// 0x80 in byte b where label(j / K) == j % K for channel j = j0 + b (j < HS K), else 0: v_perm
// gathers the (at most two) label bytes of the 4 channels, XOR with the channel numbers, and a
// carry-free zero-byte test.
template <int K, int VK>
__device__ __forceinline__ uint32_t match4(const uint32_t (&w)[32], int j0) {
  using E = ExactK<K, VK>;
  if (j0 >= E::HS * K) return 0u;
  const int dA = (j0 / K) >> 2;
  uint32_t sel = 0, cc = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int j = j0 + b;
    const bool ok = j < E::HS * K;
    sel |= static_cast<uint32_t>(ok ? (j / K - 4 * dA) : 0x0C) << (8 * b);
    cc |= static_cast<uint32_t>(ok ? (j % K) : 0xFE) << (8 * b);
  }
  const uint32_t s1 = w[dA];
  const uint32_t s0 = (dA + 1 < E::NWX) ? w[dA + 1] : s1;
  const uint32_t x = __builtin_amdgcn_perm(s0, s1, sel) ^ cc;
  const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(t | x) & 0x80808080u;
}

// FP4 exact-K one-hot: dwords 8 kc .. 8 kc + 7 of a 256-channel super-step.  Byte b of dword q
// holds channel 8 q + b (low nibble) and 8 q + 4 + b (high nibble), 0x2 = 1.0 where it matches.
template <int K>
__device__ __forceinline__ void expand_chunk_exact_f4(const uint32_t (&w)[32], int kc, uint32_t (&o)[8]) {
#pragma unroll
  for (int qq = 0; qq < 8; ++qq) {
    const int j0 = 8 * (8 * kc + qq);
    o[qq] = (match4<K, 256>(w, j0) >> 6) | (match4<K, 256>(w, j0 + 4) >> 2);
  }
}

typedef int v8i __attribute__((ext_vector_type(8)));

// One 16-B LDS-DMA piece per lane (global_load_lds_dwordx4: lane l lands at M0 + 16 l), issued
// from inline asm with the wave-uniform LDS base in M0; completion is awaited explicitly with a
// vmcnt(0) before the barrier that publishes the data.  No compiler-generated code in these
// kernels uses M0 (the backend reserves M0, so an "m0" clobber would be ignored); the CPU test
// tests/test_isa.py checks that on the ISA of every kernel in libccmi.so.
__device__ __forceinline__ void dma16(const void* g, const void* lds_base) {
  const unsigned la = static_cast<unsigned>(reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) const char*)lds_base));
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(__builtin_amdgcn_readfirstlane(la)), "v"(g));
}

// expansion VALU interleaved per MFMA in the FP4 main loop (power-of-two / exact-K forms)
#ifndef CO_F4_V
#define CO_F4_V 10
#endif
#ifndef CO_F4_EXV
#define CO_F4_EXV 14
#endif

// One MFMA step of the tile loop on the operand pair (a, b): i8 (32 virtual k) or FP4 (64).
// FP4: v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1 operands (format 4) and unit block scales
// (E8M0 127 = 2^0); only the low 4 dwords of each operand are read for FP4.
template <bool F4, class Acc>
__device__ __forceinline__ Acc mfma_step(const v4i& a, const v4i& b, const Acc& c) {
  if constexpr (F4) {
    const v8i a8 = __builtin_shufflevector(a, a, 0, 1, 2, 3, -1, -1, -1, -1);
    const v8i b8 = __builtin_shufflevector(b, b, 0, 1, 2, 3, -1, -1, -1, -1);
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 127, 0, 127);
  } else {
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
  }
}

// Accumulator element as an unsigned count (FP4 accumulates exact integers in f32).
__device__ __forceinline__ uint32_t count_of(int v) { return static_cast<uint32_t>(v); }
__device__ __forceinline__ uint32_t count_of(float v) { return static_cast<uint32_t>(v); }

// F4: the co-association kernels (KP >= 3) contract FP4 one-hot operands, 256 virtual k per
// super-step (4 chunks of 64): the same LDS bytes and MFMA cycles per step as the i8 form's 128
// virtual k, so the LDS traffic and the matrix-pipe time per count are halved.  The co-sampling
// kernel (KP = 1, 0/1 flags of 128 resamples per step) and K <= 2 keep the i8 form.
template <int KP, bool F4>
__global__ __launch_bounds__(NT, 1) void tiles_kernel(
    const uint8_t* __restrict__ labels, int n, int ldl, int Hpad, int64_t tile_begin,
    uint16_t* __restrict__ I_tiles_out, const uint16_t* __restrict__ I_tiles_in,
    const float* __restrict__ edges, unsigned long long* __restrict__ bin_counts,
    int32_t* __restrict__ full_out, const uint16_t* __restrict__ btab, int bt_rows) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  constexpr int VK = F4 ? 256 : 128;  // virtual k per super-step
  constexpr int HS = VK / KP;  // resamples per super-step
  constexpr bool EX = (KP & (KP - 1)) != 0;  // exact-K packing (K = KP not a power of two)
  static_assert(!F4 || KP >= 3, "FP4 form: K >= 3");
  using Acc = std::conditional_t<F4, v16f, v16i>;

  CO_STAMP(st0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 2;  // 0..1 : 128-row half
  const int wc = wave & 3;   // 0..3 : 64-col quarter
  const int nb = (n + T - 1) / T;
  // XCD-aware tile order: blocks b and b + 8 share an XCD (round-robin dealing), so XCD x gets
  // the contiguous tile range [x q + min(x, r), ...): its CUs work on neighbouring tiles of one
  // row band at a time and share the A-side label rows through that XCD's L2.
  const int nblk = static_cast<int>(gridDim.x), bx = static_cast<int>(blockIdx.x);
  const int xq = nblk >> 3, xr = nblk & 7, xcd = bx & 7;
  const int64_t t = tile_begin + xcd * xq + (xcd < xr ? xcd : xr) + (bx >> 3);
  int bi, bj;
  tile_coords(t, nb, bi, bj);

  // Expansion role: one row per thread. side 0 = tile rows (A), side 1 = tile cols (B).
  const int side = tid >> 8;
  const int erow = tid & 255;
  const int grow = (side ? bj : bi) * T + erow;
  const bool evalid = grow < n;
  const uint8_t* rowp = labels + static_cast<int64_t>(evalid ? grow : 0) * ldl;
  const int erb = erow >> 5, er = erow & 31;
  char* const wbase = lds + side * SIDE + erb * KC * FRAG + er * 16;

  const int nsteps = EX ? (Hpad + HS - 1) / HS : Hpad / HS;
  Acc acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = Acc{};

  // Label prefetch depth: two steps ahead for the co-association kernels (<= 16 label bytes
  // per row and step); the co-sampling kernel (128 bytes per row and step) loads one step
  // ahead into a single buffer and expands after the MFMAs (its registers would spill).
  constexpr bool PF2 = KP > 1;
  constexpr int NWD = (HS + 3) / 4;
  uint32_t w[32], wn[PF2 ? NWD : 1], o[32];
  constexpr int KX = EX ? KP : 3;  // (a valid instantiation when unused)
  constexpr int NRW = EX ? ExactK<KX, VK>::RAW : 1;
  uint32_t raw1[NRW];  // exact K: raw chunks of step s+2 (one step in flight; two measured slower)
  // the one-hot dwords of chunk kc of the step whose labels are in w
  auto expand_kc = [&](int kc, uint32_t (&oc)[8]) __attribute__((always_inline)) {
    if constexpr (EX && F4)
      expand_chunk_exact_f4<KX>(w, kc, oc);
    else if constexpr (EX)
      expand_chunk_exact<KX>(w, kc, oc);
    else if constexpr (F4)
      expand_chunk_f4<(KP >= 4 ? KP : 4)>(w, kc, oc);
    else
      expand_chunk<KP>(w, kc, oc);
  };
  // step 0's one-hot straight into LDS buffer 0, chunk by chunk
  auto store_step0 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      uint32_t oc[8];
      expand_kc(kc, oc);
#pragma unroll
      for (int g = 0; g < 2; ++g)
        *reinterpret_cast<uint4*>(wbase + kc * FRAG + g * 512) =
            make_uint4(oc[g * 4 + 0], oc[g * 4 + 1], oc[g * 4 + 2], oc[g * 4 + 3]);
    }
  };
  if constexpr (EX) {
    load_raw<KX, VK>(rowp, 0, ldl, raw1);
    realign<KX, VK>(raw1, 0, Hpad, ldl, evalid, w);
    store_step0();
    load_raw<KX, VK>(rowp, nsteps > 1 ? 1 : 0, ldl, raw1);
    realign<KX, VK>(raw1, nsteps > 1 ? 1 : 0, Hpad, ldl, evalid, w);  // step 1
    load_raw<KX, VK>(rowp, nsteps > 2 ? 2 : 0, ldl, raw1);  // step 2
  } else if constexpr (PF2) {
    load_labels<HS>(rowp, evalid, w);
    store_step0();
  } else {
    load_labels<HS>(rowp, evalid, w);
    expand<KP>(w, o);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int g = 0; g < 2; ++g)
        *reinterpret_cast<uint4*>(wbase + kc * FRAG + g * 512) =
            make_uint4(o[kc * 8 + g * 4 + 0], o[kc * 8 + g * 4 + 1], o[kc * 8 + g * 4 + 2],
                       o[kc * 8 + g * 4 + 3]);
  }
  if constexpr (PF2 && !EX) {
    load_labels<HS>(rowp + (nsteps > 1 ? HS : 0), evalid, w);  // step 1
    uint32_t t32[32];
    load_labels<HS>(rowp + (nsteps > 2 ? 2 * HS : 0), evalid, t32);  // step 2
#pragma unroll
    for (int q = 0; q < NWD; ++q) wn[q] = t32[q];
  }
  __syncthreads();
  CO_STAMP(st1);
  CO_ACC(0, st0, st1);

  for (int s = 0; s < nsteps; ++s) {
    const bool more = (s + 1) < nsteps;
    const char* rb = lds + (s & 1) * BUF;
    char* wb = wbase + ((s + 1) & 1) * BUF;
    if constexpr (!PF2)
      if (more) load_labels<HS>(rowp + (s + 1) * HS, evalid, w);
    // operand fragments double-buffered across the k-chunks: the reads of chunk kc+1 are in
    // flight while chunk kc's MFMAs issue (only the first chunk's read latency is exposed)
    v4i a[2][4], b[2][2];
    auto frags = [&](int kc, v4i (&fa)[4], v4i (&fb)[2]) __attribute__((always_inline)) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
        fa[mi] = *reinterpret_cast<const v4i*>(rb + ((wr * 4 + mi) * KC + kc) * FRAG + lane * 16);
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
        fb[nj] = *reinterpret_cast<const v4i*>(rb + SIDE + ((wc * 2 + nj) * KC + kc) * FRAG +
                                               lane * 16);
    };
    frags(0, a[0], b[0]);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int cb = kc & 1;
      if (kc + 1 < KC) frags(kc + 1, a[cb ^ 1], b[cb ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj)
          acc[mi][nj] = mfma_step<F4>(a[cb][mi], b[cb][nj], acc[mi][nj]);
      if constexpr (PF2) {
        // one-hot expansion of step s+1 (labels prefetched two steps ahead) interleaved with
        // this step's MFMAs: chunk kc's 8 dwords are expanded and stored right after chunk
        // kc's MFMAs issue, so the vector work runs in the MFMA shadows
        // (the stores are unconditional: on the last step they land in the buffer nobody reads)
        uint32_t oc[8];
        expand_kc(kc, oc);
#pragma unroll
        for (int g = 0; g < 2; ++g)
          *reinterpret_cast<uint4*>(wb + kc * FRAG + g * 512) =
              make_uint4(oc[g * 4 + 0], oc[g * 4 + 1], oc[g * 4 + 2], oc[g * 4 + 3]);
        // issue order: each MFMA followed by a few expansion VALU ops, which then execute in
        // that MFMA's 32-cycle shadow instead of after the whole MFMA block
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, F4 ? (EX ? CO_F4_EXV : CO_F4_V) : ((EX && KP >= 10) ? 9 : 6), 0);  // VALU per MFMA
        }
        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);    // the 2 LDS stores
      }
    }
    if constexpr (EX) {
      // w <- step s+2 (loaded one step ago), raw1 <- step s+3
      realign<KX, VK>(raw1, (s + 2) < nsteps ? s + 2 : s, Hpad, ldl, evalid, w);
      load_raw<KX, VK>(rowp, (s + 3) < nsteps ? s + 3 : s, ldl, raw1);
    } else if constexpr (PF2) {
      // rotate the label prefetch: w <- step s+2, wn <- step s+3 (clamped re-reads at the end)
#pragma unroll
      for (int q = 0; q < NWD; ++q) w[q] = wn[q];
      uint32_t t32[32];
      load_labels<HS>(rowp + ((s + 3) < nsteps ? s + 3 : s) * HS, evalid, t32);
#pragma unroll
      for (int q = 0; q < NWD; ++q) wn[q] = t32[q];
    } else if (more) {
      expand<KP>(w, o);
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          *reinterpret_cast<uint4*>(wb + kc * FRAG + g * 512) =
              make_uint4(o[kc * 8 + g * 4 + 0], o[kc * 8 + g * 4 + 1], o[kc * 8 + g * 4 + 2],
                         o[kc * 8 + g * 4 + 3]);
    }
    __syncthreads();
  }

  // ---- epilogue ------------------------------------------------------------
  CO_STAMP(st2);
  CO_ACC(1, st1, st2);
  const int64_t tl = t - tile_begin;
  const bool diag = (bi == bj);
  const int row0 = bi * T + wr * 128 + 4 * (lane >> 5);
  const int col0 = bj * T + wc * 64 + (lane & 31);

  if constexpr (KP == 1) {
    // thread-contiguous tile layout: thread tid's 128 accumulator elements, in (mi, nj, v)
    // order, are elements 128 tid .. 128 tid + 127 (16 x 16-B stores; the co-association
    // epilogue reads them back with 16-B loads)
    uint4* it4 = reinterpret_cast<uint4*>(I_tiles_out + tl * (T * T) + 128 * tid);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint32_t pk[4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            pk[q] = (static_cast<uint32_t>(acc[mi][nj][8 * h + 2 * q]) & 0xFFFFu) |
                    (static_cast<uint32_t>(acc[mi][nj][8 * h + 2 * q + 1]) << 16);
          it4[(mi * 2 + nj) * 2 + h] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int val = acc[mi][nj][v];
          if (full_out) {
            const int i = row0 + mi * 32 + (v & 3) + 8 * (v >> 2);
            const int j = col0 + nj * 32;
            if (i < n && j < n) {
              full_out[static_cast<int64_t>(i) * n + j] = val;
              if (!diag) full_out[static_cast<int64_t>(j) * n + i] = val;
            }
          }
        }
  } else {
    // [NBINS][NT] private counters, the 21 edges, the per-wave sums and (small H) the bin
    // threshold table, reusing the operand LDS.
    uint32_t* hist = reinterpret_cast<uint32_t*>(lds);
    float* es = reinterpret_cast<float*>(lds + NBINS * NT * sizeof(uint32_t));
    uint16_t* tab = reinterpret_cast<uint16_t*>(lds + BT_OFF);
    const uint32_t* ptab = reinterpret_cast<const uint32_t*>(lds + BT_OFF);
    const uint8_t* ttab = reinterpret_cast<const uint8_t*>(lds + BT_OFF);
    const int form = bt_form(bt_rows);  // launch-uniform
    // the staged form's bytes and where it sits in the global table; the reciprocals follow it
    const int64_t fbytes = form == BT_TRI ? bt_tri_bytes(bt_rows)
                                          : (form == BT_PAIR ? bt_pair_bytes(bt_rows) : bt_u16_bytes(bt_rows));
    const int64_t fsrc = form == BT_TRI ? bt_u16_bytes(bt_rows) + bt_pair_bytes(bt_rows)
                                        : (form == BT_PAIR ? bt_u16_bytes(bt_rows) : 0);
    float* rtab_w = reinterpret_cast<float*>(lds + BT_OFF + fbytes);
    if (btab) {
      // the table by LDS-DMA, every 1-KiB piece in flight at once (lane l of wave w copies 16 B
      // of pieces w, w + 8, ...): the copy loop it replaces waited on each 16-B load before
      // its LDS store, 4-6 dependent L2 round trips per tile
      const int vecs = static_cast<int>(fbytes / 16);
      const char* src = reinterpret_cast<const char*>(btab) + fsrc;
      for (int pc = wave; pc * 64 < vecs; pc += NW)
        if (pc * 64 + lane < vecs) dma16(src + (static_cast<int64_t>(pc) * 64 + lane) * 16, lds + BT_OFF + pc * 1024);
    }
#pragma unroll
    for (int b = 0; b < NBINS; ++b) hist[b * NT + tid] = 0;
    if (tid <= NBINS) es[tid] = edges[tid];
    if (btab && form != BT_TRI)
      for (int r = tid; r < bt_rows; r += NT)
        rtab_w[r] = r > 0 ? 20.0f * __builtin_amdgcn_rcpf(static_cast<float>(r)) : 0.0f;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the DMA pieces (opaque to the compiler) landed
    __syncthreads();
    CO_STAMP(st3);
    CO_ACC(2, st2, st3);
    const float* rtab = rtab_w;
    const uint4* it4 = reinterpret_cast<const uint4*>(I_tiles_in + tl * (T * T) + 128 * tid);
    // Interior tiles (off the diagonal, every column < n; all but a sliver of the triangle)
    // bin every element with no pair mask, through the staged table: batched LDS passes per
    // block of 16 elements (all reads of a pass in flight together, then the counter adds).
    const bool interior = btab && !diag && (bj + 1) * T <= n && !full_out;
    if (interior && form == BT_TRI) {
      // the next block's two co-sampling loads are issued before this block's table reads and
      // counter adds (one block ahead: each block waited on its own HBM round trip)
      uint4 n0 = it4[0], n1 = it4[1];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj) {
          const int blk = mi * 2 + nj;
          const uint4 q0 = n0, q1 = n1;
          if (blk < 7) {
            n0 = it4[(blk + 1) * 2];
            n1 = it4[(blk + 1) * 2 + 1];
          }
          const uint32_t iw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
          uint32_t bb[16];
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const uint32_t iv = (iw[v >> 1] >> (16 * (v & 1))) & 0xFFFFu;
            bb[v] = tri_bin(count_of(acc[mi][nj][v]), iv, ttab);
          }
#pragma unroll
          for (int v = 0; v < 16; ++v) asm volatile("" : "+v"(bb[v]));
#pragma unroll
          for (int v = 0; v < 16; ++v) atomicAdd(&hist[bb[v] * NT + tid], 1u);
        }
    } else if (interior && form == BT_PAIR) {
      uint4 n0 = it4[0], n1 = it4[1];  // one block ahead, as above
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj) {
          const int blk = mi * 2 + nj;
          const uint4 q0 = n0, q1 = n1;
          if (blk < 7) {
            n0 = it4[(blk + 1) * 2];
            n1 = it4[(blk + 1) * 2 + 1];
          }
          const uint32_t iw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
          uint32_t ival[16];
          float rc[16];
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            ival[v] = (iw[v >> 1] >> (16 * (v & 1))) & 0xFFFFu;
            rc[v] = rtab[ival[v]];
          }
#pragma unroll
          for (int v = 0; v < 16; ++v) asm volatile("" : "+v"(rc[v]));
          int g[16];
          uint32_t pr[16];
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            g[v] = static_cast<int>(acc[mi][nj][v] * rc[v]);  // the accumulator is the exact count
            g[v] = g[v] > NBINS - 1 ? NBINS - 1 : g[v];
            pr[v] = ptab[ival[v] * NBINS + g[v]];
          }
#pragma unroll
          for (int v = 0; v < 16; ++v) asm volatile("" : "+v"(pr[v]));
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const uint32_t m = count_of(acc[mi][nj][v]);
            const int b = g[v] - (m < (pr[v] & 0xFFFFu) ? 1 : 0) + (m >= (pr[v] >> 16) ? 1 : 0);
            atomicAdd(&hist[b * NT + tid], 1u);
          }
        }
    } else if (interior) {
      uint4 n0 = it4[0], n1 = it4[1];  // one block ahead, as above
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj) {
          const int blk = mi * 2 + nj;
          const uint4 q0 = n0, q1 = n1;
          if (blk < 7) {
            n0 = it4[(blk + 1) * 2];
            n1 = it4[(blk + 1) * 2 + 1];
          }
          const uint32_t iw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
          // table_bin_r for the block's 16 elements in three batched LDS passes (reciprocals,
          // then both thresholds, then the counter adds): one element at a time, every
          // element was two dependent LDS round trips, each behind the previous add
          uint32_t ival[16];
          float rc[16];
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            ival[v] = (iw[v >> 1] >> (16 * (v & 1))) & 0xFFFFu;
            rc[v] = rtab[ival[v]];
          }
#pragma unroll
          for (int v = 0; v < 16; ++v) asm volatile("" : "+v"(rc[v]));
          int g[16];
          uint32_t lo[16], hi[16];
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const uint32_t m = count_of(acc[mi][nj][v]);
            g[v] = static_cast<int>(static_cast<float>(m) * rc[v]);
            g[v] = g[v] > NBINS - 1 ? NBINS - 1 : g[v];
            const uint16_t* row = tab + ival[v] * BT_ROW;
            lo[v] = row[g[v]];
            hi[v] = row[g[v] + 1];
          }
#pragma unroll
          for (int v = 0; v < 16; ++v) asm volatile("" : "+v"(lo[v]), "+v"(hi[v]));
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const uint32_t m = count_of(acc[mi][nj][v]);
            const int b = g[v] - (m < lo[v] ? 1 : 0) + (m >= hi[v] ? 1 : 0);
            atomicAdd(&hist[b * NT + tid], 1u);
          }
        }
    } else {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj) {
        const uint4 q0 = it4[(mi * 2 + nj) * 2], q1 = it4[(mi * 2 + nj) * 2 + 1];
        const uint32_t iw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const uint32_t ival = (iw[v >> 1] >> (16 * (v & 1))) & 0xFFFFu;
          const int val = static_cast<int>(count_of(acc[mi][nj][v]));
          const int i = row0 + mi * 32 + (v & 3) + 8 * (v >> 2);
          const int j = col0 + nj * 32;
          if (i < j && j < n) {
            const int b = !btab ? consensus_bin(static_cast<uint32_t>(val), ival, es)
                        : form == BT_TRI ? tri_bin(static_cast<uint32_t>(val), ival, ttab)
                        : form == BT_PAIR ? pair_bin(static_cast<uint32_t>(val), ival, ptab, rtab)
                                          : table_bin(static_cast<uint32_t>(val), ival, tab);
            atomicAdd(&hist[b * NT + tid], 1u);
          }
          if (full_out && i < n && j < n) {
            full_out[static_cast<int64_t>(i) * n + j] = val;
            if (!diag) full_out[static_cast<int64_t>(j) * n + i] = val;
          }
        }
      }
    }
    CO_STAMP(st4);
    CO_ACC(3, st3, st4);
    // per-bin totals: 16 threads per bin sum its 512 counters from LDS (16-B reads, the 16
    // threads of a bin cover 256 contiguous bytes per read: conflict-free), then reduce
    // within their 16 lanes: one global atomic per bin and tile (20 contended words: keep it
    // at one per bin)
    __syncthreads();
    if (tid < NBINS * 16) {
      const int b = tid >> 4, part = tid & 15;
      const uint4* src = reinterpret_cast<const uint4*>(hist + b * NT) + part;
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < NT / 64; ++k) {
        const uint4 v = src[16 * k];
        c += v.x + v.y + v.z + v.w;
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) c += __shfl_xor(c, o);
      if (part == 0 && c) atomicAdd(&bin_counts[b], static_cast<unsigned long long>(c));
    }
    CO_STAMP(st5);
    CO_ACC(4, st4, st5);
  }
}

__global__ void scatter_labels_kernel(const int32_t* __restrict__ idx, const int32_t* __restrict__ lab,
                                      int H, int m, int n, uint8_t* __restrict__ out, int ldl) {
  const int64_t total = static_cast<int64_t>(H) * m;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int h = static_cast<int>(e / m);
    const int row = idx[e];
    if (row < 0 || row >= n) continue;
    out[static_cast<int64_t>(row) * ldl + h] = lab ? static_cast<uint8_t>(lab[e]) : 0;
  }
}

// dst[r * ld_dst + col_dst + j] = src[r * ld_src + col_src + j] for r < rows, j < width: a
// window of resample columns between two sample-major label matrices (the multi-GPU label
// exchange packs a rank's own columns before the all-gather and places every rank's columns
// after it).  One thread per byte of the window; consecutive threads read consecutive bytes.
__global__ void copy_label_columns_kernel(const uint8_t* __restrict__ src, int64_t ld_src, int col_src,
                                          uint8_t* __restrict__ dst, int64_t ld_dst, int col_dst,
                                          int64_t rows, int width) {
  const int64_t total = rows * width;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t r = e / width;
    const int j = static_cast<int>(e - r * width);
    dst[r * ld_dst + col_dst + j] = src[r * ld_src + col_src + j];
  }
}

// C = f32(M) / f32(f64(I) + 1e-6), C_ii = 1 (CC.py:372-373), one HBM stream of 12 bytes per
// element.  n % 4 == 0 and 16-B aligned M, I, C (then every row is): a workgroup per row (grid-stride over rows), each
// thread 4 elements per access (dwordx4 loads of M and I, one dwordx4 store), 4 accesses in flight;
// no per-element index division.  Otherwise the flat form below.
typedef int cc_i4 __attribute__((ext_vector_type(4)));
typedef float cc_f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) consensus_rows_kernel(const int32_t* __restrict__ M,
                                                             const int32_t* __restrict__ I, int n,
                                                             float* __restrict__ C) {
  constexpr int U = 4;
  const int nv = n >> 2;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const size_t rb = static_cast<size_t>(i) * static_cast<size_t>(nv);
    const cc_i4* Mr = reinterpret_cast<const cc_i4*>(M) + rb;
    const cc_i4* Ir = reinterpret_cast<const cc_i4*>(I) + rb;
    cc_f4* Cr = reinterpret_cast<cc_f4*>(C) + rb;
    for (int v0 = threadIdx.x; v0 < nv; v0 += U * 256) {
      cc_i4 mv[U], iv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int v = v0 + u * 256;
        if (v < nv) {
          mv[u] = __builtin_nontemporal_load(Mr + v);
          iv[u] = __builtin_nontemporal_load(Ir + v);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int v = v0 + u * 256;
        if (v < nv) {
          cc_f4 c;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float fi = static_cast<float>(static_cast<double>(iv[u][q]) + 1e-6);
            c[q] = (4 * v + q == i) ? 1.0f : static_cast<float>(mv[u][q]) / fi;
          }
          __builtin_nontemporal_store(c, Cr + v);
        }
      }
    }
  }
}

__global__ void consensus_kernel(const int32_t* __restrict__ M, const int32_t* __restrict__ I,
                                 int n, float* __restrict__ C) {
  const int64_t total = static_cast<int64_t>(n) * n;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t i = e / n, j = e - i * n;
    const float fi = static_cast<float>(static_cast<double>(I[e]) + 1e-6);
    C[e] = (i == j) ? 1.0f : static_cast<float>(M[e]) / fi;
  }
}

int check_common(const char* fn, const void* labels, int n, int ldl, int Hpad, int64_t tb,
                 int64_t te) {
  if (!labels || n <= 0 || Hpad <= 0 || Hpad % 128 != 0 || ldl < Hpad || ldl % 16 != 0) {
    cc::set_error(std::string(fn) + ": bad labels/n/ldl/Hpad (Hpad % 128 == 0, ldl >= Hpad, ldl % 16 == 0)");
    return CC_ERR_ARG;
  }
  if (reinterpret_cast<uintptr_t>(labels) & 15) {
    cc::set_error(std::string(fn) + ": labels_nh must be 16-B aligned (16-B row loads)");
    return CC_ERR_ARG;
  }
  if (Hpad > 65535) {
    cc::set_error(std::string(fn) + ": Hpad > 65535 overflows the uint16 co-sampling tiles");
    return CC_ERR_ARG;
  }
  const int64_t nt = cc_num_tiles(n);
  if (tb < 0 || te < tb || te > nt) {
    cc::set_error(std::string(fn) + ": tile range outside [0, num_tiles]");
    return CC_ERR_ARG;
  }
  return CC_OK;
}

int launch_status(const char* fn) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cc::set_error(std::string(fn) + ": " + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}

template <int KP, bool F4 = false>
void launch_tiles(dim3 grid, hipStream_t st, const uint8_t* lab, int n, int ldl, int Hpad,
                  int64_t tb, uint16_t* Iout, const uint16_t* Iin, const float* edges,
                  unsigned long long* counts, int32_t* full, const uint16_t* btab = nullptr,
                  int bt_rows = 0) {
  hipLaunchKernelGGL((tiles_kernel<KP, F4>), grid, dim3(NT), 0, st, lab, n, ldl, Hpad, tb, Iout, Iin,
                     edges, counts, full, btab, bt_rows);
}

}  // namespace

extern "C" int64_t cc_num_tiles(int n) {
  if (n <= 0) return 0;
  const int64_t nb = (n + T - 1) / T;
  return nb * (nb + 1) / 2;
}

extern "C" int cc_scatter_labels(const int32_t* idx_hm, const int32_t* labels_hm, int H, int m,
                                 int n, int8_t* labels_nh, int ldl, void* stream) {
  if (!idx_hm || !labels_nh || H < 0 || m < 0 || n <= 0 || ldl < H) {
    cc::set_error("cc_scatter_labels: bad arguments (ldl >= H required)");
    return CC_ERR_ARG;
  }
  const int64_t total = static_cast<int64_t>(H) * m;
  if (total == 0) return CC_OK;
  int blocks = static_cast<int>(std::min<int64_t>((total + 255) / 256, 8192));
  hipLaunchKernelGGL(scatter_labels_kernel, dim3(blocks), dim3(256), 0,
                     static_cast<hipStream_t>(stream), idx_hm, labels_hm, H, m, n,
                     reinterpret_cast<uint8_t*>(labels_nh), ldl);
  return launch_status("cc_scatter_labels");
}

extern "C" int cc_copy_label_columns(const uint8_t* src, int64_t ld_src, int col_src, uint8_t* dst,
                                     int64_t ld_dst, int col_dst, int64_t rows, int width, void* stream) {
  if (rows < 0 || width < 0 || col_src < 0 || col_dst < 0 || col_src + static_cast<int64_t>(width) > ld_src ||
      col_dst + static_cast<int64_t>(width) > ld_dst || ((!src || !dst) && rows * width > 0)) {
    cc::set_error("cc_copy_label_columns: bad arguments (the window must lie inside both row strides)");
    return CC_ERR_ARG;
  }
  const int64_t total = rows * width;
  if (total == 0) return CC_OK;
  const int blocks = static_cast<int>(std::min<int64_t>((total + 255) / 256, 16384));
  hipLaunchKernelGGL(copy_label_columns_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     src, ld_src, col_src, dst, ld_dst, col_dst, rows, width);
  return launch_status("cc_copy_label_columns");
}

extern "C" int cc_cosample(const int8_t* labels_nh, int n, int ldl, int Hpad, int64_t tile_begin,
                           int64_t tile_end, uint16_t* I_tiles, int32_t* I_full, void* stream) {
  int rc = check_common("cc_cosample", labels_nh, n, ldl, Hpad, tile_begin, tile_end);
  if (rc) return rc;
  if (tile_end == tile_begin) return CC_OK;  // an empty band (a rank with no tiles)
  if (!I_tiles || (reinterpret_cast<uintptr_t>(I_tiles) & 15)) {
    cc::set_error("cc_cosample: I_tiles is NULL or not 16-B aligned");
    return CC_ERR_ARG;
  }
  const int64_t ntl = tile_end - tile_begin;
  if (ntl == 0) return CC_OK;
  if (ntl > 0x7fffffff) {
    cc::set_error("cc_cosample: too many tiles for one launch");
    return CC_ERR_ARG;
  }
  launch_tiles<1>(dim3(static_cast<unsigned>(ntl)), static_cast<hipStream_t>(stream),
                  reinterpret_cast<const uint8_t*>(labels_nh), n, ldl, Hpad, tile_begin, I_tiles,
                  nullptr, nullptr, nullptr, I_full);
  return launch_status("cc_cosample");
}

// table: rows * 21 uint16, allocated to a multiple of 16 B (cc_coassoc copies it in 16-B pieces)
extern "C" size_t cc_bin_table_bytes(int rows) {
  if (rows <= 0 || rows > BT_MAX_ROWS) return 0;
  return static_cast<size_t>(bt_u16_bytes(rows) + bt_pair_bytes(rows) + bt_tri_bytes(rows));
}

extern "C" int cc_bin_table(int rows, const float* edges, uint16_t* table, size_t table_bytes, void* stream) {
  if (rows <= 0 || rows > BT_MAX_ROWS || !edges || !table || table_bytes < cc_bin_table_bytes(rows)) {
    cc::set_error("cc_bin_table: bad arguments (1 <= rows <= cc_bin_table_max_rows(), "
                  "table_bytes >= cc_bin_table_bytes(rows))");
    return CC_ERR_ARG;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const int total = rows * BT_ROW;
  hipLaunchKernelGGL(bin_table_kernel, dim3((total + 255) / 256), dim3(256), 0, st, rows, edges, table);
  const int64_t packed = std::max<int64_t>(bt_pair_bytes(rows) ? static_cast<int64_t>(rows) * NBINS : 0,
                                           bt_tri_bytes(rows) ? static_cast<int64_t>(rows) * (rows + 1) / 2 : 0);
  if (packed > 0)
    hipLaunchKernelGGL(bin_table_pack_kernel, dim3(static_cast<unsigned>((packed + 255) / 256)), dim3(256), 0, st,
                       rows, table);
  return launch_status("cc_bin_table");
}

extern "C" int cc_bin_table_max_rows(void) { return BT_MAX_ROWS; }

extern "C" int cc_bin_table_form_rows(int form) {
  return form == BT_TRI ? BT_TRI_ROWS : (form == BT_PAIR ? BT_PAIR_ROWS : (form == BT_U16 ? BT_MAX_ROWS : 0));
}

extern "C" int cc_bin_selftest(int rows, const float* edges, const uint16_t* table,
                               unsigned long long* mismatches, void* stream) {
  if (rows <= 0 || rows > BT_MAX_ROWS || !edges || !table || !mismatches) {
    cc::set_error("cc_bin_selftest: bad arguments (1 <= rows <= cc_bin_table_max_rows())");
    return CC_ERR_ARG;
  }
  hipLaunchKernelGGL(bin_selftest_kernel, dim3(rows), dim3(256), 0, static_cast<hipStream_t>(stream),
                     rows, edges, table, mismatches);
  return launch_status("cc_bin_selftest");
}

extern "C" int cc_coassoc(const int8_t* labels_nh, int n, int ldl, int Hpad, int K,
                          int64_t tile_begin, int64_t tile_end, const uint16_t* I_tiles,
                          const float* edges, unsigned long long* bin_counts, int32_t* M_full,
                          const uint16_t* bin_table, int table_rows, void* stream) {
  int rc = check_common("cc_coassoc", labels_nh, n, ldl, Hpad, tile_begin, tile_end);
  if (rc) return rc;
  if (K < 1 || K > 127) {
    cc::set_error("cc_coassoc: K must be in [1, 127]");
    return CC_ERR_ARG;
  }
  if (tile_end == tile_begin) return CC_OK;  // an empty band (a rank with no tiles)
  if (!I_tiles || !edges || !bin_counts) {
    cc::set_error("cc_coassoc: I_tiles, edges and bin_counts are required");
    return CC_ERR_ARG;
  }
  if ((reinterpret_cast<uintptr_t>(I_tiles) | reinterpret_cast<uintptr_t>(bin_table)) & 15) {
    cc::set_error("cc_coassoc: I_tiles and bin_table must be 16-B aligned (16-B tile and table copies)");
    return CC_ERR_ARG;
  }
  if (bin_table && (table_rows < Hpad + 1 || table_rows > BT_MAX_ROWS)) {
    cc::set_error("cc_coassoc: bin_table needs Hpad + 1 <= table_rows <= cc_bin_table_max_rows()");
    return CC_ERR_ARG;
  }
  const int64_t ntl = tile_end - tile_begin;
  if (ntl == 0) return CC_OK;
  if (ntl > 0x7fffffff) {
    cc::set_error("cc_coassoc: too many tiles for one launch");
    return CC_ERR_ARG;
  }
  const dim3 grid(static_cast<unsigned>(ntl));
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const uint8_t* lab = reinterpret_cast<const uint8_t*>(labels_nh);
  // K <= 2: i8 one-hot (KP = 2, 64 resamples per step).  K >= 3: FP4 one-hot, 256 virtual k
  // per step, channels padded to the next power of two KP >= 4, or exact-K packing (ExactK) for
  // K = 17, 18, where it saves over 40 % of the super-steps.  Measured at C3
  // (tools/co_only.py, profiles/r03/coassoc_fp4_first.txt): the exact form's expansion costs
  // more VALU per step, and below K = 17 its register demand spills, so K = 5, 9, 10, 11, 19, 20
  // ran 5-100 % slower exact than padded; only K = 17, 18 are built exact.
  // CCMI_CO_PACK=pow2 / exact forces one form for those two (diagnostics; identical counts).
  int kp = K <= 2 ? 2 : 4;
  while (kp < K) kp <<= 1;
  if (K == 17 || K == 18) {
    const int hs = 256 / K, se = (Hpad + hs - 1) / hs, sp = Hpad / (256 / kp);
    const char* pk = std::getenv("CCMI_CO_PACK");
    const bool force_pow2 = pk && pk[0] == 'p', force_exact = pk && pk[0] == 'e';
    if (force_exact || (!force_pow2 && 5 * se <= 3 * sp)) kp = K;
  }
  switch (kp) {
#define CC_F4(k) case k: launch_tiles<k, true>(grid, st, lab, n, ldl, Hpad, tile_begin, nullptr, I_tiles, edges, bin_counts, M_full, bin_table, table_rows); break;
    CC_F4(4) CC_F4(8) CC_F4(16) CC_F4(17) CC_F4(18) CC_F4(32) CC_F4(64)
#undef CC_F4
    case 2: launch_tiles<2>(grid, st, lab, n, ldl, Hpad, tile_begin, nullptr, I_tiles, edges, bin_counts, M_full, bin_table, table_rows); break;
    default: launch_tiles<128, true>(grid, st, lab, n, ldl, Hpad, tile_begin, nullptr, I_tiles, edges, bin_counts, M_full, bin_table, table_rows); break;
  }
  return launch_status("cc_coassoc");
}

#ifdef CC_CO_STAMPS
extern "C" int cc_co_stamps(unsigned long long* out8, int reset) {
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(cc_co_stamp_acc), 8 * sizeof(unsigned long long)) != hipSuccess)
    return CC_ERR_HIP;
  if (reset) {
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(cc_co_stamp_acc), z, sizeof(z)) != hipSuccess) return CC_ERR_HIP;
  }
  return CC_OK;
}
#endif

extern "C" int cc_consensus(const int32_t* M, const int32_t* I, int n, float* C, void* stream) {
  if (!M || !I || !C || n <= 0) {
    cc::set_error("cc_consensus: bad arguments");
    return CC_ERR_ARG;
  }
  const int64_t total = static_cast<int64_t>(n) * n;
  const bool al16 = ((reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(I) |
                     reinterpret_cast<uintptr_t>(C)) & 15) == 0;  // the row form's 16-B accesses
  if (n % 4 == 0 && al16) {
    const int blocks = std::min(n, 8192);  // 32 resident 256-thread workgroups per CU
    hipLaunchKernelGGL(consensus_rows_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), M, I, n, C);
  } else {
    int blocks = static_cast<int>(std::min<int64_t>((total + 255) / 256, 16384));
    hipLaunchKernelGGL(consensus_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       M, I, n, C);
  }
  return launch_status("cc_consensus");
}
