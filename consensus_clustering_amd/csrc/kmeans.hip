// Batched k-means for every (resample, K, init) problem of a consensus fit, on gfx950 (v3).
//
// Replaces the per-(K, h) `clusterer.fit_predict(X[indices])` of the reference
// (consensus_clustering_parallelised.py:282, default clusterer KMeans(), CC.py:88-90,
// with set_params(random_state=seed, n_init=3), CC.py:212-214).  The algorithm is
// scikit-learn's KMeans (sklearn/cluster/_kmeans.py):
//   * k-means++ seeding (:174-262): first centre from RandomState(seed).choice (resolved on
//     the host), then per centre 2+floor(ln K) candidates drawn by
//     searchsorted(cumsum(closest d^2), u * pot), the candidate minimising the potential
//     kept; every fit of one K replays the same RandomState(seed) stream;
//   * Lloyd (:624-752, _k_means_lloyd.pyx:23-212): labels = argmin_c |c|^2 - 2 x.c (strict
//     <, lowest index on ties), centres = sums * f32(1/count), empty clusters relocated to
//     the farthest points (_k_means_common.pyx:167-212), strict convergence on unchanged
//     labels else sum(shift^2) <= tol, tol = 1e-4 * mean var, a final E-step when not
//     strictly converged;
//   * best of n_init: lower inertia AND a different clustering (:1525-1531).
//
// Mapping (v3).  A persistent grid (one 512-thread workgroup per CU, ~150 KiB LDS) pulls
// UNITS = (resample h, subset of the (K, init) problems) from an atomic counter and runs a
// unit's whole set of fits on-chip.  A unit is driven as a problem ENGINE: every SWEEP
// streams the resample's rows once through LDS (32-row tiles) and serves up to 256 centroid
// "slots": the candidate columns of problems that are seeding (k-means++) and the centres of
// problems in Lloyd.  Between sweeps the engine retires converged problems, admits new ones
// and packs the next sweep round-robin, so no slot idles behind a group's slowest init.
//
// Arithmetic.  Rows and centres enter the MFMA as f16 hi/lo pairs of x * 2^s (the exact
// power-of-two scale keeps the pair inside f16 range): x.c = xh.ch + xh.cl + xl.ch, three
// v_mfma_f32_32x32x16_f16 per 16 dims with f32 accumulation (22 significant bits per
// operand, the accuracy class of sklearn's own float32 sgemm), 5.3x the f32-MFMA rate.  The
// M-step sums are a one-hot x (xh + xl) f16 MFMA (exact one-hot products, f32 sums), the
// counts a one-hot x ones MFMA.  All decisions (argmin, potentials, convergence, relocation,
// best-of-init) are f32/f64 as in sklearn.
//
// The 8 waves have two roles, one wave of each per SIMD, each role in its own tile loop (one
// barrier per tile in both, so their register sets never overlap and one role's vector chain
// runs while the other's MFMAs occupy the matrix pipe).  Per tile iteration t:
//   distance waves 0..3: the gather of tile t+1 into a 4-slot ring (LDS-DMA), the distance
//     MFMAs of tile t for slot tiles w and w+4 (register-resident f16 A fragments, one B read
//     per k-step for both) -> LDS distance tile (double buffer), and a share of the E-steps;
//   E/M waves 4..7: most E-steps of tile t-1 (thread = (row, work item); argmin per Lloyd
//     problem, min-with-closest per seeding candidate) and the M-steps of tile t-2 for slot
//     tiles q and q+4 (one-hot A from the E-step labels, B = the X tile read back with
//     ds_read_b64_tr_b16 from the same swizzled image the distance reads row-wise, one B read
//     for both tiles).
// The E-steps are dealt by LPT on a cost model in which the distance waves start with the cost
// of their MFMAs (KM_COST_DIST per slot tile) and the E/M waves with their M-steps.
// Nothing crosses workgroups, so results do not depend on scheduling, on how the units are
// split over launches or over GPUs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <vector>

#include "ccmi_internal.h"

namespace {

typedef float v16f __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

constexpr int NT = 512;
constexpr int NW = 8;
constexpr int NDW = 4;              // distance waves 0..3 (gather + distance MFMAs), one per SIMD
constexpr int NEW = NW - NDW;       // E/M waves 4..7 (E-steps + M-step MFMAs), one per SIMD
constexpr int RT = 32;              // rows per tile (one MFMA row block)
constexpr int CW = 256;             // centroid slots per sweep (8 slot tiles of 32)
constexpr int NLS = 8;              // E-step Lloyd steps per E/M wave (one Lloyd item each)
constexpr int NSS = 8;              // E-step seeding steps per E/M wave (two seeding items each)
constexpr int NLS_D = 3;            // ... per distance wave (they take a share of the E-steps;
constexpr int NSS_D = 2;            //     more spill their A fragments at d = 128)
constexpr int IMAX = 128;           // work items per sweep (80 seeding candidates + 44 Lloyd steps fit)
constexpr int PMAX = CC_KM_PMAX;    // problems per unit
constexpr int LSN = PMAX;           // label hand-off rows per buffer (indexed by problem)
constexpr int TMAX = 6;             // max local trials: 2 + floor(ln 127)
constexpr int KMAX = 127;
constexpr int DSD = CW + 4;         // distance-tile row stride (floats): 16-B rows, conflict-free b128
constexpr int NRING = 4;            // X tile ring: t+1 (gather), t (dist), t-2 (M-step)
// Pair mode (d <= 64, sweeps of at most 4 slot tiles = 128 slots): each barrier interval moves
// two row tiles (2p, 2p+1) through every stage, sequentially on the same waves, so the narrow
// sweeps at the end of a unit pay half the barriers and twice the work per wave chain.  Row
// tile 2p+1's distances sit in the same distance buffer at column offset 128 (the +inf chunk at
// CW stays shared), the ring holds 8 tiles and the label buffers 4.  Every row's arithmetic,
// every item's wave and every accumulation order are those of the one-tile loop, so the
// results are identical.
#ifndef KM_PAIR
#define KM_PAIR 1
#endif
template <int DP>
constexpr bool kPair = KM_PAIR && DP <= 64;
template <int DP>
constexpr int kRing = kPair<DP> ? 8 : NRING;
template <int DP>
constexpr int kLsb = kPair<DP> ? 4 : 2;  // label buffers of the E-step -> M-step hand-off
constexpr int US = CC_KM_USTRIDE;
// step-dealing cost units (a Lloyd step of K = 20 costs 80, a seeding step 20): the distance
// MFMAs and the M-step of a wave's own slots, measured in the same units from the phase stamps
#ifndef KM_COST_DIST
#define KM_COST_DIST 80  // at d = 128; the MFMA count scales with d (dist_cost)
#endif
#ifndef KM_COST_MSTEP
#define KM_COST_MSTEP 50
#endif
#ifndef KM_COST_LBASE
#define KM_COST_LBASE 32
#endif
#ifndef KM_COST_LCHUNK
#define KM_COST_LCHUNK 16
#endif
#ifndef KM_COST_SSTEP
#define KM_COST_SSTEP 20
#endif
#ifndef KM_COST_DIST_NARROW
#define KM_COST_DIST_NARROW KM_COST_DIST * DP / 128
#endif
// The sparse M-step pays at d = 128 only: at d = 32 / 64 the M-step MFMAs it removes are cheap
// (one or two 32-dim blocks) against the post-sweep work that grows with m (C5 k-means 314 ->
// 538 ms with it, C2 89 -> 92 ms).
template <int DP>
constexpr bool kSparse = DP == 128;
// The distance waves' starting cost per active slot tile for feature padding DP.
template <int DP>
__host__ __device__ constexpr int dist_cost() { return KM_COST_DIST_NARROW; }

// Diagnostic build only (-DCC_KM_STAMPS): per-wave cycle accounting of the sweep phases of
// workgroup 0, added into stats[8 + 8 * wave + k] (k: issue, dist, estep, mstep, commit,
// barrier) and stats[72..75] (sweep prologue, post-processing, unit setup, output).
#ifdef CC_KM_STAMPS
#define KM_STAMP(var)                  \
  __builtin_amdgcn_sched_barrier(0);   \
  const unsigned long long var = __builtin_amdgcn_s_memtime(); \
  __builtin_amdgcn_sched_barrier(0)
#define KM_ACC(k, a, b) st_acc[k] += (b) - (a)
#else
#define KM_STAMP(var)
#define KM_ACC(k, a, b)
#endif

enum { ST_WAIT = 0, ST_SEED = 1, ST_RUN = 2, ST_FINAL = 3, ST_DONE = 4 };
enum { IK_SEED0 = 0, IK_SEED = 1, IK_RUN = 2, IK_FINAL = 3 };

struct KArgs {
  const float* X;          // [n][DP] f32 (mean-centred, zero-padded)
  const uint16_t* Xhl;     // [n][2][DP] f16 bits: hi, lo of X * 2^s
  const float* xnorm;      // [n]
  int dreal;
  float scale, inv_scale, dscale, ndinv;  // 2^s, 2^-s, 2^(1-2s), -2^(2s-1) (a kernel argument: scalar)
  const int32_t* idx;
  int m, h_begin, nh, T;
  const int32_t* units;
  int nU;
  int max_iter;
  double tol_rel;
  const double* kpp_u;
  int kpp_stride, n_init;
  const int32_t* kpp_pos;
  uint8_t* labels_out;
  int n, ldl, H;
  float* inertia_out;
  int32_t* niter_out;
  unsigned long long* stats;
  unsigned* counter;
  uint8_t* ws;
  size_t ws_per_wg, off_cen, off_cenn, off_cpos, off_dbuf, off_rdist, off_s64, off_c64, off_list;
  int Pws, Kws, Tws, seedmax;
  int lsm;   // glab row stride (m rounded up to 64)
  int lseg;  // change-list entries per problem and wave segment
};

// Diagnostics (CCMI_KM_DENSE=1 at launch): every Lloyd item runs the dense M-step, for the
// sparse-against-dense parity test.  A device global read once per sweep by the scheduling
// thread, not a KArgs field: a field moved the sweep loops' register allocation (C3 +0.8 %).
__device__ int cc_km_dense_only = 0;

struct State {
  // unit
  int unit, P;
  float tol;
  int rr;
  unsigned seedfree;
  // problems
  unsigned char K[PMAX], kidx[PMAX], init[PMAX], ntr[PMAX], st[PMAX], c[PMAX], cs[PMAX], sslot[PMAX];
  unsigned char need_sel[PMAX], to_run[PMAX], sbest[PMAX], lcur[PMAX];
  short cenoff[PMAX], pitem[PMAX];
  int iter[PMAX], amax[PMAX], nempty[PMAX];
  int pchg[PMAX];  // labels changed in the problem's last Lloyd E-step (m before the first)
  float pot32[PMAX], inert[PMAX];
  int cand[PMAX][TMAX];
  // sweep
  int nitems, ncols;
  unsigned char ikind[IMAX], iprob[IMAX], itr[IMAX];
  unsigned iw0[IMAX], iw1[IMAX];               // packed item words (see EState)
  unsigned char lstep[NW][NLS], sstep[NW][NSS][2];  // E-step steps of each wave (item; 0xFF none)
  unsigned char nlw[NW], nsw[NW];
  int4 sdesc[NW][NSS][2];  // seeding step descriptors of the sweep (see estep)
  short ioff[IMAX], incol[IMAX];
  double iinert[IMAX];
  unsigned ichanged[IMAX];
  unsigned char isparse[IMAX];  // RUN item whose sums follow its change list (no M-step MFMAs)
  unsigned lcnt[IMAX][NW];      // changed labels of a sparse item per wave segment of its rows
  short sitem[CW], scl[CW];
  int srow[CW];  // >= 0: X row (seeding candidate); < 0: -(centre row) - 1
  alignas(16) float cnorm[CW];
  float shift[CW];
  unsigned cnt[CW];
  // scratch
  double red_v[NW];
  int red_i[NW];
  int map[KMAX + 1];
  int flag;
  unsigned long long n_lloyd, n_seed, n_mrows, n_reloc, n_sweeps, n_ctiles, n_sparse, n_changes;
};

// Measured (round 5, C3): the sweep loops ran 7.5 % slower (1653 -> 1775 ms, identical results)
// with the per-sweep item fields (ikind .. nsw) at offsets 0 mod 8 instead of 4 mod 8 -- a 4-byte
// field added after ncols, or moved there, is enough; pads of 2 / 4 words were neutral.  New
// State fields go to the end (a field there measured neutral).
static_assert(offsetof(State, ikind) % 8 == 4, "State layout: see the note above");

template <int DP>
struct Lay {
  static constexpr int IMG = RT * DP * 2;     // one f16 image (hi or lo) of a tile, bytes
  static constexpr int SLOT = 2 * IMG;        // ring slot: hi image then lo image
  static constexpr int OFF_D = kRing<DP> * SLOT;  // distance tiles [2][RT][DSD] f32
  static constexpr int DBUF = RT * DSD * 4;
  static constexpr int U_END = OFF_D + 2 * DBUF;
  static constexpr int S_BYTES = CW * DP * 4;  // centre sums [CW][DP] f32, aliasing ring + D
  static_assert(S_BYTES <= U_END, "centre sums must fit in the ring + distance tiles");
  static constexpr int OFF_LS = (U_END + 32 + 15) / 16 * 16;  // labels [2][LSN][RT] u8 (32 B slack: E-step over-reads)
  static constexpr int OFF_XN = OFF_LS + kLsb<DP> * LSN * RT;  // row norms [kRing][64] f32 (DMA'd, 32 used)
  static constexpr int OFF_ST = OFF_XN + kRing<DP> * 64 * 4;
  static constexpr int TOTAL = OFF_ST + ((sizeof(State) + 15) / 16) * 16;
  static_assert(TOTAL <= 163840, "LDS budget");
  static_assert(NSS % 4 == 0 && (NSS_D < 4 || NSS_D % 4 == 0), "seeding steps are read in batches");
};

// Byte offset of 16-B chunk `ch` of tile row `row` in one f16 image (DP/8 chunks per row).
// XOR-swizzled so that both the row-wise ds_read_b128 of the distance B operand (32 rows,
// one chunk) and the ds_read_b64_tr_b16 of the M-step B operand (4 rows x 32 dims per
// 32-lane half) are bank-conflict free (bank = (addr/4) mod 64).
template <int DP>
__device__ __forceinline__ int xoff(int row, int ch) {
  if constexpr (DP == 128) return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
  else if constexpr (DP == 64) return 128 * row + 16 * (ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3)));
  else return 64 * row + 16 * (ch ^ ((row >> 2) & 3));
}

__device__ __forceinline__ double half_sum(double v) {  // over the 32 lanes of a half-wave
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ v16f mfma16(const h8& a, const h8& b, const v16f& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// numpy pairwise_sum of a short contiguous float32 array (n <= 128), as
// `(center_shift ** 2).sum()` evaluates it (numpy/_core/src/umath/loops_utils.h).
__device__ __forceinline__ float np_pairwise_sum(const float* a, int n) {
  if (n < 8) {
    float res = 0.f;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

// sum of squares of a centre row (sklearn row_norms: f32, sequential).
__device__ __forceinline__ float row_sq(const float* c, int dreal) {
  float s = 0.f;
  for (int d = 0; d < dreal; ++d) s = fmaf(c[d], c[d], s);
  return s;
}

// XOR value of the swizzle of xoff<DP> for a row (chunk position = ch ^ xsw(row)).
template <int DP>
__device__ __forceinline__ int xsw(int row) {
  if constexpr (DP == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  else if constexpr (DP == 64) return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
  else return (row >> 2) & 3;
}

// ---- X tile gather by LDS-DMA (global_load_lds_dwordx4: lane i of a wave-instruction writes
// 16 B at M0 + 16 i, so one instruction fills a contiguous 1-KiB piece = 1024/(2 DP) whole rows
// of the swizzled image; each lane fetches the chunk that lives at its linear position).
// The data never passes through VGPRs; rows past m load the clamped row m-1 (consumers ignore
// them: E-step rows are masked, their labels are 0xFF so the M-step one-hot is 0).
template <int DP>
struct Gather {
  static constexpr int IMG = RT * DP * 2;
  static constexpr int NI = (2 * IMG) / 1024;          // pieces per tile (hi + lo)
  static constexpr int PER = (NI + NDW - 1) / NDW;     // pieces per distance wave
  static constexpr int ROWB = 2 * DP;                  // bytes per image row
};

template <int DP>
struct TileIdx {
  int src[Gather<DP>::PER];
  int xsrc;
};

template <int DP>
__device__ __forceinline__ void idx_issue(const KArgs& a, const int32_t* idx, int r0, int wave, int lane,
                                          TileIdx<DP>& I) {
  using GA = Gather<DP>;
#pragma unroll
  for (int j = 0; j < GA::PER; ++j) {  // unsigned: the divisions by powers of two are shifts
    const unsigned k = wave + NDW * j;
    const unsigned B = 1024u * k + 16u * static_cast<unsigned>(lane);
    const unsigned off = B % GA::IMG;
    I.src[j] = idx[min(r0 + static_cast<int>(off / GA::ROWB), a.m - 1)];
  }
  I.xsrc = idx[min(r0 + lane, a.m - 1)];
}

// LDS-DMA piece issued from inline asm: opaque to the compiler's waitcnt pass, which would
// otherwise put a vmcnt(0) in front of every LDS read it cannot prove disjoint from the DMA
// (the ds_read_b64_tr_b16 of the M-step), exposing the gather latency mid-iteration.
// Untracked VMEM ops only make the compiler's own vmcnt waits stricter (the counter drains in
// order); completion is awaited explicitly by dma_wait() before the barrier that publishes the
// tile.  M0 is set inside the asm; no compiler-generated code in this kernel uses M0.  No
// "memory" clobber: the piece writes a ring slot nothing touches until the next barrier and
// reads immutable rows (a clobber makes the compiler drain vmcnt in front of every piece).
__device__ __forceinline__ void dma_piece(const void* g, const void* lds_dst, int bytes) {
  const unsigned la = static_cast<unsigned>(reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) const char*)lds_dst));
  if (bytes == 16)
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(__builtin_amdgcn_readfirstlane(la)), "v"(g));
  else
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(__builtin_amdgcn_readfirstlane(la)), "v"(g));
}

// DMA source addresses of one tile (computed before anything else is issued, so that the
// compiler's wait for the index registers, loaded one iteration earlier, precedes every piece).
template <int DP>
struct TileAddr {
  const uint16_t* src[Gather<DP>::PER];
  const float* xsrc;
};

template <int DP>
__device__ __forceinline__ void tile_addr(const KArgs& a, const TileIdx<DP>& I, int wave, int lane,
                                          TileAddr<DP>& A) {
  using GA = Gather<DP>;
  int ln = lane;
  asm volatile("" : "+v"(ln));  // recompute the per-lane chunk offsets (cheap) rather than hold them
#pragma unroll
  for (int j = 0; j < GA::PER; ++j) {  // unsigned: the divisions by powers of two are shifts
    const unsigned k = wave + NDW * j;
    const unsigned B = 1024u * k + 16u * static_cast<unsigned>(ln);
    const unsigned part = B / GA::IMG, off = B % GA::IMG;
    const unsigned row = off / GA::ROWB, ch = ((off % GA::ROWB) >> 4) ^ static_cast<unsigned>(xsw<DP>(static_cast<int>(row)));
    A.src[j] = a.Xhl + static_cast<size_t>(static_cast<unsigned>(I.src[j])) * (2 * DP) + (part * DP + 8u * ch);
  }
  A.xsrc = a.xnorm + static_cast<unsigned>(I.xsrc);
}

// Keeps the pieces' address registers allocated up to this point (after the end-of-iteration
// wait): the compiler treats an inline-asm operand as possibly still being read, and would
// put a vmcnt(0) in front of any instruction that reuses one of those registers earlier.
template <int DP>
__device__ __forceinline__ void tile_addr_hold(const TileAddr<DP>& A) {
#pragma unroll
  for (int j = 0; j < Gather<DP>::PER; ++j) asm volatile("" ::"v"(A.src[j]));
  asm volatile("" ::"v"(A.xsrc));
}

// The tile's pieces, issued last in the gather block: no VALU after them overwrites an address
// register before the end-of-iteration wait (the compiler would wait vmcnt(0) for that).
template <int DP>
__device__ __forceinline__ void tile_issue(const TileAddr<DP>& A, char* slot, float* xn, int wave) {
  using GA = Gather<DP>;
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < GA::PER; ++j)
    if (wave + NDW * j < GA::NI) dma_piece(A.src[j], slot + 1024 * (wave + NDW * j), 16);  // wave-uniform
  if (wave == NDW - 1) dma_piece(A.xsrc, xn, 4);
  __builtin_amdgcn_sched_barrier(0);
}

// vmcnt(0) through the builtin (not inline asm): the compiler's waitcnt model then knows that
// nothing is outstanding, so it puts no wait of its own after the next tile's DMA pieces (which
// it cannot see) for loads that have already landed.
__device__ __forceinline__ void dma_wait() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// A fragments of one centroid slot: lane (r, h) holds dims 16s + 8h + j of its slot's centre.
template <int DP>
__device__ __forceinline__ void afrag_load(h8 (&ah)[DP / 16], h8 (&al)[DP / 16], const float* src,
                                           bool valid, int h, float scale) {
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
    if (valid) {
      x0 = *reinterpret_cast<const float4*>(src + 16 * s + 8 * h);
      x1 = *reinterpret_cast<const float4*>(src + 16 * s + 8 * h + 4);
    }
    const float x[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xs = x[j] * scale;
      const _Float16 hi = static_cast<_Float16>(xs);
      ah[s][j] = hi;
      al[s][j] = static_cast<_Float16>(xs - static_cast<float>(hi));
    }
  }
}

// Empty-cluster relocation for problem p (rare path; _k_means_common.pyx:167-212).
// Sm holds the un-averaged sums of the problem's slots [off, off+K), cen the centres the
// labels came from, glab the problem's labels of this sweep.
template <int DP, class St>
__device__ void relocate(const KArgs& a, const int32_t* idx, int p, int off, const float* cen,
                         float* Sm, St& S, const uint8_t* glab, float* dist, int tid) {
  const int m = a.m, K = S.K[p];
  float mymax = 0.f;
  for (int r = tid; r < m; r += NT) {
    const float* x = a.X + static_cast<size_t>(idx[r]) * DP;
    const float* c = cen + (S.cenoff[p] + glab[r]) * DP;
    float s = 0.f;
    for (int d = 0; d < a.dreal; ++d) {
      const float t = x[d] - c[d];
      s = fmaf(t, t, s);
    }
    dist[r] = s;
    mymax = fmaxf(mymax, s);
  }
  for (int o = 32; o > 0; o >>= 1) mymax = fmaxf(mymax, __shfl_xor(mymax, o));
  if ((tid & 63) == 0) S.red_v[tid >> 6] = mymax;
  __syncthreads();
  double gmax = 0.0;
  for (int w = 0; w < NW; ++w) gmax = fmax(gmax, S.red_v[w]);
  // the empty clusters are fixed before any relocation (np.where(weight == 0))
  if (tid == 0) {
    int ne = 0;
    for (int c = 0; c < K; ++c)
      if (S.cnt[off + c] == 0) S.map[ne++] = c;
    S.flag = ne;
  }
  __syncthreads();
  if (gmax == 0.0) return;  // sklearn returns early when every point sits on its centre
  const int ne = S.flag;
  for (int e = 0; e < ne; ++e) {
    const int c = S.map[e];
    float bv = -1.f;
    int bi = 0x7fffffff;
    for (int r = tid; r < m; r += NT) {
      const float v = dist[r];
      if (v > bv) {
        bv = v;
        bi = r;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o);
      const int oi = __shfl_xor(bi, o);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if ((tid & 63) == 0) {
      S.red_v[tid >> 6] = bv;
      S.red_i[tid >> 6] = bi;
    }
    __syncthreads();
    double gv = -2.0;
    int gi = 0x7fffffff;
    for (int w = 0; w < NW; ++w)
      if (S.red_v[w] > gv || (S.red_v[w] == gv && S.red_i[w] < gi)) {
        gv = S.red_v[w];
        gi = S.red_i[w];
      }
    const int old = glab[gi];
    const float* x = a.X + static_cast<size_t>(idx[gi]) * DP;
    for (int d = tid; d < DP; d += NT) {
      Sm[(off + old) * DP + d] -= x[d];
      Sm[(off + c) * DP + d] = x[d];
    }
    __syncthreads();
    if (tid == 0) {
      S.cnt[off + c] = 1;
      S.cnt[off + old] -= 1;
      dist[gi] = -1.f;
      S.n_reloc += 1;
    }
    __syncthreads();
  }
}

// Wave w's part of the post-sweep label compare of a sparse item: rows [w * seg, (w + 1) * seg)
// (seg = m / 8 rounded up to 16), 16 rows per lane and load; each changed row is appended to the
// wave's segment of the item's change list as (row, old | new << 8), in row order (wave prefix
// sum of the lanes' counts).  Returns the segment's count (it may exceed the capacity `cap`:
// then only the count is meaningful).
__device__ unsigned list_changes(const uint8_t* cur, const uint8_t* old, int m, int w, int lane, uint2* seg,
                                 unsigned cap) {
  const int rs = (((m + NW - 1) / NW) + 15) & ~15;
  const int r0 = w * rs, r1 = min(m, r0 + rs);
  unsigned n = 0;
  for (int b = r0; b < r1; b += 16 * 64) {  // wave-uniform
    const int r = b + 16 * lane;
    unsigned msk = 0;
    uint4 x = make_uint4(0, 0, 0, 0), y = x;
    if (r < r1) {  // r1 - r is a multiple of 16 except at m (rows past m hold 0xFF in both buffers)
      x = *reinterpret_cast<const uint4*>(cur + r);
      y = *reinterpret_cast<const uint4*>(old + r);
      const unsigned xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned dq = xs[q] ^ ys[q];
#pragma unroll
        for (int k = 0; k < 4; ++k) msk |= ((dq >> (8 * k)) & 0xFFu) ? (1u << (4 * q + k)) : 0u;
      }
    }
    const unsigned c = __popc(msk);
    unsigned pre = c;  // inclusive wave scan of the counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned t = __shfl_up(pre, o);
      if (lane >= o) pre += t;
    }
    unsigned pos = n + pre - c;
    const unsigned xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
    while (msk) {
      const int k = __builtin_ctz(msk);
      msk &= msk - 1;
      const unsigned nv = (xs[k >> 2] >> (8 * (k & 3))) & 0xFFu, ov = (ys[k >> 2] >> (8 * (k & 3))) & 0xFFu;
      if (pos < cap) seg[pos] = make_uint2(static_cast<unsigned>(r + k), ov | (nv << 8));
      ++pos;
    }
    n += __shfl(pre, 63);
  }
  return n;
}

// Sums and counts of a sparse RUN item from its change list, one wave (lane = DP / 64 dims): the
// entries (segments in wave order, each in row order) add their f32 row to the new cluster's
// row of acc and subtract it from the old one's (f32; acc = the item's own K rows of Sm, which
// the M-step leaves alone for a sparse item), 16 row loads in flight; counts by LDS atomics into
// cnt.  With `full` (a segment overflowed) every row's label `lab` counts as an entry that moved
// in from nowhere.  The order of additions depends only on the list, so the results do not
// depend on how the sweeps were packed.  The caller adds acc / cnt into the running sums.
template <int DP>
__device__ void apply_changes(const KArgs& a, const int32_t* idx, const uint2* lst, const unsigned* nseg,
                              bool full, const uint8_t* lab, float* acc, unsigned* cnt, int K, int lane) {
  constexpr int DL = DP >= 64 ? DP / 64 : 1;  // dims per lane (lanes >= 32 idle at DP = 32)
  const bool dok = lane * DL < DP;
  const int d0 = dok ? lane * DL : 0;
  for (int e = lane; e < K * DP; e += 64) acc[e] = 0.f;
  if (lane < K) cnt[lane] = 0u;
  for (int sg = 0; sg < (full ? 1 : NW); ++sg) {
    const int n = full ? a.m : static_cast<int>(nseg[sg]);
    const uint2* ls = lst + static_cast<size_t>(sg) * a.lseg;
    for (int e0 = 0; e0 < n; e0 += 64) {
      const int e = e0 + lane;
      unsigned xr = 0, o = 0xFFu, nw = 0xFFu;
      if (e < n) {
        unsigned r;
        if (full) {
          r = static_cast<unsigned>(e);
          nw = lab[e];
        } else {
          const uint2 v = ls[e];
          r = v.x;
          o = v.y & 0xFFu;
          nw = (v.y >> 8) & 0xFFu;
        }
        xr = static_cast<unsigned>(idx[r]);
        if (nw < 0xFFu) __hip_atomic_fetch_add(&cnt[nw], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (o < 0xFFu) __hip_atomic_fetch_add(&cnt[o], ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      const int ne = min(64, n - e0);
      constexpr int B = 16;
      for (int j0 = 0; j0 < ne; j0 += B) {  // wave-uniform
        float v[B][DL];
        unsigned jn[B], jo[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {  // the batch's row loads in flight together
          const int jj = min(j0 + j, ne - 1);
          const unsigned row = __builtin_amdgcn_readlane(xr, jj);
          jn[j] = (j0 + j < ne) ? __builtin_amdgcn_readlane(nw, jj) : 0xFFu;
          jo[j] = (j0 + j < ne) ? __builtin_amdgcn_readlane(o, jj) : 0xFFu;
          const float* xp = a.X + static_cast<size_t>(row) * DP + d0;
          if constexpr (DL == 2) {
            const float2 q = *reinterpret_cast<const float2*>(xp);
            v[j][0] = q.x;
            v[j][DL - 1] = q.y;
          } else {
            v[j][0] = *xp;
          }
        }
        if (dok) {
#pragma unroll
          for (int j = 0; j < B; ++j) {  // in list order (one wave's LDS accesses stay ordered)
            if (jn[j] < 0xFFu) {
              float* q = acc + jn[j] * DP + d0;
              if constexpr (DL == 2) {
                float2 t = *reinterpret_cast<float2*>(q);
                t.x += v[j][0];
                t.y += v[j][DL - 1];
                *reinterpret_cast<float2*>(q) = t;
              } else {
                *q += v[j][0];
              }
            }
            if (jo[j] < 0xFFu) {
              float* q = acc + jo[j] * DP + d0;
              if constexpr (DL == 2) {
                float2 t = *reinterpret_cast<float2*>(q);
                t.x -= v[j][0];
                t.y -= v[j][DL - 1];
                *reinterpret_cast<float2*>(q) = t;
              } else {
                *q -= v[j][0];
              }
            }
          }
        }
      }
    }
  }
}

// k-means++ candidate positions for centre S.c[p] (>= 1) of problem p, one wave:
// searchsorted(cumsum(closest), u * pot) (side='left': #{cumsum < v}), clipped to m-1.
// The cumsum is blocked by 32-row tiles: each lane sums whole tiles sequentially in f64 (the
// in-tile order of the sklearn cumsum), the wave prefix-sums the tile sums, and the crossing
// tile is walked sequentially from its prefix, so the two levels agree exactly.
template <class St>
__device__ void kpp_select(const KArgs& a, St& S, int p, const float* closest, int lane) {
  const int ntr = S.ntr[p], c = S.c[p], m = a.m, T = a.T;
  const double* u = a.kpp_u + (static_cast<size_t>(S.kidx[p]) * a.n_init + S.init[p]) * a.kpp_stride +
                    1 + static_cast<size_t>(c - 1) * ntr;
  const double pot = static_cast<double>(S.pot32[p]);
  double rv[TMAX], base[TMAX];
  int tau[TMAX];
  bool found[TMAX];
#pragma unroll
  for (int t = 0; t < TMAX; ++t) {
    rv[t] = (t < ntr) ? u[t] * pot : 0.0;
    base[t] = 0.0;
    tau[t] = T;
    found[t] = false;
  }
  double run = 0.0;
  for (int b = 0; b < T; b += 64) {
    const int j = b + lane;
    double v = 0.0;
    if (j < T) {
      const float* rowp = closest + RT * j;
      const int nr = min(RT, m - RT * j);
      if (nr == RT) {  // a full tile: all its loads in flight, then the same in-order f64 sum
        float4 q[RT / 4];
#pragma unroll
        for (int r4 = 0; r4 < RT / 4; ++r4) q[r4] = *reinterpret_cast<const float4*>(rowp + 4 * r4);
#pragma unroll
        for (int r4 = 0; r4 < RT / 4; ++r4) {
          v += static_cast<double>(q[r4].x);
          v += static_cast<double>(q[r4].y);
          v += static_cast<double>(q[r4].z);
          v += static_cast<double>(q[r4].w);
        }
      } else {
        for (int r = 0; r < nr; r += 4) {
          const float4 q = *reinterpret_cast<const float4*>(rowp + r);  // m, RT multiples of 4 or tail
          v += static_cast<double>(q.x);
          if (r + 1 < nr) v += static_cast<double>(q.y);
          if (r + 2 < nr) v += static_cast<double>(q.z);
          if (r + 3 < nr) v += static_cast<double>(q.w);
        }
      }
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double y = __shfl_up(v, o);
      if (lane >= o) v += y;
    }
    const double cum = run + v;
    const int nvalid = min(64, T - b);
#pragma unroll
    for (int t = 0; t < TMAX; ++t) {
      if (t >= ntr) continue;
      const int k = __popcll(__ballot(j < T && cum < rv[t]));
      const double prev = __shfl(cum, max(k - 1, 0));
      if (!found[t] && k < nvalid) {
        found[t] = true;
        tau[t] = b + k;
        base[t] = (k == 0) ? run : prev;
      }
    }
    run = __shfl(cum, 63);
  }
  // within the crossing tile: lane t walks its rows
#pragma unroll
  for (int t = 0; t < TMAX; ++t) {
    if (t >= ntr || lane != t) continue;
    int pos = m;
    if (found[t]) {
      const int r0 = RT * tau[t];
      double acc = base[t];
      int k = 0;
      for (; k < RT && r0 + k < m; ++k) {
        acc += static_cast<double>(closest[r0 + k]);
        if (!(acc < rv[t])) break;
      }
      pos = r0 + k;
    }
    S.cand[p][t] = min(pos, m - 1);
  }
}

// ---- E-step (all 512 threads): lane = (tile row tid & 31, half-wave hh).  The schedule deals
// the sweep's work items to the 8 waves (LPT by cost) as STEPS:
//   Lloyd steps (one item, wave-uniform): the two half-waves scan the two halves of the item's
//     slots in aligned 4-slot chunks (problems sit at 4-aligned slot offsets, K padded to a
//     multiple of 4 with +inf dummy slots, so no masking) and merge with v_permlane32_swap;
//     half-wave 0 stores the label (global, double-buffered per problem: the "labels
//     changed" test is a post-sweep compare of the two buffers) and the M-step label (LDS)
//     and accumulates the inertia;
//   seeding steps (two items, one per half-wave): min with the closest distance, stored for
//     the potential and the next k-means++ draw.
// Item words (LDS):
//   iw0 = label buffer<<30 | kind<<24 | problem<<16 | K<<8 | slot offset
//   iw1 = dbuf write slot<<11 | closest slot<<8 | trial<<5 | seeding slot
// Per-thread inertia / potential partials of the wave's E-step steps: f32 over at most 32 tiles,
// then flushed (f64 half-wave sum) into the item's f64 accumulator in LDS (S.iinert).  f32
// partials keep 8 VGPRs instead of 16: with f64 partials the kernel spilled, and every spill
// reload drained the LDS-DMA pipeline (vmcnt(0)).
template <int NL, int NS>
struct EState {
  float iaccL[NL], iaccS[NS];
};
constexpr int FLUSH = 32;  // tiles per f32 partial

// The first slot tile whose M-step E/M wave NDW + q runs (then + NDW).  Waves w and w + NDW
// share a SIMD, so the M-step of slot tile q runs on another SIMD than its distance MFMAs
// (wave q): in a narrow sweep (one slot tile) the two MFMA blocks use two matrix pipes.
__host__ __device__ constexpr int mstep_tile(int q) { return (q + 1) % NDW; }
static_assert(NEW == NDW, "one E/M wave per distance wave");

__device__ __forceinline__ int iw_off(unsigned w) { return w & 0xFF; }
__device__ __forceinline__ int iw_K(unsigned w) { return (w >> 8) & 0xFF; }
__device__ __forceinline__ int iw_prob(unsigned w) { return (w >> 16) & 0x3F; }
__device__ __forceinline__ int iw_kind(unsigned w) { return (w >> 24) & 3; }
__device__ __forceinline__ int iw_buf(unsigned w) { return (w >> 30) & 1; }

// Seeding step descriptor (one per wave, step and half-wave, every entry initialised; built
// once per sweep so that a step costs one LDS read instead of three dependent ones, and all
// steps' reads are issued together, unconditionally): x = closest-distance column read (float
// offset in dbuf), z = column written, y = w = distance column (CW, the +inf chunk, when the
// half-wave has no item) | flags << 16, flags = 1 (item) | 2 (kind IK_SEED: min with the
// closest distance).  The prefetch reads (x, y), the E-step (z, w).
__device__ __forceinline__ int4 seed_desc(const KArgs& a, const State& S, int it, int T1) {
  if (it == 0xFF) return make_int4(0, CW, 0, CW);
  const unsigned w0 = S.iw0[it], w1 = S.iw1[it];
  const int slot = w1 & 31;
  const int dcf = iw_off(w0) | ((1 | ((iw_kind(w0) == IK_SEED) ? 2 : 0)) << 16);
  return make_int4((slot * T1 + ((w1 >> 8) & 7)) * a.lsm, dcf, (slot * T1 + ((w1 >> 11) & 7)) * a.lsm, dcf);
}

// Closest distances of the seeding items of tile tp (issued one iteration before its E-step).
template <int NS>
__device__ __forceinline__ void estep_prefetch(const KArgs& a, const State& S, int tp, int T, int tidl, int ns,
                                               const float* dbuf, unsigned (&pre)[NS]) {
  const int erow = tp * RT + (tidl & (RT - 1));
  const bool eok = (tp >= 0 && tp < T) && erow < a.m;
  const int w = (tidl >> 6) & 7, hh = (tidl >> 5) & 1;  // tidl is opaque: steps re-read from LDS
#pragma unroll
  for (int i = 0; i < NS; ++i) pre[i] = 0;
#pragma unroll
  for (int i0 = 0; i0 < NS; i0 += (NS < 4 ? NS : 4)) {  // wave-uniform: only the batches in use
    if (i0 >= ns) break;
    constexpr int B = NS < 4 ? NS : 4;
    int2 d[B];
#pragma unroll
    for (int i = 0; i < B; ++i) d[i] = *reinterpret_cast<const int2*>(&S.sdesc[w][i0 + i][hh].x);  // in flight together
#pragma unroll
    for (int i = 0; i < B; ++i)
      if (eok && (d[i].y & (2 << 16))) pre[i0 + i] = __float_as_uint(dbuf[static_cast<unsigned>(d[i].x) + erow]);
  }
}

// strict-< argmin of NCH aligned chunks (4 slots each, columns col[u] .. col[u] + 3, increasing
// in u) as a tree (dependency depth 2 + log2 NCH instead of 4 NCH): ties keep the lower slot at
// every level.  EAGER: the slot indices are materialised as the values are compared and the
// result is selected without a branch; otherwise the compiler sinks the index selects under the
// final compare and keeps every compare mask live in SGPR pairs until then.  Same result either
// way; eager measured C5 275 -> 268 ms and C2 87.1 -> 86.0 ms, C3 (d = 128) unchanged within
// noise (1649 vs 1652 ms, its SGPR spills 335 -> 287 but no faster), so d = 128 keeps the sunk form.
template <int NCH, bool EAGER>
__device__ __forceinline__ void amin_chunks(const float4 (&v)[NCH], const int (&col)[NCH], float& best, int& lab) {
  float bv[NCH];
  int bi[NCH];
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    float m0 = v[u].x, m1 = v[u].z;
    int i0 = col[u], i1 = col[u] + 2;
    if (v[u].y < m0) { m0 = v[u].y; i0 = col[u] + 1; }
    if (v[u].w < m1) { m1 = v[u].w; i1 = col[u] + 3; }
    if (m1 < m0) { m0 = m1; i0 = i1; }
    bv[u] = m0;
    bi[u] = i0;
    if constexpr (EAGER) asm volatile("" : "+v"(bi[u]));
  }
#pragma unroll
  for (int st = 1; st < NCH; st *= 2)
#pragma unroll
    for (int u = 0; u + st < NCH; u += 2 * st)
      if (bv[u + st] < bv[u]) { bv[u] = bv[u + st]; bi[u] = bi[u + st]; }
  if constexpr (EAGER) {
    asm volatile("" : "+v"(bi[0]));
    const bool upd = bv[0] < best;
    best = upd ? bv[0] : best;
    lab = upd ? bi[0] : lab;
  } else if (bv[0] < best) {
    best = bv[0];
    lab = bi[0];
  }
}

// Lloyd argmin of one half-wave over chunks j0 .. j0 + NCH - 1 (those at or past cnt read the
// +inf columns CW..CW+3).
template <int NCH, bool EAGER>
__device__ __forceinline__ void amin_half(const float* drow, int base, int j0, int cnt, float& best, int& lab) {
  int col[NCH];
  float4 v[NCH];
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    col[u] = (j0 + u < cnt) ? base + 4 * (j0 + u) : CW;
    v[u] = *reinterpret_cast<const float4*>(drow + col[u]);
  }
  // all NCH reads in flight before the first wait (the scheduler otherwise reuses one register
  // quad for the chunks and serialises their LDS round trips)
#pragma unroll
  for (int u = 0; u < NCH; ++u) asm volatile("" : "+v"(v[u].x), "+v"(v[u].y), "+v"(v[u].z), "+v"(v[u].w));
  amin_chunks<NCH, EAGER>(v, col, best, lab);
}

template <int DP, int NL, int NS, bool PM = false>
__device__ __forceinline__ void estep(const KArgs& a, const State& S, int t, int T, int tidl, const float* Dt,
                                      uint8_t* Ls, const float* XN, uint8_t* glab, float* dbuf,
                                      const unsigned (&pre)[NS], const unsigned (&lw)[NL], int nl, int ns,
                                      EState<NL, NS>& es) {
  if (t < 1 || t > T) return;
  const int m = a.m;
  const int te = t - 1;
  const int ler = tidl & (RT - 1);
  const int w = (tidl >> 6) & 7, hh = (tidl >> 5) & 1;
  const int erow = te * RT + ler;
  const bool eok = erow < m;
  // pair mode: tile te's distances in buffer (te >> 1) & 1 at column offset 128 (te & 1), its
  // labels in buffer te & 3
  const int coff = PM ? 128 * (te & 1) : 0;
  const float* drow = Dt + (PM ? ((te >> 1) & 1) : (te & 1)) * (RT * DSD) + ler * DSD;
  uint8_t* lsb = Ls + (PM ? (te & 3) : (te & 1)) * (LSN * RT);
  const float xnr = XN[(te % kRing<DP>) * 64 + ler];
  constexpr float INF = __builtin_huge_valf();
  // seeding steps first (one item per half-wave): descriptors and distances of every step in
  // flight together, then min with the closest distance, store for the potential and the next
  // k-means++ draw
#pragma unroll
  for (int i0 = 0; i0 < NS; i0 += (NS < 4 ? NS : 4)) {  // wave-uniform: only the batches in use
    if (i0 >= ns) break;
    constexpr int B = NS < 4 ? NS : 4;
    int2 d[B];
    float dd[B];
#pragma unroll
    for (int i = 0; i < B; ++i) d[i] = *reinterpret_cast<const int2*>(&S.sdesc[w][i0 + i][hh].z);
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int col = d[i].y & 0xFFFF;
      dd[i] = drow[(PM && col != CW) ? col + coff : col];
    }
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const float dist = fmaxf(xnr + dd[i], 0.f);
      const float dm = (d[i].y & (2 << 16)) ? fminf(__uint_as_float(pre[i0 + i]), dist) : dist;
      if (eok && (d[i].y & (1 << 16))) {
        dbuf[static_cast<unsigned>(d[i].x) + erow] = dm;
        es.iaccS[i0 + i] += dm;
      }
    }
  }
  // Lloyd steps (wave-uniform words, hoisted for the sweep)
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    if (i >= nl) break;
    const unsigned ww = lw[i];
    const int off = iw_off(ww), C = (iw_K(ww) + 3) >> 2, h0 = (C + 1) >> 1;
    const int base = off + coff + (hh ? 4 * h0 : 0), cnt = hh ? C - h0 : h0;
    float best = INF;
    int lab = 0;
    // wave-uniform (one item per wave): the item's chunk count per half-wave
    constexpr bool EAGER = DP < 128;
    if (h0 <= 2) {
      amin_half<2, EAGER>(drow, base, 0, cnt, best, lab);
    } else if (h0 <= 3) {
      amin_half<3, EAGER>(drow, base, 0, cnt, best, lab);
    } else {
      for (int j0 = 0; j0 < h0; j0 += 4) amin_half<4, EAGER>(drow, base, j0, cnt, best, lab);  // 4 reads in flight
    }
    // merge the halves (v_permlane32_swap: lane i <-> i^32 without LDS): lower value, ties to
    // the lower slot.  Half 0 holds the lower slots, so its lanes take the other half's minimum
    // only when strictly lower and half 1's lanes on ties too: both halves end with the same
    // (best, lab), and the stores below need no half-wave mask (both write the same byte)
    const auto bs = __builtin_amdgcn_permlane32_swap(__float_as_uint(best), __float_as_uint(best), false, false);
    const auto ls = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(lab), static_cast<unsigned>(lab), false, false);
    const float ob = __uint_as_float(hh ? bs[0] : bs[1]);
    const int ol = static_cast<int>(hh ? ls[0] : ls[1]);
    const bool upd = hh ? !(best < ob) : (ob < best);
    best = upd ? ob : best;
    lab = upd ? ol : lab;
    lab -= off + coff;
    const uint8_t lb = eok ? static_cast<uint8_t>(lab) : static_cast<uint8_t>(0xFF);  // 0xFF: rows past m
    glab[(static_cast<size_t>(2 * iw_prob(ww) + iw_buf(ww))) * a.lsm + erow] = lb;
    es.iaccL[i] += (eok && hh == 0) ? xnr + best : 0.f;
    lsb[iw_prob(ww) * RT + ler] = lb;  // M-step labels, by problem
  }
}

// Add the f32 partials into the items' f64 accumulators (each item has exactly one
// contributing half-wave, so lane 0 of it is the only writer) and restart them.
template <int NL, int NS>
__device__ __forceinline__ void estep_flush(State& S, int tid, EState<NL, NS>& es) {
  const int er = tid & (RT - 1), hh = (tid >> 5) & 1, w = tid >> 6;
  const int nl = S.nlw[w], ns = S.nsw[w];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const double v = half_sum(static_cast<double>(es.iaccL[i]));
    if (i < nl && er == 0 && hh == 0) S.iinert[S.lstep[w][i]] += v;
    es.iaccL[i] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const double v = half_sum(static_cast<double>(es.iaccS[i]));
    if (i < ns && er == 0 && S.sstep[w][i][hh] != 0xFF) S.iinert[S.sstep[w][i][hh]] += v;
    es.iaccS[i] = 0.f;
  }
}

// A fragments of slot sl (register-resident for the sweep): a candidate row (exact f32 row of
// X), a running centre, or a dummy / alignment / unused slot (zero centre, +inf norm).
template <int DP>
__device__ __forceinline__ void slot_frags(const KArgs& a, const State& S, const float* cen, int sl, int ncols,
                                           int hh, h8 (&ah)[DP / 16], h8 (&al)[DP / 16]) {
  int sr = INT_MIN;
  if (sl < ncols) sr = S.srow[sl];
  const bool ok = sr != INT_MIN;
  const float* src = (sr >= 0) ? a.X + static_cast<size_t>(sr) * DP
                               : cen + static_cast<size_t>(ok ? -sr - 1 : 0) * DP;
  afrag_load<DP>(ah, al, src, ok, hh, a.scale);
}

// Distance wave: x.c of the tile's 32 rows against NS slot tiles (w, w + NDW) on f16 MFMA
// (xh.ch + xh.cl + xl.ch), one B operand read per k-step shared by the NS tiles, then
// D = |c|^2 - 2 x.c into the LDS distance tile (row lr, 4 slots per b128 store).
template <int DP, int NS>
__device__ __forceinline__ void dist_tiles(const KArgs& a, const State& S, const char* xs, float* dtile, int w,
                                           int lane, const h8 (&ah0)[DP / 16], const h8 (&al0)[DP / 16],
                                           const h8 (&ah1)[DP / 16], const h8 (&al1)[DP / 16]) {
  using LY = Lay<DP>;
  __builtin_amdgcn_s_setprio(1);  // MFMA-dense block first in the SIMD arbiter
  int lno = lane;
  asm volatile("" : "+v"(lno));  // per-lane offsets recomputed here (cheap), never held or spilled
  const int lro = lno & 31, hh = lno >> 5;
  // The accumulators start at -|c|^2 / dscale (exact: dscale is a power of two), so that
  // D = -dscale * acc = |c|^2 - dscale x.c needs no LDS read after the MFMAs (reads of |c|^2
  // between the distance-tile stores were serialised into one LDS round trip per 8 bytes by
  // the register-starved scheduler).
  v16f acc0, acc1 = {};
  {
    // d = 128: the scalar kernel argument (a VGPR copy of -1/dscale was spilled and reloaded
    // with a vmcnt(0) before the first MFMA); d = 32 / 64 keep the per-lane value (fewer spills)
    const float ninv = DP == 128 ? a.ndinv : -1.0f / a.dscale;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const float* cn = S.cnorm + 32 * (w + NDW * j) + 4 * hh;
      v16f& acc = j ? acc1 : acc0;
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // slots 8g + 4hh .. +3 of the tile
        const float4 c4 = *reinterpret_cast<const float4*>(cn + 8 * g);
        acc[4 * g] = c4.x * ninv;
        acc[4 * g + 1] = c4.y * ninv;
        acc[4 * g + 2] = c4.z * ninv;
        acc[4 * g + 3] = c4.w * ninv;
      }
    }
  }
  // B operands PD k-steps ahead of the MFMAs.  Two slot tiles: one step (6 MFMAs cover the
  // read; 16 VGPRs in flight).  One slot tile (narrow sweeps, where this wave's chain sets the
  // tile time): three MFMAs per step do not cover an LDS read under DMA traffic, so three steps
  // ahead, in the registers the second accumulator leaves free.
  constexpr int KS = DP / 16, PD = NS == 1 ? 2 : 1;
  h8 bh[KS], bl[KS];
#pragma unroll
  for (int s = 0; s < PD && s < KS; ++s) {
    const int off = xoff<DP>(lro, 2 * s + hh);
    bh[s] = *reinterpret_cast<const h8*>(xs + off);
    bl[s] = *reinterpret_cast<const h8*>(xs + LY::IMG + off);
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (s + PD < KS) {
      const int off = xoff<DP>(lro, 2 * (s + PD) + hh);
      bh[s + PD] = *reinterpret_cast<const h8*>(xs + off);
      bl[s + PD] = *reinterpret_cast<const h8*>(xs + LY::IMG + off);
    }
    acc0 = mfma16(ah0[s], bl[s], acc0);
    if constexpr (NS == 2) acc1 = mfma16(ah1[s], bl[s], acc1);
    acc0 = mfma16(al0[s], bh[s], acc0);
    if constexpr (NS == 2) acc1 = mfma16(al1[s], bh[s], acc1);
    acc0 = mfma16(ah0[s], bh[s], acc0);
    if constexpr (NS == 2) acc1 = mfma16(ah1[s], bh[s], acc1);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const v16f& acc = j ? acc1 : acc0;
    float* drow = dtile + lro * DSD + 32 * (w + NDW * j) + 4 * hh;
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // slots 8g + 4hh .. +3 of the tile: one b128 store
      float4 d;
      d.x = -a.dscale * acc[4 * g];
      d.y = -a.dscale * acc[4 * g + 1];
      d.z = -a.dscale * acc[4 * g + 2];
      d.w = -a.dscale * acc[4 * g + 3];
      *reinterpret_cast<float4*>(drow + 8 * g) = d;
    }
  }
  __builtin_amdgcn_s_setprio(0);
}

// E/M wave: one-hot A operand of the lane's slot (cluster mycl) for 8 rows of its 16-row k-block
// s2 of a tile (f16 1.0 where label == mycl), and their count.
// Packed: per 4 labels, XOR with the cluster replicated in every byte, a carry-free zero-byte
// test (0x80 where the label matches), the flags scaled to 0x3C (f16 1.0 = 0x3C00) and placed
// into the high byte of each f16 by v_perm; the count is a popcount of the flags.  A cluster of
// -1 (no running centre) compares against 0xFE, which no label takes (labels are < 127, 0xFF
// marks rows past m).
__device__ __forceinline__ h8 onehot8(const uint8_t* lsb, int s2, int hh, int mycl, unsigned& mcnt) {
  const uint2 lab = *reinterpret_cast<const uint2*>(lsb + 16 * s2 + 8 * hh);
  const unsigned rep = static_cast<unsigned>(mycl < 0 ? 0xFE : mycl) * 0x01010101u;
  u32x4 ohu;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const unsigned y = (h ? lab.y : lab.x) ^ rep;
    const unsigned z = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;  // 0x80: byte == 0
    mcnt += __builtin_popcount(z);
    const unsigned t = z >> 7;               // 0 / 1 per byte
    const unsigned f = (t << 6) - (t << 2);  // 0 / 0x3C per byte (no borrow across bytes)
    // f16 pairs: label 2i -> bits 15:8 of dword i, label 2i+1 -> bits 31:24 (selector 12 = 0x00)
    ohu[2 * h] = __builtin_amdgcn_perm(0u, f, 0x010C000Cu);
    ohu[2 * h + 1] = __builtin_amdgcn_perm(0u, f, 0x030C020Cu);
  }
  return __builtin_bit_cast(h8, ohu);
}

// E/M wave: M-step of NS slot tiles over one X tile: sums += one-hot(labels == cluster of the
// lane's slot) x (xh + xl) on f16 MFMA, counts by popcount.  B is the X tile read back
// transposed with ds_read_b64_tr_b16 from the swizzled image, once for the NS tiles.
// lsb0 / lsb1: the labels of the problem each tile's lane slot belongs to.  act1 (wave-uniform):
// the second tile has a running centre; without one its MFMAs are skipped (narrow sweeps; d = 128
// only).
template <int DP, int NS>
__device__ __forceinline__ void mstep_tiles(const char* xs, const uint8_t* lsb0, const uint8_t* lsb1, int lane,
                                            int mycl0, int mycl1, v16f (&sacc0)[DP / 32], v16f (&sacc1)[DP / 32],
                                            unsigned& mcnt0, unsigned& mcnt1, bool act1) {
  using LY = Lay<DP>;
  int lanel = lane;
  asm volatile("" : "+v"(lanel));
  const int G = lanel >> 4, q = (lanel >> 2) & 3, pp = lanel & 3, hh = lanel >> 5;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    __builtin_amdgcn_sched_barrier(0);  // bounded working set: one k-half at a time
    const h8 oh0 = onehot8(lsb0, s2, hh, mycl0, mcnt0);
    h8 oh1 = oh0;
    if constexpr (NS == 2) oh1 = onehot8(lsb1, s2, hh, mycl1, mcnt1);
    const int row0 = 16 * s2 + 8 * (G >> 1) + q;
    // transposed B reads one feature block ahead of its MFMAs
    auto rd = [&](int dt, s4 (&r)[4]) __attribute__((always_inline)) {
      const int chn = 4 * dt + 2 * (G & 1) + (pp >> 1);
      const int a0 = xoff<DP>(row0, chn) + 8 * (pp & 1);
      const int a1 = xoff<DP>(row0 + 4, chn) + 8 * (pp & 1);
      r[0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(xs + a0));
      r[1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(xs + a1));
      r[2] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(xs + LY::IMG + a0));
      r[3] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(xs + LY::IMG + a1));
    };
    s4 rc[4], rn[4];
    rd(0, rc);
#pragma unroll
    for (int dt = 0; dt < DP / 32; ++dt) {
      if (dt + 1 < DP / 32) rd(dt + 1, rn);
      const h8 bh = __builtin_bit_cast(h8, __builtin_shufflevector(rc[0], rc[1], 0, 1, 2, 3, 4, 5, 6, 7));
      const h8 bl = __builtin_bit_cast(h8, __builtin_shufflevector(rc[2], rc[3], 0, 1, 2, 3, 4, 5, 6, 7));
      sacc0[dt] = mfma16(oh0, bl, sacc0[dt]);
      if constexpr (NS == 2)
        if (DP < 128 || act1) {  // the skip costs spills at d = 32 / 64 (C2 +7 %, C5 +3 %)
          sacc1[dt] = mfma16(oh1, bl, sacc1[dt]);
          sacc1[dt] = mfma16(oh1, bh, sacc1[dt]);
        }
      sacc0[dt] = mfma16(oh0, bh, sacc0[dt]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 4; ++k) rc[k] = rn[k];
    }
  }
}

// E/M wave, after the sweep: the un-averaged sums of slot tile ct into Sm, the counts of its
// slots into S.cnt.
template <int DP>
__device__ __forceinline__ void msum_out(const KArgs& a, State& S, float* Sm, const v16f (&sacc)[DP / 32],
                                         unsigned mcnt, int ct, int msl, int lr, int hh) {
#pragma unroll
  for (int dt = 0; dt < DP / 32; ++dt)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int s2 = 32 * ct + (v & 3) + 8 * (v >> 2) + 4 * hh;
      Sm[s2 * DP + 32 * dt + lr] = sacc[dt][v] * a.inv_scale;
    }
  const unsigned tot = mcnt + __shfl_xor(mcnt, 32);
  if (hh == 0) S.cnt[msl] = tot;
}

// Thread 0: admit waiting problems into free seeding slots, then pack the next sweep:
// seeding candidates first (they are on every problem's critical path), then Lloyd
// problems round-robin from S.rr, first fit into the CW slots.
__device__ void schedule(const KArgs& a, State& S, const int32_t* idx, int dist_cost, bool sparse_ok) {
  const int P = S.P;
  for (int p = 0; p < P && S.seedfree; ++p) {
    if (S.st[p] != ST_WAIT) continue;
    const int s = __ffs(S.seedfree) - 1;
    S.seedfree &= ~(1u << s);
    S.sslot[p] = static_cast<unsigned char>(s);
    S.st[p] = ST_SEED;
    S.c[p] = 0;
  }
  int ni = 0, nc = 0, nls = 0, nss2 = 0;  // items, slots, Lloyd steps, seeding half-steps
  unsigned long long nseed = 0, nlloyd = 0, nm = 0;
  for (int p = 0; p < P; ++p) S.pitem[p] = -1;
  for (int p = 0; p < P; ++p) {
    if (S.st[p] != ST_SEED) continue;
    const int c = S.c[p];
    const int nt = (c == 0) ? 1 : S.ntr[p];
    if (nc + nt > CW || ni + nt > IMAX || nss2 + nt > 2 * (NEW * NSS + NDW * NSS_D)) continue;
    nss2 += nt;
    S.pitem[p] = static_cast<short>(ni);
    for (int t = 0; t < nt; ++t) {
      const int kind = (c == 0) ? IK_SEED0 : IK_SEED;
      S.ikind[ni] = static_cast<unsigned char>(kind);
      S.iprob[ni] = static_cast<unsigned char>(p);
      S.ioff[ni] = static_cast<short>(nc);
      S.incol[ni] = 1;
      S.itr[ni] = static_cast<unsigned char>(t);
      const int cs = (kind == IK_SEED0) ? 0 : S.cs[p];
      const int wslot = (kind == IK_SEED0) ? 0 : ((t < cs) ? t : t + 1);
      S.iw0[ni] = (static_cast<unsigned>(kind) << 24) | (static_cast<unsigned>(p) << 16) | (1u << 8) |
                  static_cast<unsigned>(nc);
      S.iw1[ni] = (static_cast<unsigned>(wslot) << 11) | (static_cast<unsigned>(cs) << 8) |
                  (static_cast<unsigned>(t) << 5) | static_cast<unsigned>(S.sslot[p]);
      const int pos = (c == 0) ? a.kpp_pos[S.kidx[p] * a.n_init + S.init[p]] : S.cand[p][t];
      S.sitem[nc] = static_cast<short>(ni);
      S.scl[nc] = -1;
      S.srow[nc] = idx[pos];
      ++ni;
      ++nc;
    }
    nseed += static_cast<unsigned long long>(nt) * a.m;
  }
  // Lloyd problems: 4-aligned offsets, K padded to a multiple of 4 with dummy (+inf) slots
  int first_skip = -1, last = -1;
  for (int j = 0; j < P; ++j) {
    const int p = (S.rr + j) % P;
    const int st = S.st[p];
    if (st != ST_RUN && st != ST_FINAL) continue;
    const int K = S.K[p], K4 = (K + 3) & ~3;
    const int off = (nc + 3) & ~3;
    if (off + K4 > CW || ni + 1 > IMAX || nls + 1 > NEW * NLS + NDW * NLS_D) {
      if (first_skip < 0) first_skip = p;
      continue;
    }
    for (int c = nc; c < off; ++c) {  // alignment gap
      S.sitem[c] = -1;
      S.scl[c] = -1;
      S.srow[c] = INT_MIN;
    }
    S.pitem[p] = static_cast<short>(ni);
    const int kind = (st == ST_RUN) ? IK_RUN : IK_FINAL;
    // sparse: the sums follow the labels that changed (few moved in the last E-step; no M-step
    // MFMAs); dense: the M-step recomputes them (the first iteration, after a burst of changes)
    const bool sparse = sparse_ok && st == ST_RUN && S.pchg[p] <= a.m / 8;
    S.isparse[ni] = static_cast<unsigned char>(sparse);
    S.ikind[ni] = static_cast<unsigned char>(kind);
    S.iprob[ni] = static_cast<unsigned char>(p);
    S.ioff[ni] = static_cast<short>(off);
    S.incol[ni] = static_cast<short>(K);
    S.itr[ni] = 0;
    S.iw0[ni] = (static_cast<unsigned>(1 - S.lcur[p]) << 30) | (static_cast<unsigned>(kind) << 24) |
                (static_cast<unsigned>(p) << 16) | (static_cast<unsigned>(K) << 8) | static_cast<unsigned>(off);
    S.iw1[ni] = 0;
    for (int c = 0; c < K4; ++c) {
      S.sitem[off + c] = static_cast<short>(c < K ? ni : -1);
      S.scl[off + c] = static_cast<short>((st == ST_RUN && !sparse && c < K) ? c : -1);  // M-step slots
      S.srow[off + c] = (c < K) ? -(S.cenoff[p] + c) - 1 : INT_MIN;
    }
    ++ni;
    ++nls;
    nc = off + K4;
    last = p;
    nlloyd += static_cast<unsigned long long>(K) * a.m;
    if (st == ST_RUN) nm += a.m;
    S.n_sparse += sparse;
  }
  S.rr = (first_skip >= 0) ? first_skip : (last >= 0 ? (last + 1) % P : S.rr);
  // deal the E-steps to the waves (LPT: heaviest first onto the least loaded wave).  Distance
  // wave w starts with the cost of its slot tiles' MFMAs (and takes at most NLS_D / NSS_D
  // steps), E/M wave NDW + q with the M-steps of slot tiles mstep_tile(q) and + NDW
  int wcost[NW];
  for (int w = 0; w < NW; ++w) {
    wcost[w] = 0;
    if (w < NDW)
      for (int j = w; j < CW / 32; j += NDW) wcost[w] += (32 * j < nc) ? dist_cost : 0;
    else
      for (int j = mstep_tile(w - NDW); j < CW / 32; j += NEW)
        for (int c = 32 * j; c < min(nc, 32 * j + 32); ++c)
          if (S.scl[c] >= 0) {
            wcost[w] += KM_COST_MSTEP;
            break;
          }
    S.nlw[w] = S.nsw[w] = 0;
    for (int i = 0; i < NLS; ++i) S.lstep[w][i] = 0xFF;
    for (int i = 0; i < NSS; ++i) S.sstep[w][i][0] = S.sstep[w][i][1] = 0xFF;
  }
  for (int it = 0; it < ni; ++it) {  // Lloyd items were appended after the seeding items
    if (S.ikind[it] < IK_RUN) continue;
    int w = -1;
    for (int q = 0; q < NW; ++q)
      if (S.nlw[q] < (q < NDW ? NLS_D : NLS) && (w < 0 || wcost[q] < wcost[w])) w = q;
    S.lstep[w][S.nlw[w]++] = static_cast<unsigned char>(it);
    wcost[w] += (S.incol[it] + 7) / 8 * KM_COST_LCHUNK + KM_COST_LBASE;
  }
  int open_w = -1;
  for (int it = 0; it < ni; ++it) {
    if (S.ikind[it] >= IK_RUN) continue;
    if (open_w >= 0) {  // second half of an open seeding step
      S.sstep[open_w][S.nsw[open_w] - 1][1] = static_cast<unsigned char>(it);
      open_w = -1;
      continue;
    }
    int w = -1;
    for (int q = 0; q < NW; ++q)
      if (S.nsw[q] < (q < NDW ? NSS_D : NSS) && (w < 0 || wcost[q] < wcost[w])) w = q;
    S.sstep[w][S.nsw[w]++][0] = static_cast<unsigned char>(it);
    wcost[w] += KM_COST_SSTEP;
    open_w = w;
  }
  S.nitems = ni;
  S.ncols = nc;
  S.n_seed += nseed;
  S.n_lloyd += nlloyd;
  S.n_mrows += nm;
  if (ni > 0) {
    S.n_sweeps += 1;
    S.n_ctiles += static_cast<unsigned long long>((nc + 31) / 32) * a.T;
  }
}

template <int DP>
__global__ __launch_bounds__(NT, 1) void kmeans_kernel(KArgs a) {
  using LY = Lay<DP>;
  __shared__ __attribute__((aligned(16))) char smem[LY::TOTAL];
  char* ring = smem;
  float* Dt = reinterpret_cast<float*>(smem + LY::OFF_D);   // [2][RT][DSD]
  float* Sm = reinterpret_cast<float*>(smem);               // [CW][DP] sums (aliases ring + D)
  uint8_t* Ls = reinterpret_cast<uint8_t*>(smem + LY::OFF_LS);
  float* XN = reinterpret_cast<float*>(smem + LY::OFF_XN);
  State& S = *reinterpret_cast<State*>(smem + LY::OFF_ST);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = a.m, T = a.T;
  uint8_t* wsb = a.ws + static_cast<size_t>(blockIdx.x) * a.ws_per_wg;
  uint8_t* glab = wsb;                                                  // [2 Pws][lsm]
  double* s64 = reinterpret_cast<double*>(wsb + a.off_s64);             // [Cws][DP] running sums
  int* c64 = reinterpret_cast<int*>(wsb + a.off_c64);                   // [Cws] running counts
  uint2* clist = reinterpret_cast<uint2*>(wsb + a.off_list);            // [Pws][NW][lseg] changes
  float* cen = reinterpret_cast<float*>(wsb + a.off_cen);               // [Cws][DP]
  float* cenn = reinterpret_cast<float*>(wsb + a.off_cenn);             // [Cws]
  int32_t* cpos = reinterpret_cast<int32_t*>(wsb + a.off_cpos);         // [Pws][Kws]
  float* dbuf = reinterpret_cast<float*>(wsb + a.off_dbuf);             // [seedmax][Tws+1][m]
  float* rdist = reinterpret_cast<float*>(wsb + a.off_rdist);           // [m]
  const int T1 = a.Tws + 1;
  if (tid == 0) S.n_lloyd = S.n_seed = S.n_mrows = S.n_reloc = S.n_sweeps = S.n_ctiles = S.n_sparse = S.n_changes = 0;

  for (;;) {
    __syncthreads();
    if (tid == 0) S.unit = static_cast<int>(atomicAdd(a.counter, 1u));
    __syncthreads();
    const int unit = S.unit;
    if (unit >= a.nh * a.nU) break;
    const int hb = unit / a.nU, g = unit - hb * a.nU;
    const int h = a.h_begin + hb;
    const int32_t* idx = a.idx + static_cast<size_t>(h) * m;
    const int32_t* gd = a.units + g * US;

    // ---- problem table --------------------------------------------------------
    if (tid == 0) {
      const int P = gd[0];
      S.P = P;
      int o = 0;
      for (int p = 0; p < P; ++p) {
        S.K[p] = static_cast<unsigned char>(gd[1 + 4 * p]);
        S.kidx[p] = static_cast<unsigned char>(gd[2 + 4 * p]);
        S.init[p] = static_cast<unsigned char>(gd[3 + 4 * p]);
        S.ntr[p] = static_cast<unsigned char>(gd[4 + 4 * p]);
        S.st[p] = ST_WAIT;
        S.iter[p] = 0;
        S.pchg[p] = a.m;
        S.lcur[p] = 0;
        S.cenoff[p] = static_cast<short>(o);
        o += S.K[p];
      }
      S.rr = 0;
      S.seedfree = (a.seedmax >= 32) ? 0xFFFFFFFFu : ((1u << a.seedmax) - 1u);
    }
    __syncthreads();
    const int P = S.P;
    for (size_t e = tid; e < static_cast<size_t>(2 * P) * a.lsm; e += NT) glab[e] = 0xFF;  // 2 buffers per problem

    // ---- tol = tol_rel * mean(var(X_sub, axis=0)) (sklearn _tolerance, :270-278) --
    {
      double* red = reinterpret_cast<double*>(ring);  // [NT/DP][DP]
      double* mean = reinterpret_cast<double*>(ring) + NT;
      constexpr int NPH = NT / DP;
      const int d = tid % DP, ph = tid / DP;
      double s = 0.0;
      for (int r = ph; r < m; r += NPH) s += static_cast<double>(a.X[static_cast<size_t>(idx[r]) * DP + d]);
      red[ph * DP + d] = s;
      __syncthreads();
      if (tid < DP) {
        double t = 0.0;
        for (int k = 0; k < NPH; ++k) t += red[k * DP + tid];
        mean[tid] = t / m;
      }
      __syncthreads();
      const double mu = mean[d];
      double q = 0.0;
      for (int r = ph; r < m; r += NPH) {
        const double v = static_cast<double>(a.X[static_cast<size_t>(idx[r]) * DP + d]) - mu;
        q += v * v;
      }
      __syncthreads();
      red[ph * DP + d] = q;
      __syncthreads();
      if (tid == 0) {
        double tot = 0.0;
        for (int dd = 0; dd < a.dreal; ++dd) {
          double t = 0.0;
          for (int k = 0; k < NPH; ++k) t += red[k * DP + dd];
          tot += t / m;
        }
        S.tol = static_cast<float>(static_cast<float>(tot / a.dreal) * a.tol_rel);
      }
      __syncthreads();
    }

    // ---- sweeps -----------------------------------------------------------------
    for (;;) {
      KM_STAMP(swp);
      if (tid == 0) {
        // d <= 64 (pair mode): the larger kernel body would leave these helpers out of line and
        // the KArgs copied to scratch; inline them there (at d = 128 the default choice stands)
        if constexpr (kPair<DP>) {
          [[clang::always_inline]] schedule(a, S, idx, dist_cost<DP>(), kSparse<DP> && !cc_km_dense_only);
        } else {
          schedule(a, S, idx, dist_cost<DP>(), kSparse<DP> && !cc_km_dense_only);
        }
      }
      __syncthreads();
      const int nitems = S.nitems, ncols = S.ncols;
      if (nitems == 0) break;

      // slot norms: centres from the last write-back, candidates from xnorm
      if (tid < ncols) {
        const int sr = S.srow[tid];
        S.cnorm[tid] = (sr >= 0) ? a.xnorm[sr] : (sr == INT_MIN ? __builtin_huge_valf() : cenn[-sr - 1]);
      }
      if (tid < 2 * RT * 4) Dt[(tid >> 2) * DSD + CW + (tid & 3)] = __builtin_huge_valf();  // +inf chunk
      if (tid < IMAX) S.iinert[tid] = 0.0;  // visible to the flushes after the prologue barrier
      if (tid < NW * NSS * 2) {  // seeding step descriptors
        const int w = tid / (2 * NSS), i = (tid / 2) % NSS, h = tid & 1;
        S.sdesc[w][i][h] = seed_desc(a, S, S.sstep[w][i][h], T1);
      }
      const int hh = lane >> 5, lr = lane & 31;
      const bool pm = kPair<DP> && ncols <= 4 * 32;  // block-uniform
      const int TP = (T + 1) >> 1;                    // row-tile pairs (pair mode)
#ifdef CC_KM_STAMPS
      unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
      // Role-specialised waves, one of each role per SIMD.  Waves 0..NDW-1 gather the X tiles
      // and run the distance MFMAs of slot tiles w and w + NDW; waves NDW..NW-1 run the E-steps
      // dealt to them and the M-steps of slot tiles q and q + NDW (q = w - NDW).  Each role has
      // its own loop (one barrier per tile in both), so their register sets never overlap and
      // the vector chain of one role runs while the other role's MFMAs occupy the matrix pipe.
      if (wave < NDW) {
        const int nsub = __builtin_amdgcn_readfirstlane(static_cast<int>(32 * wave < ncols) +
                                                        static_cast<int>(32 * (wave + NDW) < ncols));
        h8 ah0[DP / 16], al0[DP / 16], ah1[DP / 16], al1[DP / 16];
        slot_frags<DP>(a, S, cen, 32 * wave + lr, ncols, hh, ah0, al0);
        slot_frags<DP>(a, S, cen, 32 * (wave + NDW) + lr, ncols, hh, ah1, al1);
        // the distance wave's share of the E-steps (at most NLS_D Lloyd, NSS_D seeding steps)
        EState<NLS_D, NSS_D> es;
#pragma unroll
        for (int i = 0; i < NLS_D; ++i) es.iaccL[i] = 0.f;
#pragma unroll
        for (int i = 0; i < NSS_D; ++i) es.iaccS[i] = 0.f;
        const int nl = __builtin_amdgcn_readfirstlane(S.nlw[wave]);
        const int ns = __builtin_amdgcn_readfirstlane(S.nsw[wave]);
        unsigned lw[NLS_D];
#pragma unroll
        for (int i = 0; i < NLS_D; ++i)
          lw[i] = __builtin_amdgcn_readfirstlane(i < nl ? S.iw0[S.lstep[wave][i]] : 0u);
        unsigned pre[NSS_D];
#pragma unroll
        for (int i = 0; i < NSS_D; ++i) pre[i] = 0;
        if (!pm) {
        // pipeline prologue: tile 0 in the ring, indices of tile 1
        TileIdx<DP> nI;
        {
          TileIdx<DP> I0;
          TileAddr<DP> A0;
          idx_issue<DP>(a, idx, 0, wave, lane, I0);
          tile_addr<DP>(a, I0, wave, lane, A0);
          tile_issue<DP>(A0, ring, XN, wave);
          idx_issue<DP>(a, idx, RT, wave, lane, nI);
          dma_wait();
          tile_addr_hold<DP>(A0);
        }
        __syncthreads();
        KM_STAMP(sw0);
        KM_ACC(6, swp, sw0);
        for (int t = 0; t <= T + 1; ++t) {
          KM_STAMP(s0);
          if (t < T) {  // distances of tile t (MFMA) -> D[t & 1]
            const char* xs = ring + (t % kRing<DP>) * LY::SLOT;
            float* dtile = Dt + (t & 1) * (RT * DSD);
            if (nsub == 2)
              dist_tiles<DP, 2>(a, S, xs, dtile, wave, lane, ah0, al0, ah1, al1);
            else if (nsub == 1)
              dist_tiles<DP, 1>(a, S, xs, dtile, wave, lane, ah0, al0, ah1, al1);
          }
          KM_STAMP(s1);
          // rows of tile t+1 by LDS-DMA, after the distance MFMAs so that the pieces' address
          // registers (held to the end-of-iteration wait) do not overlap the A fragments'
          // busiest stretch: addresses of t+1 (consuming the index registers loaded last
          // iteration), the index loads of t+2 into them, then the pieces (all unconditional
          // but the pieces, so no branch lets the compiler reorder them; past the end the index
          // loads are clamped to row m-1 and unused).  The pieces land under the E-step share.
          TileAddr<DP> An;
          tile_addr<DP>(a, nI, wave, lane, An);
          idx_issue<DP>(a, idx, (t + 2) * RT, wave, lane, nI);
          if (t + 1 < T) tile_issue<DP>(An, ring + ((t + 1) % kRing<DP>) * LY::SLOT, XN + ((t + 1) % kRing<DP>) * 64, wave);
          KM_STAMP(s2);
          {
            int tidl = tid;
            asm volatile("" : "+v"(tidl));
            unsigned npre[NSS_D];
            estep_prefetch<NSS_D>(a, S, t, T, tidl, ns, dbuf, npre);
            estep<DP, NLS_D, NSS_D>(a, S, t, T, tidl, Dt, Ls, XN, glab, dbuf, pre, lw, nl, ns, es);
            if ((t % FLUSH) == FLUSH - 1) estep_flush(S, tid, es);
#pragma unroll
            for (int i = 0; i < NSS_D; ++i) pre[i] = npre[i];
          }
          KM_STAMP(s2e);
          dma_wait();  // tile t+1 and the indices of t+2 have landed
          tile_addr_hold<DP>(An);
          KM_STAMP(s3);
          __syncthreads();
          KM_STAMP(s4);
          KM_ACC(1, s0, s1);
          KM_ACC(0, s1, s2);
          KM_ACC(2, s2, s2e);
          KM_ACC(4, s2e, s3);
          KM_ACC(5, s3, s4);
        }
        } else if constexpr (kPair<DP>) {
          // pair mode: prologue tiles 0, 1 in the ring, indices of tiles 2, 3; per interval the
          // distances of tiles 2p, 2p+1 (this wave's one slot tile, A fragments shared), the
          // gather of 2p+2, 2p+3, the E-step share of 2p-2, 2p-1
          TileIdx<DP> nI0, nI1;
          unsigned preB[NSS_D];
#pragma unroll
          for (int i = 0; i < NSS_D; ++i) preB[i] = 0;
          {
            TileIdx<DP> I0, I1;
            TileAddr<DP> A0, A1;
            idx_issue<DP>(a, idx, 0, wave, lane, I0);
            idx_issue<DP>(a, idx, RT, wave, lane, I1);
            tile_addr<DP>(a, I0, wave, lane, A0);
            tile_addr<DP>(a, I1, wave, lane, A1);
            tile_issue<DP>(A0, ring, XN, wave);
            if (T > 1) tile_issue<DP>(A1, ring + LY::SLOT, XN + 64, wave);
            idx_issue<DP>(a, idx, 2 * RT, wave, lane, nI0);
            idx_issue<DP>(a, idx, 3 * RT, wave, lane, nI1);
            dma_wait();
            tile_addr_hold<DP>(A0);
            tile_addr_hold<DP>(A1);
          }
          __syncthreads();
          for (int pr = 0; pr <= TP + 1; ++pr) {
            const int tA = 2 * pr, tB = tA + 1;
            if (nsub == 1) {
              float* dtile = Dt + (pr & 1) * (RT * DSD);
              if (tA < T) dist_tiles<DP, 1>(a, S, ring + (tA % kRing<DP>) * LY::SLOT, dtile, wave, lane, ah0, al0, ah1, al1);
              if (tB < T) dist_tiles<DP, 1>(a, S, ring + (tB % kRing<DP>) * LY::SLOT, dtile + 128, wave, lane, ah0, al0, ah1, al1);
            }
            TileAddr<DP> An0, An1;
            tile_addr<DP>(a, nI0, wave, lane, An0);
            tile_addr<DP>(a, nI1, wave, lane, An1);
            idx_issue<DP>(a, idx, (tA + 4) * RT, wave, lane, nI0);
            idx_issue<DP>(a, idx, (tA + 5) * RT, wave, lane, nI1);
            if (tA + 2 < T)
              tile_issue<DP>(An0, ring + ((tA + 2) % kRing<DP>) * LY::SLOT, XN + ((tA + 2) % kRing<DP>) * 64, wave);
            if (tB + 2 < T)
              tile_issue<DP>(An1, ring + ((tB + 2) % kRing<DP>) * LY::SLOT, XN + ((tB + 2) % kRing<DP>) * 64, wave);
            {
              int tidl = tid;
              asm volatile("" : "+v"(tidl));
              unsigned npre[NSS_D], npreB[NSS_D];
              estep_prefetch<NSS_D>(a, S, tA, T, tidl, ns, dbuf, npre);
              estep_prefetch<NSS_D>(a, S, tB, T, tidl, ns, dbuf, npreB);
              estep<DP, NLS_D, NSS_D, true>(a, S, tA - 1, T, tidl, Dt, Ls, XN, glab, dbuf, pre, lw, nl, ns, es);
              if (((tA - 1) % FLUSH) == FLUSH - 1) estep_flush(S, tid, es);
              estep<DP, NLS_D, NSS_D, true>(a, S, tA, T, tidl, Dt, Ls, XN, glab, dbuf, preB, lw, nl, ns, es);
              if ((tA % FLUSH) == FLUSH - 1) estep_flush(S, tid, es);
#pragma unroll
              for (int i = 0; i < NSS_D; ++i) {
                pre[i] = npre[i];
                preB[i] = npreB[i];
              }
            }
            dma_wait();  // tiles 2p+2, 2p+3 and the indices of 2p+4, 2p+5 have landed
            tile_addr_hold<DP>(An0);
            tile_addr_hold<DP>(An1);
            __syncthreads();
          }
        }
        estep_flush(S, tid, es);
      } else {
        const int q = mstep_tile(wave - NDW);
        EState<NLS, NSS> es;
#pragma unroll
        for (int i = 0; i < NLS; ++i) es.iaccL[i] = 0.f;
#pragma unroll
        for (int i = 0; i < NSS; ++i) es.iaccS[i] = 0.f;
        // this wave's Lloyd step words, wave-uniform for the whole sweep
        const int nl = __builtin_amdgcn_readfirstlane(S.nlw[wave]);
        const int ns = __builtin_amdgcn_readfirstlane(S.nsw[wave]);
        unsigned lw[NLS];
#pragma unroll
        for (int i = 0; i < NLS; ++i)
          lw[i] = __builtin_amdgcn_readfirstlane(i < nl ? S.iw0[S.lstep[wave][i]] : 0u);
        // M-step slot tiles q and q + NDW: the lane's slot, its cluster and item
        const int msl0 = 32 * q + lr, msl1 = 32 * (q + NDW) + lr;
        int mycl0 = -1, myit0 = 0, mycl1 = -1, myit1 = 0;
        // (myit: the problem whose M-step labels the lane's slot reads; 0 when the slot is idle)
        if (msl0 < ncols) {
          mycl0 = S.scl[msl0];
          if (mycl0 >= 0) myit0 = S.iprob[S.sitem[msl0]];
        }
        if (msl1 < ncols) {
          mycl1 = S.scl[msl1];
          if (mycl1 >= 0) myit1 = S.iprob[S.sitem[msl1]];
        }
        const bool mact0 = __ballot(mycl0 >= 0) != 0ull;  // wave-uniform: any running centre
        const bool mact1 = __ballot(mycl1 >= 0) != 0ull;
        v16f sacc0[DP / 32], sacc1[DP / 32];
#pragma unroll
        for (int dt = 0; dt < DP / 32; ++dt) sacc0[dt] = sacc1[dt] = v16f{};
        unsigned mcnt0 = 0, mcnt1 = 0;
        unsigned pre[NSS];  // closest distances of the seeding steps of tile t-1 (loaded in t-1)
#pragma unroll
        for (int i = 0; i < NSS; ++i) pre[i] = 0;
        __syncthreads();
        KM_STAMP(sw0);
        KM_ACC(6, swp, sw0);
        if (!pm) {
        for (int t = 0; t <= T + 1; ++t) {
          KM_STAMP(s0);
          int tidl = tid;
          asm volatile("" : "+v"(tidl));
          // E-step operands of tile t (consumed next iteration)
          unsigned npre[NSS];
          estep_prefetch<NSS>(a, S, t, T, tidl, ns, dbuf, npre);
          KM_STAMP(s1);
          estep<DP, NLS, NSS>(a, S, t, T, tidl, Dt, Ls, XN, glab, dbuf, pre, lw, nl, ns, es);
          KM_STAMP(s2);
          // M-steps of tile t-2 (one-hot x X on f16 MFMA; counts by popcount)
          if (t >= 2) {
            const int tm = t - 2;
            const char* xs = ring + (tm % kRing<DP>) * LY::SLOT;
            const uint8_t* lsb = Ls + (tm & 1) * (LSN * RT);
            if (mact0 || mact1)  // both tiles share the transposed X reads (a tile without running
                                 // centres has an all-zero one-hot)
              mstep_tiles<DP, 2>(xs, lsb + myit0 * RT, lsb + myit1 * RT, lane, mycl0, mycl1, sacc0, sacc1, mcnt0, mcnt1, mact1);
          }
          if ((t % FLUSH) == FLUSH - 1) estep_flush(S, tid, es);
          KM_STAMP(s3);
#pragma unroll
          for (int i = 0; i < NSS; ++i) pre[i] = npre[i];
          __syncthreads();
          KM_STAMP(s4);
          KM_ACC(0, s0, s1);
          KM_ACC(2, s1, s2);
          KM_ACC(3, s2, s3);
          KM_ACC(5, s3, s4);
        }
        } else if constexpr (kPair<DP>) {
          // pair mode: per interval the E-steps of tiles 2p-2, 2p-1 and the M-steps of 2p-4,
          // 2p-3, in tile order
          unsigned preB[NSS];
#pragma unroll
          for (int i = 0; i < NSS; ++i) preB[i] = 0;
          for (int pr = 0; pr <= TP + 1; ++pr) {
            const int tA = 2 * pr, tB = tA + 1;
            int tidl = tid;
            asm volatile("" : "+v"(tidl));
            unsigned npre[NSS], npreB[NSS];
            estep_prefetch<NSS>(a, S, tA, T, tidl, ns, dbuf, npre);
            estep_prefetch<NSS>(a, S, tB, T, tidl, ns, dbuf, npreB);
            estep<DP, NLS, NSS, true>(a, S, tA - 1, T, tidl, Dt, Ls, XN, glab, dbuf, pre, lw, nl, ns, es);
            if (((tA - 1) % FLUSH) == FLUSH - 1) estep_flush(S, tid, es);
            estep<DP, NLS, NSS, true>(a, S, tA, T, tidl, Dt, Ls, XN, glab, dbuf, preB, lw, nl, ns, es);
            if ((tA % FLUSH) == FLUSH - 1) estep_flush(S, tid, es);
#pragma unroll
            for (int g = 0; g < 2; ++g) {
              const int tm = tA - 4 + g;
              if (tm >= 0 && tm < T && (mact0 || mact1)) {
                const char* xs = ring + (tm % kRing<DP>) * LY::SLOT;
                const uint8_t* lsb = Ls + (tm & 3) * (LSN * RT);
                mstep_tiles<DP, 2>(xs, lsb + myit0 * RT, lsb + myit1 * RT, lane, mycl0, mycl1, sacc0, sacc1, mcnt0, mcnt1, mact1);
              }
            }
#pragma unroll
            for (int i = 0; i < NSS; ++i) {
              pre[i] = npre[i];
              preB[i] = npreB[i];
            }
            __syncthreads();
          }
        }
        estep_flush(S, tid, es);
        dma_wait();  // label and closest-distance stores land before the post-sweep reads
        // sums -> Sm (aliases the ring and D: every reader passed the last loop barrier); counts
        if (mact0) msum_out<DP>(a, S, Sm, sacc0, mcnt0, q, msl0, lr, hh);
        if (mact1) msum_out<DP>(a, S, Sm, sacc1, mcnt1, q + NDW, msl1, lr, hh);
      }
#ifdef CC_KM_STAMPS
#ifdef CC_KM_STAMPS_NARROW
      if (ncols <= 32 && lane == 0 && a.stats)  // narrow sweeps only, every workgroup
#else
      if (blockIdx.x == 0 && lane == 0 && a.stats)
#endif
        for (int k = 0; k < 7; ++k) atomicAdd(&a.stats[8 + 8 * wave + k], st_acc[k]);
#endif
      __syncthreads();

      KM_STAMP(pp0);
      // ---- seeding decisions (thread per problem) -----------------------------------
      if (tid < P) {
        const int p = tid;
        S.need_sel[p] = 0;
        S.to_run[p] = 0;
        if (S.st[p] == ST_SEED && S.pitem[p] >= 0) {
          const int it0 = S.pitem[p], c = S.c[p];
          const int nt = (c == 0) ? 1 : S.ntr[p];
          int best = 0;
          float bv = static_cast<float>(S.iinert[it0]);
          for (int t = 1; t < nt; ++t) {
            const float v = static_cast<float>(S.iinert[it0 + t]);
            if (v < bv) {
              bv = v;
              best = t;
            }
          }
          S.pot32[p] = bv;
          const int cs = S.cs[p];
          S.cs[p] = static_cast<unsigned char>((c == 0) ? 0 : ((best < cs) ? best : best + 1));
          S.sbest[p] = static_cast<unsigned char>(best);
          cpos[p * a.Kws + c] = (c == 0) ? a.kpp_pos[S.kidx[p] * a.n_init + S.init[p]] : S.cand[p][best];
          S.c[p] = static_cast<unsigned char>(c + 1);
          if (c + 1 == S.K[p]) {
            S.to_run[p] = 1;  // seeding slot released below (single writer)
          } else {
            S.need_sel[p] = 1;
          }
        }
      }
      __syncthreads();
      if (tid == 0) {
        for (int p = 0; p < P; ++p)
          if (S.to_run[p]) {
            S.seedfree |= 1u << S.sslot[p];
            S.st[p] = ST_RUN;
            S.iter[p] = 0;
            S.pchg[p] = a.m;
          }
      }
      // candidate selection: one wave per problem
      {
        int j = 0;
        for (int p = 0; p < P; ++p) {
          if (!S.need_sel[p]) continue;
          if ((j++ % NW) != wave) continue;
          const int ss = S.sslot[p];
          if constexpr (kPair<DP>) {
            [[clang::always_inline]] kpp_select(a, S, p, dbuf + (static_cast<size_t>(ss) * T1 + S.cs[p]) * a.lsm, lane);
          } else {
            kpp_select(a, S, p, dbuf + (static_cast<size_t>(ss) * T1 + S.cs[p]) * a.lsm, lane);
          }
        }
      }
      // initial centres of problems leaving seeding: the chosen rows (exact f32)
      for (int p = 0; p < P; ++p) {
        if (!S.to_run[p]) continue;
        const int K = S.K[p];
        for (int e = tid; e < K * DP; e += NT) {
          const int c = e / DP, d = e - c * DP;
          cen[(S.cenoff[p] + c) * DP + d] = a.X[static_cast<size_t>(idx[cpos[p * a.Kws + c]]) * DP + d];
        }
        if (tid < K) cenn[S.cenoff[p] + tid] = row_sq(a.X + static_cast<size_t>(idx[cpos[p * a.Kws + tid]]) * DP, a.dreal);
      }

      KM_STAMP(ppA);
      // ---- labels changed? (RUN items): compare this sweep's label buffer with the previous
      // one, 16 B per thread and load, every item in one pass (flags set by any thread that sees
      // a difference: one barrier for all items instead of one per item); then this sweep's
      // buffer becomes the current one
      // ---- labels changed? (RUN items): compare this sweep's label buffer with the previous
      // one, each wave over its eighth of the rows; the changed rows of a sparse item go to its
      // change list (a dense item's are only counted); then this sweep's buffer becomes the
      // current one
      if constexpr (kSparse<DP>) {
        for (int it = 0; it < nitems; ++it) {
          if (S.ikind[it] != IK_RUN) continue;
          const int p = S.iprob[it];
          const uint8_t* cur = glab + static_cast<size_t>(2 * p + 1 - S.lcur[p]) * a.lsm;
          const uint8_t* old = glab + static_cast<size_t>(2 * p + S.lcur[p]) * a.lsm;
          const unsigned nc = list_changes(cur, old, m, wave, lane, clist + (static_cast<size_t>(p) * NW + wave) * a.lseg,
                                           S.isparse[it] ? static_cast<unsigned>(a.lseg) : 0u);
          if (lane == 0) S.lcnt[it][wave] = nc;
        }
        __syncthreads();
        if (tid < nitems) {
          const int it = tid;
          S.ichanged[it] = 0;
          if (S.ikind[it] == IK_RUN) {
            unsigned tot = 0;
            bool over = false;
            for (int w = 0; w < NW; ++w) {
              tot += S.lcnt[it][w];
              over |= S.lcnt[it][w] > static_cast<unsigned>(a.lseg);
            }
            S.pchg[S.iprob[it]] = static_cast<int>(tot);
            S.ichanged[it] = (tot != 0) | ((S.isparse[it] && over) ? 2u : 0u);  // 2: rebuild the sums
          }
        }
      } else {  // flags only: 16 B per thread and load, every item in one pass
        if (tid < nitems) S.ichanged[tid] = 0;
        __syncthreads();
        for (int it = 0; it < nitems; ++it) {
          if (S.ikind[it] != IK_RUN) continue;
          const int p = S.iprob[it];
          const uint4* cur = reinterpret_cast<const uint4*>(glab + static_cast<size_t>(2 * p + 1 - S.lcur[p]) * a.lsm);
          const uint4* old = reinterpret_cast<const uint4*>(glab + static_cast<size_t>(2 * p + S.lcur[p]) * a.lsm);
          bool diff = false;
          for (int e = tid; e < (m + 15) / 16; e += NT) {
            const uint4 x = cur[e], y = old[e];
            diff |= (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
          }
          if (diff) S.ichanged[it] = 1;
        }
      }
      __syncthreads();
      if (tid == 0)
        for (int it = 0; it < nitems; ++it)
          if (S.ikind[it] >= IK_RUN) {
            S.lcur[S.iprob[it]] = static_cast<unsigned char>(1 - S.lcur[S.iprob[it]]);
            if (S.ikind[it] == IK_RUN) S.n_changes += static_cast<unsigned>(S.pchg[S.iprob[it]]);
          }
      __syncthreads();
      KM_STAMP(ppB);

      // ---- running sums (d = 128): dense items take the M-step's sums; sparse items add their
      // change lists (one wave per item) into the f64 sums, which then feed the centre update below
      if constexpr (kSparse<DP>) {
        for (int e = tid; e < ncols * DP; e += NT) {
          const int sl = e / DP, d = e - sl * DP;
          const int it = S.sitem[sl];
          if (it < 0 || S.ikind[it] != IK_RUN || S.isparse[it] || sl - S.ioff[it] >= S.K[S.iprob[it]]) continue;
          const int row = S.cenoff[S.iprob[it]] + (sl - S.ioff[it]);
          s64[static_cast<size_t>(row) * DP + d] = static_cast<double>(Sm[e]);
          if (d == 0) c64[row] = static_cast<int>(S.cnt[sl]);
        }
        {
          int j = 0;
          for (int it = 0; it < nitems; ++it) {
            if (S.ikind[it] != IK_RUN || !S.isparse[it]) continue;
            if ((j++ % NW) != wave) continue;
            const int p = S.iprob[it], off = S.ioff[it];
            apply_changes<DP>(a, idx, clist + static_cast<size_t>(p) * NW * a.lseg, S.lcnt[it], (S.ichanged[it] & 2u) != 0,
                              glab + static_cast<size_t>(2 * p + S.lcur[p]) * a.lsm, Sm + static_cast<size_t>(off) * DP,
                              S.cnt + off, S.K[p], lane);
          }
        }
        __syncthreads();
        for (int e = tid; e < ncols * DP; e += NT) {  // sparse items: f64 sums += the f32 deltas
          const int sl = e / DP, d = e - sl * DP;
          const int it = S.sitem[sl];
          if (it < 0 || S.ikind[it] != IK_RUN || !S.isparse[it] || sl - S.ioff[it] >= S.K[S.iprob[it]]) continue;
          const int row = S.cenoff[S.iprob[it]] + (sl - S.ioff[it]);
          const bool full = (S.ichanged[it] & 2u) != 0;
          double* sp = s64 + static_cast<size_t>(row) * DP + d;
          const double t = (full ? 0.0 : *sp) + static_cast<double>(Sm[e]);
          *sp = t;
          Sm[e] = static_cast<float>(t);
          if (d == 0) {
            const int c = (full ? 0 : c64[row]) + static_cast<int>(S.cnt[sl]);
            c64[row] = c;
            S.cnt[sl] = static_cast<unsigned>(c);
          }
        }
        __syncthreads();
      }

      KM_STAMP(ppC);
      // ---- Lloyd M-step completion (RUN items) ------------------------------------
      if (tid == 0) {
        int f = 0;
        for (int it = 0; it < nitems; ++it) {
          if (S.ikind[it] != IK_RUN) continue;
          const int p = S.iprob[it], off = S.ioff[it];
          int ne = 0;
          for (int c = 0; c < S.K[p]; ++c) ne += (S.cnt[off + c] == 0);
          S.nempty[p] = ne;
          f |= (ne > 0);
        }
        S.flag = f;
      }
      __syncthreads();
      if (S.flag) {
        for (int it = 0; it < nitems; ++it) {
          if (S.ikind[it] != IK_RUN) continue;
          const int p = S.iprob[it];
          if (S.nempty[p] == 0) continue;
          if constexpr (kPair<DP>) {
            [[clang::always_inline]] relocate<DP>(a, idx, p, S.ioff[it], cen, Sm, S,
                                                  glab + static_cast<size_t>(2 * p + S.lcur[p]) * a.lsm, rdist, tid);
          } else {
            relocate<DP>(a, idx, p, S.ioff[it], cen, Sm, S, glab + static_cast<size_t>(2 * p + S.lcur[p]) * a.lsm,
                         rdist, tid);
          }
          __syncthreads();
        }
      }
      // first argmax of counts per problem (for clusters still empty: _average_centers)
      if (tid < nitems && S.ikind[tid] == IK_RUN) {
        const int p = S.iprob[tid], off = S.ioff[tid];
        int am = 0;
        for (int c = 1; c < S.K[p]; ++c)
          if (S.cnt[off + c] > S.cnt[off + am]) am = c;
        S.amax[p] = am;
      }
      __syncthreads();
      // _average_centers (_k_means_common.pyx:215-237) runs j in order: an empty cluster
      // j copies centre argmax(weight), which is still a raw sum when j < argmax.
      for (int e = tid; e < ncols * DP; e += NT) {
        const int sl = e / DP, d = e - sl * DP;
        const int it = S.sitem[sl];
        if (it < 0 || S.ikind[it] != IK_RUN || S.cnt[sl] != 0) continue;
        const int p = S.iprob[it], off = S.ioff[it];
        if (sl - off > S.amax[p]) continue;
        Sm[sl * DP + d] = Sm[(off + S.amax[p]) * DP + d];
      }
      __syncthreads();
      for (int e = tid; e < ncols * DP; e += NT) {
        const int sl = e / DP;
        if (S.sitem[sl] < 0 || S.ikind[S.sitem[sl]] != IK_RUN) continue;
        const unsigned cn = S.cnt[sl];
        if (cn > 0) {
          const float alpha = static_cast<float>(1.0 / static_cast<double>(static_cast<float>(cn)));
          Sm[e] *= alpha;
        }
      }
      __syncthreads();
      for (int e = tid; e < ncols * DP; e += NT) {
        const int sl = e / DP, d = e - sl * DP;
        const int it = S.sitem[sl];
        if (it < 0 || S.ikind[it] != IK_RUN || S.cnt[sl] != 0) continue;
        const int p = S.iprob[it], off = S.ioff[it];
        if (sl - off < S.amax[p]) continue;
        Sm[sl * DP + d] = Sm[(off + S.amax[p]) * DP + d];
      }
      __syncthreads();
      // centre shifts (sklearn _euclidean_dense_dense, 4-way unrolled f32)
      if (tid < ncols && S.sitem[tid] >= 0 && S.ikind[S.sitem[tid]] == IK_RUN) {
        const int sl = tid;
        const int it = S.sitem[sl];
        const int p = S.iprob[it];
        const float* cnw = Sm + sl * DP;
        const float* co = cen + (S.cenoff[p] + (sl - S.ioff[it])) * DP;
        float res = 0.f;
        const int n4 = a.dreal / 4, rem = a.dreal % 4;
        for (int i = 0; i < n4; ++i) {
          const float d0 = cnw[4 * i] - co[4 * i], d1 = cnw[4 * i + 1] - co[4 * i + 1];
          const float d2 = cnw[4 * i + 2] - co[4 * i + 2], d3 = cnw[4 * i + 3] - co[4 * i + 3];
          res += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
        }
        for (int i = 0; i < rem; ++i) {
          const float dd = cnw[4 * n4 + i] - co[4 * n4 + i];
          res += dd * dd;
        }
        const float sh = sqrtf(res);
        S.shift[sl] = sh * sh;
      }
      __syncthreads();
      // convergence decisions (_kmeans_single_lloyd :697-736)
      if (tid < nitems && S.ikind[tid] >= IK_RUN) {
        const int it = tid, p = S.iprob[it];
        if (S.ikind[it] == IK_RUN) {
          S.iter[p] += 1;
          if (!S.ichanged[it]) {
            S.st[p] = ST_DONE;  // strict convergence: final labels are this sweep's
            S.inert[p] = static_cast<float>(S.iinert[it]);
          } else {
            const float tot = np_pairwise_sum(S.shift + S.ioff[it], S.K[p]);
            S.st[p] = (tot <= S.tol || S.iter[p] >= a.max_iter) ? ST_FINAL : ST_RUN;
          }
        } else {
          S.st[p] = ST_DONE;
          S.inert[p] = static_cast<float>(S.iinert[it]);
        }
      }
      __syncthreads();
      // write back the centres (and norms) of problems that sweep again
      for (int e = tid; e < ncols * DP; e += NT) {
        const int sl = e / DP, d = e - sl * DP;
        const int it = S.sitem[sl];
        if (it < 0 || S.ikind[it] != IK_RUN) continue;
        const int p = S.iprob[it];
        if (S.st[p] == ST_DONE) continue;
        cen[(S.cenoff[p] + (sl - S.ioff[it])) * DP + d] = Sm[e];
      }
      if (tid < ncols) {
        const int it = S.sitem[tid];
        if (it >= 0 && S.ikind[it] == IK_RUN) {
          const int p = S.iprob[it];
          if (S.st[p] != ST_DONE) cenn[S.cenoff[p] + (tid - S.ioff[it])] = row_sq(Sm + tid * DP, a.dreal);
        }
      }
      __syncthreads();
#ifdef CC_KM_STAMPS
      KM_STAMP(pp1);
      if (blockIdx.x == 0 && tid == 0 && a.stats) {
        atomicAdd(&a.stats[73], pp1 - pp0);
        // post-processing phases: seeding, label compare, running sums, centre update
        atomicAdd(&a.stats[106], ppA - pp0);
        atomicAdd(&a.stats[107], ppB - ppA);
        atomicAdd(&a.stats[108], ppC - ppB);
        atomicAdd(&a.stats[109], pp1 - ppC);
      }
      // sweep cycles and counts by width (active 32-slot waves 1..8), all workgroups
      if (tid == 0 && a.stats) {
        const int wv = (ncols + 31) / 32;
        atomicAdd(&a.stats[80 + wv], pp1 - swp);
        atomicAdd(&a.stats[96 + wv], 1ull);
      }
#endif
    }

    // ---- best of n_init per K, output (KMeans.fit :1495-1531) -------------------
    for (int p0 = 0; p0 < P; p0 += a.n_init) {
      int best = p0;
      for (int i = 1; i < a.n_init; ++i) {
        const int p = p0 + i;
        if (!(S.inert[p] < S.inert[best])) continue;
        // _is_same_clustering(labels_p, labels_best): labels_p -> labels_best must be a function
        if (tid <= KMAX) S.map[tid] = -1;
        if (tid == 0) S.flag = 0;
        __syncthreads();
        const uint8_t* l1 = glab + static_cast<size_t>(2 * p + S.lcur[p]) * a.lsm;
        const uint8_t* l2 = glab + static_cast<size_t>(2 * best + S.lcur[best]) * a.lsm;
        for (int r = tid; r < m; r += NT) S.map[l1[r]] = l2[r];
        __syncthreads();
        bool bad = false;
        for (int r = tid; r < m; r += NT) bad |= (S.map[l1[r]] != l2[r]);
        if (bad) S.flag = 1;
        __syncthreads();
        if (S.flag) best = p;
        __syncthreads();
      }
      const int kidx = S.kidx[p0];
      const uint8_t* lb = glab + static_cast<size_t>(2 * best + S.lcur[best]) * a.lsm;
      uint8_t* out = a.labels_out + static_cast<size_t>(kidx) * a.n * a.ldl + h;
      for (int r = tid; r < m; r += NT) out[static_cast<size_t>(idx[r]) * a.ldl] = lb[r];
      if (tid == 0) {
        if (a.inertia_out) a.inertia_out[static_cast<size_t>(kidx) * a.H + h] = S.inert[best];
        if (a.niter_out) a.niter_out[static_cast<size_t>(kidx) * a.H + h] = S.iter[best];
      }
    }
  }
  if (tid == 0 && a.stats) {
    atomicAdd(&a.stats[0], S.n_lloyd);
    atomicAdd(&a.stats[1], S.n_seed);
    atomicAdd(&a.stats[2], S.n_mrows);
    atomicAdd(&a.stats[3], S.n_reloc);
    atomicAdd(&a.stats[4], S.n_sweeps);
    atomicAdd(&a.stats[5], S.n_ctiles);
    atomicAdd(&a.stats[6], S.n_sparse);
    atomicAdd(&a.stats[7], S.n_changes);
  }
}

// f16 hi/lo image of the rows: Xhl[r][0][d] = f16(x s), Xhl[r][1][d] = f16(x s - hi), s = 2^e.
__global__ void split_kernel(const float* X, long long total, int dpad, float scale, uint16_t* Xhl) {
  const long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long long row = i / dpad;
  const int d = static_cast<int>(i - row * dpad);
  const float xs = X[i] * scale;
  const _Float16 hi = static_cast<_Float16>(xs);
  const _Float16 lo = static_cast<_Float16>(xs - static_cast<float>(hi));
  Xhl[row * 2 * dpad + d] = __builtin_bit_cast(uint16_t, hi);
  Xhl[row * 2 * dpad + dpad + d] = __builtin_bit_cast(uint16_t, lo);
}

int local_trials(int K) { return 2 + static_cast<int>(std::log(static_cast<double>(K))); }

struct WsLayout {
  int Pws = 0, Cws = 0, Kws = 0, Tws = 0, lseg = 0;
  size_t off_cen = 0, off_cenn = 0, off_cpos = 0, off_dbuf = 0, off_rdist = 0, off_s64 = 0, off_c64 = 0,
         off_list = 0, per_wg = 0;
};

// Change-list entries per problem and wave segment (a segment covers m / 8 rows): a sparse
// iteration expects at most m / 8 changed labels (the scheduler's threshold); a segment that
// overflows makes the post-sweep phase rebuild the sums from every label instead.
int list_seg(int m) { return std::max(16, ((m / 16) + 15) & ~15); }

constexpr size_t WS_HEADER = 256;  // the work counter

WsLayout ws_layout(int m, int dpad, const int32_t* units, int nU, int seedmax) {
  WsLayout L;
  for (int g = 0; g < nU; ++g) {
    const int32_t* gd = units + static_cast<size_t>(g) * US;
    L.Pws = std::max(L.Pws, gd[0]);
    int cols = 0;
    for (int p = 0; p < gd[0]; ++p) {
      L.Kws = std::max(L.Kws, gd[1 + 4 * p]);
      L.Tws = std::max(L.Tws, gd[4 + 4 * p]);
      cols += gd[1 + 4 * p];
    }
    L.Cws = std::max(L.Cws, cols);
  }
  auto al = [](size_t x) { return (x + 255) & ~static_cast<size_t>(255); };
  L.off_cen = al(static_cast<size_t>(2 * L.Pws) * ((m + 63) & ~63));
  L.off_cenn = L.off_cen + al(static_cast<size_t>(L.Cws) * dpad * sizeof(float));
  L.off_cpos = L.off_cenn + al(static_cast<size_t>(L.Cws) * sizeof(float));
  L.off_dbuf = L.off_cpos + al(static_cast<size_t>(L.Pws) * L.Kws * sizeof(int32_t));
  L.off_rdist = L.off_dbuf + al(static_cast<size_t>(seedmax) * (L.Tws + 1) * ((m + 63) & ~63) * sizeof(float));
  // the sparse M-step's running sums, counts and change lists (d = 128 only, kSparse)
  const bool sp = dpad == 128;
  L.off_s64 = L.off_rdist + al(static_cast<size_t>(m) * sizeof(float));
  L.off_c64 = L.off_s64 + (sp ? al(static_cast<size_t>(L.Cws) * dpad * sizeof(double)) : 0);
  L.off_list = L.off_c64 + (sp ? al(static_cast<size_t>(L.Cws) * sizeof(int)) : 0);
  L.lseg = list_seg(m);
  L.per_wg = L.off_list + (sp ? al(static_cast<size_t>(L.Pws) * NW * L.lseg * sizeof(uint2)) : 0);
  return L;
}

template <int DP>
void launch(const KArgs& a, unsigned blocks, hipStream_t st) {
  hipLaunchKernelGGL(kmeans_kernel<DP>, dim3(blocks), dim3(NT), 0, st, a);
}

}  // namespace

extern "C" int cc_kmeans_plan(const int32_t* Ks, int nK, int n_init, int n_sub, int32_t* units,
                              int max_units) {
  if (!Ks || nK <= 0 || n_init <= 0 || n_sub <= 0 || !units || max_units <= 0) {
    cc::set_error("cc_kmeans_plan: bad arguments");
    return CC_ERR_ARG;
  }
  if (n_init > PMAX) {
    cc::set_error("cc_kmeans_plan: n_init must be <= 64");
    return CC_ERR_UNSUPPORTED;
  }
  std::vector<int> order(nK);
  for (int i = 0; i < nK; ++i) {
    if (Ks[i] < 1 || Ks[i] > KMAX) {
      cc::set_error("cc_kmeans_plan: need 1 <= K <= 127");
      return CC_ERR_UNSUPPORTED;
    }
    order[i] = i;
  }
  // every unit must hold <= PMAX problems: at least ceil(nK*n_init / PMAX) units
  const int per_unit = PMAX / n_init;  // K groups per unit
  const int nU = std::max(n_sub, (nK + per_unit - 1) / per_unit);
  if (nU > max_units) {
    cc::set_error("cc_kmeans_plan: max_units too small");
    return CC_ERR_ARG;
  }
  // largest K first (longest critical paths admitted first); greedy balance of K^2 cost
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return Ks[x] > Ks[y]; });
  std::vector<double> cost(nU, 0.0);
  std::vector<int> probs(nU, 0);
  std::fill(units, units + static_cast<size_t>(nU) * US, 0);
  for (int k : order) {
    int g = -1;
    for (int u = 0; u < nU; ++u) {
      if (probs[u] + n_init > PMAX) continue;
      if (g < 0 || cost[u] < cost[g]) g = u;
    }
    if (g < 0) {
      cc::set_error("cc_kmeans_plan: internal packing failure");
      return CC_ERR_ARG;
    }
    int32_t* gd = units + static_cast<size_t>(g) * US;
    for (int i = 0; i < n_init; ++i) {
      const int p = probs[g] + i;
      gd[1 + 4 * p] = Ks[k];
      gd[2 + 4 * p] = k;
      gd[3 + 4 * p] = i;
      gd[4 + 4 * p] = local_trials(Ks[k]);
    }
    probs[g] += n_init;
    gd[0] = probs[g];
    cost[g] += static_cast<double>(Ks[k]) * (Ks[k] + 8) * n_init;
  }
  // drop empty units (n_sub larger than the number of K groups)
  int w = 0;
  for (int u = 0; u < nU; ++u) {
    if (units[static_cast<size_t>(u) * US] == 0) continue;
    if (w != u) std::copy(units + static_cast<size_t>(u) * US, units + static_cast<size_t>(u + 1) * US,
                          units + static_cast<size_t>(w) * US);
    ++w;
  }
  return w;
}

extern "C" size_t cc_kmeans_workspace_bytes(int m, int dpad, const int32_t* units_host, int nU,
                                            int seedmax, int grid) {
  if (m <= 0 || !units_host || nU <= 0 || seedmax <= 0 || grid <= 0) return 0;
  return WS_HEADER + ws_layout(m, dpad, units_host, nU, seedmax).per_wg * static_cast<size_t>(grid);
}

extern "C" int cc_split_f16(const float* X, int n, int dpad, int scale_exp, uint16_t* Xhl, void* stream) {
  if (!X || !Xhl || n <= 0 || dpad <= 0 || scale_exp < -62 || scale_exp > 62) {
    cc::set_error("cc_split_f16: bad arguments");
    return CC_ERR_ARG;
  }
  const long long total = static_cast<long long>(n) * dpad;
  const unsigned blocks = static_cast<unsigned>((total + 255) / 256);
  hipLaunchKernelGGL(split_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), X, total,
                     dpad, std::ldexp(1.0f, scale_exp), Xhl);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_split_f16: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}

extern "C" int cc_kmeans_batched(const float* X, const uint16_t* Xhl, const float* xnorm, int n,
                                 int dreal, int dpad, int scale_exp, const int32_t* idx_hm, int H,
                                 int m, int h_begin, int h_end, const int32_t* units,
                                 const int32_t* units_host, int nU, int n_init, int max_iter,
                                 double tol_rel, const double* kpp_u, int kpp_stride,
                                 const int32_t* kpp_pos, uint8_t* labels_nh, int ldl, float* inertia,
                                 int32_t* n_iter, unsigned long long* stats, void* workspace,
                                 size_t ws_bytes, int grid, int seedmax, void* stream) {
  if (!X || !Xhl || !xnorm || !idx_hm || !units || !units_host || !kpp_u || !kpp_pos || !labels_nh ||
      n <= 0 || m <= 0 || m > n || H <= 0 || h_begin < 0 || h_end > H || h_end < h_begin || nU <= 0 ||
      n_init <= 0 || max_iter <= 0 || dreal <= 0 || dreal > dpad || ldl < H || grid <= 0 ||
      seedmax <= 0 || seedmax > 32 || scale_exp < -62 || scale_exp > 62) {
    cc::set_error("cc_kmeans_batched: bad arguments");
    return CC_ERR_ARG;
  }
  if (((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Xhl) | reinterpret_cast<uintptr_t>(workspace)) & 15) != 0) {
    cc::set_error("cc_kmeans_batched: X, Xhl and the workspace must be 16-B aligned (16-B row and LDS-DMA loads)");
    return CC_ERR_ARG;
  }
  if (dpad != 32 && dpad != 64 && dpad != 128) {
    cc::set_error("cc_kmeans_batched: dpad must be 32, 64 or 128 (d <= 128 in this build)");
    return CC_ERR_UNSUPPORTED;
  }
  int kmax = 0, tmax = 0;
  for (int g = 0; g < nU; ++g) {
    const int32_t* gd = units_host + static_cast<size_t>(g) * US;
    if (gd[0] <= 0 || gd[0] > PMAX || gd[0] % n_init != 0) {
      cc::set_error("cc_kmeans_batched: malformed unit descriptor");
      return CC_ERR_ARG;
    }
    for (int p = 0; p < gd[0]; ++p) {
      const int K = gd[1 + 4 * p];
      if (K < 1 || K > KMAX || K > m || gd[4 + 4 * p] != local_trials(K) || gd[4 + 4 * p] > TMAX ||
          gd[3 + 4 * p] < 0 || gd[3 + 4 * p] >= n_init || gd[2 + 4 * p] < 0 || gd[2 + 4 * p] > 255) {
        cc::set_error("cc_kmeans_batched: bad problem in unit (1 <= K <= min(127, m))");
        return CC_ERR_ARG;
      }
      kmax = std::max(kmax, K);
      tmax = std::max(tmax, gd[4 + 4 * p]);
    }
  }
  if (kpp_stride < 1 + (kmax - 1) * tmax) {
    cc::set_error("cc_kmeans_batched: kpp_stride too small");
    return CC_ERR_ARG;
  }
  const int nh = h_end - h_begin;
  if (nh == 0) return CC_OK;
  const WsLayout L = ws_layout(m, dpad, units_host, nU, seedmax);
  if (static_cast<double>(seedmax) * (L.Tws + 1) * ((m + 63) & ~63) >= 4294967296.0) {
    cc::set_error("cc_kmeans_batched: closest-distance buffers exceed 2^32 floats (lower seedmax)");
    return CC_ERR_UNSUPPORTED;
  }
  if (!workspace || ws_bytes < WS_HEADER + L.per_wg * static_cast<size_t>(grid)) {
    cc::set_error("cc_kmeans_batched: workspace too small");
    return CC_ERR_ARG;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(workspace, 0, sizeof(unsigned), st);
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_kmeans_batched: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  KArgs a{};
  a.X = X;
  a.Xhl = Xhl;
  a.xnorm = xnorm;
  a.dreal = dreal;
  a.scale = std::ldexp(1.0f, scale_exp);
  a.inv_scale = std::ldexp(1.0f, -scale_exp);
  a.dscale = std::ldexp(1.0f, 1 - 2 * scale_exp);
  a.ndinv = -std::ldexp(1.0f, 2 * scale_exp - 1);
  a.idx = idx_hm;
  a.m = m;
  a.h_begin = h_begin;
  a.nh = nh;
  a.T = (m + RT - 1) / RT;
  a.units = units;
  a.nU = nU;
  a.max_iter = max_iter;
  a.tol_rel = tol_rel;
  a.kpp_u = kpp_u;
  a.kpp_stride = kpp_stride;
  a.n_init = n_init;
  a.kpp_pos = kpp_pos;
  a.labels_out = labels_nh;
  a.n = n;
  a.ldl = ldl;
  a.H = H;
  a.inertia_out = inertia;
  a.niter_out = n_iter;
  a.stats = stats;
  a.counter = static_cast<unsigned*>(workspace);
  a.ws = static_cast<uint8_t*>(workspace) + WS_HEADER;
  a.ws_per_wg = L.per_wg;
  a.off_cen = L.off_cen;
  a.off_cenn = L.off_cenn;
  a.off_cpos = L.off_cpos;
  a.off_dbuf = L.off_dbuf;
  a.off_rdist = L.off_rdist;
  a.off_s64 = L.off_s64;
  a.off_c64 = L.off_c64;
  a.off_list = L.off_list;
  a.lseg = L.lseg;
  a.Pws = L.Pws;
  a.Kws = L.Kws;
  a.Tws = L.Tws;
  a.seedmax = seedmax;
  a.lsm = (m + 63) & ~63;
  {
    static int dense_set = 0;  // the value last written to the device global
    const char* dm = std::getenv("CCMI_KM_DENSE");
    const int dense = (dm && dm[0] == '1') ? 1 : 0;
    if (dense != dense_set) {
      e = hipMemcpyToSymbolAsync(HIP_SYMBOL(cc_km_dense_only), &dense, sizeof(int), 0, hipMemcpyHostToDevice, st);
      if (e != hipSuccess) {
        cc::set_error(std::string("cc_kmeans_batched: ") + hipGetErrorString(e));
        return CC_ERR_HIP;
      }
      dense_set = dense;
    }
  }
  const unsigned blocks = static_cast<unsigned>(std::min<long long>(grid, static_cast<long long>(nh) * nU));
  switch (dpad) {
    case 32: launch<32>(a, blocks, st); break;
    case 64: launch<64>(a, blocks, st); break;
    default: launch<128>(a, blocks, st); break;
  }
  e = hipGetLastError();
  if (e != hipSuccess) {
    cc::set_error(std::string("cc_kmeans_batched: ") + hipGetErrorString(e));
    return CC_ERR_HIP;
  }
  return CC_OK;
}
