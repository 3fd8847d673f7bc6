// Batched k-means for wide rows (d > 128) on gfx950: the distance-GEMM-bound path of BASELINE
// config 4 (n = 5k samples x d = 20k features).
//
// The same fits and decisions as kmeans.hip (scikit-learn KMeans: k-means++ seeding
// sklearn/cluster/_kmeans.py:174-262, Lloyd :624-752 with _k_means_lloyd.pyx:23-212, empty
// cluster relocation _k_means_common.pyx:167-212, best of n_init :1495-1531) for every
// `clusterer.fit_predict(X[indices])` of the reference (consensus_clustering_parallelised.py:282),
// organised for rows that do not fit on chip.  Work advances in ROUNDS; one round moves every
// active (resample, K, init) problem of a batch of resamples by one step (one k-means++ centre,
// or one Lloyd iteration, or the final E-step) with three launches:
//   E  distance GEMM [rows x slots] over the whole feature axis on f16 hi/lo MFMA
//      (x.c = xh.ch + xh.cl + xl.ch, f32 accumulation, as kmeans.hip), fused with the E-step:
//      strict-< argmin labels per Lloyd problem, min-with-closest per k-means++ candidate, and
//      per-tile partial inertia / potential sums (f64, fixed order);
//   M  centre sums = one-hot(labels)^T x X (f16 MFMA, f32 sums), per 256-feature stripe;
//   P  one workgroup per resample: k-means++ decisions and draws, new centres, relocation,
//      averaging, shifts, convergence, best-of-init output, and the packing of the next round.
// A resample's SLOTS (the centres of its Lloyd problems, the candidates of its seeding
// problems) are packed into 256-wide COLUMN TILES, so E and M read the resample's rows once per
// round for all of its problems.  E workgroups that share a column tile are dealt to one XCD
// (blocks b and b+8 share an XCD), so the tile's centre stripes are read from HBM once and
// served to the other row tiles from that XCD's L2.
// Nothing depends on scheduling: every sum has a fixed order, so results are deterministic and
// independent of the batch size and of the GPU count.
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
constexpr int ER = 128;          // rows per E workgroup
constexpr int CWW = 256;         // slots per column tile
constexpr int IMW = 128;         // work items per column tile
constexpr int KC = 32;           // features per E stage
constexpr int DS = CWW + 4;      // distance-tile row stride (floats)
constexpr int MDW = 256;         // features per M workgroup
constexpr int MRS = 32;          // rows per M stage
constexpr int MP = 576;          // LDS pitch (bytes) of one staged 256-feature f16 row: conflict-free tr reads
constexpr int PMAX = CC_KM_PMAX;
constexpr int TMAX = 6;
constexpr int KMAX = 127;
constexpr int CTMAX = 8;
constexpr int CNMAX = CTMAX * CWW;
constexpr int RTB = 32;          // k-means++ cumsum block (rows)
#ifndef KW_ALIGN
#define KW_ALIGN 1               // align the problems' Lloyd phases (schedule)
#endif

enum { ST_SEED = 1, ST_RUN = 2, ST_FINAL = 3, ST_DONE = 4 };
enum { IK_SEED0 = 0, IK_SEED = 1, IK_RUN = 2, IK_FINAL = 3 };

// Item words: iw0 = label buffer<<30 | kind<<24 | problem<<16 | K<<8 | slot offset,
//             iw1 = dbuf write slot<<8 | closest slot<<4 | trial (seeding items).
__device__ __forceinline__ int iw_off(unsigned w) { return w & 0xFF; }
__device__ __forceinline__ int iw_K(unsigned w) { return (w >> 8) & 0xFF; }
__device__ __forceinline__ int iw_prob(unsigned w) { return (w >> 16) & 0x3F; }
__device__ __forceinline__ int iw_kind(unsigned w) { return (w >> 24) & 3; }
__device__ __forceinline__ int iw_buf(unsigned w) { return (w >> 30) & 1; }

// One column tile of a round (global; written by P, read by E and M of the next round).
struct WTile {
  int nslots, nitems, nrun, pad;
  unsigned iw0[IMW], iw1[IMW];
  int srow[CWW];             // >= 0: X row (candidate); < 0: -(centre row) - 1; INT_MIN: dummy
  float cnorm[CWW];          // |slot|^2 (+inf for dummies)
  short scl[CWW];            // Lloyd RUN slot: its cluster; -1 otherwise (M-step one-hot)
  short sdst[CWW];           // Lloyd RUN slot: row of its sums in cen [2][Cn]; -1 otherwise
  unsigned char sitem[CWW];  // item of the slot (0xFF none)
};

struct WProb {
  unsigned char K, kidx, init, ntr, st, c, cs, lcur, ccur, need_sel, to_run, changed;
  short cenoff, item;  // item: flat index ct * IMW + it of this round's first item, -1 none
  int iter, amax, nempty;
  float pot32, inert;
  int cand[TMAX];
};

struct WState {
  int P, Cn, finished, round;  // round: P launches so far (the init is round 0)
  float tol;
  int kmax;                    // largest K of the resample's problems
  int pad2[2];
  WProb pr[PMAX];
};

struct WArgs {
  const float* X;          // [n][dpad] f32 (mean-centred, zero-padded)
  const uint16_t* Xhl;     // [n][2][dpad] f16 bits: hi, lo of X * 2^s
  const float* xnorm;      // [n]
  int n, dreal, dpad;
  float scale, inv_scale, dscale;
  const int32_t* idx;      // [H][m]
  int m, H, h0, nb;
  const int32_t* probs;    // [P][4]: K, kidx, init, ntr
  int P, Cn, nct, ndb, kws, RE, DT, lsm;
  int max_iter;
  double tol_rel;
  const double* kpp_u;
  int kpp_stride, n_init;
  const int32_t* kpp_pos;
  uint8_t* labels_out;
  int ldl;
  float* inertia_out;
  int32_t* niter_out;
  unsigned long long* stats;
  int* active;             // scheduled column tiles of the next round (summed by P)
  int reloc_full;          // diagnostics (CCMI_WIDE_RELOC_FULL): relocation reads every row exactly
  uint8_t* ws;
  size_t ws_per, off_tolp, off_tiles, off_part, off_glab, off_dbuf, off_cpos, off_cen, off_cenhl, off_cenn, off_rdist;
};

struct RP {  // one resample's workspace
  WState* st;
  WTile* tiles;
  double* part;     // [nct][IMW][RE]
  uint8_t* glab;    // [P][2][lsm]
  float* dbuf;      // [P][ndb][lsm]
  int32_t* cpos;    // [P][kws]
  float* cen;       // [2][Cn][dpad]
  uint16_t* cenhl;  // [Cn][2][dpad]
  float* cenn;      // [Cn]
  float* rdist;     // [lsm]
};

__device__ __forceinline__ RP rp(const WArgs& a, int b) {
  uint8_t* base = a.ws + static_cast<size_t>(b) * a.ws_per;
  RP r;
  r.st = reinterpret_cast<WState*>(base);
  r.tiles = reinterpret_cast<WTile*>(base + a.off_tiles);
  r.part = reinterpret_cast<double*>(base + a.off_part);
  r.glab = base + a.off_glab;
  r.dbuf = reinterpret_cast<float*>(base + a.off_dbuf);
  r.cpos = reinterpret_cast<int32_t*>(base + a.off_cpos);
  r.cen = reinterpret_cast<float*>(base + a.off_cen);
  r.cenhl = reinterpret_cast<uint16_t*>(base + a.off_cenhl);
  r.cenn = reinterpret_cast<float*>(base + a.off_cenn);
  r.rdist = reinterpret_cast<float*>(base + a.off_rdist);
  return r;
}

__device__ __forceinline__ v16f mfma16(const h8& a, const h8& b, const v16f& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// strict-< argmin update with the 4 values of an aligned chunk at slot c
__device__ __forceinline__ void amin4(const float4& v, int c, float& best, int& lab) {
  if (v.x < best) { best = v.x; lab = c; }
  if (v.y < best) { best = v.y; lab = c + 1; }
  if (v.z < best) { best = v.z; lab = c + 2; }
  if (v.w < best) { best = v.w; lab = c + 3; }
}

// numpy pairwise_sum of a short float32 array (n <= 128): `(center_shift ** 2).sum()`.
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

// LDS-DMA piece from inline asm (lane i writes 16 B at M0 + 16 i), opaque to the compiler's
// waitcnt pass; completion is awaited explicitly with dma_wait_n (vmcnt drains in order).  M0
// is set inside the asm; nothing else in these kernels uses M0.
__device__ __forceinline__ void dma_piece16(const void* g, const void* lds_dst) {
  const unsigned la = static_cast<unsigned>(reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) const char*)lds_dst));
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(__builtin_amdgcn_readfirstlane(la)), "v"(g));
}

template <int N>
__device__ __forceinline__ void dma_wait_n() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  static_assert(N == 0 || N == 6, "six pieces per wave and stage");
}

// ============================================================================================
// E: distances of a 256-row tile to a 256-slot column tile, then the E-step.
// Waves: 4 slot groups (64 slots) x 2 row groups (128 rows); per 32-feature stage each wave does
// 2 k-steps x (2 x 4 blocks) x 3 MFMAs from register-staged LDS images: 0.5 fragment reads per
// MFMA (the 128-row form read 0.67, and its LDS traffic per stage was about its MFMA time).  Every
// output's MFMA chain (stage and k-step order, xh.cl then xl.ch then xh.ch) is the 128-row form's,
// so the distances are bit-identical.  The E-step runs per 64-row quarter of the tile (the distance
// tile of a quarter fits in the operand ring); a quarter's per-item sums are the wave sums of the
// 128-row form's waves, and each 128-row half writes its own partial (part[.][2 rt + half]), so
// the potentials and inertias keep their order too.
// ============================================================================================
constexpr int ER2 = 2 * ER;  // rows per E workgroup
__global__ __launch_bounds__(NT, 1) void wide_estep(WArgs a) {
  // ring of 2 stages; a stage = A (slots) hi/lo planes + B (rows) hi/lo planes, 64-B rows
  // (32 features) with the 16-B chunks XOR-swizzled by (row >> 2) & 3: conflict-free b128
  // fragment reads, and lane-linear 1-KiB pieces (16 rows of a plane) for the LDS-DMA fill
  constexpr int RB = KC * 2;                    // 64 B per row and plane
  constexpr int APL = CWW * RB, BPL = ER2 * RB;  // 16 KiB, 16 KiB
  constexpr int STG = 2 * APL + 2 * BPL;        // 64 KiB
  constexpr int NSTG = 2;
  constexpr int QR = 64;                        // rows per E-step quarter
  constexpr int DBYTES = QR * DS * 4;
  constexpr int UN = (NSTG * STG > DBYTES) ? NSTG * STG : DBYTES;
  constexpr int NPC = STG / 1024 / NW;          // pieces per wave and stage (8)
  __shared__ __attribute__((aligned(16))) char sm[UN];
  __shared__ int s_srow[CWW];
  __shared__ __attribute__((aligned(16))) float s_cn[CWW];
  __shared__ unsigned s_iw0[IMW], s_iw1[IMW];
  __shared__ int s_gidx[ER2];
  __shared__ float s_xn[ER2];
  __shared__ double s_red[IMW][2];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = a.nb * a.nct;
  const int RE2 = (a.RE + 1) >> 1;
  const int bid = blockIdx.x, xcd = bid & 7, jb = bid >> 3;
  const int rt = jb % RE2, g = (jb / RE2) * 8 + xcd;
  if (g >= G) return;
  const int b = g / a.nct, ct = g - b * a.nct;
  const RP R = rp(a, b);
  const WTile* T = R.tiles + ct;
  const int nslots = __builtin_amdgcn_readfirstlane(T->nslots);
  if (nslots == 0) return;
  const int nitems = __builtin_amdgcn_readfirstlane(T->nitems);
  const int m = a.m, dpad = a.dpad;
  const int32_t* idx = a.idx + static_cast<size_t>(a.h0 + b) * m;
  for (int s = tid; s < CWW; s += NT) {
    s_srow[s] = (s < nslots) ? T->srow[s] : INT_MIN;
    s_cn[s] = T->cnorm[s];
  }
  for (int i = tid; i < nitems; i += NT) {
    s_iw0[i] = T->iw0[i];
    s_iw1[i] = T->iw1[i];
  }
  if (tid < ER2) {
    const int r = rt * ER2 + tid;
    const int gi = idx[min(r, m - 1)];
    s_gidx[tid] = gi;
    s_xn[tid] = a.xnorm[gi];
  }
  __syncthreads();

  // LDS-DMA fill: per stage 64 pieces of 1 KiB (A: 2 planes x 16, B: 2 planes x 16), eight per
  // wave; lane i of a piece writes 16 B at piece base + 16 i, i.e. row i/4, physical chunk i%4,
  // so it fetches logical chunk (i%4) ^ ((row >> 2) & 3) of its row.  The source rows are fixed
  // for the workgroup: the per-lane pointers are advanced by 64 B per stage.  Dummy slots and
  // slots past nslots read a valid X row (their distances are +inf or unread).
  const int S = dpad / KC;
  const char* psrc[NPC];
  int pdst[NPC];
#pragma unroll
  for (int k = 0; k < NPC; ++k) {
    const int pc = wave + NW * k;  // piece of the stage
    const int plane = (pc >> 4) & 1, row = (pc & 15) * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 2) & 3);
    const uint16_t* src;
    if (pc < 32) {
      const int sr = s_srow[row];
      if (sr >= 0) src = a.Xhl + (static_cast<size_t>(sr) * 2 + plane) * dpad;
      else if (sr != INT_MIN) src = R.cenhl + (static_cast<size_t>(-sr - 1) * 2 + plane) * dpad;
      else src = a.Xhl + (static_cast<size_t>(s_gidx[0]) * 2 + plane) * dpad;
      pdst[k] = plane * APL + (pc & 15) * 1024;
    } else {
      src = a.Xhl + (static_cast<size_t>(s_gidx[row]) * 2 + plane) * dpad;
      pdst[k] = 2 * APL + plane * BPL + (pc & 15) * 1024;
    }
    psrc[k] = reinterpret_cast<const char*>(src) + 16 * chunk;
  }
  auto issue = [&](int st) __attribute__((always_inline)) {
    const char* ring = sm + (st % NSTG) * STG;
#pragma unroll
    for (int k = 0; k < NPC; ++k) dma_piece16(psrc[k] + static_cast<size_t>(st) * (2 * KC), ring + pdst[k]);
  };

  const int ws = wave >> 1, wr = wave & 1, lr = lane & 31, hh = lane >> 5;
  // waves w and w+4 share a SIMD: with ws = w >> 1 they hold different slot groups, so a tile
  // with few slots (k-means++ rounds) still keeps every SIMD's matrix pipe busy
  const bool wact = 64 * ws < nslots;  // wave-uniform
  v16f acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v16f{};
  auto fo = [](int row, int c) { return row * RB + 16 * (c ^ ((row >> 2) & 3)); };
  auto compute = [&](int st) __attribute__((always_inline)) {
    if (!wact) return;
    const char* base = sm + (st % NSTG) * STG;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      h8 ah[2], al[2], bh[4], bl[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = fo(64 * ws + 32 * i + lr, 2 * ks + hh);
        ah[i] = *reinterpret_cast<const h8*>(base + o);
        al[i] = *reinterpret_cast<const h8*>(base + APL + o);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = 2 * APL + fo(128 * wr + 32 * j + lr, 2 * ks + hh);
        bh[j] = *reinterpret_cast<const h8*>(base + o);
        bl[j] = *reinterpret_cast<const h8*>(base + BPL + o);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          acc[i][j] = mfma16(ah[i], bl[j], acc[i][j]);
          acc[i][j] = mfma16(al[i], bh[j], acc[i][j]);
          acc[i][j] = mfma16(ah[i], bh[j], acc[i][j]);
        }
    }
  };
  // stage s: wait for its pieces (issued one stage earlier), barrier (everyone's pieces landed,
  // and every wave is done with stage s-1, whose slot the next issue refills), issue stage s+1,
  // compute stage s
  issue(0);
  for (int st = 0; st < S; ++st) {
    dma_wait_n<0>();
    __syncthreads();
    if (st + 1 < S) issue(st + 1);
    compute(st);
  }
  __syncthreads();

  // per 64-row quarter: the distance tile D[row][slot] = |c|^2 - 2 x.c of its rows (aliases the
  // stages), then the E-step; thread = (row of the quarter, item group of 8)
  float* D = reinterpret_cast<float*>(sm);
  constexpr float INF = __builtin_huge_valf();
  const int qrow = tid & (QR - 1), grp = tid >> 6;
  for (int q = 0; q < ER2 / QR; ++q) {
    if (wact && wr == (q >> 1)) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int j = 2 * (q & 1) + jj;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const int slot0 = 64 * ws + 32 * i + 8 * gq + 4 * hh;
            const int row = 32 * jj + lr;
            const float4 c4 = *reinterpret_cast<const float4*>(s_cn + slot0);
            float4 d;
            d.x = c4.x - a.dscale * acc[i][j][4 * gq];
            d.y = c4.y - a.dscale * acc[i][j][4 * gq + 1];
            d.z = c4.z - a.dscale * acc[i][j][4 * gq + 2];
            d.w = c4.w - a.dscale * acc[i][j][4 * gq + 3];
            *reinterpret_cast<float4*>(D + row * DS + slot0) = d;
          }
      }
    }
    __syncthreads();
    const int lrow = QR * q + qrow;  // row of the 256-row tile
    const int r = rt * ER2 + lrow;
    const bool ok = r < m;
    const float xnr = s_xn[lrow];
    const float* drow = D + qrow * DS;
    for (int it = grp; it < nitems; it += NW) {
      const unsigned w0 = s_iw0[it];
      const int kind = iw_kind(w0), p = iw_prob(w0), off = iw_off(w0);
      double v = 0.0;
      if (kind >= IK_RUN) {
        const int K = iw_K(w0);
        float best = INF;
        int lab = 0;
        for (int c = 0; c < K; c += 4) amin4(*reinterpret_cast<const float4*>(drow + off + c), c, best, lab);
        if (ok) {
          R.glab[(static_cast<size_t>(p) * 2 + iw_buf(w0)) * a.lsm + r] = static_cast<uint8_t>(lab);
          v = static_cast<double>(xnr) + static_cast<double>(best);
          // the row's squared distance to its centre as the E-step has it (dbuf slot 0 is free
          // once a problem runs Lloyd): relocate() filters its candidates with it
          R.dbuf[static_cast<size_t>(p) * a.ndb * a.lsm + r] = xnr + best;
        }
      } else {
        const float dist = fmaxf(xnr + drow[off], 0.f);
        const unsigned w1 = s_iw1[it];
        if (ok) {
          float dm = dist;
          if (kind == IK_SEED) dm = fminf(R.dbuf[(static_cast<size_t>(p) * a.ndb + ((w1 >> 4) & 15)) * a.lsm + r], dist);
          R.dbuf[(static_cast<size_t>(p) * a.ndb + ((w1 >> 8) & 15)) * a.lsm + r] = dm;
          v = static_cast<double>(dm);
        }
      }
      v = wave_sum(v);  // the 64 rows of the quarter, in the 128-row form's lane order
      if (lane == 0) s_red[it][q & 1] = v;
    }
    __syncthreads();
    // a 128-row half done: its per-item partial, as the 128-row form wrote it
    const int rth = 2 * rt + (q >> 1);
    if ((q & 1) && tid < nitems && rth < a.RE)
      R.part[(static_cast<size_t>(ct) * IMW + tid) * a.RE + rth] = s_red[tid][0] + s_red[tid][1];
  }
}

// ============================================================================================
// M: sums[slot][f] = sum_r [label_r == cluster(slot)] * x_r[f] for the Lloyd RUN slots of a
// column tile and a 256-feature stripe.  Waves: 4 slot groups (64) x 2 feature groups (128).
// A = one-hot from the labels (LDS), B = the rows read back transposed with ds_read_b64_tr_b16.
// ============================================================================================
__global__ __launch_bounds__(NT, 1) void wide_mstep(WArgs a) {
  constexpr int PL = MRS * MP;  // one plane of a stage
  constexpr int STG = 2 * PL;
  __shared__ __attribute__((aligned(16))) char sm[2 * STG];
  __shared__ __attribute__((aligned(16))) uint8_t Lb[2][IMW + 1][MRS];  // row IMW: sink of idle loaders
  __shared__ short s_scl[CWW], s_dst[CWW];
  __shared__ unsigned char s_item[CWW];
  __shared__ int s_ritem[IMW], s_lofs[IMW];
  __shared__ int s_nr, s_gact[4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int DT = a.DT;
  const int g = blockIdx.x / DT, dt = blockIdx.x - g * DT;
  if (g >= a.nb * a.nct) return;
  const int b = g / a.nct, ct = g - b * a.nct;
  const RP R = rp(a, b);
  const WTile* T = R.tiles + ct;
  if (__builtin_amdgcn_readfirstlane(T->nrun) == 0) return;
  const int nslots = T->nslots;
  const int m = a.m, dpad = a.dpad;
  const int32_t* idx = a.idx + static_cast<size_t>(a.h0 + b) * m;
  if (tid < 4) s_gact[tid] = 0;
  __syncthreads();
  for (int s = tid; s < CWW; s += NT) {
    const bool in = s < nslots;
    const short cl = in ? T->scl[s] : static_cast<short>(-1);
    s_scl[s] = cl;
    s_dst[s] = in ? T->sdst[s] : static_cast<short>(-1);
    const unsigned char itm = in ? T->sitem[s] : static_cast<unsigned char>(0xFF);
    s_item[s] = (itm == 0xFF) ? 0 : itm;
    if (cl >= 0) s_gact[s >> 6] = 1;
  }
  if (tid == 0) {
    int nr = 0;
    const int ni = T->nitems;
    for (int it = 0; it < ni; ++it) {
      const unsigned w0 = T->iw0[it];
      if (iw_kind(w0) != IK_RUN) continue;
      s_ritem[nr] = it;
      s_lofs[nr] = (iw_prob(w0) * 2 + iw_buf(w0)) * a.lsm;
      ++nr;
    }
    s_nr = nr;
  }
  __syncthreads();
  const int nr = s_nr;

  // loaders: X = row tid>>4, plane (tid>>3)&1, 32-feature piece tid&7 (64 B); labels = RUN item
  // tid>>1, 16-B half tid&1
  const int xr = tid >> 4, xp = (tid >> 3) & 1, xq = tid & 7;
  // every lane loads (exact vmcnt counting): pieces past dpad re-read the last piece (their
  // columns are never stored), idle label loaders read item 0's labels into the sink row
  const int f0 = min(dt * MDW + 32 * xq, dpad - 32);
  const int xoffl = xp * PL + xr * MP + 64 * xq;
  const bool lon = tid < 2 * nr;
  const uint8_t* lsrc = R.glab + (lon ? s_lofs[tid >> 1] : 0) + 16 * (tid & 1);
  uint8_t* ldst0 = &Lb[0][lon ? s_ritem[tid >> 1] : IMW][16 * (tid & 1)];
  // a register set carries one stage's loads and the row index of the stage 3 later (by value:
  // see wide_estep)
  struct MSet {  // named fields: an array member makes the set a scratch object
    uint4 x0, x1, x2, x3, l;
    int gi;
  };
  auto gload = [&](int s, const MSet R) __attribute__((always_inline)) -> MSet {
    MSet Rg;
    const uint4* p = reinterpret_cast<const uint4*>(a.Xhl + (static_cast<size_t>(R.gi) * 2 + xp) * dpad + f0);
    Rg.x0 = p[0];
    Rg.x1 = p[1];
    Rg.x2 = p[2];
    Rg.x3 = p[3];
    Rg.l = *reinterpret_cast<const uint4*>(lsrc + MRS * s);
    Rg.gi = idx[min((s + 3) * MRS + xr, m - 1)];
    return Rg;
  };
  auto lstore = [&](int buf, const MSet Rg) __attribute__((always_inline)) {
    uint4* p = reinterpret_cast<uint4*>(sm + buf * STG + xoffl);
    p[0] = Rg.x0;
    p[1] = Rg.x1;
    p[2] = Rg.x2;
    p[3] = Rg.x3;
    *reinterpret_cast<uint4*>(ldst0 + buf * ((IMW + 1) * MRS)) = Rg.l;
  };

  const int ws = wave >> 1, wd = wave & 1, lr = lane & 31, hh = lane >> 5;  // as wide_estep
  const int fw = dt * MDW + 128 * wd;
  const int nbd = min(4, max(0, (dpad - fw) / 32));  // feature blocks of this wave (uniform)
  const bool wact = s_gact[ws] && nbd > 0;
  int cl[2], itm[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int slot = 64 * ws + 32 * i + lr;
    cl[i] = s_scl[slot];
    itm[i] = s_item[slot];
  }
  v16f acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v16f{};
  const int S = (m + MRS - 1) / MRS;
  const int Gq = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  auto compute = [&](int s) __attribute__((always_inline)) {
    if (!wact) return;
    const char* base = sm + (s & 1) * STG;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      h8 oh[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const unsigned long long lab8 =
            *reinterpret_cast<const unsigned long long*>(&Lb[s & 1][itm[i]][16 * ks + 8 * hh]);
        u32x4 ohu;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int b0 = static_cast<int>((lab8 >> (16 * j)) & 0xFFu);
          const int b1 = static_cast<int>((lab8 >> (16 * j + 8)) & 0xFFu);
          ohu[j] = ((b0 == cl[i]) ? 0x3C00u : 0u) | ((b1 == cl[i]) ? 0x3C000000u : 0u);
        }
        oh[i] = __builtin_bit_cast(h8, ohu);
      }
      const int row0 = 16 * ks + 8 * (Gq >> 1) + q;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= nbd) break;
        const int a0 = row0 * MP + 2 * (128 * wd + 32 * j + 16 * (Gq & 1) + 4 * pp);
        const int a1 = a0 + 4 * MP;
        const s4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + a0));
        const s4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + a1));
        const s4 l0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + PL + a0));
        const s4 l1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + PL + a1));
        const h8 bh = __builtin_bit_cast(h8, __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7));
        const h8 bl = __builtin_bit_cast(h8, __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          acc[i][j] = mfma16(oh[i], bl, acc[i][j]);
          acc[i][j] = mfma16(oh[i], bh, acc[i][j]);
        }
      }
    }
  };
  MSet R0, R1, R2;
  R0.gi = idx[min(xr, m - 1)];
  R1.gi = idx[min(MRS + xr, m - 1)];
  R2.gi = idx[min(2 * MRS + xr, m - 1)];
  R0 = gload(0, R0);
  lstore(0, R0);
  R1 = gload(min(1, S - 1), R1);
  R2 = gload(min(2, S - 1), R2);
  R0 = gload(min(3, S - 1), R0);
  __syncthreads();
  auto step = [&](int s, const MSet Rg) __attribute__((always_inline)) -> MSet {
    compute(s);
    lstore((s + 1) & 1, Rg);
    __builtin_amdgcn_sched_barrier(0);
    const MSet Rn = gload(min(s + 4, S - 1), Rg);
    __syncthreads();
    return Rn;
  };
  int s = 0;
  for (; s + 3 <= S; s += 3) {
    R1 = step(s, R1);
    R2 = step(s + 1, R2);
    R0 = step(s + 2, R0);
  }
  if (s < S) R1 = step(s, R1);
  if (s + 1 < S) R2 = step(s + 1, R2);
  if (wact) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= nbd) break;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int slot = 64 * ws + 32 * i + 8 * (v >> 2) + 4 * hh + (v & 3);
          const int dst = s_dst[slot];
          if (dst >= 0) R.cen[static_cast<size_t>(dst) * dpad + fw + 32 * j + lr] = acc[i][j][v] * a.inv_scale;
        }
      }
  }
}

// ============================================================================================
// tol pre-pass: sum over a 512-feature chunk of var(X_sub[:, f]) (f64, one pass, fixed order),
// one workgroup per (resample, chunk); the init sums the chunks in order.
// ============================================================================================
__global__ __launch_bounds__(NT) void wide_tol(WArgs a) {
  __shared__ double red[NW];
  const int NTC = (a.dreal + NT - 1) / NT;
  const int b = blockIdx.x / NTC, ch = blockIdx.x - b * NTC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int d = ch * NT + tid, m = a.m;
  const int32_t* idx = a.idx + static_cast<size_t>(a.h0 + b) * m;
  double v = 0.0;
  if (d < a.dreal) {
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    const float* col = a.X + d;
    int r = 0;
    for (; r + 4 <= m; r += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double x = static_cast<double>(col[static_cast<size_t>(idx[r + u]) * a.dpad]);
        s1[u] += x;
        s2[u] += x * x;
      }
    }
    for (; r < m; ++r) {
      const double x = static_cast<double>(col[static_cast<size_t>(idx[r]) * a.dpad]);
      s1[0] += x;
      s2[0] += x * x;
    }
    const double mu = ((s1[0] + s1[1]) + (s1[2] + s1[3])) / m;
    v = fmax(((s2[0] + s2[1]) + (s2[2] + s2[3])) / m - mu * mu, 0.0);
  }
  v = wave_sum(v);
  if (lane == 0) red[wave] = v;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < NW; ++w) t += red[w];
    reinterpret_cast<double*>(a.ws + static_cast<size_t>(b) * a.ws_per + a.off_tolp)[ch] = t;
  }
}

// ============================================================================================
// P: per-resample round processing (one workgroup per resample).
// ============================================================================================
struct PS {
  WState S;
  unsigned iw0[CTMAX][IMW], iw1[CTMAX][IMW];
  int nit[CTMAX];
  double iinert[CTMAX * IMW];
  unsigned cnt[CNMAX];
  float shift[CNMAX];
  int map[KMAX + 1];
  double red_v[NW];
  int red_i[NW];
  int flag;
  unsigned char ranf[PMAX];  // ran a Lloyd RUN item this round
  unsigned long long n_lloyd, n_seed, n_mrows, n_reloc;
  WTile tn[CTMAX];
};

// k-means++ candidate positions for centre c (>= 1) of problem p, one wave:
// searchsorted(cumsum(closest), u * pot) (side='left'), clipped to m-1.  The cumsum is blocked
// by 32-row blocks (f64 block sums in row order, a wave prefix over blocks, then a walk of the
// crossing block), so the two levels agree exactly.
__device__ void kpp_select(const WArgs& a, WProb& q, const float* closest, int lane) {
  const int ntr = q.ntr, c = q.c, m = a.m, T = (m + RTB - 1) / RTB;
  const double* u = a.kpp_u + (static_cast<size_t>(q.kidx) * a.n_init + q.init) * a.kpp_stride + 1 +
                    static_cast<size_t>(c - 1) * ntr;
  const double pot = static_cast<double>(q.pot32);
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
  for (int b0 = 0; b0 < T; b0 += 64) {
    const int j = b0 + lane;
    double v = 0.0;
    if (j < T) {
      const int r0 = RTB * j, nr = min(RTB, m - r0);
      for (int k = 0; k < nr; ++k) v += static_cast<double>(closest[r0 + k]);
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double y = __shfl_up(v, o);
      if (lane >= o) v += y;
    }
    const double cum = run + v;
    const int nvalid = min(64, T - b0);
#pragma unroll
    for (int t = 0; t < TMAX; ++t) {
      if (t >= ntr) continue;
      const int k = __popcll(__ballot(j < T && cum < rv[t]));
      const double prev = __shfl(cum, max(k - 1, 0));
      if (!found[t] && k < nvalid) {
        found[t] = true;
        tau[t] = b0 + k;
        base[t] = (k == 0) ? run : prev;
      }
    }
    run = __shfl(cum, 63);
  }
#pragma unroll
  for (int t = 0; t < TMAX; ++t) {
    if (t >= ntr || lane != t) continue;
    int pos = m;
    if (found[t]) {
      const int r0 = RTB * tau[t];
      double acc = base[t];
      int k = 0;
      for (; k < RTB && r0 + k < m; ++k) {
        acc += static_cast<double>(closest[r0 + k]);
        if (!(acc < rv[t])) break;
      }
      pos = r0 + k;
    }
    q.cand[t] = min(pos, m - 1);
  }
}


// One new centre row (one wave): nw <- nw * alpha (the f32 _average_centers scaling, in
// place), shift = |nw - od|^2 (f64 sum -> f32, squared back from its f32 root as
// _euclidean_dense_dense + `** 2`), the f16 hi/lo image and the f32 squared norm.  Four 16-B
// pieces per lane in flight.
__device__ void update_row(const WArgs& a, float* nw, const float* od, float alpha, uint16_t* hl,
                           float* norm, float* shift, int lane) {
  const int n4 = a.dpad / 4;
  double sh = 0.0, nn = 0.0;
  for (int q0 = lane; q0 < n4; q0 += 256) {
    float4 x[4], o[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int qi = q0 + 64 * u;
      if (qi < n4) {
        x[u] = reinterpret_cast<const float4*>(nw)[qi];
        o[u] = reinterpret_cast<const float4*>(od)[qi];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int qi = q0 + 64 * u;
      if (qi >= n4) continue;
      const float v[4] = {x[u].x * alpha, x[u].y * alpha, x[u].z * alpha, x[u].w * alpha};
      const float w[4] = {o[u].x, o[u].y, o[u].z, o[u].w};
      reinterpret_cast<float4*>(nw)[qi] = make_float4(v[0], v[1], v[2], v[3]);
      uint16_t h[4], l[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (4 * qi + k < a.dreal) {
          const double t = static_cast<double>(v[k]) - static_cast<double>(w[k]);
          sh += t * t;
          nn += static_cast<double>(v[k]) * static_cast<double>(v[k]);
        }
        const float xs = v[k] * a.scale;
        const _Float16 hi = static_cast<_Float16>(xs);
        const _Float16 lo = static_cast<_Float16>(xs - static_cast<float>(hi));
        h[k] = __builtin_bit_cast(uint16_t, hi);
        l[k] = __builtin_bit_cast(uint16_t, lo);
      }
      reinterpret_cast<uint2*>(hl)[qi] = make_uint2(h[0] | (static_cast<uint32_t>(h[1]) << 16),
                                                    h[2] | (static_cast<uint32_t>(h[3]) << 16));
      reinterpret_cast<uint2*>(hl + a.dpad)[qi] = make_uint2(l[0] | (static_cast<uint32_t>(l[1]) << 16),
                                                             l[2] | (static_cast<uint32_t>(l[3]) << 16));
    }
  }
  sh = wave_sum(sh);
  nn = wave_sum(nn);
  if (lane == 0) {
    const float r = sqrtf(static_cast<float>(sh));
    *shift = r * r;
    *norm = static_cast<float>(nn);
  }
}

// Empty-cluster relocation for problem p (rare; _k_means_common.pyx:167-212).  sums: the
// problem's un-averaged sums [K][dpad]; cold: the centres the labels came from; est: the E-step's
// squared distance of each row to its centre, cn: the squared norms of cold.
//
// The clusters take the farthest rows by the exact distance (f64 sum of the f32 squared
// differences, below), which reads every row in full: 320 MB per problem at C4, one workgroup,
// ~25 ms.  Only rows that can be among the ne farthest are read: |est - exact| <= b_r with
//   b_r = (2 d + 64) 2^-24 (|x| + |c|)^2 + 2^-22 sqrt(d) (|x| + |c|) / scale
// (f32 accumulation of the f16 hi/lo products over d terms, their 2^-22 split error, the f32
// norms and the f16 subnormal spacing of the scaled operands; the exact value's own rounding is
// below the first term), so a row whose est + b_r is below the ne-th largest est - b is never
// picked, and the candidates get their exact distance; the rest are excluded (-2).
__device__ void relocate(const WArgs& a, PS& L, const int32_t* idx, int p, float* sums, const float* cold,
                         const uint8_t* lab, const float* est, const float* cn, float* dist, int tid) {
  WProb& q = L.S.pr[p];
  const int m = a.m, K = q.K, dpad = a.dpad, off = q.cenoff;
  const int lane = tid & 63, wave = tid >> 6, n4 = dpad / 4;
  const float gam = static_cast<float>((2.0 * a.dreal + 64.0) * 0x1p-24);
  const float gab = 0x1p-22f * sqrtf(static_cast<float>(a.dreal)) * a.inv_scale;
  auto bound = [&](int r) -> float {
    const float s = sqrtf(a.xnorm[idx[r]]) + sqrtf(cn[lab[r]]);
    return gam * s * s + gab * s;
  };
  // pv = the ne-th largest lower bound est - b (ties by lower row), ne = the empty count
  int ne0 = 0;
  for (int c = 0; c < K; ++c) ne0 += (L.cnt[off + c] == 0);
  float pv = __builtin_huge_valf();
  int pi = -1;
  for (int e = 0; e < ne0; ++e) {
    float bv = -__builtin_huge_valf();
    int bi = 0x7fffffff;
    for (int r = tid; r < m; r += NT) {
      const float lo = est[r] - bound(r);
      if ((lo < pv || (lo == pv && r > pi)) && (lo > bv || (lo == bv && r < bi))) {
        bv = lo;
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
    if (lane == 0) {
      L.red_v[wave] = bv;
      L.red_i[wave] = bi;
    }
    __syncthreads();
    double gv = -__builtin_huge_val();
    int gi = 0x7fffffff;
    for (int w = 0; w < NW; ++w)
      if (L.red_v[w] > gv || (L.red_v[w] == gv && L.red_i[w] < gi)) {
        gv = L.red_v[w];
        gi = L.red_i[w];
      }
    __syncthreads();
    pv = static_cast<float>(gv);
    pi = gi;
  }
  if (ne0 == 0 || a.reloc_full) pv = -__builtin_huge_valf();
  // the candidates (est + b >= pv) get their exact squared distance to the centre they were
  // assigned to: one wave per row, coalesced 16-B reads, f64 sum of the f32 squared differences
  float mymax = 0.f;
  for (int r = wave; r < m; r += NW) {
    if (!(est[r] + bound(r) >= pv)) {
      if (lane == 0) dist[r] = -2.f;
      continue;
    }
    const float4* x = reinterpret_cast<const float4*>(a.X + static_cast<size_t>(idx[r]) * dpad);
    const float4* c = reinterpret_cast<const float4*>(cold + static_cast<size_t>(lab[r]) * dpad);
    double acc = 0.0;
    for (int q = lane; q < n4; q += 64) {
      const float4 xv = x[q], cv = c[q];
      const float t[4] = {xv.x - cv.x, xv.y - cv.y, xv.z - cv.z, xv.w - cv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (4 * q + k < a.dreal) acc += static_cast<double>(t[k]) * static_cast<double>(t[k]);
    }
    const float sd = static_cast<float>(wave_sum(acc));
    if (lane == 0) dist[r] = sd;
    mymax = fmaxf(mymax, sd);
  }
  if ((tid & 63) == 0) L.red_v[tid >> 6] = mymax;
  __syncthreads();
  double gmax = 0.0;
  for (int w = 0; w < NW; ++w) gmax = fmax(gmax, L.red_v[w]);
  if (tid == 0) {
    int ne = 0;
    for (int c = 0; c < K; ++c)
      if (L.cnt[off + c] == 0) L.map[ne++] = c;
    L.flag = ne;
  }
  __syncthreads();
  if (gmax == 0.0) return;
  const int ne = L.flag;
  for (int e = 0; e < ne; ++e) {
    const int c = L.map[e];
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
      L.red_v[tid >> 6] = bv;
      L.red_i[tid >> 6] = bi;
    }
    __syncthreads();
    double gv = -2.0;
    int gi = 0x7fffffff;
    for (int w = 0; w < NW; ++w)
      if (L.red_v[w] > gv || (L.red_v[w] == gv && L.red_i[w] < gi)) {
        gv = L.red_v[w];
        gi = L.red_i[w];
      }
    const int old = lab[gi];
    const float* x = a.X + static_cast<size_t>(idx[gi]) * dpad;
    for (int d = tid; d < dpad; d += NT) {
      sums[static_cast<size_t>(old) * dpad + d] -= x[d];
      sums[static_cast<size_t>(c) * dpad + d] = x[d];
    }
    __syncthreads();
    if (tid == 0) {
      L.cnt[off + c] = 1;
      L.cnt[off + old] -= 1;
      dist[gi] = -1.f;
      L.n_reloc += 1;
    }
    __syncthreads();
  }
}

// Thread 0: pack the next round.  Lloyd problems first (4-aligned offsets, K padded to a
// multiple of 4 with +inf dummies: no alignment gaps), then the seeding candidates; first fit
// over the column tiles; a problem that does not fit waits for the next round.
__device__ void schedule(const WArgs& a, PS& L, const int32_t* idx, const float* cenn) {
  WState& S = L.S;
  const int P = S.P, nct = a.nct, Cn = S.Cn;
  for (int ct = 0; ct < nct; ++ct) L.tn[ct].nslots = L.tn[ct].nitems = L.tn[ct].nrun = 0;
  for (int p = 0; p < P; ++p) S.pr[p].item = -1;
  for (int p = 0; p < P; ++p) {
    WProb& q = S.pr[p];
    if (q.st != ST_RUN && q.st != ST_FINAL) continue;
    const int K = q.K, K4 = (K + 3) & ~3;
    int ct = 0;
    while (ct < nct && (L.tn[ct].nslots + K4 > CWW || L.tn[ct].nitems + 1 > IMW)) ++ct;
    if (ct == nct) continue;
    WTile& t = L.tn[ct];
    const int off = t.nslots, it = t.nitems;
    const int kind = (q.st == ST_RUN) ? IK_RUN : IK_FINAL;
    t.iw0[it] = (static_cast<unsigned>(1 - q.lcur) << 30) | (static_cast<unsigned>(kind) << 24) |
                (static_cast<unsigned>(p) << 16) | (static_cast<unsigned>(K) << 8) | static_cast<unsigned>(off);
    t.iw1[it] = 0;
    for (int c = 0; c < K4; ++c) {
      const int sl = off + c;
      if (c < K) {
        t.srow[sl] = -(q.cenoff + c) - 1;
        t.cnorm[sl] = cenn[q.cenoff + c];
        t.scl[sl] = static_cast<short>(kind == IK_RUN ? c : -1);
        t.sdst[sl] = static_cast<short>(kind == IK_RUN ? (1 - q.ccur) * Cn + q.cenoff + c : -1);
        t.sitem[sl] = static_cast<unsigned char>(it);
      } else {
        t.srow[sl] = INT_MIN;
        t.cnorm[sl] = __builtin_huge_valf();
        t.scl[sl] = -1;
        t.sdst[sl] = -1;
        t.sitem[sl] = 0xFF;
      }
    }
    q.item = static_cast<short>(ct * IMW + it);
    t.nslots = off + K4;
    t.nitems = it + 1;
    if (kind == IK_RUN) {
      t.nrun += 1;
      L.n_mrows += a.m;
    }
    L.n_lloyd += static_cast<unsigned long long>(K) * a.m;
  }
  for (int p = 0; p < P; ++p) {
    WProb& q = S.pr[p];
    if (q.st != ST_SEED) continue;
#if KW_ALIGN
    // a problem starts seeding at round kmax - K, so that every problem's Lloyd iterations fall
    // in the same rounds: the M launch streams all rows of a resample whenever any problem runs
    // Lloyd, so rounds with Lloyd work are the ones to have fewest of (the order of problems
    // changes no result)
    if (q.c == 0 && S.round < S.kmax - static_cast<int>(q.K)) continue;
#endif
    const int c = q.c, nt = (c == 0) ? 1 : q.ntr;
    int ct = 0;
    while (ct < nct && (L.tn[ct].nslots + nt > CWW || L.tn[ct].nitems + nt > IMW)) ++ct;
    if (ct == nct) continue;
    WTile& t = L.tn[ct];
    q.item = static_cast<short>(ct * IMW + t.nitems);
    for (int tr = 0; tr < nt; ++tr) {
      const int sl = t.nslots, it = t.nitems;
      const int kind = (c == 0) ? IK_SEED0 : IK_SEED;
      const int cs = (c == 0) ? 0 : q.cs;
      const int wslot = (c == 0) ? 0 : ((tr < cs) ? tr : tr + 1);
      t.iw0[it] = (static_cast<unsigned>(kind) << 24) | (static_cast<unsigned>(p) << 16) | (1u << 8) |
                  static_cast<unsigned>(sl);
      t.iw1[it] = (static_cast<unsigned>(wslot) << 8) | (static_cast<unsigned>(cs) << 4) | static_cast<unsigned>(tr);
      const int pos = (c == 0) ? a.kpp_pos[q.kidx * a.n_init + q.init] : q.cand[tr];
      const int xr = idx[pos];
      t.srow[sl] = xr;
      t.cnorm[sl] = a.xnorm[xr];
      t.scl[sl] = -1;
      t.sdst[sl] = -1;
      t.sitem[sl] = static_cast<unsigned char>(it);
      t.nslots = sl + 1;
      t.nitems = it + 1;
    }
    L.n_seed += static_cast<unsigned long long>(nt) * a.m;
  }
}

__device__ void post_body(const WArgs& a, PS& L, bool init) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x, h = a.h0 + b, m = a.m, dpad = a.dpad;
  const RP R = rp(a, b);
  WState& S = L.S;
  const int32_t* idx = a.idx + static_cast<size_t>(h) * m;
  if (tid == 0) L.n_lloyd = L.n_seed = L.n_mrows = L.n_reloc = 0;
  if (init) {
    if (tid == 0) {
      S.P = a.P;
      S.Cn = a.Cn;
      S.finished = 0;
      S.round = 0;
      S.kmax = 0;
      for (int p = 0; p < a.P; ++p) S.kmax = max(S.kmax, a.probs[4 * p]);
      int o = 0;
      for (int p = 0; p < a.P; ++p) {
        WProb& q = S.pr[p];
        q.K = static_cast<unsigned char>(a.probs[4 * p]);
        q.kidx = static_cast<unsigned char>(a.probs[4 * p + 1]);
        q.init = static_cast<unsigned char>(a.probs[4 * p + 2]);
        q.ntr = static_cast<unsigned char>(a.probs[4 * p + 3]);
        q.st = ST_SEED;
        q.c = q.cs = q.lcur = q.ccur = 0;
        q.need_sel = q.to_run = q.changed = 0;
        q.iter = 0;
        q.cenoff = static_cast<short>(o);
        q.item = -1;
        o += q.K;
      }
    }
    for (size_t e = tid; e < static_cast<size_t>(2 * a.P) * a.lsm; e += NT) R.glab[e] = 0xFF;
    // tol = tol_rel * mean(var(X_sub, axis=0)) (sklearn _tolerance, :270-278), from wide_tol
    if (tid == 0) {
      const double* tp = reinterpret_cast<const double*>(a.ws + static_cast<size_t>(b) * a.ws_per + a.off_tolp);
      double tot = 0.0;
      for (int ch = 0; ch < (a.dreal + NT - 1) / NT; ++ch) tot += tp[ch];
      S.tol = static_cast<float>(static_cast<float>(tot / a.dreal) * a.tol_rel);
    }
    __syncthreads();
  } else {
    {
      const int* src = reinterpret_cast<const int*>(R.st);
      int* dst = reinterpret_cast<int*>(&S);
      for (int i = tid; i < static_cast<int>(sizeof(WState) / 4); i += NT) dst[i] = src[i];
    }
    __syncthreads();
    if (S.finished) return;
    if (tid == 0) S.round += 1;
    const int P = S.P, Cn = S.Cn;
    for (int ct = 0; ct < a.nct; ++ct) {
      const WTile* t = R.tiles + ct;
      const int ni = t->nitems;
      if (tid == 0) L.nit[ct] = ni;
      for (int it = tid; it < ni; it += NT) {
        L.iw0[ct][it] = t->iw0[it];
        L.iw1[ct][it] = t->iw1[it];
      }
    }
    __syncthreads();
    for (int fi = tid; fi < a.nct * IMW; fi += NT) {
      const int ct = fi / IMW, it = fi - ct * IMW;
      if (it >= L.nit[ct]) continue;
      const double* pr = R.part + static_cast<size_t>(fi) * a.RE;
      double s = 0.0;
      for (int rt = 0; rt < a.RE; ++rt) s += pr[rt];
      L.iinert[fi] = s;
    }
    __syncthreads();

    // ---- seeding decisions (thread per problem) ----------------------------------------
    if (tid < P) {
      WProb& q = S.pr[tid];
      q.need_sel = 0;
      q.to_run = 0;
      if (q.st == ST_SEED && q.item >= 0) {
        const int fi0 = q.item, c = q.c;
        const int nt = (c == 0) ? 1 : q.ntr;
        int best = 0;
        float bv = static_cast<float>(L.iinert[fi0]);
        for (int t = 1; t < nt; ++t) {
          const float v = static_cast<float>(L.iinert[fi0 + t]);
          if (v < bv) {
            bv = v;
            best = t;
          }
        }
        q.pot32 = bv;
        const int cs = q.cs;
        q.cs = static_cast<unsigned char>((c == 0) ? 0 : ((best < cs) ? best : best + 1));
        R.cpos[tid * a.kws + c] = (c == 0) ? a.kpp_pos[q.kidx * a.n_init + q.init] : q.cand[best];
        q.c = static_cast<unsigned char>(c + 1);
        if (c + 1 == q.K) {
          q.to_run = 1;
          q.st = ST_RUN;
          q.iter = 0;
        } else {
          q.need_sel = 1;
        }
      }
    }
    __syncthreads();
    {  // candidate draws: one wave per problem
      int j = 0;
      for (int p = 0; p < P; ++p) {
        if (!S.pr[p].need_sel) continue;
        if ((j++ % NW) != wave) continue;
        WProb& q = S.pr[p];
        kpp_select(a, q, R.dbuf + (static_cast<size_t>(p) * a.ndb + q.cs) * a.lsm, lane);
      }
    }
    // initial centres of problems leaving seeding: the chosen rows (exact f32), their f16 image
    // and norm (one wave per row; a lane reads back only what it wrote)
    {
      int j = 0;
      for (int p = 0; p < P; ++p) {
        const WProb& q = S.pr[p];
        if (!q.to_run) continue;
        for (int c = 0; c < q.K; ++c) {
          if ((j++ % NW) != wave) continue;
          const int row = q.cenoff + c;
          const float4* src = reinterpret_cast<const float4*>(a.X + static_cast<size_t>(idx[R.cpos[p * a.kws + c]]) * dpad);
          float* dst = R.cen + (static_cast<size_t>(q.ccur) * Cn + row) * dpad;
          for (int d = lane; d < dpad / 4; d += 64) reinterpret_cast<float4*>(dst)[d] = src[d];
          update_row(a, dst, dst, 1.f, R.cenhl + static_cast<size_t>(row) * 2 * dpad, R.cenn + row,
                     L.shift + row, lane);
        }
      }
    }

    // ---- labels changed? (RUN), then the written buffer becomes the current one ----------
    for (int p = 0; p < P; ++p) {
      WProb& q = S.pr[p];
      if (q.item < 0 || (q.st != ST_RUN && q.st != ST_FINAL) || q.to_run) continue;
      const unsigned w0 = L.iw0[q.item / IMW][q.item % IMW];
      bool diff = false;
      if (iw_kind(w0) == IK_RUN) {
        const uint4* cur = reinterpret_cast<const uint4*>(R.glab + (static_cast<size_t>(p) * 2 + 1 - q.lcur) * a.lsm);
        const uint4* old = reinterpret_cast<const uint4*>(R.glab + (static_cast<size_t>(p) * 2 + q.lcur) * a.lsm);
        for (int e = tid; e < (m + 15) / 16; e += NT) {
          const uint4 x = cur[e], y = old[e];
          diff |= (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
        }
      }
      const int any = __syncthreads_or(diff);
      if (tid == 0) {
        q.changed = any != 0;
        q.lcur = static_cast<unsigned char>(1 - q.lcur);
      }
    }
    __syncthreads();

    // ---- Lloyd M-step completion (problems that ran a RUN item) ---------------------------
    if (tid < P) {
      const WProb& q = S.pr[tid];
      L.ranf[tid] = q.item >= 0 && q.st == ST_RUN && !q.to_run && iw_kind(L.iw0[q.item / IMW][q.item % IMW]) == IK_RUN;
    }
    for (int e = tid; e < Cn; e += NT) L.cnt[e] = 0;
    __syncthreads();
    auto ran = [&](int p) -> bool { return L.ranf[p] != 0; };
    for (int p = 0; p < P; ++p) {
      if (!ran(p)) continue;
      const WProb& q = S.pr[p];
      const uint8_t* lab = R.glab + (static_cast<size_t>(p) * 2 + q.lcur) * a.lsm;
      for (int r = tid; r < m; r += NT) atomicAdd(&L.cnt[q.cenoff + lab[r]], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      int f = 0;
      for (int p = 0; p < P; ++p) {
        if (!ran(p)) continue;
        WProb& q = S.pr[p];
        int ne = 0;
        for (int c = 0; c < q.K; ++c) ne += (L.cnt[q.cenoff + c] == 0);
        q.nempty = ne;
        f |= (ne > 0);
      }
      L.flag = f;
    }
    __syncthreads();
    if (L.flag) {
      for (int p = 0; p < P; ++p) {
        if (!ran(p) || S.pr[p].nempty == 0) continue;
        const WProb& q = S.pr[p];
        relocate(a, L, idx, p, R.cen + (static_cast<size_t>(1 - q.ccur) * Cn + q.cenoff) * dpad,
                 R.cen + (static_cast<size_t>(q.ccur) * Cn + q.cenoff) * dpad,
                 R.glab + (static_cast<size_t>(p) * 2 + q.lcur) * a.lsm,
                 R.dbuf + static_cast<size_t>(p) * a.ndb * a.lsm, R.cenn + q.cenoff, R.rdist, tid);
        __syncthreads();
      }
    }
    if (tid < P && ran(tid)) {
      WProb& q = S.pr[tid];
      int am = 0;
      for (int c = 1; c < q.K; ++c)
        if (L.cnt[q.cenoff + c] > L.cnt[q.cenoff + am]) am = c;
      q.amax = am;
    }
    __syncthreads();
    // _average_centers (_k_means_common.pyx:215-237) runs j in order: an empty cluster j copies
    // centre argmax(weight), which is still a raw sum when j < argmax (pass 0 here, rare) and
    // the averaged one when j > argmax (pass 2 below, rare).  Pass 1, the scaling of every
    // other row, is fused with the centre shift, the f16 image and the norm: one wave per
    // row, 16-B accesses, one read of the new and the old row.
    for (int p = 0; p < P; ++p) {
      if (!ran(p) || S.pr[p].nempty == 0) continue;
      const WProb& q = S.pr[p];
      float* base = R.cen + (static_cast<size_t>(1 - q.ccur) * Cn + q.cenoff) * dpad;
      for (int c = 0; c < q.amax; ++c) {
        if (L.cnt[q.cenoff + c] != 0) continue;
        const float* src = base + static_cast<size_t>(q.amax) * dpad;
        for (int d = tid; d < dpad; d += NT) base[static_cast<size_t>(c) * dpad + d] = src[d];
      }
    }
    __syncthreads();
    auto finish_rows = [&](bool late) {
      int j = 0;
      for (int p = 0; p < P; ++p) {
        if (!ran(p)) continue;
        const WProb& q = S.pr[p];
        for (int c = 0; c < q.K; ++c) {
          const unsigned cn = L.cnt[q.cenoff + c];
          if (late != (cn == 0 && c > q.amax)) continue;  // pass-2 rows are finished after it
          if ((j++ % NW) != wave) continue;
          const int row = q.cenoff + c;
          const float alpha =
              (cn > 0 && !late) ? static_cast<float>(1.0 / static_cast<double>(static_cast<float>(cn))) : 1.f;
          update_row(a, R.cen + (static_cast<size_t>(1 - q.ccur) * Cn + row) * dpad,
                     R.cen + (static_cast<size_t>(q.ccur) * Cn + row) * dpad, alpha,
                     R.cenhl + static_cast<size_t>(row) * 2 * dpad, R.cenn + row, L.shift + row, lane);
        }
      }
    };
    finish_rows(false);
    __syncthreads();
    {
      bool any = false;
      for (int p = 0; p < P; ++p) any |= ran(p) && S.pr[p].nempty > 0;
      if (any) {
        for (int p = 0; p < P; ++p) {
          if (!ran(p) || S.pr[p].nempty == 0) continue;
          const WProb& q = S.pr[p];
          float* base = R.cen + (static_cast<size_t>(1 - q.ccur) * Cn + q.cenoff) * dpad;
          for (int c = q.amax + 1; c < q.K; ++c) {
            if (L.cnt[q.cenoff + c] != 0) continue;
            const float* src = base + static_cast<size_t>(q.amax) * dpad;
            for (int d = tid; d < dpad; d += NT) base[static_cast<size_t>(c) * dpad + d] = src[d];
          }
        }
        __syncthreads();
        finish_rows(true);
        __syncthreads();
      }
    }
    // convergence decisions (_kmeans_single_lloyd :697-736)
    if (tid < P) {
      WProb& q = S.pr[tid];
      if (q.item >= 0 && !q.to_run && (q.st == ST_RUN || q.st == ST_FINAL)) {
        const int kind = iw_kind(L.iw0[q.item / IMW][q.item % IMW]);
        const float inert = static_cast<float>(L.iinert[q.item]);
        if (kind == IK_RUN) {
          q.iter += 1;
          if (!q.changed) {
            q.st = ST_DONE;  // strict convergence: the final labels are this round's
            q.inert = inert;
          } else {
            const float tot = np_pairwise_sum(L.shift + q.cenoff, q.K);
            q.st = (tot <= S.tol || q.iter >= a.max_iter) ? ST_FINAL : ST_RUN;
            q.ccur = static_cast<unsigned char>(1 - q.ccur);  // the averaged sums are the centres now
          }
        } else {
          q.st = ST_DONE;
          q.inert = inert;
        }
      }
    }
    __syncthreads();
    // ---- all problems done: best of n_init per K, output (KMeans.fit :1495-1531) ----------
    bool all_done = true;
    for (int p = 0; p < P; ++p) all_done &= (S.pr[p].st == ST_DONE);
    if (all_done) {
      for (int p0 = 0; p0 < P; p0 += a.n_init) {
        int best = p0;
        for (int i = 1; i < a.n_init; ++i) {
          const int p = p0 + i;
          if (!(S.pr[p].inert < S.pr[best].inert)) continue;
          // _is_same_clustering(labels_p, labels_best): labels_p -> labels_best must be a function
          if (tid <= KMAX) L.map[tid] = -1;
          if (tid == 0) L.flag = 0;
          __syncthreads();
          const uint8_t* l1 = R.glab + (static_cast<size_t>(p) * 2 + S.pr[p].lcur) * a.lsm;
          const uint8_t* l2 = R.glab + (static_cast<size_t>(best) * 2 + S.pr[best].lcur) * a.lsm;
          for (int r = tid; r < m; r += NT) L.map[l1[r]] = l2[r];
          __syncthreads();
          bool bad = false;
          for (int r = tid; r < m; r += NT) bad |= (L.map[l1[r]] != l2[r]);
          if (bad) L.flag = 1;
          __syncthreads();
          if (L.flag) best = p;
          __syncthreads();
        }
        const int kidx = S.pr[p0].kidx;
        const uint8_t* lb = R.glab + (static_cast<size_t>(best) * 2 + S.pr[best].lcur) * a.lsm;
        uint8_t* out = a.labels_out + static_cast<size_t>(kidx) * a.n * a.ldl + h;
        for (int r = tid; r < m; r += NT) out[static_cast<size_t>(idx[r]) * a.ldl] = lb[r];
        if (tid == 0) {
          if (a.inertia_out) a.inertia_out[static_cast<size_t>(kidx) * a.H + h] = S.pr[best].inert;
          if (a.niter_out) a.niter_out[static_cast<size_t>(kidx) * a.H + h] = S.pr[best].iter;
        }
      }
      if (tid == 0) S.finished = 1;
    }
    __syncthreads();
  }

  // ---- next round -----------------------------------------------------------------------------
  if (tid == 0) {
    if (S.finished) {
      for (int ct = 0; ct < a.nct; ++ct) L.tn[ct].nslots = L.tn[ct].nitems = L.tn[ct].nrun = 0;
    } else {
      schedule(a, L, idx, R.cenn);
    }
    int na = 0;
    for (int ct = 0; ct < a.nct; ++ct) na += L.tn[ct].nslots > 0;
    if (na) atomicAdd(a.active, na);
    if (a.stats) {
      atomicAdd(&a.stats[0], L.n_lloyd);
      atomicAdd(&a.stats[1], L.n_seed);
      atomicAdd(&a.stats[2], L.n_mrows);
      atomicAdd(&a.stats[3], L.n_reloc);
      if (na) atomicAdd(&a.stats[4], 1ull);
      atomicAdd(&a.stats[5], static_cast<unsigned long long>(na));
    }
  }
  __syncthreads();
  {
    const int* src = reinterpret_cast<const int*>(L.tn);
    int* dst = reinterpret_cast<int*>(R.tiles);
    const int nw = static_cast<int>(sizeof(WTile) / 4) * a.nct;
    for (int i = tid; i < nw; i += NT) dst[i] = src[i];
    const int* s2 = reinterpret_cast<const int*>(&S);
    int* d2 = reinterpret_cast<int*>(R.st);
    for (int i = tid; i < static_cast<int>(sizeof(WState) / 4); i += NT) d2[i] = s2[i];
  }
}

__global__ __launch_bounds__(NT, 1) void wide_init(WArgs a) {
  __shared__ PS L;
  post_body(a, L, true);
}

__global__ __launch_bounds__(NT, 1) void wide_post(WArgs a) {
  __shared__ PS L;
  post_body(a, L, false);
}

int local_trials(int K) { return 2 + static_cast<int>(std::log(static_cast<double>(K))); }

constexpr size_t HDR = 4096;  // active counter + problem table

struct WL {
  int P = 0, Cn = 0, nct = 0, ndb = 0, kws = 0, RE = 0, DT = 0, lsm = 0;
  size_t off_tolp = 0, off_tiles = 0, off_part = 0, off_glab = 0, off_dbuf = 0, off_cpos = 0, off_cen = 0, off_cenhl = 0,
         off_cenn = 0, off_rdist = 0, per = 0;
};

// returns false (with the error set) when the problem set does not fit the wide path
bool wide_layout(int m, int dpad, const int32_t* Ks, int nK, int n_init, WL& L) {
  L.P = nK * n_init;
  if (L.P > PMAX) {
    cc::set_error("cc_kmeans_wide: at most 64 (K, init) problems per call");
    return false;
  }
  int slots = 0, items = 0, tmax = 0, kmax = 0;
  for (int k = 0; k < nK; ++k) {
    const int K = Ks[k], t = local_trials(K);
    if (K < 1 || K > KMAX || K > m) {
      cc::set_error("cc_kmeans_wide: need 1 <= K <= min(127, m)");
      return false;
    }
    slots += n_init * std::max((K + 3) & ~3, t);
    items += n_init * t;
    L.Cn += n_init * K;
    tmax = std::max(tmax, t);
    kmax = std::max(kmax, K);
  }
  int nct = std::max((slots + CWW - 1) / CWW, (items + IMW - 1) / IMW);
  if (nct > 1) nct += 1;  // first-fit slack
  if (nct > CTMAX || L.Cn > CNMAX) {
    cc::set_error("cc_kmeans_wide: too many centroids for one call (split K_range)");
    return false;
  }
  L.nct = nct;
  L.ndb = tmax + 1;
  L.kws = kmax;
  L.RE = (m + ER - 1) / ER;
  L.DT = (dpad + MDW - 1) / MDW;
  L.lsm = (m + 63) & ~63;
  auto al = [](size_t x) { return (x + 255) & ~static_cast<size_t>(255); };
  size_t o = al(sizeof(WState));
  L.off_tolp = o;
  o += al(sizeof(double) * ((dpad + NT - 1) / NT));
  L.off_tiles = o;
  o += al(sizeof(WTile) * nct);
  L.off_part = o;
  o += al(sizeof(double) * nct * IMW * L.RE);
  L.off_glab = o;
  o += al(static_cast<size_t>(L.P) * 2 * L.lsm);
  L.off_dbuf = o;
  o += al(sizeof(float) * L.P * L.ndb * static_cast<size_t>(L.lsm));
  L.off_cpos = o;
  o += al(sizeof(int32_t) * L.P * L.kws);
  L.off_cen = o;
  o += al(sizeof(float) * 2 * static_cast<size_t>(L.Cn) * dpad);
  L.off_cenhl = o;
  o += al(sizeof(uint16_t) * 2 * static_cast<size_t>(L.Cn) * dpad);
  L.off_cenn = o;
  o += al(sizeof(float) * L.Cn);
  L.off_rdist = o;
  o += al(sizeof(float) * L.lsm);
  L.per = o;
  return true;
}

int hip_fail(const char* what, hipError_t e) {
  cc::set_error(std::string("cc_kmeans_wide: ") + what + ": " + hipGetErrorString(e));
  return CC_ERR_HIP;
}

}  // namespace

extern "C" size_t cc_kmeans_wide_workspace_bytes(int m, int dpad, const int32_t* Ks, int nK, int n_init,
                                                 int batch) {
  if (m <= 0 || dpad <= 0 || !Ks || nK <= 0 || n_init <= 0 || batch <= 0) return 0;
  WL L;
  if (!wide_layout(m, dpad, Ks, nK, n_init, L)) return 0;
  return HDR + L.per * static_cast<size_t>(batch);
}

extern "C" int cc_kmeans_wide(const float* X, const uint16_t* Xhl, const float* xnorm, int n, int dreal,
                              int dpad, int scale_exp, const int32_t* idx_hm, int H, int m, int h_begin,
                              int h_end, const int32_t* Ks, int nK, int n_init, int max_iter, double tol_rel,
                              const double* kpp_u, int kpp_stride, const int32_t* kpp_pos, uint8_t* labels_nh,
                              int ldl, float* inertia, int32_t* n_iter, unsigned long long* stats,
                              void* workspace, size_t ws_bytes, int batch, void* stream) {
  if (!X || !Xhl || !xnorm || !idx_hm || !Ks || !kpp_u || !kpp_pos || !labels_nh || n <= 0 || m <= 0 ||
      m > n || H <= 0 || h_begin < 0 || h_end > H || h_end < h_begin || nK <= 0 || n_init <= 0 ||
      max_iter <= 0 || dreal <= 0 || dreal > dpad || dpad % KC != 0 || ldl < H || batch <= 0 ||
      scale_exp < -62 || scale_exp > 62) {
    cc::set_error("cc_kmeans_wide: bad arguments");
    return CC_ERR_ARG;
  }
  if (((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Xhl) | reinterpret_cast<uintptr_t>(workspace)) & 15) != 0) {
    cc::set_error("cc_kmeans_wide: X, Xhl and the workspace must be 16-B aligned (16-B row and LDS-DMA loads)");
    return CC_ERR_ARG;
  }
  WL L;
  if (!wide_layout(m, dpad, Ks, nK, n_init, L)) return CC_ERR_UNSUPPORTED;
  int kmax = 0, tmax = 0;
  for (int k = 0; k < nK; ++k) {
    kmax = std::max(kmax, Ks[k]);
    tmax = std::max(tmax, local_trials(Ks[k]));
  }
  if (kpp_stride < 1 + (kmax - 1) * tmax) {
    cc::set_error("cc_kmeans_wide: kpp_stride too small");
    return CC_ERR_ARG;
  }
  const int nh = h_end - h_begin;
  if (nh == 0) return CC_OK;
  batch = std::min(batch, nh);
  if (!workspace || ws_bytes < HDR + L.per * static_cast<size_t>(batch)) {
    cc::set_error("cc_kmeans_wide: workspace too small");
    return CC_ERR_ARG;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<int32_t> probs(4 * L.P);
  for (int k = 0; k < nK; ++k)
    for (int i = 0; i < n_init; ++i) {
      const int p = k * n_init + i;
      probs[4 * p] = Ks[k];
      probs[4 * p + 1] = k;
      probs[4 * p + 2] = i;
      probs[4 * p + 3] = local_trials(Ks[k]);
    }
  uint8_t* base = static_cast<uint8_t*>(workspace);
  int* active = reinterpret_cast<int*>(base);
  int32_t* probs_d = reinterpret_cast<int32_t*>(base + 256);
  hipError_t e = hipMemcpyAsync(probs_d, probs.data(), probs.size() * sizeof(int32_t), hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return hip_fail("problem table", e);

  WArgs a{};
  a.X = X;
  a.Xhl = Xhl;
  a.xnorm = xnorm;
  a.n = n;
  a.dreal = dreal;
  a.dpad = dpad;
  a.scale = std::ldexp(1.0f, scale_exp);
  a.inv_scale = std::ldexp(1.0f, -scale_exp);
  a.dscale = std::ldexp(1.0f, 1 - 2 * scale_exp);
  a.idx = idx_hm;
  a.m = m;
  a.H = H;
  a.probs = probs_d;
  a.P = L.P;
  a.Cn = L.Cn;
  a.nct = L.nct;
  a.ndb = L.ndb;
  a.kws = L.kws;
  a.RE = L.RE;
  a.DT = L.DT;
  a.lsm = L.lsm;
  a.max_iter = max_iter;
  a.tol_rel = tol_rel;
  a.kpp_u = kpp_u;
  a.kpp_stride = kpp_stride;
  a.n_init = n_init;
  a.reloc_full = std::getenv("CCMI_WIDE_RELOC_FULL") != nullptr;
  a.kpp_pos = kpp_pos;
  a.labels_out = labels_nh;
  a.ldl = ldl;
  a.inertia_out = inertia;
  a.niter_out = n_iter;
  a.stats = stats;
  a.active = active;
  a.ws = base + HDR;
  a.ws_per = L.per;
  a.off_tolp = L.off_tolp;
  a.off_tiles = L.off_tiles;
  a.off_part = L.off_part;
  a.off_glab = L.off_glab;
  a.off_dbuf = L.off_dbuf;
  a.off_cpos = L.off_cpos;
  a.off_cen = L.off_cen;
  a.off_cenhl = L.off_cenhl;
  a.off_cenn = L.off_cenn;
  a.off_rdist = L.off_rdist;
  // every problem needs at most K seeding rounds + max_iter Lloyd rounds + 1 final E-step; the
  // first-fit packing may defer a problem by a round now and then
  const long long round_cap = 4LL * (max_iter + KMAX + 8) + 64;
  for (int h0 = h_begin; h0 < h_end; h0 += batch) {
    const int nb = std::min(batch, h_end - h0);
    a.h0 = h0;
    a.nb = nb;
    if ((e = hipMemsetAsync(active, 0, sizeof(int), st)) != hipSuccess) return hip_fail("memset", e);
    hipLaunchKernelGGL(wide_tol, dim3(nb * ((dreal + NT - 1) / NT)), dim3(NT), 0, st, a);
    hipLaunchKernelGGL(wide_init, dim3(nb), dim3(NT), 0, st, a);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail("init launch", e);
    const int G = nb * L.nct;
    const unsigned eblocks = static_cast<unsigned>(8 * ((L.RE + 1) / 2) * ((G + 7) / 8));  // 256-row E tiles
    const unsigned mblocks = static_cast<unsigned>(G * L.DT);
    for (long long round = 0;; ++round) {
      int act = 0;
      if ((e = hipMemcpyAsync(&act, active, sizeof(int), hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_fail("active count", e);
      if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail("round sync", e);
      if (act == 0) break;
      if (round >= round_cap) {
        cc::set_error("cc_kmeans_wide: round cap exceeded");
        return CC_ERR_HIP;
      }
      hipLaunchKernelGGL(wide_estep, dim3(eblocks), dim3(NT), 0, st, a);
      hipLaunchKernelGGL(wide_mstep, dim3(mblocks), dim3(NT), 0, st, a);
      if ((e = hipMemsetAsync(active, 0, sizeof(int), st)) != hipSuccess) return hip_fail("memset", e);
      hipLaunchKernelGGL(wide_post, dim3(nb), dim3(NT), 0, st, a);
      if ((e = hipGetLastError()) != hipSuccess) return hip_fail("round launch", e);
    }
  }
  return CC_OK;
}
