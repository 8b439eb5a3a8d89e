// Batched augmented Gram (SYRK) on f64 MFMA — kernel K1 of SURVEY.md §2.5.
//
// For every local worker n with shard H_n (m x d, row-major) and labels y_n (m):
//     A_n = H_n^T H_n  (d x d, full symmetric),  b_n = H_n^T y_n,  yy_n = y_n^T y_n
// computed as ONE lower-triangular SYRK of the augmented matrix [H_n | y_n] (D = d+1 columns), so
// the shard is streamed exactly once. The reference recomputes H^T H inside every closed-form solve
// (group_ADMM_closedForm.m:43,45,82,84); here it is loop-invariant set-up.
//
// Tiling (gfx950): a 256-thread workgroup owns one BT x BT tile of the lower triangle; its 4 waves
// are 2 x 2, each wave (BT/2) x (BT/2) as (BT/32)^2 tiles of v_mfma_f64_16x16x4_f64. K is staged
// through LDS in BK = 16-row slabs (rows padded by 16 doubles: conflict-free ds_read_b64 — lanes
// 0..15 read row r and lanes 16..31 row r+1 of the same half-wave), with the next slab prefetched
// into registers while the MFMAs of the current one issue. Tall shards are split along K into
// `ksplit` partial slabs that a second kernel reduces in a fixed order (deterministic; no f64
// atomics). Workgroup ids are XCD-remapped so consecutive tiles share an L2.
//
// f64 MFMA fragment maps (cdna_hip_programming.md §3): A/B one f64 per lane, A[i=l&15][k=l>>4],
// B[k=l>>4][j=l&15]; C/D col = l&15, row = (l>>4) + 4*reg.
#include <stdlib.h>
#include "gadmm_common.h"

namespace {

constexpr int BK = 16;
constexpr int PAD = 16;

// Lower-triangular tile id -> (ti, tj), ti >= tj, in SUPERTILE order: the tiles of an ST x ST block of
// the triangle (rows [ST I, ST I + ST), columns [ST J, ST J + ST), J <= I) get consecutive ids, blocks
// in row-major order over the triangle. With the XCD remap, the workgroups one XCD runs together are
// then a square-ish block of tiles that share 2 ST column panels of the shard (ST^2 tiles from 2 ST
// panels) instead of a strip of one tile row (~64 tiles from ~65 panels): 3-4x fewer distinct shard
// bytes per K row through that XCD's L2 (the d = 10k Gram was operand-bandwidth bound at ~52 TF/s).
// ST = 0: the plain row-major triangle order.
__device__ __forceinline__ void tri_of(int t, int& ti, int& tj) {
  ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  while (ti * (ti + 1) / 2 > t) --ti;
  tj = t - ti * (ti + 1) / 2;
}

__device__ __forceinline__ void tile_of(int tile, int nt, int ST, int& ti, int& tj) {
  if (ST <= 1 || nt <= ST) {
    tri_of(tile, ti, tj);
    return;
  }
  // walk the supertile rows: block row I holds I full ST x ST blocks (J < I) and one diagonal block
  const int nbr = (nt + ST - 1) / ST;
  int base = 0;
  for (int I = 0; I < nbr; ++I) {
    const int rows = (I + 1) * ST <= nt ? ST : nt - I * ST;  // tile rows in this block row
    const int rlo = I * ST;
    // tiles of block row I: sum over its rows r of (r + 1) = the rows' triangle widths
    const int in_row = rows * rlo + rows * (rows + 1) / 2;
    if (tile >= base + in_row) {
      base += in_row;
      continue;
    }
    const int off = tile - base;
    const int full = I * ST * rows;  // the I full blocks (J < I), each rows x ST tiles
    if (off < full) {
      const int J = off / (rows * ST), o = off % (rows * ST);
      ti = rlo + o / ST;
      tj = J * ST + o % ST;
    } else {
      int a, b;
      tri_of(off - full, a, b);  // the diagonal block: a lower triangle of rows x rows tiles
      ti = rlo + a;
      tj = rlo + b;
    }
    return;
  }
  ti = tj = 0;  // unreachable for tile < ntiles
}

// NT threads = NT/64 waves arranged WR x 2; a wave owns a (BT/WR) x (BT/2) sub-tile of MFMA tiles.
template <int BT, int NT>
struct GramTile {
  static constexpr int NWAVE = NT / 64;
  static constexpr int WR = NWAVE / 2;      // wave rows
  static constexpr int WTR = BT / WR;       // wave tile rows
  static constexpr int WTC = BT / 2;        // wave tile cols
  static constexpr int TMR = WTR / 16;      // MFMA tiles per wave (rows)
  static constexpr int TMC = WTC / 16;      // MFMA tiles per wave (cols)
  static constexpr int LDSROW = BT + PAD;   // doubles per LDS row
  static constexpr int PER_THREAD = BK * BT / NT;
};

// The K loop of one tile: slabs of BK rows staged through two LDS buffers. DIAG (uniform per
// workgroup: a diagonal tile reads one panel) is a template parameter and the full slabs of an
// interior tile run a loop with NO branch around the next slab's global loads, so those loads stay in
// flight across the current slab's MFMAs (the wait lands right before the stash). With a branch (the
// old `if (interior) ... else ...` / `if (!diag)` fetch), the compiler merged the two paths' registers
// with moves right after the loads and drained vmcnt(0) there, exposing the load latency on every slab.
// Tiles with columns past the shard (the y column, the zero padding) run the same pipelined loop with
// clamped loads + selects (CLAMP); only the partial last slab takes the synchronous clamped path.
// Same MFMA order either way (bit-identical results).
template <int BT, int NT, bool DIAG, bool CLAMP>
__device__ __forceinline__ void gram_slabs(const double* __restrict__ H, const double* __restrict__ yv, int d,
                                           long kbeg, long kend, long nfull, int row0, int col0,
                                           double (*lds)[2 * BK * GramTile<BT, NT>::LDSROW],
                                           f64x4 (&acc)[GramTile<BT, NT>::TMR][GramTile<BT, NT>::TMC]) {
  using T = GramTile<BT, NT>;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  double ri[T::PER_THREAD], rj[T::PER_THREAD];
  auto fetch_in = [&](long k0) {  // branch-free 8-B loads (every column < d, every row < kend)
#pragma unroll
    for (int p = 0; p < T::PER_THREAD / 2; ++p) {
      const int e2 = tid + NT * p;
      const int r = e2 / (BT / 2), c = (e2 % (BT / 2)) * 2;
      const double* src = H + (k0 + r) * (long)d;
      ri[2 * p] = src[row0 + c];
      ri[2 * p + 1] = src[row0 + c + 1];
      if constexpr (!DIAG) {
        rj[2 * p] = src[col0 + c];
        rj[2 * p + 1] = src[col0 + c + 1];
      }
    }
  };
  auto fetch_cl = [&](long k0) {  // clamped loads + selects: the y column, zero padding, rows past kend
#pragma unroll
    for (int p = 0; p < T::PER_THREAD / 2; ++p) {
      const int e2 = tid + NT * p;
      const int r = e2 / (BT / 2), c = (e2 % (BT / 2)) * 2;
      const long k = k0 + r;
      const long kk = k < kend ? k : (kend - 1);
      const double yk = yv[kk];
      const bool kin = k < kend;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ca = row0 + c + q, cb = col0 + c + q;
        const double va = H[kk * d + (ca < d ? ca : d - 1)];
        ri[2 * p + q] = kin ? (ca < d ? va : (ca == d ? yk : 0.0)) : 0.0;
        if constexpr (!DIAG) {
          const double vb = H[kk * d + (cb < d ? cb : d - 1)];
          rj[2 * p + q] = kin ? (cb < d ? vb : (cb == d ? yk : 0.0)) : 0.0;
        }
      }
    }
  };
  // CLAMP tiles in the pipelined loop: raw clamped loads at the top of a slab (fetch_raw), the selects
  // (y column, zero padding, rows past kend) applied at the stash, after the MFMAs, so the loads stay
  // in flight across them like fetch_in's
  double yr[CLAMP ? T::PER_THREAD / 2 : 1];
  long kraw = 0;
  auto fetch_raw = [&](long k0) {
    kraw = k0;
#pragma unroll
    for (int p = 0; p < T::PER_THREAD / 2; ++p) {
      const int e2 = tid + NT * p;
      const int r = e2 / (BT / 2), c = (e2 % (BT / 2)) * 2;
      const long k = k0 + r;
      const long kk = k < kend ? k : (kend - 1);
      yr[p] = yv[kk];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ca = row0 + c + q, cb = col0 + c + q;
        ri[2 * p + q] = H[kk * d + (ca < d ? ca : d - 1)];
        if constexpr (!DIAG) rj[2 * p + q] = H[kk * d + (cb < d ? cb : d - 1)];
      }
    }
  };
  auto select_raw = [&]() {
#pragma unroll
    for (int p = 0; p < T::PER_THREAD / 2; ++p) {
      const int e2 = tid + NT * p;
      const int r = e2 / (BT / 2), c = (e2 % (BT / 2)) * 2;
      const bool kin = kraw + r < kend;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ca = row0 + c + q, cb = col0 + c + q;
        ri[2 * p + q] = kin ? (ca < d ? ri[2 * p + q] : (ca == d ? yr[p] : 0.0)) : 0.0;
        if constexpr (!DIAG) rj[2 * p + q] = kin ? (cb < d ? rj[2 * p + q] : (cb == d ? yr[p] : 0.0)) : 0.0;
      }
    }
  };
  auto stash = [&](int buf) {
    if constexpr (CLAMP) select_raw();
    double* Si = lds[buf];
    double* Sj = lds[buf] + BK * T::LDSROW;
#pragma unroll
    for (int p = 0; p < T::PER_THREAD / 2; ++p) {
      const int e2 = tid + NT * p;
      const int r = e2 / (BT / 2), c = (e2 % (BT / 2)) * 2;
      *reinterpret_cast<double2*>(Si + r * T::LDSROW + c) = make_double2(ri[2 * p], ri[2 * p + 1]);
      if constexpr (!DIAG) *reinterpret_cast<double2*>(Sj + r * T::LDSROW + c) = make_double2(rj[2 * p], rj[2 * p + 1]);
    }
  };
  auto mma = [&](int buf) {
    const double* Ci = lds[buf];
    const double* Cb = DIAG ? Ci : lds[buf] + BK * T::LDSROW;
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double a[T::TMR], b[T::TMC];
#pragma unroll
      for (int t = 0; t < T::TMR; ++t) a[t] = Ci[kr * T::LDSROW + wr * T::WTR + t * 16 + (lane & 15)];
#pragma unroll
      for (int t = 0; t < T::TMC; ++t) b[t] = Cb[kr * T::LDSROW + wc * T::WTC + t * 16 + (lane & 15)];
#pragma unroll
      for (int x = 0; x < T::TMR; ++x)
#pragma unroll
        for (int yq = 0; yq < T::TMC; ++yq)
          acc[x][yq] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], b[yq], acc[x][yq], 0, 0, 0);
    }
  };

  auto fetch = [&](long k0) {
    if constexpr (CLAMP) fetch_raw(k0);
    else fetch_in(k0);
  };
  int cur = 0;
  long k0 = kbeg;
  if (nfull > 0) {
    fetch(k0);
    stash(0);
    lds_barrier();
    for (long s = 1; s < nfull; ++s) {  // slab s - 1 in LDS buffer cur; slab s loads during its MFMAs
      fetch(k0 + BK);
      mma(cur);
      stash(cur ^ 1);  // the other buffer: nobody reads it during this slab
      lds_barrier();   // slab s visible, and every wave is done reading slab s - 1
      cur ^= 1;
      k0 += BK;
    }
    mma(cur);
    lds_barrier();  // every wave is done with the last full slab before any buffer is rewritten
    cur ^= 1;
    k0 += BK;
  }
  for (; k0 < kend; k0 += BK) {  // synchronous clamped slabs, alternating buffers (one barrier each)
    if constexpr (CLAMP) fetch_raw(k0);  // selected by the stash
    else fetch_cl(k0);
    stash(cur);
    lds_barrier();
    mma(cur);
    cur ^= 1;
  }
}

template <int BT, int NT>
__global__ void __launch_bounds__(NT)
gram_aug_kernel(const double* __restrict__ X, const double* __restrict__ Y, int m, int d,
                int ntiles, int ksplit, long rows_per_split,
                double* __restrict__ A, double* __restrict__ B, double* __restrict__ YY,
                double* __restrict__ slab, int nt, int ST) {
  using T = GramTile<BT, NT>;
  // two LDS buffers (double buffering): slab s is read from buffer s&1 while slab s+1 is written
  // into the other one, so each K step needs ONE LDS-only barrier and the staging stores issue
  // behind the MFMAs instead of between two barriers
  __shared__ __attribute__((aligned(16))) double lds[2][2 * BK * T::LDSROW];

  const int nwg = gridDim.x;
  const int gid = xcd_remap(blockIdx.x, nwg);
  const int tile = gid % ntiles;
  const int rest = gid / ntiles;
  const int split = rest % ksplit;
  const int n = rest / ksplit;

  int ti, tj;
  tile_of(tile, nt, ST, ti, tj);
  const bool diag = (ti == tj);
  const int row0 = ti * BT, col0 = tj * BT;

  const double* H = X + (long)n * m * d;
  const double* yv = Y + (long)n * m;
  const long kbeg = (long)split * rows_per_split;
  long kend = kbeg + rows_per_split;
  if (kend > m) kend = m;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;  // T::WR x 2 waves
  const int D = d + 1;

  f64x4 acc[T::TMR][T::TMC];
#pragma unroll
  for (int a = 0; a < T::TMR; ++a)
#pragma unroll
    for (int b = 0; b < T::TMC; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};

  // every tile runs its full slabs in the pipelined loop: interior tiles (every column < d) with
  // branch-free loads, boundary tiles (the y column, zero padding) with the clamped ones; see gram_slabs
  const bool cols_in = (row0 + BT <= d) && (diag || col0 + BT <= d);
  const long nfull = kend > kbeg ? (kend - kbeg) / BK : 0;
  if (kbeg < kend) {
    if (cols_in) {
      if (diag) gram_slabs<BT, NT, true, false>(H, yv, d, kbeg, kend, nfull, row0, col0, lds, acc);
      else gram_slabs<BT, NT, false, false>(H, yv, d, kbeg, kend, nfull, row0, col0, lds, acc);
    } else {
      if (diag) gram_slabs<BT, NT, true, true>(H, yv, d, kbeg, kend, nfull, row0, col0, lds, acc);
      else gram_slabs<BT, NT, false, true>(H, yv, d, kbeg, kend, nfull, row0, col0, lds, acc);
    }
  }

  // epilogue
#pragma unroll
  for (int x = 0; x < T::TMR; ++x)
#pragma unroll
    for (int yq = 0; yq < T::TMC; ++yq)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int lr = wr * T::WTR + x * 16 + (lane >> 4) + 4 * reg;  // row within tile
        const int lc = wc * T::WTC + yq * 16 + (lane & 15);          // col within tile
        const double v = acc[x][yq][reg];
        if (ksplit > 1) {
          slab[(((long)n * ntiles + tile) * ksplit + split) * (BT * BT) + lr * BT + lc] = v;
          continue;
        }
        const int r = row0 + lr, c = col0 + lc;
        if (r >= D || c >= D || c > r) continue;  // lower triangle (incl. diagonal) only
        if (r < d && c < d) {
          double* An = A + (long)n * d * d;
          An[(long)r * d + c] = v;
          An[(long)c * d + r] = v;
        } else if (r == d && c < d) {
          B[(long)n * d + c] = v;
        } else if (r == d && c == d) {
          YY[n] = v;
        }
      }
}

// Fixed-order reduction of the split-K slabs + symmetric scatter into (A, b, yy).
template <int BT>
__global__ void __launch_bounds__(256)
gram_reduce_kernel(const double* __restrict__ slab, int d, int ntiles, int ksplit,
                   double* __restrict__ A, double* __restrict__ B, double* __restrict__ YY, int nt, int ST) {
  const int tile = blockIdx.x, n = blockIdx.y;
  int ti, tj;
  tile_of(tile, nt, ST, ti, tj);
  const int D = d + 1;
  const double* s = slab + ((long)n * ntiles + tile) * ksplit * (BT * BT);
  for (int e = threadIdx.x; e < BT * BT; e += blockDim.x) {
    const int lr = e / BT, lc = e % BT;
    const int r = ti * BT + lr, c = tj * BT + lc;
    if (r >= D || c >= D || c > r) continue;
    double v = 0.0;
    for (int k = 0; k < ksplit; ++k) v += s[(long)k * BT * BT + e];
    if (r < d && c < d) {
      double* An = A + (long)n * d * d;
      An[(long)r * d + c] = v;
      An[(long)c * d + r] = v;
    } else if (r == d && c < d) {
      B[(long)n * d + c] = v;
    } else if (r == d && c == d) {
      YY[n] = v;
    }
  }
}

template <int BT>
int launch_gram(const double* X, const double* Y, int N, int m, int d, int ksplit, double* A,
                double* B, double* YY, double* slab, hipStream_t st) {
  const int D = d + 1;
  const int nt = (D + BT - 1) / BT;
  const int ntiles = nt * (nt + 1) / 2;
  if (ksplit < 1) ksplit = 1;
  long rows = ((long)m + ksplit - 1) / ksplit;
  rows = ((rows + BK - 1) / BK) * BK;
  ksplit = (int)(((long)m + rows - 1) / rows);
  if (ksplit < 1) ksplit = 1;
  const long nwg = (long)ntiles * ksplit * N;
  static const int nt_env = getenv("GADMM_GRAM_NT") ? atoi(getenv("GADMM_GRAM_NT")) : 0;  // A/B switch
  const int nthr = nt_env == 256 || nt_env == 512 ? nt_env : (BT == 128 ? 512 : 256);
  // tile order: row-major over the triangle (tile_of's supertile order, ST = 8, measured 0.5 % slower
  // at 2 x 625000 x 10000: profiles/r03_gram; the LDS-DMA ring variants measured ~1 % slower:
  // profiles/r03_gram_glds, r04_gram -- both removed in round 6)
  const int ST = 0;
  if (nthr == 512)
    hipLaunchKernelGGL((gram_aug_kernel<BT, 512>), dim3((unsigned)nwg), dim3(512), 0, st, X, Y, m, d, ntiles, ksplit,
                       rows, A, B, YY, slab, nt, ST);
  else
    hipLaunchKernelGGL((gram_aug_kernel<BT, 256>), dim3((unsigned)nwg), dim3(256), 0, st, X, Y, m, d, ntiles, ksplit,
                       rows, A, B, YY, slab, nt, ST);
  if (ksplit > 1) {
    hipLaunchKernelGGL(gram_reduce_kernel<BT>, dim3(ntiles, N), dim3(256), 0, st, slab, d, ntiles,
                       ksplit, A, B, YY, nt, ST);
  }
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // namespace

extern "C" {

// Workspace (doubles) needed for a given split; 0 when ksplit == 1.
long gadmm_gram_workspace(int N, int m, int d, int ksplit) {
  if (ksplit <= 1) return 0;
  const int BT = (d + 1 <= 64) ? 64 : 128;
  const int nt = (d + 1 + BT - 1) / BT;
  return (long)N * (nt * (nt + 1) / 2) * ksplit * BT * BT;
}

// Heuristic split so that the grid covers the chip (>= ~2 workgroups per CU) for tall shards.
int gadmm_gram_pick_ksplit(int N, int m, int d) {
  // Split K so the grid fills whole "waves" of resident workgroups: with W workgroups and S
  // resident slots the run takes ceil(W / S) rounds, efficiency W / (rounds * S). Pick the
  // smallest split reaching the target (default 97 %, env GADMM_GRAM_EFF; the split-K reduce pass
  // is cheap next to the SYRK itself). At the real10m shape (2 x 625000 x 10000) a 90 % target
  // picked 1 split: 13 rounds whose last ran 176 of 512 slots (5 % of the Gram idle); 2 splits run
  // 25 rounds at 98.75 %.
  const int BT = (d + 1 <= 64) ? 64 : 128;
  const int nt = (d + 1 + BT - 1) / BT;
  const long tiles = (long)N * (nt * (nt + 1) / 2);
  int cus = gadmm_cu_count();
  if (cus <= 0) cus = 256;
  // 2 resident workgroups per CU (LDS / VGPR bound)
  const long slots = (long)cus * 2;
  long maxk = (m + 255) / 256;       // keep >= 256 rows per split
  if (maxk > 64) maxk = 64;
  if (maxk < 1) maxk = 1;
  static const double target = getenv("GADMM_GRAM_EFF") ? atof(getenv("GADMM_GRAM_EFF")) : 0.97;
  long best = 1;
  double best_eff = 0.0;
  for (long k = 1; k <= maxk; ++k) {
    const long W = tiles * k;
    const long rounds = (W + slots - 1) / slots;
    const double eff = (double)W / (double)(rounds * slots);
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = k;
    }
    if (eff >= target && W >= slots) {
      best = k;
      break;
    }
  }
  return (int)best;
}

int gadmm_gram_f64(const double* X, const double* Y, int N, int m, int d, int ksplit, double* A,
                   double* B, double* YY, double* slab, hipStream_t st) {
  if (N <= 0 || m <= 0 || d <= 0) return 0;
  if (ksplit > 1 && slab == nullptr) {
    gadmm_set_error("gram: ksplit=%d needs a workspace", ksplit);
    return -1;
  }
  if (d + 1 <= 64) return launch_gram<64>(X, Y, N, m, d, ksplit, A, B, YY, slab, st);
  return launch_gram<128>(X, Y, N, m, d, ksplit, A, B, YY, slab, st);
}

}  // extern "C"
