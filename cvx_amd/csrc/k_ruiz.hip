// k_ruiz.hip — every Ruiz sweep of MatrixUtils.scala:240-268 in ONE persistent launch, H held in registers.
//
// The multi-launch form (k_vec.hip: k_ruiz_tiles + k_ruiz_rows per sweep) streams the lower triangle of H from HBM
// once per sweep and pays two launches per sweep; the C3 loop runs 13 sweeps (~245 us per Newton step).  Here each
// workgroup claims a run of lower 64 x 64 tiles once and keeps them in VGPRs (RZ_MT tiles = 288 VGPRs per lane: 2080
// tiles over 256 workgroups at n = 4096); a sweep is then a dataflow step in which every hand-off is a data-tagged
// 16-B granule {value, tag(k)} (tag(k) = launch generation << 8 | sweep), polled directly by its consumer -- no
// flags, no drains, no atomics on the sweep's path:
//   tile (I, J), sweep k:  polls d^(k) of blocks I and J (dbuf[k]); writes the partials S[J][rows of I] (row sums)
//                          and S[I][rows of J] (column sums) as granules tagged k
//   block X, sweep k:      the workgroup owning the diagonal tile (X, X) polls S[0..nbn)[rows of X] for tag k, adds
//                          them, and writes d^(k+1) of block X (dbuf[k+1]) and the block's max |1 - u| (rhop[k+1][X])
// Every partial, sum and d entry is computed by the same expressions in the same order as k_ruiz_tiles /
// k_ruiz_rows, so d, rho and the sweep count are bitwise those of the multi-launch loop.
//
// Termination (sweep k runs iff rho[k] > 1e-6, rho[0] = 1, rho[k] = max_X rhop[k][X]): the reference's test runs one
// sweep behind here -- sweep k runs while rho[k-1] > 1e-6, polled from rhop[k-1] (written by the reductions of sweep
// k-2, which every sweep-(k-1) tile waited for) -- so the sweep K with rho[K] <= 1e-6 runs too, writing dbuf[K+1] and
// rhop[K+1], which nobody reads; k_ruiz_loop_final finds K and copies dbuf[K].  d of every sweep has its own buffer;
// the partial slots are reused from sweep to sweep, which is safe: tile (I, J) of sweep k+1 needs d^(k+1) of I and J,
// i.e. the sweep-k reductions that read both of its slots.
//
// Deadlock freedom: a workgroup claims tiles (an atomic counter) until the pool is empty before it starts sweeping, so
// every tile, and every block's reduction, belongs to a running workgroup whatever the residency (claims beyond RZ_MT
// are streamed from H each sweep; the host takes this path only while RZ_LIST holds every tile).  A workgroup runs its
// tiles of sweep k, then its reductions of sweep k: a reduction waits only on sweep-k tiles, which wait only on
// sweep-(k-1) reductions.  Polls are bounded (SPIN_LIMIT_TICKS): on a timeout the abort word is raised, every
// workgroup leaves, and the final pass reports ruiz_sweeps = -2.
#include <algorithm>

#include "potrf64.hpp"
#include "ruiz_tile.hpp"

namespace cvxg {

constexpr int RZ_MT = 9;        // tiles a workgroup keeps in registers
constexpr int RZ_LIST = 8192;   // tiles a workgroup can own (registers + streamed)
constexpr int RZ_OWN = 128;     // diagonal tiles (block reductions) a workgroup can own

size_t ruiz_loop_work_ints(int) { return 2; }
bool ruiz_loop_fits(int nbn) { return nbn <= RZ_OWN && (size_t)nbn * (nbn + 1) / 2 <= (size_t)RZ_LIST; }
size_t ruiz_loop_doubles(int nbn) {  // 16-B granules of dbuf, the partials and rhop
  const size_t ld = (size_t)nbn * NB;
  return 2 * ((RUIZ_MAX + 1) * ld + (size_t)nbn * ld + (RUIZ_MAX + 1) * (size_t)nbn);
}

namespace {

__device__ __forceinline__ int rz_poll(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ double rz_tag(unsigned long long gen, int k) {
  return __longlong_as_double((long long)((gen << 8) | (unsigned long long)k));
}
__device__ __forceinline__ bool rz_is(f64x2 g, double tag) {
  return __double_as_longlong(g[1]) == __double_as_longlong(tag);
}

// a granule array (16 B each) behind an sc1 buffer descriptor
struct Gran {
  __amdgpu_buffer_rsrc_t r;
  __device__ Gran(double* base, size_t count) : r(uniform_rsrc(base, (unsigned)(count * 16))) {}
  __device__ __forceinline__ f64x2 ld(int i) const {
    return __builtin_bit_cast(f64x2, __builtin_amdgcn_raw_buffer_load_b128(r, i * 16, 0, AUX_SC1));
  }
  __device__ __forceinline__ void st(int i, double v, double tag) const {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f64x2{v, tag}), r, i * 16, 0, AUX_SC1);
  }
};

struct RzShared {
  int tile[RZ_LIST];             // claimed tiles, (I << 16) | J
  int own[RZ_OWN];               // blocks whose reduction this workgroup runs (its diagonal tiles)
  int nt, nown, ok, stop;
  double d[2 * RZ_MT][NB];       // d^(k) of the batch's blocks: tile t's I at 2t, J at 2t + 1
  double cred[RZ_MT][8][NB];     // column partials per row group
  double red[4][NB];
};

struct RzArgs {
  int n, nbn;
  double* dbuf;  // (RUIZ_MAX + 1) x nbn NB granules: d^(k)
  double* part;  // nbn x nbn NB granules: S[P][row]
  double* rhop;  // (RUIZ_MAX + 1) x nbn granules: rhop[k][X] = max |1 - u| over block X in sweep k - 1
  int* abortw;
  unsigned long long gen;
};

// Every thread loads its granules i < G with bit i of `need` set (index idx(i)) and polls until each carries `tag`;
// false on abort / timeout (abort word raised).
template <int G, class Idx>
__device__ __forceinline__ bool rz_wait_all(f64x2 (&g)[G], unsigned need, double tag, const Gran& src, Idx idx,
                                            int* abortw, int code, bool loaded = false) {
  if (!loaded) {
#pragma unroll
    for (int i = 0; i < G; ++i)
      if (need >> i & 1) g[i] = src.ld(idx(i));
  }
  const unsigned long long t0 = spin_clock();
  for (unsigned spins = 0;; ++spins) {
    unsigned miss = 0;
#pragma unroll
    for (int i = 0; i < G; ++i)
      if ((need >> i & 1) && !rz_is(g[i], tag)) miss |= 1u << i;
    if (!miss) return true;
    if ((spins & 15) == 15 && rz_poll(abortw)) return false;
    if (spin_expired(spins, t0)) {
      __hip_atomic_store(abortw, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
#pragma unroll
    for (int i = 0; i < G; ++i)
      if (miss >> i & 1) g[i] = src.ld(idx(i));
  }
}

// Block-uniform verdict of per-thread waits (false anywhere -> false everywhere); a barrier on both sides.
__device__ __forceinline__ bool rz_agree(bool mine, RzShared& sh) {
  __syncthreads();
  if (threadIdx.x == 0) sh.ok = 1;
  __syncthreads();
  if (!mine) sh.ok = 0;
  __syncthreads();
  return sh.ok != 0;
}

// One sweep over a batch of nb <= MT tiles whose entries are in h (k_ruiz_tiles' per-thread layout: row g + 8 q,
// columns 2 c2, 2 c2 + 1).  False: stop (the loop is done) or abort.
// the thread index through an empty asm: the compiler cannot prove it loop-invariant, so the many addresses derived
// from it are recomputed per sweep instead of being held (and spilled) across the sweep loop
__device__ __forceinline__ int rz_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

template <int MT>
__device__ __forceinline__ bool rz_batch(const f64x2 (&h)[MT][8], int nb, const int* tiles, int k, const RzArgs& a,
                                         RzShared& sh, bool check_stop, unsigned long long* dstamp = nullptr) {
  const int tid = rz_tid(), lane = tid & 63, wid = tid >> 6;
  const int c2 = tid & 31, g = tid >> 5;
  const int nbn = a.nbn, ldS = nbn * NB;
  const Gran dk(a.dbuf + (size_t)k * ldS * 2, ldS), S(a.part, (size_t)nbn * ldS);
  const double tk = rz_tag(a.gen, k);
  // d^(k) of the batch's blocks: each thread polls its granules (2 MT 64 entries over 256 threads)
  constexpr int G = (2 * MT * NB + 255) / 256;
  f64x2 gd[G];
  unsigned need = 0;
#pragma unroll
  for (int i = 0; i < G; ++i)
    if (k > 0 && tid + 256 * i < nb * 2 * NB) need |= 1u << i;
  auto didx = [&](int i) {
    const int e = tid + 256 * i, t = e / (2 * NB), w = (e / NB) & 1;
    return (w ? (tiles[t] & 0xffff) : (tiles[t] >> 16)) * NB + (e & (NB - 1));
  };
  // d loads first (in flight while wave 0 polls the stop test)
#pragma unroll
  for (int i = 0; i < G; ++i)
    if (need >> i & 1) gd[i] = dk.ld(didx(i));
  // the stop test: rho[k-1] = max_X rhop[k-1][X], polled by wave 0 (k >= 2; rho[0] = 1)
  bool ok = true;
  if (check_stop && k >= 2 && wid == 0) {
    const Gran rp(a.rhop + (size_t)(k - 1) * nbn * 2, (size_t)nbn);
    const double tr = rz_tag(a.gen, k - 1);
    f64x2 gr[2];
    const unsigned nr = (lane < nbn ? 1u : 0u) | (lane + 64 < nbn ? 2u : 0u);
    ok = rz_wait_all<2>(gr, nr, tr, rp, [&](int i) { return lane + 64 * i; }, a.abortw, 0x10000 | k << 8);
    double m = 0.0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (nr >> i & 1) m = fmax(m, gr[i][0]);
    m = wave_max(m);
    if (lane == 0) sh.stop = !(m > 1e-6);
  } else if (tid == 0) {
    sh.stop = 0;
  }
  ok = ok && rz_wait_all<G>(gd, need, tk, dk, didx, a.abortw, 0x20000 | k << 8, true);
  if (!rz_agree(ok, sh)) return false;
  if (sh.stop) return false;
  if (dstamp && tid == 0) *dstamp = __builtin_amdgcn_s_memrealtime();
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int e = tid + 256 * i;
    if (e < nb * 2 * NB) sh.d[e / NB][e & (NB - 1)] = (k == 0) ? 1.0 : gd[i][0];
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    if (t < nb) {
      const int I = tiles[t] >> 16, J = tiles[t] & 0xffff;
      const f64x2 dj = {sh.d[2 * t + 1][2 * c2], sh.d[2 * t + 1][2 * c2 + 1]};
      f64x2 csum = {0.0, 0.0};
      double rs[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {  // ruiz_tile.hpp's arithmetic, as k_ruiz_tiles (the 8 sums side by side)
        const double di = sh.d[2 * t][g + 8 * q];
        const f64x2 av = dj * h[t][q];
        rs[q] = av[0] * av[0] + av[1] * av[1];
        const f64x2 bv = h[t][q] * di;
        csum = __builtin_elementwise_fma(bv, bv, csum);
      }
      rz_rowgroup_sum8(rs);
      if (c2 == RZ_ROW_LANE) {
#pragma unroll
        for (int q = 0; q < 8; ++q) S.st(J * ldS + I * NB + g + 8 * q, rs[q], tk);
      }
      if (I != J) {
        sh.cred[t][g][2 * c2] = csum[0];
        sh.cred[t][g][2 * c2 + 1] = csum[1];
      }
    }
  }
  __syncthreads();
  if (tid < NB) {
    for (int t = 0; t < nb; ++t) {
      const int I = tiles[t] >> 16, J = tiles[t] & 0xffff;
      if (I != J) {
        double v = sh.cred[t][0][tid];
#pragma unroll
        for (int r = 1; r < 8; ++r) v += sh.cred[t][r][tid];
        S.st(I * ldS + J * NB + tid, v, tk);
      }
    }
  }
  return true;
}

// The reduction of block X in sweep k (k_ruiz_rows' sums in its order): d^(k+1) of the block, its max |1 - u|.
__device__ __forceinline__ bool rz_reduce(int X, int k, const RzArgs& a, RzShared& sh) {
  const int tid = rz_tid(), lane = tid & 63, wid = tid >> 6;
  const int nbn = a.nbn, ldS = nbn * NB;
  const Gran S(a.part, (size_t)nbn * ldS), dk(a.dbuf + (size_t)k * ldS * 2, ldS),
      dn(a.dbuf + (size_t)(k + 1) * ldS * 2, ldS), rp(a.rhop + (size_t)(k + 1) * nbn * 2, (size_t)nbn);
  const double tk = rz_tag(a.gen, k), tn = rz_tag(a.gen, k + 1);
  const int row = X * NB + lane;
  const bool live = row < a.n;
  // wave q's partials P = q, q + 4, ..., polled 16 at a time (nbn <= 128: at most two rounds), summed in
  // k_ruiz_rows' order: s0..s3 over P, P + 4, P + 8, P + 12 while P + 12 < nbn (P += 16), then the tail into s0
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  bool ok = true, main = true;
  for (int half = 0; half < 2 && ok; ++half) {
    const int P0 = wid + 64 * half;
    if (!live || P0 >= nbn) break;
    f64x2 gp[16];
    unsigned nd = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (P0 + 4 * i < nbn) nd |= 1u << i;
    ok = rz_wait_all<16>(gp, nd, tk, S, [&](int i) { return (P0 + 4 * i) * ldS + row; }, a.abortw,
                         0x30000 | k << 8 | X);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int P = P0 + 16 * c;
      if (main && P + 12 < nbn) {
        s0 += gp[4 * c][0];
        s1 += gp[4 * c + 1][0];
        s2 += gp[4 * c + 2][0];
        s3 += gp[4 * c + 3][0];
      } else if (main) {
        main = false;
#pragma unroll
        for (int jj = 0; jj < 3; ++jj)
          if (P + 4 * jj < nbn) s0 += gp[4 * c + jj][0];
      }
    }
  }
  // d^(k) of the block's rows (wave 0; the workgroup's own diagonal tile polled it this sweep)
  f64x2 gdi[1];
  const unsigned ndi = (wid == 0 && live && k > 0) ? 1u : 0u;
  ok = ok && rz_wait_all<1>(gdi, ndi, tk, dk, [&](int) { return row; }, a.abortw, 0x40000 | k << 8 | X);
  sh.red[wid][lane] = (s0 + s1) + (s2 + s3);
  if (!rz_agree(ok, sh)) return false;
  if (wid == 0) {
    double m = 0.0;
    if (live) {
      const double di = (k == 0) ? 1.0 : gdi[0][0];
      const double ssum = ((sh.red[0][lane] + sh.red[1][lane]) + sh.red[2][lane]) + sh.red[3][lane];
      const double u = sqrt(di * sqrt(ssum));    // MatrixUtils.scala:258
      const double v = (u > 0) ? 1.0 / u : 1.0;  // :259
      dn.st(row, di * v, tn);                    // :260
      m = fabs(1.0 - u);                         // :261-262
    } else {
      dn.st(row, 1.0, tn);
    }
    m = wave_max(m);
    if (lane == 0) rp.st(X, m, tn);
  }
  __syncthreads();  // (sh.red is reused by the next reduction)
  return true;
}

__device__ __forceinline__ void rz_load_tile(f64x2 (&h)[8], const double* H, int ld, int IJ) {
  const int tid = threadIdx.x, c2 = tid & 31, g = tid >> 5;
  const double* tile = H + (size_t)(IJ >> 16) * NB * ld + (size_t)(IJ & 0xffff) * NB;
#pragma unroll
  for (int q = 0; q < 8; ++q) h[q] = *reinterpret_cast<const f64x2*>(tile + (size_t)(g + 8 * q) * ld + 2 * c2);
}

}  // namespace

// work: [0] claim counter, [1] abort word -- zeroed by k_ruiz_loop_init
// trace (instrumentation, CVXG_RUIZ_TRACE): per workgroup and sweep, 4 timestamps: batch start, its d in hand,
// its tiles done, its reductions done (s_memrealtime, 100 MHz); [nwg][RUIZ_MAX][4]
__global__ __launch_bounds__(256, 1) void k_ruiz_loop(const double* __restrict__ H, int ld, int n, int nbn,
                                                      double* __restrict__ gbuf, int* __restrict__ work, int batch,
                                                      unsigned long long gen, unsigned long long* __restrict__ trace) {
  __shared__ RzShared sh;
  const int tid = threadIdx.x;
  const int ntiles = nbn * (nbn + 1) / 2;
  const size_t ldS = (size_t)nbn * NB;
  auto claim = [&](int nt) {  // thread 0: one run of `batch` tiles (row-major over the lower triangle)
    const int t0 = __hip_atomic_fetch_add(work, batch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int t = t0; t < min(ntiles, t0 + batch); ++t) {
      int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      while (I * (I + 1) / 2 > t) --I;
      const int J = t - I * (I + 1) / 2;
      sh.tile[nt++] = (I << 16) | J;
      if (I == J) sh.own[sh.nown++] = I;  // (nbn <= RZ_OWN: ruiz_loop_fits)
    }
    return nt;
  };
  if (tid == 0) {
    sh.nown = 0;
    sh.nt = claim(0);
  }
  __syncthreads();
  const int nreg = min(sh.nt, RZ_MT);
  if (nreg == 0) return;
  f64x2 h[RZ_MT][8];
#pragma unroll
  for (int t = 0; t < RZ_MT; ++t)
    if (t < nreg) rz_load_tile(h[t], H, ld, sh.tile[t]);
  // the rest of the pool (normally empty by now: every resident workgroup made its first claim while these loads
  // were in flight), streamed from H every sweep
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0 && sh.nt == batch) {
    int nt = sh.nt;
    for (;;) {
      const int m = claim(nt);
      if (m == nt) break;
      nt = m;
    }
    sh.nt = nt;
  }
  __syncthreads();
  const int nt = sh.nt, nown = sh.nown;
  RzArgs a{n, nbn, gbuf, gbuf + (RUIZ_MAX + 1) * ldS * 2, gbuf + (RUIZ_MAX + 1 + (size_t)nbn) * ldS * 2, work + 1, gen};
  auto stamp = [&](int k, int f) {
    if (trace && tid == 0) trace[((size_t)blockIdx.x * RUIZ_MAX + k) * 4 + f] = __builtin_amdgcn_s_memrealtime();
  };
  for (int k = 0; k < RUIZ_MAX; ++k) {
    stamp(k, 0);
    if (!rz_batch<RZ_MT>(h, nreg, sh.tile, k, a, sh, true, trace ? trace + ((size_t)blockIdx.x * RUIZ_MAX + k) * 4 + 1 : nullptr))
      return;
    stamp(k, 2);
    for (int b = nreg; b < nt; ++b) {  // (the claims beyond the first batch: its register tiles are 0 .. nreg-1)
      f64x2 hs[1][8];
      rz_load_tile(hs[0], H, ld, sh.tile[b]);
      if (!rz_batch<1>(hs, 1, sh.tile + b, k, a, sh, false)) return;
    }
    for (int o = 0; o < nown; ++o)
      if (!rz_reduce(sh.own[o], k, a, sh)) return;
    stamp(k, 3);
  }
}

// dbuf[0] = {1, tag(0)} over nbn NB rows; the claim counter and abort word zeroed.
__global__ void k_ruiz_loop_init(double* __restrict__ gbuf, int rows, int* __restrict__ work, unsigned long long gen) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < rows) reinterpret_cast<f64x2*>(gbuf)[i] = f64x2{1.0, rz_tag(gen, 0)};
  if (i < 2) work[i] = 0;
}

// K = the first k >= 1 with rho[k] = max_X rhop[k][X] <= 1e-6 (present for every k <= K: sweeps 0..K-1 ran), else
// RUIZ_MAX; dfin = dbuf[K] (1 beyond the blocks), ruiz_sweeps = K (-2 when the loop aborted).  One workgroup.
__global__ __launch_bounds__(256) void k_ruiz_loop_final(const double* __restrict__ gbuf, int nbn, int np,
                                                         double* __restrict__ dfin, DevCtrl* ctrl,
                                                         const int* __restrict__ work, unsigned long long gen) {
  __shared__ int sK;
  const int tid = threadIdx.x;
  const size_t ldS = (size_t)nbn * NB;
  const f64x2* rhop = reinterpret_cast<const f64x2*>(gbuf) + (RUIZ_MAX + 1 + (size_t)nbn) * ldS;
  if (tid < 64) {
    int K = RUIZ_MAX;
    for (int k = 1; k <= RUIZ_MAX; ++k) {
      double m = 0.0;
      bool present = true;
      for (int X = tid; X < nbn; X += 64) {
        const f64x2 gr = rhop[(size_t)k * nbn + X];
        present = present && rz_is(gr, rz_tag(gen, k));
        m = fmax(m, gr[0]);
      }
      m = wave_max(m);
      present = __ballot(!present) == 0;
      if (!present || !(m > 1e-6)) {
        K = k;
        break;
      }
    }
    if (tid == 0) sK = K;
  }
  __syncthreads();
  const int K = sK;
  const f64x2* dK = reinterpret_cast<const f64x2*>(gbuf) + (size_t)K * ldS;
  for (int i = tid; i < np; i += 256) dfin[i] = (i < (int)ldS) ? dK[i][0] : 1.0;
  if (tid == 0) {
    ctrl->ruiz_sweeps = work[1] ? -2 : K;
    ctrl->ruiz_abort = work[1];
  }
}

void launch_ruiz_loop(hipStream_t s, const double* H, int ld, int n, int np, double* gbuf, int* work, double* dfin,
                      DevCtrl* ctrl, int nwg, unsigned long long gen, unsigned long long* trace) {
  const int nbn = (n + NB - 1) / NB;
  const int ntiles = nbn * (nbn + 1) / 2;
  const int batch = std::max(1, std::min(RZ_MT, (ntiles + nwg - 1) / nwg));
  const int rows = nbn * NB;
  k_ruiz_loop_init<<<(rows + 255) / 256, 256, 0, s>>>(gbuf, rows, work, gen);
  k_ruiz_loop<<<nwg, 256, 0, s>>>(H, ld, n, nbn, gbuf, work, batch, gen, trace);
  k_ruiz_loop_final<<<1, 256, 0, s>>>(gbuf, nbn, np, dfin, ctrl, work, gen);
}

}  // namespace cvxg
