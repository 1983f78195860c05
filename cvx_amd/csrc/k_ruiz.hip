// k_ruiz.hip — every Ruiz sweep of MatrixUtils.scala:240-268 in ONE persistent launch, H held in registers.
//
// The multi-launch form (k_vec.hip: k_ruiz_tiles + k_ruiz_rows per sweep) streams the lower triangle of H from HBM
// once per sweep and pays two launches per sweep; the C3 loop runs 13 sweeps (~245 us per Newton step).  Here each
// workgroup claims a run of lower 64 x 64 tiles once, keeps them in VGPRs (RZ_MT tiles = 288 VGPRs per lane: 2080
// tiles over 256 workgroups at n = 4096), and every sweep is a dataflow step over per-block flags:
//   tile (I, J), sweep k:  needs d^(k) of blocks I and J (dver[X] >= k); writes the partials S_k[J][rows of I]
//                          (row sums) and S_k[I][rows of J] (column sums), then adds one contribution to cnt[I] and
//                          cnt[J]: block X has exactly nbn contributions per sweep (tiles (X, J <= X) and (I > X, X))
//   block X, sweep k:      the workgroup whose contribution completes cnt[X] (== (k+1) nbn) adds S_k[0..nbn)[rows of X]
//                          and writes d^(k+1) of block X and its share of rho[k+1], then raises dver[X] = k + 1.
// Every partial, sum and d entry is computed by the same expressions in the same order as k_ruiz_tiles /
// k_ruiz_rows, so d, rho and the sweep count are bitwise those of the multi-launch loop.
//
// Termination (sweep k runs iff rho[k] > 1e-6, rho[0] = 1): a tile of sweep k has waited for some d^(k) block, whose
// reduction needed every sweep k-1 tile of its block row and column, which needed d^(k-1) of every block: so rho[k-1]
// is complete when any sweep-k tile may start, and every workgroup reads the same value.  Sweep k therefore runs
// while rho[k-1] > 1e-6 -- one sweep ahead of the reference's test: the sweep K with rho[K] <= 1e-6 runs too, writing
// d^(K+1) into the buffer of d^(K-1) and nothing else anyone reads; k_ruiz_final then picks d^(K) (buffer K & 1).
// The S and d buffers alternate by sweep parity: a sweep-(k+2) tile of block X runs after block X's sweep-k and
// sweep-(k+1) reductions, so nothing it overwrites is still to be read.
//
// Deadlock freedom: a workgroup claims tiles (an atomic counter) until the pool is empty before it starts sweeping, so
// every tile belongs to a running workgroup whatever the residency (claims beyond RZ_MT are streamed from H each
// sweep; the host takes this path only while RZ_LIST holds every tile); reductions run inline in whichever workgroup
// completes a block, and waits only ever point at earlier sweeps.  Waits are bounded (SPIN_LIMIT_TICKS): on a timeout
// the abort word is raised, every workgroup leaves, and k_ruiz_final reports ruiz_sweeps = -2.
//
// Hand-off protocol as k_dataflow.hip: sc1 loads / stores of S and d, each storing wave drains, a workgroup barrier,
// one lane stores the flag; a consumer polls the flag, barrier, then sc1 loads.
#include <algorithm>

#include "potrf64.hpp"

namespace cvxg {

constexpr int RZ_MT = 9;        // tiles a workgroup keeps in registers
constexpr int RZ_LIST = 8192;   // tiles a workgroup can own (registers + streamed)

size_t ruiz_loop_work_ints(int nbn) { return 2 + 2 * (size_t)nbn; }
bool ruiz_loop_fits(int nbn) { return (size_t)nbn * (nbn + 1) / 2 <= (size_t)RZ_LIST; }

namespace {

__device__ __forceinline__ int rz_poll(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void rz_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct RzShared {
  int tile[RZ_LIST];             // claimed tiles, (I << 16) | J
  int nt, ok, stop, nred;
  int redX[2 * RZ_MT];
  double d[2 * RZ_MT][NB];       // d^(k) of the batch's blocks: tile t's I at 2t, J at 2t + 1
  double cred[RZ_MT][4][NB];     // column partials per wave
  double red[4][NB];
};

struct RzArgs {
  const double* H;
  int ld, n, nbn;
  double* d0;
  double* d1;
  double* S;  // two parity buffers of nbn x (nbn NB)
  DevCtrl* ctrl;
  int* cnt;
  int* dver;
  int* abortw;
};

// One sweep over a batch of nb <= MT tiles whose entries are in h (k_ruiz_tiles' per-thread layout: row g + 8 q,
// columns 2 c2, 2 c2 + 1).  False: stop (the loop is done) or abort.
template <int MT>
__device__ __forceinline__ bool rz_batch(const f64x2 (&h)[MT][8], int nb, const int* tiles, int k, const RzArgs& a, RzShared& sh) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int c2 = tid & 31, g = tid >> 5;
  const int nbn = a.nbn, ldS = nbn * NB;
  const unsigned dbytes = (unsigned)(ldS * 8);
  const Sc1Mem dc((k & 1) ? a.d1 : a.d0, dbytes), dn((k & 1) ? a.d0 : a.d1, dbytes);
  const Sc1Mem Sk(a.S + (size_t)(k & 1) * nbn * ldS, (unsigned)((size_t)nbn * ldS * 8));
  // wave 0: lane q < 2 nb polls the flag of block q & 1 ? J : I of tile q >> 1, all of them in flight together
  // (2 nb <= 2 RZ_MT < 64), until every one has reached sweep k
  if (wid == 0) {
    const bool act = lane < 2 * nb;
    const int X = act ? ((lane & 1) ? (tiles[lane >> 1] & 0xffff) : (tiles[lane >> 1] >> 16)) : 0;
    bool ok = true;
    if (k > 0) {
      const unsigned long long t0 = spin_clock();
      for (unsigned spins = 0;; ++spins) {
        const bool mine = !act || rz_poll(a.dver + X) >= k;
        if (__ballot(!mine) == 0) break;
        if ((spins & 15) == 15 && rz_poll(a.abortw)) {
          ok = false;
          break;
        }
        if (spin_expired(spins, t0)) {
          if (lane == 0) __hip_atomic_store(a.abortw, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (lane == 0) {
      sh.ok = ok;
      // rho[k-1] is complete here (header): sweep k runs while it exceeds 1e-6
      sh.stop = ok && k > 0 &&
                !(__longlong_as_double((long long)__hip_atomic_load(&a.ctrl->ruiz_rho[k - 1], __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT)) > 1e-6);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
  if (!sh.ok || sh.stop) return false;
  // d^(k) of the batch's blocks into LDS (one round trip)
  for (int e = tid; e < nb * 2 * NB; e += 256) {
    const int t = e / (2 * NB), w = (e / NB) & 1, r = e & (NB - 1);
    const int X = w ? (tiles[t] & 0xffff) : (tiles[t] >> 16);
    sh.d[2 * t + w][r] = dc.ld(X * NB + r);
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
      for (int q = 0; q < 8; ++q) {
        const double di = sh.d[2 * t][g + 8 * q];
        const f64x2 av = dj * h[t][q];
        rs[q] = av[0] * av[0] + av[1] * av[1];
        const f64x2 bv = h[t][q] * di;
        csum = __builtin_elementwise_fma(bv, bv, csum);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        double v = rs[q];
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        rs[q] = v;
      }
      if (c2 == 0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) Sk.st(J * ldS + I * NB + g + 8 * q, rs[q]);
      }
      if (I != J) {
        csum[0] += __shfl_xor(csum[0], 32, 64);
        csum[1] += __shfl_xor(csum[1], 32, 64);
        if (lane < 32) {
          sh.cred[t][wid][2 * c2] = csum[0];
          sh.cred[t][wid][2 * c2 + 1] = csum[1];
        }
      }
    }
  }
  __syncthreads();
  if (tid < NB) {
    for (int t = 0; t < nb; ++t) {
      const int I = tiles[t] >> 16, J = tiles[t] & 0xffff;
      if (I != J)
        Sk.st(I * ldS + J * NB + tid,
              ((sh.cred[t][0][tid] + sh.cred[t][1][tid]) + sh.cred[t][2][tid]) + sh.cred[t][3][tid]);
    }
  }
  rz_drain();
  __syncthreads();
  // contributions, one lane of wave 0 per (tile, block), all in flight together: the one completing a block reduces it
  if (wid == 0) {
    const int full = (k + 1) * nbn - 1;
    const int I = lane < 2 * nb ? tiles[lane >> 1] >> 16 : 0, J = lane < 2 * nb ? tiles[lane >> 1] & 0xffff : 0;
    const bool act = lane < 2 * nb && !((lane & 1) && I == J);  // (a diagonal tile contributes to its block once)
    const int X = (lane & 1) ? J : I;
    bool red = false;
    if (act) red = __hip_atomic_fetch_add(a.cnt + X, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == full;
    const unsigned long long mask = __ballot(red);
    if (red) sh.redX[__popcll(mask & ((1ull << lane) - 1))] = X;
    if (lane == 0) sh.nred = __popcll(mask);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
  const int nred = sh.nred;
  for (int r = 0; r < nred; ++r) {  // k_ruiz_rows' sums, in its order
    const int X = sh.redX[r];
    const int row = X * NB + lane;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    if (row < a.n) {
      int P = wid;
      for (; P + 12 < nbn; P += 16) {
        s0 += Sk.ld(P * ldS + row);
        s1 += Sk.ld((P + 4) * ldS + row);
        s2 += Sk.ld((P + 8) * ldS + row);
        s3 += Sk.ld((P + 12) * ldS + row);
      }
      for (; P < nbn; P += 4) s0 += Sk.ld(P * ldS + row);
    }
    sh.red[wid][lane] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (wid == 0) {
      double m = 0.0;
      if (row < a.n) {
        const double ssum = ((sh.red[0][lane] + sh.red[1][lane]) + sh.red[2][lane]) + sh.red[3][lane];
        const double di = dc.ld(row);
        const double u = sqrt(di * sqrt(ssum));  // MatrixUtils.scala:258
        const double v = (u > 0) ? 1.0 / u : 1.0;  // :259
        dn.st(row, di * v);                        // :260
        m = fabs(1.0 - u);                         // :261-262
      } else {
        dn.st(row, 1.0);
      }
      m = wave_max(m);
      if (lane == 0 && m > 0.0) atomic_max_pos(&a.ctrl->ruiz_rho[k + 1], m);
    }
    __syncthreads();
  }
  if (nred > 0) {
    rz_drain();
    __syncthreads();
    if (tid == 0)
      for (int r = 0; r < nred; ++r) __hip_atomic_store(a.dver + sh.redX[r], k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

__device__ __forceinline__ void rz_load_tile(f64x2 (&h)[8], const double* H, int ld, int IJ) {
  const int tid = threadIdx.x, c2 = tid & 31, g = tid >> 5;
  const double* tile = H + (size_t)(IJ >> 16) * NB * ld + (size_t)(IJ & 0xffff) * NB;
#pragma unroll
  for (int q = 0; q < 8; ++q) h[q] = *reinterpret_cast<const f64x2*>(tile + (size_t)(g + 8 * q) * ld + 2 * c2);
}

}  // namespace

// work: [0] claim counter, [1] abort word, [2, 2 + nbn) cnt, [2 + nbn, 2 + 2 nbn) dver -- zeroed by k_ruiz_init
__global__ __launch_bounds__(256, 1) void k_ruiz_loop(const double* __restrict__ H, int ld, int n, int nbn,
                                                      double* __restrict__ d0, double* __restrict__ d1,
                                                      double* __restrict__ S, DevCtrl* ctrl, int* __restrict__ work,
                                                      int batch) {
  __shared__ RzShared sh;
  const int tid = threadIdx.x;
  const int ntiles = nbn * (nbn + 1) / 2;
  auto claim = [&](int nt) {  // thread 0: one run of `batch` tiles (row-major over the lower triangle)
    const int t0 = __hip_atomic_fetch_add(work, batch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int t = t0; t < min(ntiles, t0 + batch); ++t) {
      int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      while (I * (I + 1) / 2 > t) --I;
      sh.tile[nt++] = (I << 16) | (t - I * (I + 1) / 2);
    }
    return nt;
  };
  if (tid == 0) sh.nt = claim(0);
  __syncthreads();
  const int nreg = min(sh.nt, RZ_MT);
  if (nreg == 0) return;
  f64x2 h[RZ_MT][8];
#pragma unroll
  for (int t = 0; t < RZ_MT; ++t)
    if (t < nreg) rz_load_tile(h[t], H, ld, sh.tile[t]);
  // the rest of the pool (normally empty by now: every resident workgroup made its first claim while these loads
  // were in flight), streamed from H every sweep
  rz_drain();
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
  const int nt = sh.nt;
  RzArgs a{H, ld, n, nbn, d0, d1, S, ctrl, work + 2, work + 2 + nbn, work + 1};
  for (int k = 0; k < RUIZ_MAX; ++k) {
    if (!rz_batch<RZ_MT>(h, nreg, sh.tile, k, a, sh)) return;
    for (int b = RZ_MT; b < nt; ++b) {
      f64x2 hs[1][8];
      rz_load_tile(hs[0], H, ld, sh.tile[b]);
      if (!rz_batch<1>(hs, 1, sh.tile + b, k, a, sh)) return;
    }
  }
}

void launch_ruiz_loop(hipStream_t s, const double* H, int ld, int n, double* d0, double* d1, double* S, DevCtrl* ctrl,
                      int* work, int nwg) {
  const int nbn = (n + NB - 1) / NB;
  const int ntiles = nbn * (nbn + 1) / 2;
  const int batch = std::max(1, std::min(RZ_MT, (ntiles + nwg - 1) / nwg));
  k_ruiz_loop<<<nwg, 256, 0, s>>>(H, ld, n, nbn, d0, d1, S, ctrl, work, batch);
}

}  // namespace cvxg
