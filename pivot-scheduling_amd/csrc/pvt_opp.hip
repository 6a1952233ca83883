// pvt_opp.hip — opportunistic policy (reference scheduler/opportunistic.py:11-20) on gfx950.
//
// Exactness argument: within a window the snapshot feasibility of a host that
// no task has committed to is unchanged, and a committed ("touched") host can only lose
// feasibility. So the current feasible count of task t is its snapshot count minus the touched
// hosts that fitted at the snapshot but no longer fit, and the k-th current feasible host is
// found by walking snapshot counts corrected by those "lost" hosts.
//
// RandomState.choice(list) == randint(0, n) (numpy legacy): no draw when n == 1; otherwise
// 32-bit MT19937 outputs masked to the next power of two minus one, rejected while > n - 1.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "pvt_device.h"
#include "pvt_kernels.h"
#include "pvt_mt.h"
#include "pvt_opp.h"

namespace pvt {

// ------------------------------------------------------------------------------------------
// Count kernel: block = 4 waves, each wave OPP_TW tasks over one host segment of seg_q chunks
// (a power of two <= OPP_SUP, so a segment lies inside one super-chunk); blockIdx % S picks the
// segment (all task tiles of a segment on one XCD's L2). For every (task, 256-host chunk) it
// stores the chunk's feasibility bitmap (the four wave ballots, 32 B) and adds the segment's
// feasible count to its super-chunk's (zeroed first), task-major: the walk's read of one
// super-chunk's 64 chunk bitmaps for one task is then 2 KiB contiguous. A chunk's host loads
// are issued one chunk ahead (register double buffer, clamped indices instead of branches).
// Segments are sized for ~2048 blocks: with whole super-chunks per segment a 64-task window
// was 124 blocks, each walking 64 chunks with its load latency exposed (136 us per window).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void opp_count_kernel(OppCountArgs A) {
  constexpr int U = OPP_CH / WAVE;
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int seg = blockIdx.x % A.S, tile = blockIdx.x / A.S;
  const int t0 = (tile * 4 + wave) * OPP_TW;
  if (t0 >= A.nt) return;
  const int nt = min(OPP_TW, A.nt - t0);
  double d0[OPP_TW], d1[OPP_TW], d2[OPP_TW], d3[OPP_TW];
#pragma unroll
  for (int k = 0; k < OPP_TW; k++) {
    if (k < nt) {
      const double* dp = A.dem + (size_t)(t0 + k) * 4;
      d0[k] = dp[0]; d1[k] = dp[1]; d2[k] = dp[2]; d3[k] = dp[3];
    } else {
      d0[k] = d1[k] = d2[k] = d3[k] = DINF;
    }
  }
  const int qlo = A.sq_lo * OPP_SUP, qhi = min(A.nq, A.sq_hi * OPP_SUP);
  const int qa = qlo + seg * A.seg_q, qb = min(qhi, qa + A.seg_q);
  double n0[U], n1[U], n2[U], n3[U];
  auto fetch = [&](int q) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int h = min(q * OPP_CH + u * WAVE + lane, A.H - 1);
      n0[u] = A.avail[h]; n1[u] = A.avail[(size_t)A.H + h];
      n2[u] = A.avail[2 * (size_t)A.H + h]; n3[u] = A.avail[3 * (size_t)A.H + h];
    }
  };
  if (qa < qb) fetch(qa);
  int sup[OPP_TW];
#pragma unroll
  for (int k = 0; k < OPP_TW; k++) sup[k] = 0;
  for (int q = qa; q < qb; q++) {
    double a0[U], a1[U], a2[U], a3[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const bool ok = q * OPP_CH + u * WAVE + lane < A.H;
      a0[u] = ok ? n0[u] : -DINF; a1[u] = n1[u]; a2[u] = n2[u]; a3[u] = n3[u];
    }
    if (q + 1 < qb) fetch(q + 1);
    uint64_t mine[U];
#pragma unroll
    for (int u = 0; u < U; u++) mine[u] = 0;
#pragma unroll
    for (int k = 0; k < OPP_TW; k++) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t b = __ballot(fits<false>(a0[u], a1[u], a2[u], a3[u], d0[k], d1[k], d2[k], d3[k]));
        sup[k] += __popcll(b);
        if (lane == k) mine[u] = b;
      }
    }
    if (lane < nt) {
      uint64_t* o = A.bm + ((size_t)(t0 + lane) * A.ldq + (q - qlo)) * U;
#pragma unroll
      for (int u = 0; u < U; u++) o[u] = mine[u];
    }
    if ((q + 1) % OPP_SUP == 0 || q + 1 == qb) {   // super-chunk (or segment) end
      const int Q = q / OPP_SUP;
      int v = 0;
#pragma unroll
      for (int k = 0; k < OPP_TW; k++) {
        if (lane == k) v = sup[k];
        sup[k] = 0;
      }
      if (lane < nt && v != 0) atomicAdd(&A.sc[(size_t)(t0 + lane) * A.lds + (Q - A.sq_lo)], v);
    }
  }
}

void launch_opp_count(const OppCountArgs& a0, hipStream_t st) {
  OppCountArgs a = a0;
  const int tiles = (a.nt + 4 * OPP_TW - 1) / (4 * OPP_TW);
  const int nqr = std::max(1, std::min(a.nq, a.sq_hi * OPP_SUP) - a.sq_lo * OPP_SUP);
  a.seg_q = OPP_SUP;
  while (a.seg_q > 1 && (long long)tiles * ((nqr + a.seg_q - 1) / a.seg_q) < 2048) a.seg_q >>= 1;
  a.S = (nqr + a.seg_q - 1) / a.seg_q;
  (void)hipMemsetAsync(a.sc, 0, sizeof(int32_t) * (size_t)a.nt * a.lds, st);
  PVT_LAUNCH(opp_count_kernel, dim3(tiles * a.S), dim3(256), 0, st, a);
}

// ------------------------------------------------------------------------------------------
// Commit walk: speculative ranges (one workgroup of OPP_NW waves).
//
// The walk takes a window's tasks in ranges of up to OPP_R. For a range starting at task s,
// every task's draw and candidates are computed up front, in parallel, on the state at s:
//   n_j  snapshot count minus the touched hosts that stopped fitting ("lost" at s),
//   k_j  randint(0, n_j), drawn in task order from the live MT19937 state,
//   c_j  the OPP_C hosts feasible at s from position k_j on, in host order, inside k_j's
//        super-chunk, with their availability loaded from HBM.
// One wave then walks the range in order without a memory round trip. A commit of host h by
// task i can only take h out of a later task's feasible set ("new lost"); every lane (= a later
// task of the range) records that from h's capacities before and after the commit. Task i:
//   * n_true = n_i - (new lost of i). randint draws masked outputs until one is <= n - 1, so
//     with the same mask and k_i <= n_true - 1 the true draw consumed the same outputs and
//     returned k_i (every output rejected for n_i is rejected for n_true < n_i);
//   * the k-th feasible host: m = new lost hosts below c_i[0] shift it to the m-th candidate
//     that still fits (a candidate touched in this walk reads its capacity from the LDS hash).
// A task whose draw changed or whose candidates ran out starts a new range (the MT19937 state
// saved at the range start is restored and the range's consumed outputs replayed). A range's
// first task always verifies, so every range makes progress. Measured (config 5):
// the single-wave walk it replaces spent ~8000 cycles per task, most of it on two dependent HBM
// loads (the drawn super-chunk's bitmaps, then the chosen host) and a rescan of every touched
// host per task.
// ------------------------------------------------------------------------------------------
constexpr int OPP_R = 64;               // tasks per speculation range (one walker lane each)
constexpr int OPP_C = 16;               // candidates per task (4 lanes each load one)
constexpr int OPP_NW = 16;              // waves of the walk workgroup (4 range tasks each in
                                        // the parallel passes; measured: 12.3 ms -> 11.4 ms at
                                        // config 5 against 8 waves, EXPERIMENTS.md)
constexpr int OPP_TB = OPP_R / OPP_NW;  // range tasks per wave in the parallel passes
constexpr int OPP_MAXT = 2 * OPP_MAXW;  // touched hosts: inherited + own
constexpr int OPP_HASH_BITS = 11;
constexpr int OPP_HASH = 1 << OPP_HASH_BITS;
static_assert(OPP_C * 4 == WAVE, "one lane per (candidate, resource)");
static_assert(OPP_HASH >= 4 * OPP_MAXT, "touched-host hash load factor");

struct OppLDS {
  int32_t hkey[OPP_HASH];
  int32_t hval[OPP_HASH];
  int32_t tid[OPP_MAXT];
  int32_t own[OPP_MAXT];        // touched by this walk
  double sa[4][OPP_MAXT];       // touched hosts in the count pass's view
  double ta[4][OPP_MAXT];       // current
  double sb[4][OPP_MAXT];       // when this walk started (pipelined hand-off)
  double cav[OPP_R][4][OPP_C];  // candidates' availability at the walk's start (HBM)
  int32_t cand[OPP_R][OPP_C];
  int32_t nspec[OPP_R];
  uint32_t kdraw[OPP_R];
  int32_t cnt[OPP_R];           // MT19937 outputs the draw consumed
  int32_t ccount[OPP_R];
  int32_t dl[OPP_R];            // pass 2: the range's draw tasks (n >= 2), in order
  uint32_t mt[625];
  uint32_t mtb[625];            // state at the range start
  int32_t pl[OPP_MAXW];         // placements of the window, written out when the walk ends
  int32_t lhist[OPP_NW][WAVE];  // per wave: a task's lost hosts per super-chunk (pass 3)
  // wl and lclr overlap ACROSS waves (with OPP_NW = 16, wave w's lclr covers the wl rows of
  // waves 2w and 2w + 1), not only within a wave. That is safe only because of the block
  // barriers between pass 1 (every wave reads its wl rows into registers) and pass 3 (lclr
  // written), and at the end of each range (before the next pass 1 writes wl): an edit that
  // removes or moves one of those __syncthreads lets one wave clobber another's lost-host list.
  union {
    int32_t wl[OPP_NW][OPP_TB][WAVE];                // per wave and task: its lost hosts (pass 1)
    uint64_t lclr[OPP_NW][OPP_SUP][OPP_CH / WAVE];   // per wave: lost bits of the drawn super-chunk
  };
  int32_t ctl[4];               // next range start, touched count
};

static_assert(sizeof(OppLDS) <= 160 * 1024, "opportunistic walk LDS exceeds a CU's 160 KiB");

__device__ __forceinline__ uint32_t ohslot(int32_t id) {
  return ((uint32_t)id * 2654435761u) >> (32 - OPP_HASH_BITS);
}
__device__ __forceinline__ int ohash_find(const OppLDS& S, int32_t id) {
  uint32_t p = ohslot(id);
  for (;;) {
    const int32_t k = S.hkey[p];
    if (k == id) return S.hval[p];
    if (k < 0) return -1;
    p = (p + 1) & (OPP_HASH - 1);
  }
}
__device__ __forceinline__ void ohash_put(OppLDS& S, int32_t id, int32_t v) {
  uint32_t p = ohslot(id);
  while (S.hkey[p] >= 0) p = (p + 1) & (OPP_HASH - 1);
  S.hkey[p] = id;
  S.hval[p] = v;
}

// A wave-uniform double (an LDS broadcast) as a scalar.
__device__ __forceinline__ double rfl_d(double v) {
  union { double d; uint64_t u; } x;
  x.d = v;
  x.u = rfl_u64(x.u);
  return x.d;
}

// Position of the r-th (0-based) set bit of x (r < popcount(x)).
__device__ __forceinline__ int select_bit(uint64_t x, int r) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w > 0; w >>= 1) {
    const uint64_t lo = x & ((w == 64 ? ~0ull : (1ull << w)) - 1);
    const int c = __popcll(lo);
    if (r >= c) { r -= c; x >>= w; pos += w; }
    else x = lo;
  }
  return pos;
}

// numpy legacy randint's mask for range rng: the next power of two minus one.
__device__ __forceinline__ uint32_t rint_mask(uint32_t rng) {
  rng |= rng >> 1; rng |= rng >> 2; rng |= rng >> 4; rng |= rng >> 8; rng |= rng >> 16;
  return rng;
}
// mt_randint that also counts the outputs it consumed. The rejection loop runs over the wave's
// 64 buffered outputs at once: the first buffered output (from w.used on) whose masked value
// is <= rng is the draw (a ballot), so a draw costs one ballot per buffer instead of one
// readlane per output.
__device__ inline uint32_t mt_randint_cnt(uint32_t* key, MtWave& w, uint32_t n, int& used) {
  const uint32_t rng = n - 1;
  if (rng == 0) return 0;
  const uint32_t mask = rint_mask(rng);
  const int lane = lane_id();
  for (;;) {
    if (w.used >= w.limit) mt_refill(key, w);
    const uint64_t ok = __ballot(lane >= w.used && lane < w.limit && (w.buf & mask) <= rng);
    if (ok) {
      const int j = __builtin_ctzll(ok);
      used += j + 1 - w.used;
      w.used = j + 1;
      return (uint32_t)__builtin_amdgcn_readlane((int)w.buf, j) & mask;
    }
    used += w.limit - w.used;
    w.used = w.limit;
  }
}

// The touched hosts [q0, q0 + 64) lost for demand d -- they fitted in the count pass's view and
// no longer fit -- as a ballot over lanes; th = lane's host id.
__device__ __forceinline__ uint64_t lost_piece(const OppLDS& S, int m, int q0, double d0, double d1,
                                               double d2, double d3, int32_t& th) {
  const int q = q0 + lane_id(), qq = min(q, m - 1);
  const bool lf = q < m &&
                  fits<false>(S.sa[0][qq], S.sa[1][qq], S.sa[2][qq], S.sa[3][qq], d0, d1, d2, d3) &&
                  !fits<false>(S.ta[0][qq], S.ta[1][qq], S.ta[2][qq], S.ta[3][qq], d0, d1, d2, d3);
  th = S.tid[qq];
  return __ballot(lf);
}
__device__ __forceinline__ int count_lost(const OppLDS& S, int m, double d0, double d1, double d2,
                                          double d3) {
  int n = 0;
  for (int q0 = 0; q0 < m; q0 += WAVE) {
    int32_t th;
    n += __popcll(lost_piece(S, m, q0, d0, d1, d2, d3, th));
  }
  return n;
}

#ifdef PVT_STAMPS
__device__ __forceinline__ uint64_t ostamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define OSTAMP(k)                         \
  do {                                    \
    const uint64_t t_ = ostamp();         \
    ph[k] += t_ - tl;                     \
    tl = t_;                              \
  } while (0)
#else
#define OSTAMP(k) do {} while (0)
#endif

// One wave orders its own LDS operations: a compiler fence plus lgkmcnt(0). (__syncthreads
// would also wait vmcnt(0).)
__device__ __forceinline__ void wave_lds_fence() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__global__ __launch_bounds__(OPP_NW * WAVE) void opp_commit_kernel(OppCommitArgs A) {
  constexpr int U = OPP_CH / WAVE;
  constexpr int SUPH = OPP_SUP * OPP_CH;
  constexpr int NT = OPP_NW * WAVE;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  OppLDS& S = *reinterpret_cast<OppLDS*>(smem);
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tx = threadIdx.x;
  for (int i = tx; i < OPP_HASH; i += NT) S.hkey[i] = -1;
  for (int i = tx; i < A.nt; i += NT) S.pl[i] = -1;
  for (int i = tx; i < 625; i += NT) S.mt[i] = A.mt[i];
  __syncthreads();
  // the previous walk's commits (already in global availability, launch_opp_apply): touched,
  // with the count pass's snapshot as sa
  const int m0 = A.in ? A.in->n : 0;
  for (int q = tx; q < m0; q += NT) {
    const int32_t h = A.in->tid[q];
    for (int r = 0; r < 4; r++) {
      const double t = A.in->ta[r][q];
      S.sa[r][q] = A.in->sb[r][q];
      S.ta[r][q] = t;
      S.sb[r][q] = t;
    }
    S.tid[q] = h;
    S.own[q] = 0;
    uint32_t p = ohslot(h);
    while (atomicCAS(&S.hkey[p], -1, h) != -1) p = (p + 1) & (OPP_HASH - 1);
    S.hval[p] = q;
  }
  if (tx == 0) { S.ctl[0] = 0; S.ctl[1] = m0; }
  __syncthreads();
  const bool fast = A.nsq <= WAVE;   // one super-chunk count per lane (H <= 1,048,576)
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#ifdef PVT_STAMPS
  uint64_t ph[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tl = ostamp();
#endif

  int s = 0;
  while (s < A.nt) {
    const int e = min(A.nt, s + OPP_R);
    const int m = __builtin_amdgcn_readfirstlane(S.ctl[1]);
    // ---- pass 1 (all waves): n_j = snapshot count - lost, for the range's tasks; each task's
    // lost hosts stay in a register (lane l = the l-th; nlost > 64: rescanned in pass 3)
    // Lanes = touched hosts: a 64-host piece of the table is read from LDS once and tested
    // against the wave's OPP_TB tasks (demands broadcast from registers).
    double dv[OPP_TB];
    int scr[OPP_TB], lh[OPP_TB], nlost[OPP_TB];
#pragma unroll
    for (int t = 0; t < OPP_TB; t++) {
      const int j = s + wave * OPP_TB + t;
      const bool ok = j < e;
      dv[t] = ok ? A.dem[(size_t)j * 4 + (lane & 3)] : 0.0;
      scr[t] = (ok && fast && lane < A.nsq) ? A.sc[(size_t)j * A.nsq + lane] : 0;
      nlost[t] = 0;
    }
    const int ntw = max(0, min(OPP_TB, e - (s + wave * OPP_TB)));   // this wave's tasks
    for (int q0 = 0; q0 < m; q0 += WAVE) {
      const int q = q0 + lane, qq = min(q, m - 1);
      const double a0 = S.sa[0][qq], a1 = S.sa[1][qq], a2 = S.sa[2][qq], a3 = S.sa[3][qq];
      const double b0 = S.ta[0][qq], b1 = S.ta[1][qq], b2 = S.ta[2][qq], b3 = S.ta[3][qq];
      const int32_t th = S.tid[qq];
      const uint64_t vm = __ballot(q < m);
#pragma unroll
      for (int t = 0; t < OPP_TB; t++) {
        if (t >= ntw) break;
        const double d0 = readlane_d(dv[t], 0), d1 = readlane_d(dv[t], 1);
        const double d2 = readlane_d(dv[t], 2), d3 = readlane_d(dv[t], 3);
        // fitted in the count pass's view (sa), no longer fits (ta); fits<false> per lane =
        // the AND of the per-dimension ballots
        const uint64_t b = vm & __ballot(a0 >= d0) & __ballot(a1 >= d1) & __ballot(a2 >= d2) &
                           __ballot(a3 >= d3) &
                           ~(__ballot(b0 >= d0) & __ballot(b1 >= d1) & __ballot(b2 >= d2) &
                             __ballot(b3 >= d3));
        const int pos = nlost[t] + __popcll(b & below);
        if (((b >> lane) & 1) && pos < WAVE) S.wl[wave][t][pos] = th;
        nlost[t] += __popcll(b);
      }
    }
    wave_lds_fence();
#pragma unroll
    for (int t = 0; t < OPP_TB; t++) {
      const int j = s + wave * OPP_TB + t;
      lh[t] = -1;
      if (j < e) {
        long long tot = 0;
        if (fast) {
          tot = __builtin_amdgcn_readlane(wave_incl_scan_dpp(scr[t]), 63);
        } else {
          for (int Q0 = 0; Q0 < A.nsq; Q0 += WAVE) {
            const int Q = Q0 + lane;
            tot += wave_sum_ll(Q < A.nsq ? (long long)A.sc[(size_t)j * A.nsq + Q] : 0);
          }
        }
        lh[t] = lane < nlost[t] ? S.wl[wave][t][lane] : -1;
        if (lane == 0) S.nspec[j - s] = (int)(tot - nlost[t]);
      }
    }
    __syncthreads();
    OSTAMP(0);
    // ---- pass 2 (wave 0): the draws, in task order, from the live state (saved first). Most
    // draws accept their first output (n is close to the mask's power of two), so each pending
    // draw is first tried against one buffered output (lane q: the (q - used)-th pending draw);
    // the accepted prefix commits at once and the first rejected draw runs the rejection loop.
    // Draws for n = 1 consume nothing (randint's range 0), as in mt_randint_cnt.
    if (wave == 0) {
      for (int i = lane; i < 625; i += WAVE) S.mtb[i] = S.mt[i];
      const int R = e - s;
      const int nsv = lane < R ? S.nspec[lane] : 0;
      if (lane < R) { S.kdraw[lane] = nsv == 1 ? 0u : 0xffffffffu; S.cnt[lane] = 0; }
      const uint64_t dm = __ballot(lane < R && nsv >= 2);
      if ((dm >> lane) & 1ull) S.dl[__popcll(dm & below)] = lane;
      wave_lds_fence();
      const int nd = __popcll(dm);
      MtWave mw;
      mw.buf = 0; mw.used = 0; mw.limit = 0;
      int d = 0;
      while (d < nd) {
        if (mw.used >= mw.limit) mt_refill(S.mt, mw);
        const int r = d + lane - mw.used;
        const bool in = lane >= mw.used && lane < mw.limit && r < nd;
        const int t = in ? S.dl[r] : 0;
        const uint32_t rg = (uint32_t)(S.nspec[t] - 1), mk = rint_mask(rg);
        const uint32_t kq = mw.buf & mk;
        const uint64_t inm = __ballot(in), bad = __ballot(in && kq > rg);
        const uint64_t acc = bad ? (inm & ((1ull << __builtin_ctzll(bad)) - 1ull)) : inm;
        if ((acc >> lane) & 1ull) { S.kdraw[t] = kq; S.cnt[t] = 1; }
        const int na = __popcll(acc);
        d += na;
        mw.used += na;
        if (bad) {   // draw d rejects its first output: the rejection loop from that output
          const int tb = __builtin_amdgcn_readfirstlane(S.dl[d]);
          int used = 0;
          const uint32_t k = mt_randint_cnt(S.mt, mw, (uint32_t)__builtin_amdgcn_readfirstlane(S.nspec[tb]), used);
          if (lane == 0) { S.kdraw[tb] = k; S.cnt[tb] = used; }
          d++;
        }
      }
      mt_unbuffer(S.mt, mw);
    }
    __syncthreads();
    OSTAMP(1);
    // ---- pass 3 (all waves): super-chunk of k_j, its bitmaps, the OPP_C candidates from k_j on
    int qsel[OPP_TB], ksel[OPP_TB];
    uint64_t bits[OPP_TB][U];
#pragma unroll
    for (int t = 0; t < OPP_TB; t++) {
      const int j = s + wave * OPP_TB + t;
      qsel[t] = -1; ksel[t] = 0;
#pragma unroll
      for (int u = 0; u < U; u++) bits[t][u] = 0;
      if (j >= e) continue;
      const int n = __builtin_amdgcn_readfirstlane(S.nspec[j - s]);
      if (n <= 0) continue;
      const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.kdraw[j - s]);
      int Qs = -1;
      long long acc = 0;
      if (fast) {
        // one super-chunk per lane: its snapshot count minus the task's lost hosts in it, the
        // lost hosts counted by an LDS histogram (one atomic per lost host, not a readlane loop)
        const bool none = nlost[t] == 0;   // (common: no lost host, the snapshot counts hold)
        if (!none) {
          S.lhist[wave][lane] = 0;
          wave_lds_fence();
        }
        if (none) {
        } else if (nlost[t] <= WAVE) {
          if (lane < nlost[t]) atomicAdd(&S.lhist[wave][lh[t] / SUPH], 1);
        } else {   // (rare) rescan, with the demand reloaded
          const double dv = A.dem[(size_t)j * 4 + (lane & 3)];
          const double f0 = readlane_d(dv, 0), f1 = readlane_d(dv, 1);
          const double f2 = readlane_d(dv, 2), f3 = readlane_d(dv, 3);
          for (int p0 = 0; p0 < m; p0 += WAVE) {
            int32_t th;
            const uint64_t b = lost_piece(S, m, p0, f0, f1, f2, f3, th);
            if ((b >> lane) & 1ull) atomicAdd(&S.lhist[wave][th / SUPH], 1);
          }
        }
        wave_lds_fence();
        const int v = lane < A.nsq ? scr[t] - (none ? 0 : S.lhist[wave][lane]) : 0;
        const int inc = wave_incl_scan_dpp(v);
        const int tot = __builtin_amdgcn_readlane(inc, 63);
        if ((long long)k < tot) {
          const uint64_t hit = __ballot(inc > (long long)k);
          const int L = __builtin_ctzll(hit);
          Qs = L;
          acc = __builtin_amdgcn_readlane(inc, L) - __builtin_amdgcn_readlane(v, L);
        }
      }
      for (int Q0 = 0; !fast && Q0 < A.nsq && Qs < 0; Q0 += WAVE) {
        const int Q = Q0 + lane;
        int v = 0;
        if (Q < A.nsq) v = fast ? scr[t] : A.sc[(size_t)j * A.nsq + Q];
        if (nlost[t] <= WAVE) {   // minus the lost hosts in super-chunk Q
          for (int l = 0; l < nlost[t]; l++) v -= (__builtin_amdgcn_readlane(lh[t], l) / SUPH == Q);
        } else {   // (rare) rescan, with the demand reloaded
          const double dv = A.dem[(size_t)j * 4 + (lane & 3)];
          const double f0 = readlane_d(dv, 0), f1 = readlane_d(dv, 1);
          const double f2 = readlane_d(dv, 2), f3 = readlane_d(dv, 3);
          for (int p0 = 0; p0 < m; p0 += WAVE) {
            int32_t th;
            uint64_t b = lost_piece(S, m, p0, f0, f1, f2, f3, th);
            while (b) {
              const int l = __builtin_ctzll(b);
              b &= b - 1;
              v -= (__builtin_amdgcn_readlane(th, l) / SUPH == Q);
            }
          }
        }
        const int inc = wave_incl_scan_dpp(v);
        const int tot = __builtin_amdgcn_readlane(inc, 63);
        if ((long long)k < acc + tot) {
          const uint64_t hit = __ballot(acc + inc > (long long)k);
          const int L = __builtin_ctzll(hit);
          Qs = Q0 + L;
          acc += __builtin_amdgcn_readlane(inc, L) - __builtin_amdgcn_readlane(v, L);
        } else {
          acc += tot;
        }
      }
      if (Qs < 0) continue;   // unreachable when counts are consistent (no candidates)
      qsel[t] = Qs;
      ksel[t] = (int)(k - (uint32_t)acc);
      const int q = Qs * OPP_SUP + lane;   // lane = chunk of the super-chunk
      if (q < A.nq) {
        const uint64_t* bp = A.bm + ((size_t)j * A.nq + q) * U;
#pragma unroll
        for (int u = 0; u < U; u++) bits[t][u] = bp[u];
      }
    }
    OSTAMP(5);
#pragma unroll
    for (int t = 0; t < OPP_TB; t++) {
      const int j = s + wave * OPP_TB + t;
      if (j >= e) continue;
      int cc = 0;
      const int Qs = qsel[t];
      if (Qs >= 0) {
        // current bitmaps: the snapshot's minus the lost hosts of this super-chunk (lane = its
        // chunk), collected by LDS atomics -- one per lost host -- instead of a readlane loop
        // (common: none of the task's lost hosts lies in this super-chunk -- the bitmaps hold)
        const bool clear = nlost[t] > WAVE || __ballot(lane < nlost[t] && lh[t] / SUPH == Qs) != 0;
        if (clear) {
#pragma unroll
          for (int u = 0; u < U; u++) S.lclr[wave][lane][u] = 0;
          wave_lds_fence();
          auto mark = [&](int h, bool on) {
            if (on && h / SUPH == Qs) {
              const int o = h % OPP_CH;
              atomicOr((unsigned long long*)&S.lclr[wave][(h / OPP_CH) % OPP_SUP][o / WAVE],
                       1ull << (o % WAVE));
            }
          };
          if (nlost[t] <= WAVE) {
            mark(lh[t], lane < nlost[t]);
          } else {
            const double dv = A.dem[(size_t)j * 4 + (lane & 3)];
            const double f0 = readlane_d(dv, 0), f1 = readlane_d(dv, 1);
            const double f2 = readlane_d(dv, 2), f3 = readlane_d(dv, 3);
            for (int p0 = 0; p0 < m; p0 += WAVE) {
              int32_t th;
              const uint64_t b = lost_piece(S, m, p0, f0, f1, f2, f3, th);
              mark(th, (b >> lane) & 1ull);
            }
          }
          wave_lds_fence();
#pragma unroll
          for (int u = 0; u < U; u++) bits[t][u] &= ~S.lclr[wave][lane][u];
        }
        int c = 0;
#pragma unroll
        for (int u = 0; u < U; u++) c += __popcll(bits[t][u]);
        const int inc = wave_incl_scan_dpp(c);
        int k1 = ksel[t];
        const uint64_t hit = __ballot(inc > k1);
        if (hit) {
          const int L = __builtin_ctzll(hit);
          k1 -= __builtin_amdgcn_readlane(inc, L) - __builtin_amdgcn_readlane(c, L);
          int off = -1;
          if (lane == L) {
            int r = k1;
#pragma unroll
            for (int u = 0; u < U; u++) {
              const int cu = __popcll(bits[t][u]);
              if (off < 0) {
                if (r < cu) off = u * WAVE + select_bit(bits[t][u], r);
                else r -= cu;
              }
            }
          }
          off = __builtin_amdgcn_readlane(off, L);
          // hosts from (chunk L, bit off) on, in host order: the first OPP_C are the candidates
          uint64_t kb[U];
          int c2 = 0;
#pragma unroll
          for (int u = 0; u < U; u++) {
            const int lo = u * WAVE;
            uint64_t keep;
            if (lane < L) keep = 0;
            else if (lane > L) keep = ~0ull;
            else keep = off >= lo + WAVE ? 0ull : (off <= lo ? ~0ull : (~0ull << (off - lo)));
            kb[u] = bits[t][u] & keep;
            c2 += __popcll(kb[u]);
          }
          const int inc2 = wave_incl_scan_dpp(c2);
          cc = min(OPP_C, __builtin_amdgcn_readlane(inc2, 63));
          int slot = inc2 - c2;
          if (slot < OPP_C) {
            const int base = (Qs * OPP_SUP + lane) * OPP_CH;
#pragma unroll
            for (int u = 0; u < U; u++) {
              uint64_t x = kb[u];
              while (x && slot < OPP_C) {
                const int b = __builtin_ctzll(x);
                x &= x - 1;
                S.cand[j - s][slot++] = base + u * WAVE + b;
              }
            }
          }
        }
      }
      if (lane == 0) S.ccount[j - s] = cc;
    }
    wave_lds_fence();
    OSTAMP(6);
    // candidates' capacity at the range start: lane = (candidate lane / 4, resource lane % 4);
    // touched hosts from the table, the others from HBM (the walk has not written them)
    double cv[OPP_TB];
    const int cx = lane >> 2, cr = lane & 3;
#pragma unroll
    for (int t = 0; t < OPP_TB; t++) {
      const int j = s + wave * OPP_TB + t;
      cv[t] = 0.0;
      if (j < e && cx < S.ccount[j - s]) cv[t] = A.avail[(size_t)cr * A.H + S.cand[j - s][cx]];
    }
#pragma unroll
    for (int t = 0; t < OPP_TB; t++) {
      const int j = s + wave * OPP_TB + t;
      if (j < e && cx < S.ccount[j - s]) {
        const int ws = ohash_find(S, S.cand[j - s][cx]);
        S.cav[j - s][cr][cx] = ws >= 0 ? S.ta[cr][ws] : cv[t];
      }
    }
    __syncthreads();
    OSTAMP(2);
    // ---- pass 4 (wave 0): walk the range. Lane l holds range task s + l: its demand, draw,
    // candidates (S.cav keeps their capacities current through the range's commits), the
    // candidates that stopped fitting (lm), the lost hosts below c_0 (mm) and its new-lost count
    // (nnew). Task i's draw holds while dok (same mask, k <= n - 1 for n - nnew), and its host is
    // then the mm-th candidate that still fits (the k-th feasible host, shifted by the lost hosts
    // below c_0) -- unless fewer candidates fit, when the range stops there. Every lane keeps that
    // choice (host, capacity now, capacity after) in registers, recomputed in parallel when a
    // commit takes a host from it (below its candidates) or changes a candidate's capacity, so
    // the walk itself is nine v_readlane of the committing lane's row, the fit tests of the
    // later tasks and two ballots per task (the LDS row it replaced cost ~740 cycles a commit:
    // its load latency sat on the chain). Nothing is written to the touched table until the
    // range ends.
    if (wave == 0) {
      const int R = e - s;
      const bool mine = lane < R;
      double e0 = 0.0, e1 = 0.0, e2 = 0.0, e3 = 0.0;
      int nsv = 0, ccv = 0;
      uint32_t kv = 0;
      if (mine) {
        const double* dp = A.dem + (size_t)(s + lane) * 4;
        e0 = dp[0]; e1 = dp[1]; e2 = dp[2]; e3 = dp[3];
        nsv = S.nspec[lane];
        kv = S.kdraw[lane];
        ccv = nsv > 0 ? S.ccount[lane] : 0;
      }
      // the candidates stay in S.cand (read there on the rare paths: registers kept for the walk)
      const int c0l = ccv > 0 ? S.cand[lane][0] : 0x7fffffff;
      const int cmax = ccv > 0 ? S.cand[lane][ccv - 1] : -1;   // the largest (candidates ascend)
      int nnew = 0, mm = 0;
      bool dok = true;
      uint32_t lm = 0;
      // the lane's choice: the mm-th candidate still fitting, into its registers; false if none
      // the lane's choice (host, capacity now, capacity after it) in registers: the walk reads a
      // task's row by v_readlane (no LDS round trip, no fence after a re-choice)
      int qw = 0;
      double q0 = 0.0, q1 = 0.0, q2 = 0.0, q3 = 0.0, r0 = 0.0, r1 = 0.0, r2 = 0.0, r3 = 0.0;
      auto choose = [&]() -> bool {
        const uint32_t valid = ((1u << ccv) - 1u) & ~lm;
        if (!mine || !dok || __popc(valid) <= mm) return false;
        const int xs = select_bit(valid, mm);
        const double z0 = S.cav[lane][0][xs], z1 = S.cav[lane][1][xs];
        const double z2 = S.cav[lane][2][xs], z3 = S.cav[lane][3][xs];
        qw = S.cand[lane][xs];
        q0 = z0; q1 = z1; q2 = z2; q3 = z3;
        r0 = z0 - e0; r1 = z1 - e1; r2 = z2 - e2; r3 = z3 - e3;
        return true;
      };
      // Uniform masks over the range's lanes:
      //   posm  tasks with a feasible host at s (the others place nothing and change nothing);
      //   okm   tasks whose choice holds now;  done  tasks committed.
      const uint64_t minem = __ballot(mine);
      const uint64_t posm = __ballot(mine && nsv > 0);
      uint64_t okm = __ballot(choose());
      uint64_t cmt = 0;
      int stop = e;
      OSTAMP(9);
      int L = posm ? __builtin_ctzll(posm) : R;
      while (L < R) {   // (tasks without a feasible host at s place nothing and change nothing)
        if (!((okm >> L) & 1ull)) {   // the draw changed, or the answer lies beyond the
          stop = s + L;               // candidates: the range stops here
          break;
        }
        // task L's row from lane L's registers (uniform values in SGPRs)
        const int cw = __builtin_amdgcn_readlane(qw, L);
        const double c0 = readlane_d(q0, L), c1 = readlane_d(q1, L), c2 = readlane_d(q2, L),
                     c3 = readlane_d(q3, L);
        const double m0 = readlane_d(r0, L), m1 = readlane_d(r1, L), m2 = readlane_d(r2, L),
                     m3 = readlane_d(r3, L);
        const uint64_t nx = posm & ~((2ull << L) - 1ull);
        const int Ln = nx ? __builtin_ctzll(nx) : R;
        cmt |= 1ull << L;
        // the later tasks of the range: does this commit take cw away from them (lostm: fitted
        // before, not after -- fits<false> per lane is the AND of the per-dimension ballots),
        // or is cw inside their candidates' id range (rngm; rare: a commit's host is random
        // among ~1M)? (Two commits per iteration, the second's effect computed beside the
        // first's, measured slower: 817 against 692 cycles per commit.)
        const uint64_t am = minem & ~((2ull << L) - 1ull);
        const uint64_t fw = __ballot(c0 >= e0) & __ballot(c1 >= e1) & __ballot(c2 >= e2) & __ballot(c3 >= e3);
        const uint64_t fn = __ballot(m0 >= e0) & __ballot(m1 >= e1) & __ballot(m2 >= e2) & __ballot(m3 >= e3);
        const uint64_t lostm = am & fw & ~fn;
        const uint64_t rngm = am & __ballot(cw >= c0l) & __ballot(cw <= cmax);
#ifdef PVT_STAMPS
        ph[13] += 1;
        ph[11] += lostm ? 1 : 0;
        ph[12] += rngm ? 1 : 0;
#endif
        if (lostm | rngm) {
          const bool lost = (lostm >> lane) & 1ull;
          if ((rngm >> lane) & 1ull) {   // cw's capacity is now m; a lost cw stops fitting
            for (int x = 0; x < ccv; x++) {
              if (S.cand[lane][x] == cw) {
                S.cav[lane][0][x] = m0; S.cav[lane][1][x] = m1;
                S.cav[lane][2][x] = m2; S.cav[lane][3][x] = m3;
                if (lost) lm |= 1u << x;
              }
            }
          }
          if (lost) {
            nnew += 1;
            mm += cw < c0l;
            const int ntrue = nsv - nnew;
            dok = dok & (ntrue > 0) & (rint_mask((uint32_t)(ntrue - 1)) == rint_mask((uint32_t)(nsv - 1))) &
                  (kv <= (uint32_t)(ntrue - 1));
          }
          // The choice moves only for a lane whose candidates changed (rngm) or whose lost host
          // lay below its candidates (mm grew); a lost host above them leaves it in place, and a
          // draw that no longer holds only clears the lane's ok bit.
          const bool redo = (((rngm >> lane) & 1ull) != 0) | (lost & (cw < c0l));
          bool ok = ((okm >> lane) & 1ull) & dok;
          if (redo) ok = choose();
          okm = __ballot(ok);
        }
        L = Ln;
      }
      OSTAMP(8);
      // the range's commits: lane l's row still holds its choice (later commits only rewrite
      // the rows of the tasks after them)
      int rch = -1;
      double ra0 = 0.0, ra1 = 0.0, ra2 = 0.0, ra3 = 0.0, rb0 = 0.0, rb1 = 0.0, rb2 = 0.0, rb3 = 0.0;
      if ((cmt >> lane) & 1ull) {
        rch = qw;
        rb0 = q0; rb1 = q1; rb2 = q2; rb3 = q3;
        ra0 = r0; ra1 = r1; ra2 = r2; ra3 = r3;
      }
      // A range whose first task fails cannot happen when the counts are consistent (its state
      // is exact). If it does (inconsistent counts or bitmaps), report it -- the host returns
      // PVT_EHIP -- and leave that task unplaced rather than loop.
      if (stop == s) {
        if (lane == 0 && A.fault) atomicCAS(A.fault, 0, s + 1);
        stop = s + 1;
      }
      // the range's commits: placements, then the touched table (first commit of a host
      // creates or keeps its entry with the capacity before it; its last commit sets ta)
      const int done = stop - s;
      if (lane >= done) rch = -1;
      if (rch >= 0) S.pl[s + lane] = rch;
      bool first = rch >= 0, last = rch >= 0;
      for (int l = 0; l < done; l++) {
        const int h = __builtin_amdgcn_readlane(rch, l);
        if (h >= 0 && h == rch) {
          first = first && !(l < lane);
          last = last && !(l > lane);
        }
      }
      int ws = first ? ohash_find(S, rch) : -1;
      const bool fresh = first && ws < 0;
      const uint64_t fb = __ballot(fresh);
      if (fresh) {
        ws = m + __popcll(fb & below);
        S.tid[ws] = rch;
        S.sa[0][ws] = rb0; S.sa[1][ws] = rb1; S.sa[2][ws] = rb2; S.sa[3][ws] = rb3;
        S.sb[0][ws] = rb0; S.sb[1][ws] = rb1; S.sb[2][ws] = rb2; S.sb[3][ws] = rb3;
        uint32_t p = ohslot(rch);
        while (atomicCAS(&S.hkey[p], -1, rch) != -1) p = (p + 1) & (OPP_HASH - 1);
        S.hval[p] = ws;
      }
      wave_lds_fence();
      if (last) {
        const int wl = ohash_find(S, rch);
        S.ta[0][wl] = ra0; S.ta[1][wl] = ra1; S.ta[2][wl] = ra2; S.ta[3][wl] = ra3;
        S.own[wl] = 1;
      }
      if (lane == 0) { S.ctl[0] = stop; S.ctl[1] = m + __popcll(fb); }
      if (stop < e) {   // next range at stop: the MT19937 state after the draws of [s, stop)
        wave_lds_fence();
        int skip = 0;
        for (int i = s; i < stop; i++) skip += __builtin_amdgcn_readfirstlane(S.cnt[i - s]);
        for (int i = lane; i < 625; i += WAVE) S.mt[i] = S.mtb[i];
        wave_lds_fence();
        MtWave mw;
        mw.buf = 0; mw.used = 0; mw.limit = 0;
        for (int q = 0; q < skip; q++) (void)mt_next(S.mt, mw);
        mt_unbuffer(S.mt, mw);
      }
    }
    __syncthreads();
    OSTAMP(3);
#ifdef PVT_STAMPS
    ph[4] += 1;
#endif
    s = S.ctl[0];
  }
  // the window's commits (hosts this walk touched): to global availability, or handed to the
  // next walk, which applies them once the next count pass (running now) has read the old state
  if (wave == 0) {
    const int m = __builtin_amdgcn_readfirstlane(S.ctl[1]);
    int no = 0;
    for (int q0 = 0; q0 < m; q0 += WAVE) {
      const int q = q0 + lane;
      const bool own = q < m && S.own[q];
      const uint64_t b = __ballot(own);
      if (own) {
        const int32_t h = S.tid[q];
        if (A.writeback)
          for (int r = 0; r < 4; r++) A.avail[(size_t)r * A.H + h] = S.ta[r][q];
        if (A.out) {
          const int o = no + __popcll(b & below);
          A.out->tid[o] = h;
          for (int r = 0; r < 4; r++) { A.out->sb[r][o] = S.sb[r][q]; A.out->ta[r][o] = S.ta[r][q]; }
        }
      }
      no += __popcll(b);
    }
    if (A.out && lane == 0) A.out->n = no;
  }
  for (int i = tx; i < A.nt; i += NT) A.placement[i] = S.pl[i];
  for (int i = tx; i < 625; i += NT) A.mt[i] = S.mt[i];
#ifdef PVT_STAMPS
  if (tx == 0 && A.stamps) {
    for (int k = 0; k < 14; k++)
      if (k != 7) atomicAdd((unsigned long long*)&A.stamps[k], (unsigned long long)ph[k]);
    atomicAdd((unsigned long long*)&A.stamps[7], (unsigned long long)A.nt);
  }
#endif
}

hipError_t opp_init_attrs() {
  return hipFuncSetAttribute((const void*)opp_commit_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(OppLDS));
}

void launch_opp_commit(const OppCommitArgs& a, hipStream_t st) {
  PVT_LAUNCH(opp_commit_kernel, dim3(1), dim3(OPP_NW * WAVE), sizeof(OppLDS), st, a);
}

// Rank packages -> full tables: package r holds, task-major, the chunk bitmaps ([nt][ldq][4]
// u64) then the super-chunk counts ([nt][lds] i32) of super-chunks [r * P_sq, ...).
__global__ __launch_bounds__(256) void opp_unpack_kernel(OppUnpackArgs A) {
  constexpr int U = OPP_CH / WAVE;
  const int r = blockIdx.y;
  const int s0 = r * A.P_sq, ns = min(A.P_sq, A.nsq - s0);
  if (ns <= 0) return;
  const int ldq = A.P_sq * OPP_SUP, lds = A.P_sq;
  const int q0 = s0 * OPP_SUP, nqr = min(ns * OPP_SUP, A.nq - q0);
  const uint8_t* base = A.recv + (size_t)r * A.pkg_bytes;
  const uint64_t* bm = reinterpret_cast<const uint64_t*>(base);
  const int32_t* sc = reinterpret_cast<const int32_t*>(base + sizeof(uint64_t) * U * (size_t)A.nt * ldq);
  const size_t nb = (size_t)A.nt * nqr * U;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < nb; k += (size_t)gridDim.x * blockDim.x) {
    const size_t t = k / ((size_t)nqr * U), rem = k % ((size_t)nqr * U);
    A.bm[(t * A.nq + q0) * U + rem] = bm[t * ldq * U + rem];
  }
  const size_t ns_all = (size_t)A.nt * ns;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < ns_all; k += (size_t)gridDim.x * blockDim.x) {
    const size_t t = k / ns, j = k % ns;
    A.sc[t * A.nsq + s0 + j] = sc[t * lds + j];
  }
}

void launch_opp_unpack(const OppUnpackArgs& a, hipStream_t st) {
  PVT_LAUNCH(opp_unpack_kernel, dim3(256, a.world), dim3(256), 0, st, a);
}

__global__ __launch_bounds__(256) void opp_apply_kernel(const OppTouched* t, double* avail, int H) {
  const int n = t->n;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const int32_t h = t->tid[q];
#pragma unroll
    for (int r = 0; r < 4; r++) avail[(size_t)r * H + h] = t->ta[r][q];
  }
}

void launch_opp_apply(const OppTouched* t, double* avail, int H, hipStream_t st) {
  PVT_LAUNCH(opp_apply_kernel, dim3(OPP_MAXW / 256), dim3(256), 0, st, t, avail, H);
}

}  // namespace pvt
