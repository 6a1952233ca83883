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

#include "pvt_device.h"
#include "pvt_kernels.h"
#include "pvt_mt.h"
#include "pvt_opp.h"

namespace pvt {

// ------------------------------------------------------------------------------------------
// Count kernel: block = 4 waves, each wave OPP_TW tasks over one host segment (a run of
// super-chunks); blockIdx % S picks the segment (XCD-affine, as in score_kernel). For every
// (task, 256-host chunk) it stores the chunk's feasibility bitmap (the four wave ballots,
// 32 B) and, per super-chunk, the feasible count, task-major: the walk's dependent read of one
// super-chunk's 64 chunk bitmaps for one task is then 2 KiB contiguous. A chunk's host loads are issued one chunk
// ahead (register double buffer, clamped indices instead of branches).
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
  const int Q0 = A.sq_lo + seg * A.seg_sup, Q1 = min(A.sq_hi, Q0 + A.seg_sup);
  const int qa = Q0 * OPP_SUP, qb = min(A.nq, Q1 * OPP_SUP);
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
      uint64_t* o = A.bm + ((size_t)(t0 + lane) * A.ldq + (q - A.sq_lo * OPP_SUP)) * U;
#pragma unroll
      for (int u = 0; u < U; u++) o[u] = mine[u];
    }
    if ((q + 1) % OPP_SUP == 0 || q + 1 == qb) {   // super-chunk boundary
      const int Q = q / OPP_SUP;
      int v = 0;
#pragma unroll
      for (int k = 0; k < OPP_TW; k++) {
        if (lane == k) v = sup[k];
        sup[k] = 0;
      }
      if (lane < nt) A.sc[(size_t)(t0 + lane) * A.lds + (Q - A.sq_lo)] = v;
    }
  }
}

void launch_opp_count(const OppCountArgs& a, hipStream_t st) {
  const int tiles = (a.nt + 4 * OPP_TW - 1) / (4 * OPP_TW);
  hipLaunchKernelGGL(opp_count_kernel, dim3(tiles * a.S), dim3(256), 0, st, a);
}

// ------------------------------------------------------------------------------------------
// Commit walk (one wave).
// ------------------------------------------------------------------------------------------
constexpr int OPP_HASH_BITS = 12;
constexpr int OPP_NSQ_MAX = 1024;   // super-chunks supported: 16.7M hosts
constexpr int OPP_HASH = 1 << OPP_HASH_BITS;

struct OppLDS {
  int32_t hkey[OPP_HASH];
  int32_t hval[OPP_HASH];
  int32_t tid[OPP_MAXW];
  int32_t lost[OPP_MAXW];
  double sa[4][OPP_MAXW];   // snapshot availability of touched hosts (the count pass's view)
  double ta[4][OPP_MAXW];   // current availability of touched hosts
  double sb[4][OPP_MAXW];   // availability when this walk started (pipelined hand-off)
  int32_t own[OPP_MAXW];    // touched by this walk
  int32_t slost[OPP_NSQ_MAX];   // per task: lost hosts per super-chunk
  uint64_t lmask[OPP_SUP][4];   // per task: lost hosts of the chosen super-chunk, as chunk bitmaps
  uint32_t mt[625];
  int32_t pl[OPP_MAXW];         // placements of the window, written out when the walk ends
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
// would also wait vmcnt(0), i.e. for the next task's prefetched HBM loads.)
__device__ __forceinline__ void wave_lds_fence() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__global__ __launch_bounds__(64) void opp_commit_kernel(OppCommitArgs A) {
  constexpr int U = OPP_CH / WAVE;
  constexpr int SUPH = OPP_SUP * OPP_CH;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  OppLDS& S = *reinterpret_cast<OppLDS*>(smem);
  const int lane = lane_id();
  for (int i = lane; i < OPP_HASH; i += WAVE) S.hkey[i] = -1;
  for (int i = lane; i < A.nt; i += WAVE) S.pl[i] = -1;
  for (int i = lane; i < 625; i += WAVE) S.mt[i] = A.mt[i];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  int m = 0;
  if (A.in) {
    // the previous walk's commits (already in global availability, launch_opp_apply): touched,
    // with the count pass's snapshot as sa
    m = __builtin_amdgcn_readfirstlane(A.in->n);
    for (int q = lane; q < m; q += WAVE) {
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
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const bool fast = A.nsq <= WAVE;   // one super-chunk count per lane (H <= 1,048,576)
  MtWave mw;
  mw.buf = 0; mw.used = 0; mw.limit = 0;
  // next task's super-chunk counts and demand, prefetched with vector loads (lanes 0-3 hold
  // the demand), so no scalar-memory wait is mixed with the walk's LDS traffic
  int scn = (fast && A.nt > 0 && lane < A.nsq) ? A.sc[lane] : 0;
  double dn = (A.nt > 0) ? A.dem[lane & 3] : 0.0;

#ifdef PVT_STAMPS
  uint64_t ph[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t tl = ostamp();
#endif
  for (int i = 0; i < A.nt; i++) {
    OSTAMP(6);
    const double dv = dn;
    const double d0 = readlane_d(dv, 0), d1 = readlane_d(dv, 1), d2 = readlane_d(dv, 2), d3 = readlane_d(dv, 3);
    const int scv = scn;
    if (i + 1 < A.nt) {
      dn = A.dem[(size_t)(i + 1) * 4 + (lane & 3)];
      if (fast) scn = lane < A.nsq ? A.sc[(size_t)(i + 1) * A.nsq + lane] : 0;
    }
    OSTAMP(0);
    // Touched hosts that fitted at the snapshot and no longer fit ("lost"), listed and counted
    // per super-chunk with LDS atomics (4 x 64 touched hosts per loop trip).
    // (the fences order the zeroing, the other lanes' atomics and the reads: without them the
    // compiler may forward a lane's own zero store to its later read)
    for (int Q = lane; Q < A.nsq; Q += WAVE) S.slost[Q] = 0;
    wave_lds_fence();
    int nl = 0;
    for (int q0 = 0; q0 < m; q0 += 4 * WAVE) {
      bool lf[4];
      int32_t th[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int q = q0 + u * WAVE + lane;
        const int qq = min(q, m - 1);
        th[u] = S.tid[qq];
        lf[u] = (q < m) &&
                fits<false>(S.sa[0][qq], S.sa[1][qq], S.sa[2][qq], S.sa[3][qq], d0, d1, d2, d3) &&
                !fits<false>(S.ta[0][qq], S.ta[1][qq], S.ta[2][qq], S.ta[3][qq], d0, d1, d2, d3);
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint64_t b = __ballot(lf[u]);
        if (lf[u]) {
          S.lost[nl + __popcll(b & below)] = th[u];
          atomicAdd(&S.slost[th[u] / SUPH], 1);
        }
        nl += __popcll(b);
      }
    }
    wave_lds_fence();
    OSTAMP(1);
    long long n = 0;
    if (fast) {
      n = wave_sum_ll(scv);
    } else {
      for (int Q0 = 0; Q0 < A.nsq; Q0 += WAVE) {
        const int Q = Q0 + lane;
        n += wave_sum_ll(Q < A.nsq ? (long long)A.sc[(size_t)i * A.nsq + Q] : 0);
      }
    }
    n -= nl;
    if (n <= 0) continue;
    const uint32_t k = mt_randint(S.mt, mw, (uint32_t)n);
    OSTAMP(2);
    // super-chunk
    int Qs = -1;
    long long acc = 0;
    for (int Q0 = 0; Q0 < A.nsq && Qs < 0; Q0 += WAVE) {
      const int Q = Q0 + lane;
      int v = 0;
      if (Q < A.nsq) v = (fast ? scv : A.sc[(size_t)i * A.nsq + Q]) - S.slost[Q];
      const int inc = wave_incl_scan(v);
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
    if (Qs < 0) continue;   // unreachable when counts are consistent
    OSTAMP(3);
    int k1 = (int)(k - (uint32_t)acc);
    // chunk within the super-chunk: lane = chunk; its current bitmap is the snapshot bitmap
    // minus the lost hosts, collected into per-chunk masks with LDS atomics
    const int q = Qs * OPP_SUP + lane;
    uint64_t bits[U];
#pragma unroll
    for (int u = 0; u < U; u++) bits[u] = 0;
    if (q < A.nq) {
      const uint64_t* bp = A.bm + ((size_t)i * A.nq + q) * U;
#pragma unroll
      for (int u = 0; u < U; u++) bits[u] = bp[u];
    }
#pragma unroll
    for (int u = 0; u < U; u++) S.lmask[lane][u] = 0;
    wave_lds_fence();
    for (int j = lane; j < nl; j += WAVE) {
      const int h = S.lost[j];
      if (h / SUPH == Qs) {
        const int o = h % OPP_CH;
        atomicOr((unsigned long long*)&S.lmask[(h / OPP_CH) % OPP_SUP][o / WAVE], 1ull << (o % WAVE));
      }
    }
    wave_lds_fence();
    int c = 0;
#pragma unroll
    for (int u = 0; u < U; u++) {
      bits[u] &= ~S.lmask[lane][u];
      c += __popcll(bits[u]);
    }
    const int inc = wave_incl_scan(c);
    const uint64_t hit = __ballot(inc > k1);
    if (hit == 0) continue;   // unreachable when counts are consistent
    const int L = __builtin_ctzll(hit);
    k1 -= __builtin_amdgcn_readlane(inc, L) - __builtin_amdgcn_readlane(c, L);
    int off = -1;
    if (lane == L) {
      int r = k1;
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int cu = __popcll(bits[u]);
        if (off < 0) {
          if (r < cu) off = u * WAVE + select_bit(bits[u], r);
          else r -= cu;
        }
      }
    }
    off = __builtin_amdgcn_readlane(off, L);
    const int w = (Qs * OPP_SUP + L) * OPP_CH + off;
    OSTAMP(4);
    int ws = ohash_find(S, w);
    ws = __builtin_amdgcn_readfirstlane(ws);
    double w0, w1, w2, w3;
    if (ws >= 0) {
      w0 = S.ta[0][ws]; w1 = S.ta[1][ws]; w2 = S.ta[2][ws]; w3 = S.ta[3][ws];
    } else {   // lanes 0-3 load the four resources (vector loads)
      const double av = A.avail[(size_t)(lane & 3) * A.H + w];
      w0 = readlane_d(av, 0); w1 = readlane_d(av, 1); w2 = readlane_d(av, 2); w3 = readlane_d(av, 3);
    }
    OSTAMP(5);
    const double n0 = w0 - d0, n1 = w1 - d1, n2 = w2 - d2, n3 = w3 - d3;
    if (ws < 0) {
      ws = m++;
      if (lane == 0) {
        ohash_put(S, w, ws);
        S.tid[ws] = w;
        S.sa[0][ws] = w0; S.sa[1][ws] = w1; S.sa[2][ws] = w2; S.sa[3][ws] = w3;
        S.sb[0][ws] = w0; S.sb[1][ws] = w1; S.sb[2][ws] = w2; S.sb[3][ws] = w3;
      }
    }
    // commit in LDS only: a global store here would put its round trip on the next task (the
    // next task's prefetched loads share the in-order vmcnt counter with it)
    if (lane == 0) {
      S.ta[0][ws] = n0; S.ta[1][ws] = n1; S.ta[2][ws] = n2; S.ta[3][ws] = n3;
      S.own[ws] = 1;
      S.pl[i] = w;
    }
  }
  // the window's commits (hosts this walk touched): to global availability, or handed to the
  // next walk, which applies them once the next count pass (running now) has read the old state
  __builtin_amdgcn_s_waitcnt(0xc07f);
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
  for (int i = lane; i < A.nt; i += WAVE) A.placement[i] = S.pl[i];
  mt_unbuffer(S.mt, mw);
  for (int i = lane; i < 625; i += WAVE) A.mt[i] = S.mt[i];
#ifdef PVT_STAMPS
  if (lane == 0 && A.stamps) {
    for (int k = 0; k < 7; k++) atomicAdd((unsigned long long*)&A.stamps[k], (unsigned long long)ph[k]);
    atomicAdd((unsigned long long*)&A.stamps[7], (unsigned long long)A.nt);
  }
#endif
}

hipError_t opp_init_attrs() {
  return hipFuncSetAttribute((const void*)opp_commit_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(OppLDS));
}

void launch_opp_commit(const OppCommitArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(opp_commit_kernel, dim3(1), dim3(64), sizeof(OppLDS), st, a);
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
  hipLaunchKernelGGL(opp_unpack_kernel, dim3(256, a.world), dim3(256), 0, st, a);
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
  hipLaunchKernelGGL(opp_apply_kernel, dim3(OPP_MAXW / 256), dim3(256), 0, st, t, avail, H);
}

}  // namespace pvt
