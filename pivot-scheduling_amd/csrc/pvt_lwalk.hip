// pvt_lwalk.hip — the vbp best-fit commit walk on one wave, with list cursors.
//
// vbp best-fit (reference scheduler/vbp.py:39-50): per task in sorted order, the strictly fitting
// host of least (||avail - d||2, host-id rank, index), then resc[h] -= d. With the window's
// candidate lists (exact top lists on the window's start state, pvt_band.hip + merge) the winner
// is, exactly as in the list walk (pvt_walk.hip):
//
//   min( the first list entry nobody has committed to since the lists were scored ("untouched";
//        its list state is its state), every "live" touched host rescored on its current state )
//
// where a touched host that cannot fit the window's componentwise smallest demand is dead for the
// rest of the window. vbp best-fit has almost no live touched hosts (a host's memory after its
// best-fit commit is the residual, far below any task's demand), so a task's winner is nearly
// always its list's first untouched entry -- and tasks with the same demand vector have the same
// list (the trace has few distinct demand rows, and the sorted order puts equal demands next to
// each other). So one wave walks the window holding the current list chunk in registers:
//
//   * a chunk's entries are checked against the touched-host hash ONCE, when the chunk is loaded;
//     afterwards only this walk's commits can touch them, and the walk marks its winner in the
//     chunk's flags itself;
//   * a task with the previous task's demand continues the previous task's list from the cursor
//     (every entry before it is touched); another demand loads its own list head.
//
// Per task: a ballot over the chunk's untouched flags, the (rare) scan of live touched hosts, and
// the commit in LDS. The walk stops (status[0] = tasks walked, a refill) where its lists cannot
// decide a task: a list exhausted before its bound (incomplete), or a full touched-host table; a
// window it cannot start is walked by the list walk. Capacities of the hosts it committed to are
// written back at the end, with own_ids / status[1] as the list walk reports them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"
#include "pvt_kernels.h"

namespace pvt {

constexpr int LW_HBITS = 12;
constexpr int LW_HSLOTS = 1 << LW_HBITS;   // touched-host hash (<= 2048 hosts)
constexpr int LW_TAB = 2048;               // touched hosts: inherited + committed to
constexpr int LW_EMPTY = -1;

struct LwalkLDS {
  int32_t hkey[LW_HSLOTS];
  int32_t hval[LW_HSLOTS];                 // table index of the host
  double ta[4][LW_TAB];                    // current capacities
  int32_t tid[LW_TAB];
  uint32_t ttb[LW_TAB];
  int32_t town[LW_TAB];                    // committed to by this walk
  int32_t live[LW_TAB];                    // table indices of the live hosts (any order)
  int32_t nlive, ntab, bad;
};

__device__ __forceinline__ uint32_t lw_slot(int32_t id) {
  return ((uint32_t)id * 2654435761u) >> (32 - LW_HBITS);
}
// table index of host id, or -1 (one lane)
__device__ __forceinline__ int32_t lw_find(const LwalkLDS& S, int32_t id) {
  uint32_t p = lw_slot(id);
  for (;;) {
    const int32_t k = S.hkey[p];
    if (k == id) return S.hval[p];
    if (k == LW_EMPTY) return -1;
    p = (p + 1) & (LW_HSLOTS - 1);
  }
}

__device__ __forceinline__ double rec_dw(int32_t tv, int k) {   // TaskRec double k (lanes 2k, 2k+1)
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(tv, 2 * k);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane(tv, 2 * k + 1);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ bool key_lt2(uint64_t a1, uint64_t a2, uint64_t b1, uint64_t b2) {
  return (a1 < b1) | ((a1 == b1) & (a2 < b2));
}

__device__ __forceinline__ void lw_fence() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// vbp best-fit key: (sqrt of the FMA-chain squared residual, as bits; tiebreak : id)
__device__ __forceinline__ void lw_key(double a0, double a1, double a2, double a3, double d0,
                                       double d1, double d2, double d3, uint32_t tb, int32_t id,
                                       uint64_t& k1, uint64_t& k2) {
  k1 = (uint64_t)__double_as_longlong(__builtin_sqrt(norm2_seq(a0 - d0, a1 - d1, a2 - d2, a3 - d3)));
  k2 = ((uint64_t)tb << 32) | (uint32_t)id;
}

#ifdef PVT_STAMPS
__device__ __forceinline__ uint64_t lstamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif

__global__ __launch_bounds__(WAVE) void lwalk_kernel(CommitArgs A) {
#ifdef PVT_STAMPS
  uint64_t ph[4] = {0, 0, 0, 0}, n_task = 0, n_load = 0, n_liveit = 0, n_twin = 0, n_live = 0;
  uint64_t ts = lstamp();
#define LW_PHASE(k) do { const uint64_t t2 = lstamp(); ph[k] += t2 - ts; ts = t2; } while (0)
#else
#define LW_PHASE(k) ((void)0)
#endif
  extern __shared__ __attribute__((aligned(16))) char smem[];
  LwalkLDS& S = *reinterpret_cast<LwalkLDS*>(smem);
  const int lane = lane_id();
  // an enqueued-ahead window (CommitArgs::gate): skipped when the walk before did not walk its
  // whole window; otherwise that walk's hosts are the inherited ones
  if (gate_closed(A.gate)) {
    if (lane == 0) { A.status[0] = 0; A.status[1] = 0; A.status[2] = A.nt; A.status[3] = 1; }
    return;
  }
  const int n_prev = A.gate ? __builtin_amdgcn_readfirstlane(A.gate[1]) : A.n_prev;
  for (int i = lane; i < LW_HSLOTS; i += WAVE) S.hkey[i] = LW_EMPTY;
  if (lane == 0) { S.nlive = 0; S.ntab = 0; S.bad = 0; }
  // componentwise smallest demand of the window: a touched host that cannot fit it is dead
  double m0 = DINF, m1 = DINF, m2 = DINF, m3 = DINF;
  for (int i = lane; i < A.nt; i += WAVE) {
    const double* dp = A.dem + (size_t)i * 4;
    m0 = fmin(m0, dp[0]); m1 = fmin(m1, dp[1]); m2 = fmin(m2, dp[2]); m3 = fmin(m3, dp[3]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    m0 = fmin(m0, __shfl_xor(m0, off)); m1 = fmin(m1, __shfl_xor(m1, off));
    m2 = fmin(m2, __shfl_xor(m2, off)); m3 = fmin(m3, __shfl_xor(m3, off));
  }
  m0 = readlane_d(m0, 0); m1 = readlane_d(m1, 0); m2 = readlane_d(m2, 0); m3 = readlane_d(m3, 0);
  lw_fence();
  // inherited touched hosts (the previous walk's, committed after these lists were scored):
  // their current capacities from HBM; ids are distinct
  const int np = min(n_prev, LW_TAB);
  for (int k = lane; k < np; k += WAVE) {
    const int32_t id = A.prev_ids[k];
    const double a0 = A.avail[id], a1 = A.avail[(size_t)A.H + id];
    const double a2 = A.avail[2 * (size_t)A.H + id], a3 = A.avail[3 * (size_t)A.H + id];
    S.ta[0][k] = a0; S.ta[1][k] = a1; S.ta[2][k] = a2; S.ta[3][k] = a3;
    S.tid[k] = id;
    S.ttb[k] = A.tb ? A.tb[id] : 0u;
    S.town[k] = 0;
    uint32_t p = lw_slot(id);
    while (atomicCAS(&S.hkey[p], LW_EMPTY, id) != LW_EMPTY) p = (p + 1) & (LW_HSLOTS - 1);
    S.hval[p] = k;
    if (fits<true>(a0, a1, a2, a3, m0, m1, m2, m3)) S.live[atomicAdd(&S.nlive, 1)] = k;
  }
  lw_fence();
  int ntab = np;
  int nlive = __builtin_amdgcn_readfirstlane(S.nlive);
  int n_own = 0;
  int status = A.nt;
  if (n_prev > LW_TAB) status = 0;            // (cannot hold them: the list walk decides)

  // the current list chunk (lane j: entry cbase + j of list cw) and its untouched flags
  int cw = -1, cbase = 0, ccnt = 0, cur = 0;
  bool ccomp = false;
  double ce_s = 0.0, ce0 = 0.0, ce1 = 0.0, ce2 = 0.0, ce3 = 0.0;
  uint32_t ce_tb = 0;
  int32_t ce_id = -1;
  bool ce_u = false;                          // untouched (valid entry)
  double pd0 = NAN, pd1 = NAN, pd2 = NAN, pd3 = NAN;   // the demand the chunk's list belongs to

  auto load_chunk = [&](int w, int base, int cnt) {
    const int p = base + lane;
    const bool v = p < cnt;
    const ListEntry* e = A.L.e + (size_t)w * LMAX + min(p, LMAX - 1);
    ce_s = e->s; ce_tb = e->tb; ce_id = e->id;
    ce0 = e->a[0]; ce1 = e->a[1]; ce2 = e->a[2]; ce3 = e->a[3];
    ce_u = v && lw_find(S, ce_id) < 0;
    cw = w; cbase = base; ccnt = cnt;
#ifdef PVT_STAMPS
    n_load++;
#endif
  };

  // task records, 64 per batch in lanes (lane l: task b0 + l's demand, list count, completeness,
  // caller), the next batch's loads in flight while a batch is walked
  // ri = (list count, completeness, list row, caller); representative rows (A.rowmap): the
  // demand and caller are the task's own, the list (and its count) its row's
  auto rec_load = [&](int b0, double& r0, double& r1, double& r2, double& r3, int4& ri) {
    const int w = min(b0 + lane, max(A.nt - 1, 0));
    if (A.rowmap) {
      const int row = A.rowmap[w] - A.rowbase;
      const double2 x = *reinterpret_cast<const double2*>(A.dem + (size_t)w * 4);
      const double2 y = *reinterpret_cast<const double2*>(A.dem + (size_t)w * 4 + 2);
      const int2 cc = *reinterpret_cast<const int2*>(&A.L.t[row].cnt);
      ri = make_int4(cc.x, cc.y, row, A.ordw[w]);
      r0 = x.x; r1 = x.y; r2 = y.x; r3 = y.y;
    } else {
      const TaskRec* tr = A.L.t + w;
      const double2 x = *reinterpret_cast<const double2*>(&tr->d[0]);
      const double2 y = *reinterpret_cast<const double2*>(&tr->d[2]);
      const int4 c4 = *reinterpret_cast<const int4*>(&tr->cnt);   // cnt, complete, anc, ord
      ri = make_int4(c4.x, c4.y, w, c4.w);
      r0 = x.x; r1 = x.y; r2 = y.x; r3 = y.y;
    }
  };
  double nr0, nr1, nr2, nr3;
  int4 nri;
  rec_load(0, nr0, nr1, nr2, nr3, nri);
  for (int b0 = 0; b0 < A.nt && status == A.nt; b0 += WAVE) {
  const double rd0 = nr0, rd1 = nr1, rd2 = nr2, rd3 = nr3;
  const int4 rri = nri;
  if (b0 + WAVE < A.nt) rec_load(b0 + WAVE, nr0, nr1, nr2, nr3, nri);
  const int kn = min(WAVE, A.nt - b0);
  // runs: bit k set iff batch task k has task k - 1's demand (bit for bit) and list shape
  uint64_t E;
  {
    bool eq = lane > 0 && lane < kn;
    eq &= __double_as_longlong(__shfl_up(rd0, 1)) == __double_as_longlong(rd0);
    eq &= __double_as_longlong(__shfl_up(rd1, 1)) == __double_as_longlong(rd1);
    eq &= __double_as_longlong(__shfl_up(rd2, 1)) == __double_as_longlong(rd2);
    eq &= __double_as_longlong(__shfl_up(rd3, 1)) == __double_as_longlong(rd3);
    eq &= __shfl_up(rri.x, 1) == rri.x && __shfl_up(rri.y, 1) == rri.y;
    E = __ballot(eq);
  }
  for (int k = 0; k < kn && status == A.nt; k++) {
    k = __builtin_amdgcn_readfirstlane(k);
    const int i = b0 + k;
    const double d0 = readlane_d(rd0, k), d1 = readlane_d(rd1, k);
    const double d2 = readlane_d(rd2, k), d3 = readlane_d(rd3, k);
    const int cnt = __builtin_amdgcn_readlane(rri.x, k);
    const bool comp = __builtin_amdgcn_readlane(rri.y, k) != 0;
    const int caller = __builtin_amdgcn_readlane(rri.w, k);
    const int lrow = __builtin_amdgcn_readlane(rri.z, k);
    // same demand vector (bitwise): the same list, continued from the cursor
    const bool same = cw >= 0 && __double_as_longlong(d0) == __double_as_longlong(pd0) &&
                      __double_as_longlong(d1) == __double_as_longlong(pd1) &&
                      __double_as_longlong(d2) == __double_as_longlong(pd2) &&
                      __double_as_longlong(d3) == __double_as_longlong(pd3) && cnt == ccnt &&
                      comp == ccomp;
    if (!same) {
      load_chunk(lrow, 0, cnt);
      cur = 0;
      ccomp = comp;
      pd0 = d0; pd1 = d1; pd2 = d2; pd3 = d3;
    }
#ifdef PVT_STAMPS
    n_task++;
    n_live += nlive;
#endif
    LW_PHASE(0);
    // the first untouched entry at or after the cursor
    int L = -1;
    for (;;) {
      const uint64_t m = __ballot(ce_u && cbase + lane >= cur);
      if (m) { L = __builtin_ctzll(m); break; }
      if (cbase + WAVE >= ccnt) break;          // list exhausted
      cur = cbase + WAVE;
      load_chunk(cw, cbase + WAVE, ccnt);
    }
    if (L < 0 && !ccomp) { status = i; break; }   // past the list's bound: refill from here
    // A run of tasks with this demand, no live touched host: each task's winner is simply the
    // next untouched entry (the list's order is the key order; no touched host can fit), as
    // long as every winner is dead after its commit. The run takes the chunk's untouched
    // entries from the cursor in order -- up to and including the first winner that stays alive
    // (it becomes the live host the next task must rescore) -- in one parallel commit.
    if (nlive == 0 && L >= 0 && k + 1 < kn && ((E >> (k + 1)) & 1ull)) {
      const int R = min(kn - k, 1 + (int)__builtin_ctzll(~(E >> (k + 1))));
      const uint64_t U = __ballot(ce_u && cbase + lane >= cur);
      const bool in = (U >> lane) & 1ull;
      const int rank = __popcll(U & ((1ull << lane) - 1ull));
      const double n0 = ce0 - d0, n1 = ce1 - d1, n2 = ce2 - d2, n3 = ce3 - d3;
      const uint64_t Am = __ballot(in && fits<true>(n0, n1, n2, n3, m0, m1, m2, m3));
      int Rb = min(min(R, __popcll(U)), LW_TAB - ntab);
      if (Am) Rb = min(Rb, __popcll(U & ((1ull << __builtin_ctzll(Am)) - 1ull)) + 1);
      Rb = __builtin_amdgcn_readfirstlane(Rb);
      if (Rb <= 0) { status = i; break; }         // (touched-host table full: refill)
      const bool win = in && rank < Rb;
      const int callr = __shfl(rri.w, min(k + rank, WAVE - 1));
      lw_fence();
      if (win) {
        const int t = ntab + rank;
        S.ta[0][t] = n0; S.ta[1][t] = n1; S.ta[2][t] = n2; S.ta[3][t] = n3;
        S.tid[t] = ce_id; S.ttb[t] = ce_tb; S.town[t] = 1;
        uint32_t p = lw_slot(ce_id);
        while (atomicCAS(&S.hkey[p], LW_EMPTY, ce_id) != LW_EMPTY) p = (p + 1) & (LW_HSLOTS - 1);
        S.hval[p] = t;
        A.own_ids[n_own + rank] = ce_id;
        A.placement[callr] = ce_id;
        if (((Am >> lane) & 1ull) && rank == Rb - 1) S.live[0] = t;   // the alive last winner
      }
      const uint64_t Wm = __ballot(win);
      const int last = 63 - __builtin_clzll(Wm);
      if ((Am >> last) & 1ull) nlive = 1;
      ce_u = ce_u && !win;
      cur = cbase + last + 1;
      ntab += Rb;
      n_own += Rb;
      k += Rb - 1;                               // (the loop adds the last one)
      lw_fence();
#ifdef PVT_STAMPS
      n_task += Rb - 1;
#endif
      LW_PHASE(3);
      continue;
    }
    uint64_t b1 = ~0ull, b2 = ~0ull;
    if (L >= 0) {
      b1 = readlane_u64((uint64_t)__double_as_longlong(ce_s), L);
      b2 = ((uint64_t)readlane_u(ce_tb, L) << 32) | (uint32_t)readlane_i(ce_id, L);
    }
    LW_PHASE(1);
    // live touched hosts, rescored exactly
    int wq = -1;
    for (int q0 = 0; q0 < nlive; q0 += WAVE) {
#ifdef PVT_STAMPS
      n_liveit++;
#endif
      const int qi = q0 + lane;
      const int q = qi < nlive ? S.live[qi] : 0;
      const double a0 = S.ta[0][q], a1 = S.ta[1][q], a2 = S.ta[2][q], a3 = S.ta[3][q];
      const bool f = qi < nlive && fits<true>(a0, a1, a2, a3, d0, d1, d2, d3);
      uint64_t k1 = ~0ull, k2 = ~0ull;
      if (f) lw_key(a0, a1, a2, a3, d0, d1, d2, d3, S.ttb[q], S.tid[q], k1, k2);
      // chunk minimum: (k1, k2) lexicographic
      const uint64_t mk1 = wave_min_u64(k1);
      const uint64_t mk2 = wave_min_u64(k1 == mk1 ? k2 : ~0ull);
      if (mk1 != ~0ull && key_lt2(mk1, mk2, b1, b2)) {
        const uint64_t hit = __ballot(k1 == mk1 && k2 == mk2);
        wq = readlane_i(q, __builtin_ctzll(hit));
        b1 = mk1; b2 = mk2;
      }
    }
    LW_PHASE(2);
#ifdef PVT_STAMPS
    n_twin += wq >= 0;
#endif
    if (L < 0 && wq < 0) {                     // no host fits: the task waits
      if (lane == 0) A.placement[caller] = -1;
      continue;
    }
    int32_t wid;
    if (wq >= 0) {                             // a live touched host wins
      const double n0 = S.ta[0][wq] - d0, n1 = S.ta[1][wq] - d1;
      const double n2 = S.ta[2][wq] - d2, n3 = S.ta[3][wq] - d3;
      wid = S.tid[wq];
      const bool first = S.town[wq] == 0;
      lw_fence();
      if (lane == 0) {
        S.ta[0][wq] = n0; S.ta[1][wq] = n1; S.ta[2][wq] = n2; S.ta[3][wq] = n3;
        S.town[wq] = 1;
        if (first) A.own_ids[n_own] = wid;
      }
      n_own += first ? 1 : 0;
      if (!fits<true>(n0, n1, n2, n3, m0, m1, m2, m3)) {   // dies: off the live list
        for (int q0 = 0; q0 < nlive; q0 += WAVE) {
          const int qi = q0 + lane;
          const uint64_t hit = __ballot(qi < nlive && S.live[qi] == wq);
          if (hit) {
            const int pos = q0 + __builtin_ctzll(hit);
            const int last = S.live[nlive - 1];
            lw_fence();
            if (lane == 0) S.live[pos] = last;
            nlive--;
            break;
          }
        }
      }
    } else {                                   // the list's first untouched entry wins
      if (ntab >= LW_TAB) { status = i; break; }
      const double n0 = readlane_d(ce0, L) - d0, n1 = readlane_d(ce1, L) - d1;
      const double n2 = readlane_d(ce2, L) - d2, n3 = readlane_d(ce3, L) - d3;
      wid = readlane_i(ce_id, L);
      const uint32_t wtb = readlane_u(ce_tb, L);
      const int t = ntab++;
      const bool alive = fits<true>(n0, n1, n2, n3, m0, m1, m2, m3);
      if (lane == 0) {
        S.ta[0][t] = n0; S.ta[1][t] = n1; S.ta[2][t] = n2; S.ta[3][t] = n3;
        S.tid[t] = wid; S.ttb[t] = wtb; S.town[t] = 1;
        uint32_t p = lw_slot(wid);
        while (S.hkey[p] != LW_EMPTY) p = (p + 1) & (LW_HSLOTS - 1);
        S.hkey[p] = wid;
        S.hval[p] = t;
        if (alive) S.live[nlive] = t;
        A.own_ids[n_own] = wid;
      }
      nlive += alive ? 1 : 0;
      n_own++;
      ce_u = ce_u && lane != L;                // touched now (the chunk's flags)
      cur = cbase + L + 1;
    }
    if (lane == 0) A.placement[caller] = wid;
    lw_fence();                                // this commit's LDS writes before the next reads
    LW_PHASE(3);
  }
  }
  // the capacities of the hosts this walk committed to
  lw_fence();
  for (int t = lane; t < ntab; t += WAVE)
    if (S.town[t]) {
      const int32_t id = S.tid[t];
#pragma unroll
      for (int r = 0; r < 4; r++) A.avail[(size_t)r * A.H + id] = S.ta[r][t];
    }
  if (lane == 0) {
    A.status[0] = status; A.status[1] = n_own;
    if (A.ahead) { A.status[2] = A.nt; A.status[3] = 0; }
    if (A.hflag) {
      A.hflag[1] = status;
      A.hflag[2] = n_own;
      __threadfence_system();
      __hip_atomic_store(A.hflag, A.hseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
#ifdef PVT_STAMPS
  if (lane == 0 && A.stamps) {
    for (int k = 0; k < 4; k++) atomicAdd((unsigned long long*)&A.stamps[k], (unsigned long long)ph[k]);
    atomicAdd((unsigned long long*)&A.stamps[4], (unsigned long long)n_task);
    atomicAdd((unsigned long long*)&A.stamps[5], (unsigned long long)n_load);
    atomicAdd((unsigned long long*)&A.stamps[6], (unsigned long long)n_liveit);
    atomicAdd((unsigned long long*)&A.stamps[7], (unsigned long long)n_twin);
    atomicAdd((unsigned long long*)&A.stamps[8], (unsigned long long)n_live);
  }
#endif
#undef LW_PHASE
}

constexpr size_t LWALK_LDS_BYTES = sizeof(LwalkLDS);
static_assert(LWALK_LDS_BYTES <= 160 * 1024, "list walk LDS");

hipError_t lwalk_init_attrs() {
  return hipFuncSetAttribute((const void*)lwalk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)LWALK_LDS_BYTES);
}

void launch_lwalk(const CommitArgs& a, hipStream_t st) {
  PVT_LAUNCH(lwalk_kernel, dim3(1), dim3(WAVE), LWALK_LDS_BYTES, st, a);
}

}  // namespace pvt
