// pvt_walk.hip — the commit walk: the reference's sequential placement loop over one window.
//
// Reference loops: cost_aware best-fit scheduler/cost_aware.py:84-97, first-fit :117-127,
// vbp first-fit scheduler/vbp.py:19-25, best-fit :43-49. Each visits tasks in order, picks a
// host against the CURRENT capacities and commits (resc[h] -= demand) before the next task.
//
// The candidate lists of the window were scored on a snapshot. A host nobody committed to since
// ("untouched") still has its snapshot state, so its list entry (score, feasibility) is exact;
// a committed ("touched") host can only have lost capacity. Per task:
//   best-fit   winner = min(first untouched entry of the list, every live touched host rescored
//              exactly); if the list has no untouched entry and may be missing hosts, a touched
//              host still wins exactly when it ranks at or before the list's bound, else the
//              walk stops and the host starts a new window here (a refill).
//   first-fit  winner = first entry that is untouched, or touched and still fits.
// A touched host that cannot fit the window's componentwise minimum demand can never be picked
// again in the window ("dead"); the others ("live") stay in an LDS table with their current
// capacities. Hosts committed to by the previous window, when that window's commits landed after
// this window's lists were scored, enter the walk as touched hosts (inherited).
//
// Execution: ONE workgroup on one CU, pipelined. Waves 1..PRODUCERS ("scouts") each take every
// PRODUCERS-th task: stream its list head (64 entries + task record) from HBM into an LDS ring
// slot, wait until the walk has committed every task up to i - LOOK, and then evaluate task i
// completely on that state -- touched-ness of the list entries, the deep list in HBM if needed,
// exact rescoring of the live touched hosts -- keeping the LOOK best candidates of each kind.
// Wave 0 (the walker) only patches that result with the hosts committed since (the tasks
// i - LOOK + 1 .. i - 1: at most LOOK - 1 "dirty" hosts, whose exact state it holds in
// registers), picks the winner and commits. A dirty host is dropped from the scout's lists by
// id and rescored exactly; every other host's state is what the scout saw, so LOOK candidates
// of each kind always leave a valid one.
//
// What a scout may see of a concurrent commit: the hash and the live table only grow (a host
// that dies is marked in place, never moved), and a new live entry becomes visible only through
// nl_pub, published after the entry is written. LDS operations of one wave execute in issue
// order, so a scout that reads committed >= k (or nl_pub >= n) also reads everything the walker
// wrote before. Anything torn belongs to a dirty host, which the walker re-evaluates.
// Hand-offs: a scout publishes flag[slot] = i when task i's slot and result are complete; the
// walker publishes done = i + 1 when it no longer reads slot i and committed = i + 1 after task
// i's commit. Every spin is bounded; a timeout reports status -1.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"
#include "pvt_kernels.h"

namespace pvt {

constexpr int RING = 12;                  // ring slots (task lists in LDS)
#ifndef PVT_LOOK
#define PVT_LOOK 2
#endif
#ifndef PVT_PRODUCERS
#define PVT_PRODUCERS 7
#endif
constexpr int LOOK = PVT_LOOK;            // a task is scouted on the state after task i - LOOK
constexpr int PRODUCERS = PVT_PRODUCERS;  // loader / scout waves
constexpr int PRE_CHUNKS = 4;             // list chunks a loader fetches before filtering
constexpr int WALK_THREADS = (1 + PRODUCERS) * WAVE;
constexpr int WH_BITS = 12;               // touched-host hash: 4096 slots for <= 2048 hosts
constexpr int WH_SLOTS = 1 << WH_BITS;
constexpr int LIVE_MAX = 1024;            // live touched hosts (rescored / refit every task)
constexpr int32_t H_EMPTY = -1;           // hash key of an empty slot
constexpr int32_t H_MISS = -1;            // lookup result: host not touched
constexpr int32_t H_DEAD = -2;            // hash value: touched, can no longer fit the window
constexpr int32_t H_PENDING = 0x7fffffff; // hash value before the walker writes it
constexpr int SPIN_LIMIT = 1 << 24;       // bounded spins (x s_sleep 2 ~ seconds)
constexpr int MAX_CHAIN_SEGS = 64;        // group segments per epoch chain

// A scout's result: LOOK usable list entries in list order (untouched, or for first-fit
// touched and fitting) and, for best-fit, the LOOK best live touched hosts; one 16-dword
// record per candidate (the walker reads dword k from lane k / 2 of one 64-bit load).
constexpr int RF_S = 0, RF_TB = 2, RF_ID = 3, RF_Z = 4, RF_Q = 5, RF_OWN = 6, RF_HP = 7, RF_A = 8;
constexpr int RREC = 16;                  // dwords per candidate record
constexpr int R_U = 0, R_T = LOOK * RREC, R_NU = 2 * LOOK * RREC, R_NT = R_NU + 1;
constexpr int R_WORDS = 2 * WAVE;
static_assert(R_NT < R_WORDS, "scout result exceeds 128 dwords");

struct RingSlot {
  double s[WAVE];
  double a[4][WAVE];
  int32_t id[WAVE];
  int32_t zone[WAVE];
  uint32_t tb[WAVE];
  int32_t rec[32];                        // TaskRec dwords 0-15, [16] ring entries,
                                          // [17] list position after the last one
  int32_t res[R_WORDS];                   // the scout's result
};

struct alignas(8) HK {
  int32_t key;                            // host id or H_EMPTY
  int32_t val;                            // live index or H_DEAD
};

struct WalkLDS {
  RingSlot ring[RING];
  HK hk[WH_SLOTS];
  double la[4][LIVE_MAX];                 // live touched hosts: current capacities
  int32_t lid[LIVE_MAX];
  int32_t lz[LIVE_MAX];
  int32_t lhp[LIVE_MAX];                  // hash position of the live host
  uint32_t ltb[LIVE_MAX];
  int32_t lown[LIVE_MAX];                 // 1: committed to by this walk (in own_ids)
  int32_t cseg[MAX_CHAIN_SEGS + 1];       // epoch walks: segment starts in this walk (+ nt)
  int32_t cwin[MAX_CHAIN_SEGS + 1];       //   and their first tasks' window indices
  double csum[ZMAX * ZMAX];
  double bsum[ZMAX * ZMAX];
  int32_t flag[RING];
  int32_t flagB[RING];                    // best-fit: the touched-host part of slot's task
  int32_t done;
  int32_t stop;
  int32_t nl_init;
  int32_t nl_pub;                         // live entries [0, nl_pub) are complete
  int32_t committed;                      // tasks committed (-1 until the inherited hosts are in)
};
static_assert(sizeof(WalkLDS) <= 160 * 1024, "commit walk LDS exceeds a CU's 160 KiB");

__device__ __forceinline__ uint32_t wslot(int32_t id) {
  return ((uint32_t)id * 2654435761u) >> (32 - WH_BITS);
}
// Value of `id` in the touched hash (H_MISS if absent) and the slot where the probe ended
// (the insertion point when absent).
__device__ __forceinline__ int32_t wfind(const WalkLDS& S, int32_t id, int32_t& pos) {
  uint32_t p = wslot(id);
  for (;;) {
    // key and value in ONE 64-bit LDS read (two dependent reads would double a probe's latency)
    const uint64_t kv = *reinterpret_cast<const uint64_t*>(&S.hk[p]);
    const int32_t key = (int32_t)(uint32_t)kv, val = (int32_t)(uint32_t)(kv >> 32);
    if (key == id) { pos = (int32_t)p; return val; }
    if (key == H_EMPTY) { pos = (int32_t)p; return H_MISS; }
    p = (p + 1) & (WH_SLOTS - 1);
  }
}

__device__ __forceinline__ int32_t vload(const int32_t* p) {
  return __atomic_load_n(p, __ATOMIC_RELAXED);
}
__device__ __forceinline__ void vstore(int32_t* p, int32_t v) {
  __atomic_store_n(p, v, __ATOMIC_RELAXED);
}
// Compiler-only ordering: LDS operations of one wave are executed in issue order, so keeping
// the compiler from moving loads across a hand-off flag is all the walker needs.
__device__ __forceinline__ void cbarrier() { __atomic_signal_fence(__ATOMIC_SEQ_CST); }
// The walker releases its ring slot: every read of the slot is issued before this store.
__device__ __forceinline__ void release_slot(WalkLDS& S, int32_t v) {
  cbarrier();
  vstore(&S.done, v);
  cbarrier();
}
__device__ __forceinline__ void lds_drain() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xc07f);     // lgkmcnt(0): this wave's LDS writes are done
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ void publish(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ double rec_d(int32_t tv, int k) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(tv, 2 * k);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane(tv, 2 * k + 1);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

#ifdef PVT_STAMPS
// Diagnostic build only (make stamps): per-phase cycle sums of the walker.
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP(k)                          \
  do {                                    \
    const uint64_t t_ = stamp();          \
    ph[k] += t_ - tl;                     \
    tl = t_;                              \
  } while (0)
#else
#define STAMP(k) do {} while (0)
#endif

// Window index of the walk's i-th task (epoch chains walk a subsequence of the window).
__device__ __forceinline__ int widx(const CommitArgs& A, int i) { return A.cmap ? A.cmap[i] : i; }

// ---------------------------------------------------------------- scouts (loader waves)
// Record r of a result block from lane `lane` (the lane holding the candidate): its score,
// tiebreak, host, zone, live index (-1 untouched), own flag, hash position, capacities.
__device__ __forceinline__ void put_rec(int32_t* res, int base, double s, uint32_t tb, int32_t id,
                                        int32_t z, int32_t q, int32_t own, int32_t hp, double a0,
                                        double a1, double a2, double a3) {
  int32_t* r = res + base;
  *reinterpret_cast<double*>(r + RF_S) = s;
  r[RF_TB] = (int32_t)tb; r[RF_ID] = id; r[RF_Z] = z; r[RF_Q] = q; r[RF_OWN] = own; r[RF_HP] = hp;
  double* a = reinterpret_cast<double*>(r + RF_A);
  a[0] = a0; a[1] = a1; a[2] = a2; a[3] = a3;
}

// Exact best-fit key of a host for the task: (score bits, tiebreak:id); scores are >= +0, so
// their bit patterns order like the values (cost_aware.py:83, vbp.py:45).
// The cost_aware score (c * sqrt(s2)) / bw without its square root and division where they
// cannot matter: c == 0 (a zero-cost zone pair) gives exactly +0 (finite s2, bw > 0); and when
// only a score of 0 can win (lim1 == 0, the bits of +0), c >= 2^-300, bw <= 2^300 and
// s2 >= 2^-600 prove the score positive (>= 2^-900): the key is then "beats nothing" (~0).
__device__ __forceinline__ uint64_t ca_score_bits(double c, double s2, double bw, uint64_t lim1) {
  if (c == 0.0) return 0ull;
  if (lim1 == 0ull && c >= 0x1p-300 && bw <= 0x1p300 && s2 >= 0x1p-600) return ~0ull;
  return (uint64_t)__double_as_longlong((c * __builtin_sqrt(s2)) / bw);
}

// rtrow: the task's group row of the realtime bandwidth (cost_aware.py:79), or NULL. lim1: the
// score bits a candidate must reach to matter (see ca_score_bits; ~0 = any).
template <int MODE>
__device__ __forceinline__ void bf_key(const WalkLDS& S, int Z, int anc, const double* rtrow,
                                       double a0, double a1, double a2, double a3, double d0,
                                       double d1, double d2, double d3, int32_t z, uint32_t tb,
                                       int32_t id, uint64_t lim1, uint64_t& k1, uint64_t& k2) {
  const double s2 = norm2_seq(a0 - d0, a1 - d1, a2 - d2, a3 - d3);
  if (MODE == CA_BF)
    k1 = ca_score_bits(S.csum[anc * Z + z], s2, rtrow ? rtrow[id] : S.bsum[anc * Z + z], lim1);
  else
    k1 = (uint64_t)__double_as_longlong(__builtin_sqrt(s2));
  k2 = ((uint64_t)(MODE == VBP_BF ? tb : 0u) << 32) | (uint32_t)id;
}
__device__ __forceinline__ bool key_lt(uint64_t a1, uint64_t a2, uint64_t b1, uint64_t b2) {
  return (a1 < b1) | ((a1 == b1) & (a2 < b2));
}

// Task i, after the walk has committed every task <= i - LOOK: the LOOK first usable entries of
// its list (ring, then the deep list in HBM) and, for best-fit, the LOOK best live touched hosts
// that could still win; written to R.res. PART: 0 both, 1 the list entries only, 2 the touched
// hosts only (best-fit tasks are scouted by two waves at once, one per part).
template <int MODE, int PART>
__device__ void scout(const CommitArgs& A, WalkLDS& S, RingSlot& R, int w, int k, int32_t rv,
                      const double* rtrow) {
  constexpr bool STRICT = (MODE == CA_FF || MODE == VBP_BF);
  constexpr bool BEST = (MODE == CA_BF || MODE == VBP_BF);
  const int lane = lane_id();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const double d0 = rec_d(rv, 0), d1 = rec_d(rv, 1), d2 = rec_d(rv, 2), d3 = rec_d(rv, 3);
  const int cnt = __builtin_amdgcn_readlane(rv, 8);
  const bool comp = __builtin_amdgcn_readlane(rv, 9) != 0;
  const int anc = __builtin_amdgcn_readlane(rv, 10);
  // usable ring entries (lane j: entry j)
  int nU = 0;
  uint64_t u1 = ~0ull, u2 = ~0ull;          // key of the last usable entry kept (best-fit)
  if (PART != 2) {
  const int npos = __builtin_amdgcn_readlane(R.rec[lane & 31], 17);   // own writes, in order
  {
    const bool valid = lane < k;
    const int32_t id = R.id[lane];
    int32_t hp = 0;
    const int32_t hv = valid ? wfind(S, id, hp) : H_MISS;
    // H_PENDING: the walker is inserting this host right now, so it is dirty for this task and
    // the walker re-evaluates it; first-fit keeps it (conservatively usable), best-fit does not
    // list touched hosts at all
    const bool live = hv >= 0 && hv != H_PENDING;
    const int q = live ? hv : 0;
    double c0 = R.a[0][lane], c1 = R.a[1][lane], c2 = R.a[2][lane], c3 = R.a[3][lane];
    int32_t own = 0, hpos = hp;
    bool usable;
    if (BEST) {
      usable = valid && hv == H_MISS;
    } else {
      if (live) {
        c0 = S.la[0][q]; c1 = S.la[1][q]; c2 = S.la[2][q]; c3 = S.la[3][q];
        own = S.lown[q]; hpos = S.lhp[q];
      }
      usable = valid && (hv == H_MISS || hv == H_PENDING ||
                         (live && fits<STRICT>(c0, c1, c2, c3, d0, d1, d2, d3)));
    }
    const uint64_t m = __ballot(usable);
    const int rank = __popcll(m & below);
    const double s = R.s[lane];
    const uint32_t tb = R.tb[lane];
    if (usable && rank < LOOK)
      put_rec(R.res, R_U + rank * RREC, s, tb, id, R.zone[lane], live ? hv : -1, own, hpos,
              c0, c1, c2, c3);
    nU = min(__popcll(m), LOOK);
    if (BEST && nU == LOOK) {
      const uint64_t lm = __ballot(usable && rank == LOOK - 1);
      const int L = __builtin_ctzll(lm);
      u1 = readlane_u64((uint64_t)__double_as_longlong(s), L);
      u2 = ((uint64_t)(MODE == VBP_BF ? readlane_u(tb, L) : 0u) << 32) | (uint32_t)readlane_i(id, L);
    }
  }
  // deep list (rare): entries after the ring's, by id, then their records from HBM
  const int32_t* ids = A.L.ids + (size_t)w * LMAX;
  const ListEntry* le = A.L.e + (size_t)w * LMAX;
  for (int c0 = npos; c0 < cnt && nU < LOOK; c0 += WAVE) {
    const bool v = c0 + lane < cnt;
    const int32_t id = v ? ids[c0 + lane] : 0;
    int32_t hp = 0;
    const int32_t hv = v ? wfind(S, id, hp) : H_MISS;
    const bool live = hv >= 0 && hv != H_PENDING;
    const int q = live ? hv : 0;
    bool usable;
    if (BEST) {
      usable = v && hv == H_MISS;
    } else {
      usable = v && (hv == H_MISS || hv == H_PENDING ||
                     (live && fits<STRICT>(S.la[0][q], S.la[1][q], S.la[2][q], S.la[3][q], d0, d1, d2, d3)));
    }
    const uint64_t m = __ballot(usable);
    const int rank = nU + __popcll(m & below);
    if (usable && rank < LOOK) {
      const ListEntry& x = le[c0 + lane];
      double c0_ = x.a[0], c1 = x.a[1], c2 = x.a[2], c3 = x.a[3];
      int32_t own = 0, hpos = hp;
      if (!BEST && live) {
        c0_ = S.la[0][q]; c1 = S.la[1][q]; c2 = S.la[2][q]; c3 = S.la[3][q];
        own = S.lown[q]; hpos = S.lhp[q];
      }
      put_rec(R.res, R_U + rank * RREC, x.s, x.tb, id, x.zone, live ? hv : -1, own, hpos, c0_, c1, c2, c3);
      if (BEST && rank == LOOK - 1) {
        u1 = (uint64_t)__double_as_longlong(x.s);
        u2 = ((uint64_t)(MODE == VBP_BF ? x.tb : 0u) << 32) | (uint32_t)id;
      }
    }
    if (BEST && nU + __popcll(m) >= LOOK) {
      const uint64_t lm = __ballot(usable && rank == LOOK - 1);
      const int L = __builtin_ctzll(lm);
      u1 = readlane_u64(u1, L);
      u2 = readlane_u64(u2, L);
    }
    nU = min(nU + __popcll(m), LOOK);
  }
  }   // PART != 2

  // best-fit: the LOOK best live touched hosts that rank before the bound any winner respects:
  // the LOOK-th usable entry, or with fewer the list bound (incomplete list) or nothing (the
  // touched-only part does not know the entries: the list bound, or nothing)
  int nT = 0;
  if (BEST && PART != 1) {
    uint64_t b1 = u1, b2 = u2;
    if (PART == 2 || nU < LOOK) {
      if (comp) {
        b1 = ~0ull; b2 = ~0ull;
      } else {   // every untouched host outside the list ranks at or after the bound (bid + 1)
        b1 = (uint64_t)__double_as_longlong(rec_d(rv, 6));
        b2 = (((uint64_t)(uint32_t)__builtin_amdgcn_readlane(rv, 14)) << 32) +
             (uint32_t)__builtin_amdgcn_readlane(rv, 15) + 1;
      }
    }
    uint64_t tk1[LOOK], tk2[LOOK];
    int32_t tq[LOOK];
#pragma unroll
    for (int r = 0; r < LOOK; r++) { tk1[r] = ~0ull; tk2[r] = ~0ull; tq[r] = -1; }
    const int nlp = __builtin_amdgcn_readfirstlane(vload(&S.nl_pub));
    for (int q0 = 0; q0 < nlp; q0 += WAVE) {
      const int q = q0 + lane;
      const int qq = min(q, nlp - 1);
      const double a0 = S.la[0][qq], a1 = S.la[1][qq], a2 = S.la[2][qq], a3 = S.la[3][qq];
      const bool fit = (q < nlp) && fits<STRICT>(a0, a1, a2, a3, d0, d1, d2, d3);
      if (__ballot(fit) == 0) continue;
      uint64_t k1 = ~0ull, k2 = ~0ull;
      bf_key<MODE>(S, A.Z, anc, rtrow, a0, a1, a2, a3, d0, d1, d2, d3, S.lz[qq],
                   MODE == VBP_BF ? S.ltb[qq] : 0u, S.lid[qq], b1 < tk1[LOOK - 1] ? b1 : tk1[LOOK - 1],
                   k1, k2);
      uint64_t pm = __ballot(fit && key_lt(k1, k2, b1, b2) && key_lt(k1, k2, tk1[LOOK - 1], tk2[LOOK - 1]));
      // Many candidates (a zero-cost component's touched hosts all score 0): take the chunk's
      // LOOK smallest keys by wave-wide minima (DPP) instead of inserting them one by one.
      if (__popcll(pm) > LOOK + 1) {
        bool cand = (pm >> lane) & 1ull;
        uint64_t sel = 0;
#pragma unroll
        for (int r = 0; r < LOOK; r++) {
          const uint64_t m1 = wave_min_u64(cand ? k1 : ~0ull);
          const uint64_t m2 = wave_min_u64((cand && k1 == m1) ? k2 : ~0ull);
          const uint64_t lm = __ballot(cand && k1 == m1 && k2 == m2);
          if (lm == 0) break;
          const int L = __builtin_ctzll(lm);
          sel |= 1ull << L;
          cand = cand && lane != L;
        }
        pm = sel;
      }
      while (pm) {
        const int L = __builtin_ctzll(pm);
        pm &= pm - 1;
        uint64_t c1 = readlane_u64(k1, L), c2 = readlane_u64(k2, L);
        int32_t cq = q0 + L;
        // insertion into the sorted top-LOOK (scalar)
#pragma unroll
        for (int r = 0; r < LOOK; r++) {
          if (key_lt(c1, c2, tk1[r], tk2[r])) {
            const uint64_t x1 = tk1[r], x2 = tk2[r];
            const int32_t xq = tq[r];
            tk1[r] = c1; tk2[r] = c2; tq[r] = cq;
            c1 = x1; c2 = x2; cq = xq;
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < LOOK; r++) nT += tq[r] >= 0 ? 1 : 0;
    // lane r writes record r of the touched block
    int32_t myq = -1;
    uint64_t my1 = 0;
#pragma unroll
    for (int r = 0; r < LOOK; r++)
      if (lane == r) { myq = tq[r]; my1 = tk1[r]; }
    if (lane < nT) {
      put_rec(R.res, R_T + lane * RREC, __longlong_as_double((long long)my1), S.ltb[myq], S.lid[myq],
              S.lz[myq], myq, S.lown[myq], S.lhp[myq], S.la[0][myq], S.la[1][myq], S.la[2][myq],
              S.la[3][myq]);
    }
  }
  if (lane == 0) {
    if (PART != 2) R.res[R_NU] = nU;
    if (PART != 1) R.res[R_NT] = nT;
  }
}

// A scout fills ring slot i % RING with task i's list head, skipping entries that can no longer
// be picked: best-fit drops every touched host (touched hosts compete through the live table),
// first-fit drops dead ones. Touched-ness only grows, so an entry skipped here is unusable later
// too. The ring holds the first 64 kept entries and the list position after the last of them.
// Then it waits for the walk to reach task i - LOOK and scouts task i.
//
// cost_aware best-fit tasks are scouted by two waves at once (the walker waits for both):
// split_a() waves load the ring and check its entries (part 1), the other PRODUCERS - split_a()
// scan the live touched hosts (part 2, produce_touched). Its many zero-score touched hosts make
// the live scan long; vbp best-fit rarely has live touched hosts, so there the fewer ring
// loaders in flight cost more than the split saves (walk 13.0 -> 19.7 ms;
// profiles/r02f/g11_bench_vbp_bf.log) and one wave does both parts.
#ifndef PVT_SPLIT_CA
#define PVT_SPLIT_CA 4
#endif
#ifndef PVT_SPLIT_VBP
#define PVT_SPLIT_VBP 0
#endif
template <int MODE>
__device__ constexpr int split_a() {
  return MODE == CA_BF ? PVT_SPLIT_CA : MODE == VBP_BF ? PVT_SPLIT_VBP : 0;
}
static_assert(PVT_SPLIT_CA >= 0 && PVT_SPLIT_CA < PRODUCERS, "PVT_SPLIT_CA");
static_assert(PVT_SPLIT_VBP >= 0 && PVT_SPLIT_VBP < PRODUCERS, "PVT_SPLIT_VBP");

template <int MODE>
__device__ void produce_touched(const CommitArgs& A, WalkLDS& S, int pb) {
  const int lane = lane_id();
  for (int i = pb; i < A.nt; i += PRODUCERS - split_a<MODE>()) {
    const int w = widx(A, i);
    const int32_t rv = reinterpret_cast<const int32_t*>(A.L.t + w)[lane & 15];
    const int grp = (MODE == CA_BF && A.rtb) ? __builtin_amdgcn_readfirstlane(A.grp[w]) : 0;
    const int slot = i % RING;
    for (int spin = 0; vload(&S.done) < i - RING + 1; spin++) {
      if (vload(&S.stop) || spin > SPIN_LIMIT) return;
      __builtin_amdgcn_s_sleep(2);
    }
    for (int spin = 0;; spin++) {
      const int c = vload(&S.committed);
      if (c >= 0 && c >= i - LOOK + 1) break;
      if (vload(&S.stop) || spin > SPIN_LIMIT) return;
      __builtin_amdgcn_s_sleep(1);
    }
    cbarrier();
    __builtin_amdgcn_s_setprio(2);
    scout<MODE, 2>(A, S, S.ring[slot], w, 0, rv,
                   (MODE == CA_BF && A.rtb) ? A.rtb + (size_t)grp * A.H : nullptr);
    lds_drain();
    if (lane == 0) publish(&S.flagB[slot], i);
    __builtin_amdgcn_s_setprio(0);
  }
}

template <int MODE>
__device__ void produce(const CommitArgs& A, WalkLDS& S, int pw) {
  constexpr bool BEST = (MODE == CA_BF || MODE == VBP_BF);
  constexpr int SA = split_a<MODE>();
  constexpr int NA = SA ? SA : PRODUCERS;
  if (SA && pw >= SA) { produce_touched<MODE>(A, S, pw - SA); return; }
  const int lane = lane_id();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int i = pw; i < A.nt; i += NA) {
    const int w = widx(A, i);
    const ListEntry* le = A.L.e + (size_t)w * LMAX;
    const int32_t rv = reinterpret_cast<const int32_t*>(A.L.t + w)[lane & 15];
    const int cnt = __builtin_amdgcn_readlane(rv, 8);
    // The first PRE_CHUNKS chunks of the list are in flight while the slot is busy (deep lists
    // full of touched hosts would otherwise cost one HBM round trip per chunk).
    ListEntry e[PRE_CHUNKS];
#pragma unroll
    for (int c = 0; c < PRE_CHUNKS; c++)
      if (c == 0 || c * WAVE < cnt) e[c] = le[c * WAVE + lane];
    const int slot = i % RING;
    // slot free once the walker is done with task i - RING
    for (int spin = 0; vload(&S.done) < i - RING + 1; spin++) {
      if (vload(&S.stop) || spin > SPIN_LIMIT) return;
      __builtin_amdgcn_s_sleep(2);
    }
    RingSlot& R = S.ring[slot];
    int k = 0, next_pos = cnt;
    for (int pos = 0; pos < cnt; pos += WAVE) {
      const int c = pos / WAVE;
      ListEntry x;
      if (c < PRE_CHUNKS) {
#pragma unroll
        for (int u = 0; u < PRE_CHUNKS; u++)
          if (u == c) x = e[u];
      } else {
        x = le[pos + lane];
      }
      bool keep = pos + lane < cnt;
      if (keep) {
        int32_t hp;
        const int32_t hv = wfind(S, x.id, hp);
        keep = BEST ? (hv == H_MISS) : (hv != H_DEAD);
      }
      const uint64_t m = __ballot(keep);
      const int need = WAVE - k;
      const int rank = __popcll(m & below);
      if (keep && rank < need) {
        const int j = k + rank;
        R.s[j] = x.s;
        R.a[0][j] = x.a[0]; R.a[1][j] = x.a[1]; R.a[2][j] = x.a[2]; R.a[3][j] = x.a[3];
        R.id[j] = x.id;
        R.zone[j] = x.zone;
        R.tb[j] = x.tb;
      }
      const int got = __popcll(m);
      if (got >= need) {                     // ring full: stop after the need-th kept entry
        const uint64_t lastm = __ballot(keep && rank == need - 1);
        next_pos = pos + __builtin_ctzll(lastm) + 1;
        k = WAVE;
        break;
      }
      k += got;
    }
    // realtime_bw: the task's group (the walker's patched-host rescoring reads it from rec[18])
    const int grp = (MODE == CA_BF && A.rtb) ? __builtin_amdgcn_readfirstlane(A.grp[w]) : 0;
    if (lane < 16) R.rec[lane] = rv;
    if (lane == 16) R.rec[16] = k;
    if (lane == 17) R.rec[17] = next_pos;
    if (lane == 18) R.rec[18] = grp;
    // the state this task is scouted on: every task <= i - LOOK committed
    for (int spin = 0;; spin++) {
      const int c = vload(&S.committed);
      if (c >= 0 && c >= i - LOOK + 1) break;
      if (vload(&S.stop) || spin > SPIN_LIMIT) return;
      __builtin_amdgcn_s_sleep(1);
    }
    cbarrier();
    // the scout is on the walk's critical path (the walker needs its result one task from now):
    // it outranks the other scouts' list loading, not the walker
    __builtin_amdgcn_s_setprio(2);
    scout<MODE, SA ? 1 : 0>(A, S, R, w, k, rv,
                              (MODE == CA_BF && A.rtb) ? A.rtb + (size_t)grp * A.H : nullptr);
    lds_drain();
    if (lane == 0) publish(&S.flag[slot], i);
    __builtin_amdgcn_s_setprio(0);
  }
}

// ---------------------------------------------------------------- the walker
// Reads dword k of a scout result (lane k / 2 holds dwords k & ~1, k | 1 of `rv`).
__device__ __forceinline__ int32_t rdw(uint64_t rv, int k) {
  return readlane_i((int32_t)(uint32_t)((k & 1) ? (rv >> 32) : rv), k >> 1);
}
__device__ __forceinline__ double rdd(uint64_t rv, int k) {
  return __longlong_as_double((long long)readlane_u64(rv, k >> 1));
}

// The walker's decisions are uniform: every value it branches on is a scalar (readlane of the
// scout's result, scalar state of the patched hosts), so the compiler emits scalar branches and
// the per-task chain is short. NP = LOOK - 1 patched hosts: the winners of the last NP tasks,
// newest first (x[0]); an older entry of a host that won again is stale (not rescored).
constexpr int NP = LOOK - 1;
static_assert(NP >= 1 && NP <= 2, "walker patches one or two hosts");

struct Patched {
  int32_t id, q, z, hp, anc;                // anc: anchor its c / b were read for (-1: none)
  uint32_t tb;
  bool alive;
  double a0, a1, a2, a3, c, b;
};

template <int MODE>
__device__ void walk(const CommitArgs& A, WalkLDS& S) {
  constexpr bool STRICT = (MODE == CA_FF || MODE == VBP_BF);
  constexpr bool BEST = (MODE == CA_BF || MODE == VBP_BF);
  const int lane = lane_id();
  __builtin_amdgcn_s_setprio(3);

  // Componentwise minimum demand of the window: a touched host that cannot fit it is dead.
  double m0 = DINF, m1 = DINF, m2 = DINF, m3 = DINF;
  for (int i = lane; i < A.nt; i += WAVE) {
    const double* dp = A.dem + (size_t)widx(A, i) * 4;
    m0 = fmin(m0, dp[0]); m1 = fmin(m1, dp[1]); m2 = fmin(m2, dp[2]); m3 = fmin(m3, dp[3]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    m0 = fmin(m0, __shfl_xor(m0, off)); m1 = fmin(m1, __shfl_xor(m1, off));
    m2 = fmin(m2, __shfl_xor(m2, off)); m3 = fmin(m3, __shfl_xor(m3, off));
  }
  m0 = readlane_d(m0, 0); m1 = readlane_d(m1, 0); m2 = readlane_d(m2, 0); m3 = readlane_d(m3, 0);

  // Inherited touched hosts: current capacities from HBM (the previous walk has finished).
  for (int k = lane; k < A.n_prev; k += WAVE) {
    const int32_t id = A.prev_ids[k];
    const double a0 = A.avail[id], a1 = A.avail[(size_t)A.H + id];
    const double a2 = A.avail[2 * (size_t)A.H + id], a3 = A.avail[3 * (size_t)A.H + id];
    uint32_t p = wslot(id);
    while (atomicCAS(&S.hk[p].key, H_EMPTY, id) != H_EMPTY) p = (p + 1) & (WH_SLOTS - 1);
    int32_t v = H_DEAD;
    if (fits<STRICT>(a0, a1, a2, a3, m0, m1, m2, m3)) {
      v = atomicAdd(&S.nl_init, 1);
      S.la[0][v] = a0; S.la[1][v] = a1; S.la[2][v] = a2; S.la[3][v] = a3;
      S.lid[v] = id;
      S.lz[v] = A.zone[id];
      S.ltb[v] = A.tb ? A.tb[id] : 0u;
      S.lhp[v] = (int32_t)p;
      S.lown[v] = 0;
    }
    S.hk[p].val = v;
  }
  lds_drain();
  int nl = __builtin_amdgcn_readfirstlane(vload(&S.nl_init));   // live touched hosts
  if (lane == 0) { vstore(&S.nl_pub, nl); vstore(&S.committed, 0); }
  int n_own = 0;
  int status = A.nt;
  // epoch chains: the current segment's start in this walk and in the window, the next start
  int sstart = 0, sk = 1, wbase = 0, snext = A.nt;
  if (A.wlog) { wbase = S.cwin[0]; snext = S.cseg[1]; }
  Patched X[NP];
#pragma unroll
  for (int r = 0; r < NP; r++) {
    X[r].id = -1; X[r].q = -1; X[r].z = 0; X[r].hp = 0; X[r].anc = -1; X[r].tb = 0;
    X[r].alive = false; X[r].a0 = X[r].a1 = X[r].a2 = X[r].a3 = 0.0; X[r].c = 0.0; X[r].b = 1.0;
  }

#ifdef PVT_STAMPS
  uint64_t ph[5] = {0, 0, 0, 0, 0};
  uint64_t nl_sum = 0;
  uint64_t tl = stamp();
#endif
  for (int i = 0; i < A.nt; i++) {
    const int slot = i % RING;
    for (int spin = 0; __builtin_amdgcn_readfirstlane(vload(&S.flag[slot])) != i ||
                       (split_a<MODE>() && __builtin_amdgcn_readfirstlane(vload(&S.flagB[slot])) != i);
         spin++) {
      if (spin > SPIN_LIMIT) { status = -1; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (status < 0) break;
    cbarrier();                               // no slot read may move above the flag poll
    const RingSlot& R = S.ring[slot];
    const int32_t tv = R.rec[lane & 31];
    const uint64_t rs = reinterpret_cast<const uint64_t*>(R.res)[lane];
    const double d0 = rec_d(tv, 0), d1 = rec_d(tv, 1), d2 = rec_d(tv, 2), d3 = rec_d(tv, 3);
    const bool comp = __builtin_amdgcn_readlane(tv, 9) != 0;
    const int anc = __builtin_amdgcn_readlane(tv, 10);
    const int caller = __builtin_amdgcn_readlane(tv, 11);
    const int grp = __builtin_amdgcn_readlane(tv, 18);   // realtime_bw: the task's group
    const int nU = rdw(rs, R_NU);
    STAMP(0);

    auto patched = [&](int32_t id) {
      bool p = false;
#pragma unroll
      for (int r = 0; r < NP; r++) p |= (id == X[r].id);
      return p;
    };
    // the first candidate of each scout list that is not a patched host
    int ub = -1;
#pragma unroll
    for (int r = 0; r < LOOK; r++)
      if (ub < 0 && r < nU && !patched(rdw(rs, R_U + r * RREC + RF_ID))) ub = R_U + r * RREC;
    // the patched hosts that can still take this task (the newest entry of a host only)
    bool xf[NP];
#pragma unroll
    for (int r = 0; r < NP; r++) {
      bool stale = false;
#pragma unroll
      for (int o = 0; o < r; o++) stale |= (X[o].id == X[r].id);
      xf[r] = X[r].id >= 0 && X[r].alive && !stale &&
              fits<STRICT>(X[r].a0, X[r].a1, X[r].a2, X[r].a3, d0, d1, d2, d3);
    }
    int wrec = -1, wx = -1;                   // winner: a scout record, or patched host wx
    bool none = false, refill = false;
    uint64_t wk = 0;                          // best-fit: the winner's score bits
    if (BEST) {
      const int nT = rdw(rs, R_NT);
      int tb_ = -1;
#pragma unroll
      for (int r = 0; r < LOOK; r++)
        if (tb_ < 0 && r < nT && !patched(rdw(rs, R_T + r * RREC + RF_ID))) tb_ = R_T + r * RREC;
      const bool exhausted = ub < 0 && !comp;
      uint64_t t1 = ~0ull, t2 = ~0ull;
      if (ub >= 0) {
        t1 = (uint64_t)__double_as_longlong(rdd(rs, ub + RF_S));
        t2 = ((uint64_t)(MODE == VBP_BF ? (uint32_t)rdw(rs, ub + RF_TB) : 0u) << 32) |
             (uint32_t)rdw(rs, ub + RF_ID);
        wrec = ub;
      } else if (exhausted) {
        // every untouched host outside the list ranks at or after the bound; bid + 1 turns
        // the strict comparisons below into "at or before the bound" (ids are unique)
        t1 = (uint64_t)__double_as_longlong(rec_d(tv, 6));
        t2 = (((uint64_t)(uint32_t)__builtin_amdgcn_readlane(tv, 14)) << 32) +
             (uint32_t)__builtin_amdgcn_readlane(tv, 15) + 1;
      }
      if (tb_ >= 0) {
        const uint64_t c1 = (uint64_t)__double_as_longlong(rdd(rs, tb_ + RF_S));
        const uint64_t c2 = ((uint64_t)(MODE == VBP_BF ? (uint32_t)rdw(rs, tb_ + RF_TB) : 0u) << 32) |
                            (uint32_t)rdw(rs, tb_ + RF_ID);
        if (key_lt(c1, c2, t1, t2)) { t1 = c1; t2 = c2; wrec = tb_; }
      }
      STAMP(1);
      // the patched hosts, rescored exactly (independent chains: the compiler interleaves them)
      uint64_t k1[NP], k2[NP];
#pragma unroll
      for (int r = 0; r < NP; r++) {
        k1[r] = ~0ull; k2[r] = ~0ull;
        if (xf[r]) {
          const double s2 = norm2_seq(X[r].a0 - d0, X[r].a1 - d1, X[r].a2 - d2, X[r].a3 - d3);
          if (MODE == CA_BF) {
            // its zone-table entries for this anchor (realtime_bw: its bandwidth for this group)
            const int ck = A.rtb ? grp : anc;
            if (ck != X[r].anc) {
              X[r].anc = ck;
              X[r].c = S.csum[anc * A.Z + X[r].z];
              X[r].b = A.rtb ? A.rtb[(size_t)grp * A.H + X[r].id] : S.bsum[anc * A.Z + X[r].z];
            }
            k1[r] = ca_score_bits(X[r].c, s2, X[r].b, t1);   // must beat the best so far
          } else {
            k1[r] = (uint64_t)__double_as_longlong(__builtin_sqrt(s2));
          }
          k2[r] = ((uint64_t)(MODE == VBP_BF ? X[r].tb : 0u) << 32) | (uint32_t)X[r].id;
        }
      }
#pragma unroll
      for (int r = 0; r < NP; r++)
        if (xf[r] && key_lt(k1[r], k2[r], t1, t2)) { t1 = k1[r]; t2 = k2[r]; wx = r; wrec = -1; }
      STAMP(2);
      if (wrec < 0 && wx < 0) {
        if (exhausted) refill = true;         // refill from here
        else none = true;                     // no host fits: the task waits
      }
      wk = t1;
    } else {
      // first fit: the first usable entry in list order; a patched one is re-checked exactly
#pragma unroll
      for (int r = 0; r < LOOK; r++) {
        if (wrec >= 0 || wx >= 0 || r >= nU) continue;
        const int32_t id = rdw(rs, R_U + r * RREC + RF_ID);
        int pr = -1;
#pragma unroll
        for (int o = NP - 1; o >= 0; o--) pr = (id == X[o].id) ? o : pr;   // newest entry
        if (pr < 0) {
          wrec = R_U + r * RREC;
        } else {
#pragma unroll
          for (int o = 0; o < NP; o++)
            if (o == pr && xf[o]) wx = o;
        }
      }
      STAMP(1);
      STAMP(2);
      if (wrec < 0 && wx < 0) {
        if (!comp) refill = true;
        else none = true;
      }
    }
    if (refill) { status = i; break; }
    release_slot(S, i + 1);                   // the ring slot is no longer read
    if (i >= snext) {                         // entering the chain's next segment
      while (i >= S.cseg[sk]) { sstart = S.cseg[sk]; wbase = S.cwin[sk]; sk++; }
      snext = S.cseg[sk];
    }
    if (none) {                               // nothing committed: the window slides
      if (lane == 0) {
        A.placement[caller] = -1;             // (an earlier speculative walk may have set it)
        if (A.wlog) { const int w = wbase + i - sstart; A.wlog[w].s = DINF; A.wlog[w].id = -1; A.wlog[w].sup = 0; }
      }
#pragma unroll
      for (int r = NP - 1; r > 0; r--) X[r] = X[r - 1];
      X[0].id = -1; X[0].alive = false; X[0].anc = -1;
      cbarrier();
      if (lane == 0) vstore(&S.committed, i + 1);
      STAMP(3);
      STAMP(4);
      continue;
    }

    // the winner's state
    Patched W;
    int32_t w_own;
    if (wx >= 0) {
#pragma unroll
      for (int r = 0; r < NP; r++)
        if (r == wx) W = X[r];
      w_own = 1;                              // committed to by this walk moments ago
    } else {
      W.id = rdw(rs, wrec + RF_ID); W.q = rdw(rs, wrec + RF_Q); W.z = rdw(rs, wrec + RF_Z);
      W.hp = rdw(rs, wrec + RF_HP); w_own = rdw(rs, wrec + RF_OWN); W.tb = (uint32_t)rdw(rs, wrec + RF_TB);
      W.a0 = rdd(rs, wrec + RF_A); W.a1 = rdd(rs, wrec + RF_A + 2); W.a2 = rdd(rs, wrec + RF_A + 4);
      W.a3 = rdd(rs, wrec + RF_A + 6);
      W.anc = -1; W.c = 0.0; W.b = 1.0;
      // untouched: the scout's probe ended at W.hp (empty then); only a patched host inserted
      // since can have taken that slot -- then probe again
      bool taken = false;
#pragma unroll
      for (int r = 0; r < NP; r++) taken |= (X[r].id >= 0 && X[r].hp == W.hp);
      if (W.q < 0 && taken) {
        int32_t p;
        (void)wfind(S, W.id, p);
        W.hp = __builtin_amdgcn_readfirstlane(p);
      }
    }
    STAMP(3);

    // commit: resc[h] -= t_demand (cost_aware.py:95,126; vbp.py:24,49)
    const double n0 = W.a0 - d0, n1 = W.a1 - d1, n2 = W.a2 - d2, n3 = W.a3 - d3;
    const bool alive = fits<STRICT>(n0, n1, n2, n3, m0, m1, m2, m3);
    if (W.q < 0 && alive && nl >= LIVE_MAX) { status = i; break; }   // table full: refill
    const double nr = lane == 0 ? n0 : lane == 1 ? n1 : lane == 2 ? n2 : n3;
    int32_t q_after = W.q;
    if (W.q < 0) {                            // first commit to this host in the window
      int32_t v = H_DEAD;
      if (alive) {
        v = nl++;
        if (lane < 4) S.la[lane][v] = nr;
        if (lane == 0) { S.lid[v] = W.id; S.lz[v] = W.z; S.ltb[v] = W.tb; S.lhp[v] = W.hp; S.lown[v] = 1; }
      }
      cbarrier();                             // the entry before its hash value (scouts)
      if (lane == 0) {
        S.hk[W.hp].key = W.id;
        cbarrier();
        S.hk[W.hp].val = v;
      }
      cbarrier();
      if (alive && lane == 0) vstore(&S.nl_pub, nl);   // after the entry's writes (in order)
      q_after = alive ? v : -1;
    } else {                                  // a live touched host
      if (alive) {
        if (lane < 4) S.la[lane][W.q] = nr;
        if (lane == 0) S.lown[W.q] = 1;
      } else {                                // dies: marked in place, never moved
        if (lane == 0) { S.la[0][W.q] = -DINF; S.hk[W.hp].val = H_DEAD; }
        q_after = -1;
      }
    }
    if (A.wlog) {                             // epoch walk: logged, applied once validated
      const int w = wbase + i - sstart;
      if (lane < 4) A.wlog[w].a[lane] = nr;
      if (lane == 0) {                        // (sup: set by epoch_final_kernel)
        A.wlog[w].s = __longlong_as_double((long long)wk);
        A.wlog[w].id = W.id;
      }
    } else {
      if (!w_own) {                           // first commit of this walk to the host
        if (lane == 0) A.own_ids[n_own] = W.id;
        n_own++;
      }
      if (lane < 4) A.avail[(size_t)lane * A.H + W.id] = nr;
    }
    if (lane == 0) A.placement[caller] = W.id;
    // the winner becomes the newest patched host (its c / b carry over when it was one)
#pragma unroll
    for (int r = NP - 1; r > 0; r--) X[r] = X[r - 1];
    X[0] = W;
    X[0].q = q_after; X[0].alive = alive;
    X[0].a0 = n0; X[0].a1 = n1; X[0].a2 = n2; X[0].a3 = n3;
    cbarrier();
    if (lane == 0) vstore(&S.committed, i + 1);   // after every LDS write of this commit
#ifdef PVT_STAMPS
    nl_sum += nl;
#endif
    STAMP(4);
  }
  if (lane == 0) {
    vstore(&S.stop, 1);
    A.status[0] = status;
    A.status[1] = n_own;
  }
#ifdef PVT_STAMPS
  if (lane == 0 && A.stamps) {
    for (int k = 0; k < 5; k++) atomicAdd((unsigned long long*)&A.stamps[k], (unsigned long long)ph[k]);
    atomicAdd((unsigned long long*)&A.stamps[5], (unsigned long long)(status < 0 ? 0 : status));
    atomicAdd((unsigned long long*)&A.stamps[6], (unsigned long long)nl_sum);
  }
#endif
}

template <int MODE>
__global__ __launch_bounds__(WALK_THREADS) void commit_kernel(CommitArgs A) {
  if (A.cmap) {                               // epoch walk: this workgroup's chain
    const int b = blockIdx.x;
    const int base = A.coff[b];
    A.nt = A.coff[b + 1] - base;
    A.cmap += base;
    A.status += 2 * b;
    if (A.skip_done && A.status[0] == A.nt) return;   // walked by the zero-cost frontier walk
  }
  extern __shared__ __attribute__((aligned(16))) char smem[];
  WalkLDS& S = *reinterpret_cast<WalkLDS*>(smem);
  const int tid = threadIdx.x;
  // val starts as "not dead": a loader can see a key the walker is inserting before its value
  // (loaders only act on H_DEAD, which is final, so a stale live value is merely conservative)
  for (int i = tid; i < WH_SLOTS; i += WALK_THREADS) { S.hk[i].key = H_EMPTY; S.hk[i].val = H_PENDING; }
  if (MODE == CA_BF)
    for (int i = tid; i < A.Z * A.Z; i += WALK_THREADS) { S.csum[i] = A.csum[i]; S.bsum[i] = A.bsum[i]; }
  if (tid < RING) { S.flag[tid] = -1; S.flagB[tid] = -1; }
  if (A.cmap) {                               // the chain's segment starts (chain-local), then nt
    const int s0 = A.csoff[blockIdx.x], ns = min(A.csoff[blockIdx.x + 1] - s0, MAX_CHAIN_SEGS);
    for (int k = tid; k <= MAX_CHAIN_SEGS; k += WALK_THREADS) {
      S.cseg[k] = k < ns ? A.cseg[s0 + k] : A.nt;
      S.cwin[k] = k < ns ? A.cmap[A.cseg[s0 + k]] : 0;
    }
  }
  if (tid == 0) { S.done = 0; S.stop = 0; S.nl_init = 0; S.nl_pub = 0; S.committed = -1; }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (wave == 0) walk<MODE>(A, S);
  else produce<MODE>(A, S, wave - 1);
}

// The walk asks for the whole CU's LDS so no block of a concurrently running score or merge
// kernel (pipelined windows) is placed on the walker's CU to compete for its issue slots.
constexpr size_t WALK_LDS_BYTES = 160 * 1024;
static_assert(sizeof(WalkLDS) <= WALK_LDS_BYTES, "walk LDS");
size_t commit_lds_bytes() { return WALK_LDS_BYTES; }

hipError_t init_kernel_attrs() {
  const int lds = (int)WALK_LDS_BYTES;
  hipError_t e = hipSuccess, r;
  r = hipFuncSetAttribute((const void*)commit_kernel<CA_FF>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (r != hipSuccess) e = r;
  r = hipFuncSetAttribute((const void*)commit_kernel<CA_BF>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (r != hipSuccess) e = r;
  r = hipFuncSetAttribute((const void*)commit_kernel<VBP_FF>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (r != hipSuccess) e = r;
  r = hipFuncSetAttribute((const void*)commit_kernel<VBP_BF>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (r != hipSuccess) e = r;
  return e;
}

void launch_commit(const CommitArgs& a, hipStream_t st) { launch_commit_chains(a, 1, st); }

void launch_commit_chains(const CommitArgs& a, int nchains, hipStream_t st) {
  const size_t lds = WALK_LDS_BYTES;
  const dim3 grid(nchains), block(WALK_THREADS);
  switch (a.mode) {
    case CA_FF: PVT_LAUNCH(commit_kernel<CA_FF>, grid, block, lds, st, a); break;
    case CA_BF: PVT_LAUNCH(commit_kernel<CA_BF>, grid, block, lds, st, a); break;
    case VBP_FF: PVT_LAUNCH(commit_kernel<VBP_FF>, grid, block, lds, st, a); break;
    case VBP_BF: PVT_LAUNCH(commit_kernel<VBP_BF>, grid, block, lds, st, a); break;
    default: break;
  }
}

}  // namespace pvt
