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
// Execution: ONE workgroup on one CU. Wave 0 is the walker; waves 1..PRODUCERS stream each
// task's list head (64 entries + task record) from HBM into an LDS ring ahead of the walker, so
// the walker's critical path is LDS, cross-lane and scalar work only: it never waits on HBM
// except on the rare deep-list path. Ring hand-off: a producer fills slot i % RING, waits for
// its LDS writes (lgkmcnt 0) and publishes flag[slot] = i; the walker publishes done = i + 1
// when task i no longer needs its slot. Every spin is bounded; a timeout reports status -1.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"
#include "pvt_kernels.h"

namespace pvt {

constexpr int RING = 16;                  // ring slots (task lists in LDS)
constexpr int PRODUCERS = 8;              // loader waves
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

struct RingSlot {
  double s[WAVE];
  double a[4][WAVE];
  int32_t id[WAVE];
  int32_t zone[WAVE];
  uint32_t tb[WAVE];
  int32_t rec[32];                        // TaskRec dwords 0-15, [16] ring entries,
};                                        // [17] list position after the last one

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
  double csum[ZMAX * ZMAX];
  double bsum[ZMAX * ZMAX];
  int32_t flag[RING];
  int32_t done;
  int32_t stop;
  int32_t nl_init;
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

// ---------------------------------------------------------------- loader waves
// A loader copies task i's list into ring slot i % RING, skipping entries that can no longer
// be picked: best-fit drops every touched host (touched hosts compete through the live table),
// first-fit drops dead ones. Touched-ness only grows, so an entry skipped here is unusable for
// the walker too; one the loader keeps is checked again by the walker. The ring holds the first
// 64 kept entries and the list position after the last of them (the walker's deep search, if
// needed, continues from there).
template <int MODE>
__device__ void produce(const CommitArgs& A, WalkLDS& S, int pw) {
  constexpr bool BEST = (MODE == CA_BF || MODE == VBP_BF);
  const int lane = lane_id();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int i = pw; i < A.nt; i += PRODUCERS) {
    const ListEntry* le = A.L.e + (size_t)i * LMAX;
    const int32_t rv = reinterpret_cast<const int32_t*>(A.L.t + i)[lane & 15];
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
    if (lane < 16) R.rec[lane] = rv;
    if (lane == 16) R.rec[16] = k;
    if (lane == 17) R.rec[17] = next_pos;
    lds_drain();
    if (lane == 0) publish(&S.flag[slot], i);
  }
}

// ---------------------------------------------------------------- the walker
// Everything the walk decides is wave-uniform; values are moved to scalar registers
// (readlane / readfirstlane) as soon as they are known, so branches stay scalar and no vector
// register carries a pending HBM load across the per-task loop.
template <int MODE>
__device__ void walk(const CommitArgs& A, WalkLDS& S) {
  constexpr bool STRICT = (MODE == CA_FF || MODE == VBP_BF);
  constexpr bool BEST = (MODE == CA_BF || MODE == VBP_BF);
  const int lane = lane_id();
  __builtin_amdgcn_s_setprio(3);

  // Componentwise minimum demand of the window: a touched host that cannot fit it is dead.
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
  int n_own = 0;
  int status = A.nt;

#ifdef PVT_STAMPS
  uint64_t ph[5] = {0, 0, 0, 0, 0};
  uint64_t nl_sum = 0;
  uint64_t tl = stamp();
#endif
  for (int i = 0; i < A.nt; i++) {
    const int slot = i % RING;
    for (int spin = 0; __builtin_amdgcn_readfirstlane(vload(&S.flag[slot])) != i; spin++) {
      if (spin > SPIN_LIMIT) { status = -1; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (status < 0) break;
    cbarrier();                               // no slot read may move above the flag poll
    const RingSlot& R = S.ring[slot];
    const int32_t tv = R.rec[lane & 31];
    const int32_t e_id = R.id[lane];
    const double e_s = R.s[lane];
    const uint32_t e_tb = R.tb[lane];
    const int32_t e_z = R.zone[lane];
    const double e0 = R.a[0][lane], e1 = R.a[1][lane], e2 = R.a[2][lane], e3 = R.a[3][lane];
    const double d0 = rec_d(tv, 0), d1 = rec_d(tv, 1), d2 = rec_d(tv, 2), d3 = rec_d(tv, 3);
    const int cnt = __builtin_amdgcn_readlane(tv, 8);
    const bool comp = __builtin_amdgcn_readlane(tv, 9) != 0;
    const int anc = __builtin_amdgcn_readlane(tv, 10);
    const int caller = __builtin_amdgcn_readlane(tv, 11);
    const int rcnt = __builtin_amdgcn_readlane(tv, 16);
    const int npos = __builtin_amdgcn_readlane(tv, 17);
    STAMP(0);

    // touched-ness of the ring entries (lane j: entry j)
    const bool valid = lane < rcnt;
    int32_t hp = 0;
    const int32_t hv = valid ? wfind(S, e_id, hp) : H_MISS;
    bool usable;
    if (BEST) {
      usable = valid && hv == H_MISS;
    } else {
      const int q = hv >= 0 ? hv : 0;
      usable = valid && (hv == H_MISS ||
                         (hv >= 0 && fits<STRICT>(S.la[0][q], S.la[1][q], S.la[2][q], S.la[3][q],
                                                  d0, d1, d2, d3)));
    }
    const uint64_t um = __ballot(usable);
    STAMP(1);

    // the first usable entry: (us, utb, uid), zone, snapshot capacities, hash value/position
    bool found = um != 0;
    double us = DINF, ua0 = 0, ua1 = 0, ua2 = 0, ua3 = 0;
    uint32_t utb = 0xffffffffu;
    int32_t uid = 0x7fffffff, uz = 0, uhv = H_MISS, uhp = 0;
    if (found) {
      const int ul = __builtin_ctzll(um);
      uid = readlane_i(e_id, ul); uhv = readlane_i(hv, ul); uhp = readlane_i(hp, ul);
      us = readlane_d(e_s, ul); utb = readlane_u(e_tb, ul); uz = readlane_i(e_z, ul);
      ua0 = readlane_d(e0, ul); ua1 = readlane_d(e1, ul);
      ua2 = readlane_d(e2, ul); ua3 = readlane_d(e3, ul);
    } else {
      // Deep list (rare): search the entries after the ring's by id in HBM, then read the
      // first usable one. Loaded values are consumed (moved to scalars) right here.
      const int32_t* ids = A.L.ids + (size_t)i * LMAX;
      for (int c0 = npos; c0 < cnt && !found; c0 += WAVE) {
        const bool v = c0 + lane < cnt;
        const int32_t id = v ? ids[c0 + lane] : 0;
        int32_t p2 = 0;
        const int32_t h2 = v ? wfind(S, id, p2) : H_MISS;
        bool ok;
        if (BEST) {
          ok = v && h2 == H_MISS;
        } else {
          const int q = h2 >= 0 ? h2 : 0;
          ok = v && (h2 == H_MISS ||
                     (h2 >= 0 && fits<STRICT>(S.la[0][q], S.la[1][q], S.la[2][q], S.la[3][q],
                                              d0, d1, d2, d3)));
        }
        const uint64_t mc = __ballot(ok);
        if (mc) {
          const int ul = __builtin_ctzll(mc);
          found = true;
          uhv = readlane_i(h2, ul);
          uhp = readlane_i(p2, ul);
          const ListEntry* ue = A.L.e + (size_t)i * LMAX + c0 + ul;
          const double f = (lane < 4) ? ue->a[lane] : (lane == 4) ? ue->s : 0.0;
          const int32_t g = (lane == 0) ? ue->id : (lane == 1) ? ue->zone : (int32_t)ue->tb;
          ua0 = readlane_d(f, 0); ua1 = readlane_d(f, 1); ua2 = readlane_d(f, 2);
          ua3 = readlane_d(f, 3); us = readlane_d(f, 4);
          uid = readlane_i(g, 0); uz = readlane_i(g, 1); utb = readlane_u((uint32_t)g, 2);
        }
      }
    }
    STAMP(2);

    // the winner: hash value (live index / H_MISS), hash position, capacities, zone, tiebreak,
    // and whether this walk committed to it before
    int32_t w_id, w_hv, w_hp, w_z, w_own = 0;
    uint32_t w_tb;
    double w0, w1, w2, w3;
    if (BEST) {
      // Best so far as a 128-bit key (score bits, tiebreak:id): scores are >= +0, so their bit
      // patterns order like the values, and one unsigned compare pair replaces lexless.
      const bool exhausted = !found && !comp;
      uint64_t t1 = (uint64_t)__double_as_longlong(us);
      uint64_t t2 = ((uint64_t)utb << 32) | (uint32_t)uid;
      if (exhausted) {
        // every untouched host outside the list ranks at or after the bound; bid + 1 turns
        // the strict comparison below into "at or before the bound" (ids are unique)
        t1 = (uint64_t)__double_as_longlong(rec_d(tv, 6));
        t2 = (((uint64_t)(uint32_t)__builtin_amdgcn_readlane(tv, 14)) << 32) +
             (uint32_t)__builtin_amdgcn_readlane(tv, 15) + 1;
      }
      int bq = -1;
      double b0 = 0, b1 = 0, b2 = 0, b3 = 0;
      int32_t bz = 0, bhp = 0, bown = 0;
      uint32_t btb = 0;
#ifdef PVT_STAMPS
      nl_sum += nl;
#endif
      for (int q0 = 0; q0 < nl; q0 += WAVE) {
        const int q = q0 + lane;
        const int qq = min(q, nl - 1);
        const double a0 = S.la[0][qq], a1 = S.la[1][qq], a2 = S.la[2][qq], a3 = S.la[3][qq];
        const int32_t lidq = S.lid[qq], lzq = S.lz[qq], lhq = S.lhp[qq], loq = S.lown[qq];
        const uint32_t ltq = (MODE == VBP_BF) ? S.ltb[qq] : 0u;
        const bool fit = (q < nl) && fits<STRICT>(a0, a1, a2, a3, d0, d1, d2, d3);
        if (__ballot(fit) == 0) continue;
        const double s2 = norm2_seq(a0 - d0, a1 - d1, a2 - d2, a3 - d3);
        double sc;
        if (MODE == CA_BF) {
          sc = (S.csum[anc * A.Z + lzq] * __builtin_sqrt(s2)) / S.bsum[anc * A.Z + lzq];
        } else {
          sc = __builtin_sqrt(s2);
        }
        const uint64_t k1 = (uint64_t)__double_as_longlong(sc);
        const uint64_t k2 = ((uint64_t)ltq << 32) | (uint32_t)lidq;
        uint64_t pm = __ballot(fit && (k1 < t1 || (k1 == t1 && k2 < t2)));
        while (pm) {
          const int L = __builtin_ctzll(pm);
          pm &= pm - 1;
          const uint64_t c1 = readlane_u64(k1, L), c2 = readlane_u64(k2, L);
          if ((c1 < t1) | ((c1 == t1) & (c2 < t2))) {
            t1 = c1; t2 = c2; bq = q0 + L;
            b0 = readlane_d(a0, L); b1 = readlane_d(a1, L); b2 = readlane_d(a2, L); b3 = readlane_d(a3, L);
            bz = readlane_i(lzq, L); bhp = readlane_i(lhq, L); bown = readlane_i(loq, L);
            btb = readlane_u(ltq, L);
          }
        }
      }
      STAMP(3);
      if (exhausted && bq < 0) { status = i; break; }              // refill from here
      if (!found && bq < 0) { release_slot(S, i + 1); continue; }  // no host fits: waits
      if (bq >= 0) {
        w_id = (int32_t)(uint32_t)t2; w_hv = bq; w_hp = bhp; w_z = bz; w_tb = btb; w_own = bown;
        w0 = b0; w1 = b1; w2 = b2; w3 = b3;
      } else {
        w_id = uid; w_hv = H_MISS; w_hp = uhp; w_z = uz; w_tb = utb;
        w0 = ua0; w1 = ua1; w2 = ua2; w3 = ua3;
      }
    } else {
      if (!found) {
        if (!comp) { status = i; break; }
        release_slot(S, i + 1);
        continue;
      }
      w_id = uid; w_hv = uhv; w_hp = uhp; w_z = uz; w_tb = utb;
      if (uhv >= 0) {                         // a live touched host that still fits
        const double f = (lane < 4) ? S.la[lane][uhv] : 0.0;
        w0 = readlane_d(f, 0); w1 = readlane_d(f, 1); w2 = readlane_d(f, 2); w3 = readlane_d(f, 3);
        w_own = __builtin_amdgcn_readfirstlane(S.lown[uhv]);
      } else {
        w0 = ua0; w1 = ua1; w2 = ua2; w3 = ua3;
      }
    }
    release_slot(S, i + 1);                   // the ring slot is no longer read

    // commit: resc[h] -= t_demand (cost_aware.py:95,126; vbp.py:24,49)
    const double n0 = w0 - d0, n1 = w1 - d1, n2 = w2 - d2, n3 = w3 - d3;
    const bool alive = fits<STRICT>(n0, n1, n2, n3, m0, m1, m2, m3);
    if (w_hv == H_MISS && alive && nl >= LIVE_MAX) { status = i; break; }   // table full: refill
    const double nr = lane == 0 ? n0 : lane == 1 ? n1 : lane == 2 ? n2 : n3;
    if (w_hv == H_MISS) {                     // first commit to this host in the window
      int32_t v = H_DEAD;
      if (alive) {
        v = nl++;
        if (lane < 4) S.la[lane][v] = nr;
        if (lane == 0) { S.lid[v] = w_id; S.lz[v] = w_z; S.ltb[v] = w_tb; S.lhp[v] = w_hp; S.lown[v] = 1; }
      }
      if (lane == 0) {
        S.hk[w_hp].key = w_id;
        S.hk[w_hp].val = v;
      }
    } else {                                  // a live touched host
      const int q = w_hv;
      if (alive) {
        if (lane < 4) S.la[lane][q] = nr;
        if (lane == 0) S.lown[q] = 1;
      } else {                                // swap-remove from the live table
        const int last = --nl;
        if (q != last) {
          const double mv = S.la[lane & 3][last];
          const int32_t mid = S.lid[last], mz = S.lz[last], mhp = S.lhp[last], mo = S.lown[last];
          const uint32_t mtb = S.ltb[last];
          if (lane < 4) S.la[lane][q] = mv;
          if (lane == 0) {
            S.lid[q] = mid; S.lz[q] = mz; S.ltb[q] = mtb; S.lhp[q] = mhp; S.lown[q] = mo;
            S.hk[mhp].val = q;
          }
        }
        if (lane == 0) S.hk[w_hp].val = H_DEAD;
      }
    }
    if (!w_own) {                             // first commit of this walk to the host
      if (lane == 0) A.own_ids[n_own] = w_id;
      n_own++;
    }
    if (lane < 4) A.avail[(size_t)lane * A.H + w_id] = nr;
    if (lane == 0) A.placement[caller] = w_id;
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
  extern __shared__ __attribute__((aligned(16))) char smem[];
  WalkLDS& S = *reinterpret_cast<WalkLDS*>(smem);
  const int tid = threadIdx.x;
  if (tid == 0 && A.started)    // this CU is ours: the next window's scoring may start
    __hip_atomic_store(A.started, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // val starts as "not dead": a loader can see a key the walker is inserting before its value
  // (loaders only act on H_DEAD, which is final, so a stale live value is merely conservative)
  for (int i = tid; i < WH_SLOTS; i += WALK_THREADS) { S.hk[i].key = H_EMPTY; S.hk[i].val = H_PENDING; }
  if (MODE == CA_BF)
    for (int i = tid; i < A.Z * A.Z; i += WALK_THREADS) { S.csum[i] = A.csum[i]; S.bsum[i] = A.bsum[i]; }
  if (tid < RING) S.flag[tid] = -1;
  if (tid == 0) { S.done = 0; S.stop = 0; S.nl_init = 0; }
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

void launch_commit(const CommitArgs& a, hipStream_t st) {
  const size_t lds = WALK_LDS_BYTES;
  const dim3 grid(1), block(WALK_THREADS);
  switch (a.mode) {
    case CA_FF: hipLaunchKernelGGL(commit_kernel<CA_FF>, grid, block, lds, st, a); break;
    case CA_BF: hipLaunchKernelGGL(commit_kernel<CA_BF>, grid, block, lds, st, a); break;
    case VBP_FF: hipLaunchKernelGGL(commit_kernel<VBP_FF>, grid, block, lds, st, a); break;
    case VBP_BF: hipLaunchKernelGGL(commit_kernel<VBP_BF>, grid, block, lds, st, a); break;
    default: break;
  }
}

}  // namespace pvt
