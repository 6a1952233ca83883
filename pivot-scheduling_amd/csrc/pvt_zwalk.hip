// pvt_zwalk.hip — the zero-cost frontier walk of an epoch chain (cost_aware best-fit).
//
// A cost_aware best-fit task takes the host of minimum key (score, index), score =
// (c * ||avail - d||) / bw (scheduler/cost_aware.py:85-97). Hosts in a zone its anchor reaches
// at zero egress cost (csum = 0) score exactly +0, the smallest key, so while one of them fits,
// the winner is simply the LOWEST-INDEX fitting host of those zones. An epoch chain
// (pvt_epoch.hip) holds the groups anchored in one zero-cost component, whose tasks pile onto
// the first hosts of the component's zones (config 5: the 1500 tasks of the longest chain use
// fewer than 200 of them). This kernel walks such a chain without candidate lists:
//
//   window   the first ZW_M hosts, in index order, of the zones U = the union of the chain's
//            anchors' zero-cost zones, with their capacities at the epoch start, in LDS;
//   task     the first window host (index order) that fits and scores exactly 0 -- found 64
//            hosts per step by one wave (a ballot) -- is committed in LDS and logged (WinRec);
//
// exactly the host the sequential reference picks, given three certificates checked here
// (any failure: the chain is left to the list-based walk, which then runs for it):
//
//   (1) a winner exists in the window: every zero-cost host of lower index is in the window
//       (U contains the anchor's zero-cost zones; the window is U's index-order prefix);
//   (2) no host outside U scores 0: for every zone z outside U, c = csum[a][z] >= 2^-300 and
//       bw = bsum[a][z] <= 2^300, and some capacity dimension r separates hosts from tasks,
//       min_h avail[r][h] - max_t d[r] >= 2^-288 (so s2 >= fl(x_r^2) >= 2^-578 for every such
//       pair and the score is >= 2^-900 > 0 -- the same bound ca_score_bits uses); hosts outside
//       U are never committed to by this walk, so their epoch-start state is their state;
//   (3) zero-cost scores are exactly +0: bw > 0 for the anchor's zero-cost zones and every
//       window capacity and chain demand is finite with |x| <= 2^500 (s2 finite);
//
// and window hosts of U outside the anchor's zero-cost zones are scored exactly (ca_score_bits,
// a key of 0 only when the score's bits are 0). The log and the chain's progress have the
// format of the list walk's chain mode, so validation, finality and apply are unchanged.
//
// FF: the same chain walk for cost_aware FIRST-fit with sort_hosts (scheduler/cost_aware.py:
// 99-127). A group's hosts are taken in the order of the frozen key c*df/(||avail||*bw); hosts
// of the anchor's zero-cost zones have key exactly 0 and lead that order in index order, so
// while one of them strictly fits, the winner is the lowest-index such host -- the same window,
// with strict fit, and fitting U hosts of other zones simply skipped (their key is > 0).
// Certificates: (1) as above; (2') every zone has c == 0 with bw > 0 (key exactly 0 for r > 0)
// or c >= 2^-300 with bw <= 2^300, and every host capacity is at most 2^298 (so r <= 2^299 and
// a positive key is >= 2^-899, never 0); (3') as (3), and the chain's demands are >= 0 (a host
// that strictly fits then has r > 0). Chains of different zero-cost components commit to
// disjoint hosts, none of which is zero-key for another component's anchors, so every chain's
// proven prefix is exact in the sequential order too (pvt_capi.hip ff_epoch: no validation).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pivot_place.h"
#include "pvt_device.h"
#include "pvt_kernels.h"
#include "pvt_zwin_dev.h"

namespace pvt {

constexpr int ZW_MBIG = 3072;              // the large window (a retry for chains that outgrow ZW_M)
constexpr int ZW_THREADS = 256;
constexpr int ZW_WAVES = ZW_THREADS / 64;
constexpr int ZW_SCAN = 8;                 // 16-byte zone loads (4 hosts) per thread per window-build pass
constexpr int ZW_MINB = ZW_MIN_PARTS;      // blocks of the host-minimum pass
constexpr int ZW_PR = 8;                   // chain task rows per thread per prologue pass
constexpr double ZW_BIG = 0x1p500;

#ifndef PVT_ZW_UNROLL
#define PVT_ZW_UNROLL 8
#endif
#ifndef PVT_ZW_CF
// run_bulk pass 1 in certified closed form (copies_cf): correct (t_zw green with it on) but not
// faster -- config 5 ca_bf 0.218 vs 0.210-0.215 ms, 243 of 360 runs certified; the quotient,
// the exponent tests and the certification cost about what the copy-by-copy pass does for the
// two iterations a run takes. Off by default, kept for A/B (-DPVT_ZW_CF=1).
#define PVT_ZW_CF 0
#endif
constexpr int ZW_UNROLL = PVT_ZW_UNROLL;   // run_bulk pass 1: copies per stop check
constexpr int ZW_SB = 64;                  // suffix-minimum batches (the last one holds the rest)
template <int WM>
struct ZwalkLDS {
  double wa[4][WM];                        // window capacities (live)
  int32_t wid[WM];                         // window hosts (ascending index)
  int32_t wz[WM];                          // their zones
  uint64_t zm[WM / 64];                    // current anchor: zero-cost window hosts, per chunk
  double csum[ZMAX * ZMAX], bsum[ZMAX * ZMAX];
  int32_t cnt[ZW_SCAN][ZW_WAVES];          // window build: hits per (pass row, wave)
  double red[ZW_WAVES][12];                // block reductions: max d, min d, min avail
  double smin[ZW_SB][4];                   // suffix minima of the demands, per 64-task batch
  double lg[128][4];                       // the batch's log: capacities after each commit
  int32_t lgid[128];                       //   and the host (64.. : a run carried into the next batch)
  int32_t rwho[64], rstart[64];            // run_bulk: host / start flag per run position
  uint64_t sbits[CHAIN_MAX / 64];          // chain mode: bit i = a group segment starts at task i
  uint32_t amask[ZMAX];                    // anchor -> its zero-cost zones
  uint32_t umask;
  int32_t nwin, bail;
};

// Wave reductions of doubles, uniform results: DPP row prefix steps (lane 15 of each 16-lane row
// then holds the row's result), then the four rows by readlane -- no LDS permutes.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = dpp_u32<CTRL>((uint32_t)b, (uint32_t)b);
  const uint32_t hi = dpp_u32<CTRL>((uint32_t)(b >> 32), (uint32_t)(b >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <class Op>
__device__ __forceinline__ double wave_reduce_d(double v, Op op) {
  v = op(v, dpp_d<DPP_ROW_SHR1>(v));
  v = op(v, dpp_d<DPP_ROW_SHR2>(v));
  v = op(v, dpp_d<DPP_ROW_SHR4>(v));
  v = op(v, dpp_d<DPP_ROW_SHR8>(v));
  const double r0 = readlane_d(v, 15), r1 = readlane_d(v, 31);
  const double r2 = readlane_d(v, 47), r3 = readlane_d(v, 63);
  return op(op(r0, r1), op(r2, r3));
}
__device__ __forceinline__ double wave_max_d(double v) {
  return wave_reduce_d(v, [](double a, double b) { return fmax(a, b); });
}
// NaN-propagating maximum (fmax drops a NaN operand): the FF certificate (2') must fail on a NaN
// capacity, whose frozen key would break the reference's sorted() order (cost_aware.py:116).
__device__ __forceinline__ double nan_max(double a, double b) {
  return (a != a || b <= a) ? a : b;
}
__device__ __forceinline__ double wave_nmax_d(double v) {
  return wave_reduce_d(v, [](double a, double b) { return nan_max(a, b); });
}
__device__ __forceinline__ double wave_min_d(double v) {
  return wave_reduce_d(v, [](double a, double b) { return fmin(a, b); });
}

// Per-dimension minimum capacity over hosts [lo, hi) (certificate 2), ZW_MINB partials.
__global__ __launch_bounds__(256) void host_min_kernel(const double* avail, int H, int lo, int hi,
                                                       double* part) {
  __shared__ double red[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double m[4] = {DINF, DINF, DINF, DINF};
  for (int h = lo + blockIdx.x * 256 + tid; h < hi; h += gridDim.x * 256)
#pragma unroll
    for (int r = 0; r < 4; r++) m[r] = fmin(m[r], avail[(size_t)r * H + h]);
#pragma unroll
  for (int r = 0; r < 4; r++) {
    m[r] = wave_min_d(m[r]);
    if (lane == 0) red[wave][r] = m[r];
  }
  __syncthreads();
  if (tid < 4) {
    double v = red[0][tid];
    for (int w = 1; w < 4; w++) v = fmin(v, red[w][tid]);
    part[blockIdx.x * 4 + tid] = v;
  }
}

// Fit from the minimum residual min(a - d): a >= d (best-fit) or a > d (first-fit, strict) in
// every dimension; exact in sign for finite values (certificate 3).
template <int N> struct IntC { static constexpr int value = N; };

// ---- closed-form copy counts (run_bulk pass 1) ----------------------------------------------
// Copies of a demand d > 0 a capacity x takes, subtracting sequentially: c = the largest j with
// fit(x_j), x_j = fl(x_{j-1} - d) (fit: x_j >= 0, or > 0 STRICT). In exact arithmetic that is
// floor(x / d) (STRICT: ceil(x / d) - 1). The estimate k from an approximate quotient is certified
// against the sequential values without computing them: e_j = x - j d exactly, and
//  * "nice" pairs -- x and d multiples of a power of two Q with every x - j d (j <= k + 1) below
//    2^53 Q in magnitude (cpu counts, whole MiB) -- subtract exactly: x_j == e_j, so fit(e_k) and
//    !fit(e_{k+1}) decide;
//  * otherwise |x_j - e_j| <= j 2^-53 (|x| + j d) (one rounding per subtraction, intermediates
//    below |x| + j d): e_k and e_{k+1} must clear twice that bound on their side of 0.
// Anything else is "unsure" and the caller subtracts copy by copy. (x >= d > 0 here: the lane
// fits one copy; counts are capped at ZW_CAP, more than any run takes.)
constexpr int ZW_CAP = 128;
__device__ __forceinline__ int lowbit_exp(double v) {   // exponent of v's lowest set bit (0: big)
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint64_t m = b & ((1ull << 52) - 1);
  const int e = (int)((b >> 52) & 0x7ff);
  if (e == 0) return m ? -1074 + __builtin_ctzll(m) : 4096;
  return (e - 1075) + __builtin_ctzll(m | (1ull << 52));
}
__device__ __forceinline__ int high_exp(double v) {     // floor(log2 |v|) for normal v > 0
  return (int)(((uint64_t)__double_as_longlong(v) >> 52) & 0x7ff) - 1023;
}
template <bool STRICT>
__device__ __forceinline__ int copies_cf(double x, double d, bool& sure) {
  if (__double_as_longlong(d) == 0) return ZW_CAP;      // (+0: the dimension never binds)
  const double q = x * __builtin_amdgcn_rcp(d);
  double kf = STRICT ? __builtin_ceil(q) - 1.0 : __builtin_floor(q);
  kf = __builtin_fmin(kf, (double)ZW_CAP);
  const double e0 = __builtin_fma(-kf, d, x), e1 = __builtin_fma(-(kf + 1.0), d, x);
  const double big = __builtin_fabs(x) + (kf + 1.0) * d;
  const bool nice = high_exp(big) + 2 <= min(lowbit_exp(x), lowbit_exp(d)) + 53;
  const double err = nice ? 0.0 : (kf + 2.0) * 0x1p-52 * (big + d);
  const bool fit0 = STRICT ? (e0 > err) : (e0 >= err && (nice || e0 > err));
  const bool out1 = kf >= (double)ZW_CAP || (STRICT ? (e1 <= -err && (nice || e1 < -err)) : (e1 < -err));
  sure = sure && kf >= 1.0 && fit0 && out1 && (q == q);
  return (int)kf;
}

// A branch condition the wave holds uniformly: through readfirstlane, so that the compiler's
// divergence analysis (which loses track across this walk's nested loops) keeps the branch scalar
// instead of building exec-mask loops around it.
#define UNI(c) (__builtin_amdgcn_readfirstlane((int)(c)) != 0)

template <bool STRICT>
__device__ __forceinline__ bool fit_res(double m) { return STRICT ? (m > 0.0) : (m >= 0.0); }

// One wave orders its LDS stores before its later loads (compiler fence + lgkmcnt(0)).
__device__ __forceinline__ void wave_lds_sync() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// The first WM hosts of [h_lo, h_hi), in index order, whose zone is in the mask U
// (pvt_zwin_dev.h, with this walk's workgroup and ZW_SCAN rows per pass).
template <int WM = ZW_M>
__device__ __forceinline__ void compact_zone_window(const int32_t* zone, int Z, uint32_t U,
                                                    int h_lo, int h_hi, int32_t* wid, int32_t* wz,
                                                    int32_t (*cnt)[ZW_WAVES], int32_t* nwin) {
  compact_zone_window_t<WM, ZW_THREADS, ZW_SCAN>(zone, Z, U, h_lo, h_hi, wid, wz, cnt, nwin);
}

#ifdef PVT_STAMPS
__device__ __forceinline__ uint64_t zstamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif

// KEYED: cost_aware first-fit with sort_hosts (pvt_capi.hip keyed_frontier): one group, its
// window the first ZW_M hosts of the group's zero-key prefix (perm, index order), strict fit,
// no zone certificates (the order is the keyed path's own); the window's capacities are written
// back at the end and status[0] = tasks walked.
// KEYED with STRICT = false: vbp first-fit (index order, fit >=) over a window of the first
// alive hosts (pvt_capi.hip ordered_frontier), same mechanics.
template <bool KEYED, bool STRICT, bool FF = false, int WM = ZW_M>
__global__ __launch_bounds__(ZW_THREADS) void zwalk_kernel(ZwalkArgs A) {
  static_assert(!FF || (!KEYED && STRICT), "FF: chain mode, strict fit");
  static_assert(WM == ZW_M || !KEYED, "keyed / ordered / sharded windows: ZW_M hosts");
  __shared__ ZwalkLDS<WM> S;
#ifdef PVT_STAMPS
  const uint64_t t_start = zstamp();
  uint64_t n_chunks = 0, n_switch = 0, n_bulk = 0, n_runs = 0;
  uint64_t st_search = 0, st_p1 = 0, st_p2 = 0, n_probe = 0, n_iter = 0, st_batch = 0, n_single = 0;
  uint64_t st_setup = 0, st_loop = 0, st_who = 0, st_rep = 0;   // run_bulk's parts
  uint64_t n_cf = 0;                                              // runs counted in closed form
#endif
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // chain tables: by value in the arguments (A.tab; the host sends them only for chains of at
  // most CHAIN_MAX tasks, as the epoch planner builds them), or device arrays (uploaded)
  const bool tabm = !KEYED && A.tab.nch > 0;
  const int base = KEYED ? 0 : tabm ? A.tab.coff[b] : A.coff[b];
  const int nt = KEYED ? A.knt : tabm ? A.tab.coff[b + 1] - A.tab.coff[b] : A.coff[b + 1] - base;
  // chain-local position -> epoch task (A.cmap, global): with the tables by value, this block
  // writes its chain's range of it from the segments first (read back by the same block after the
  // barrier below; the prologue's first positions come from the segments directly). (Neither a map in LDS -- the select between an LDS and a global map became a
  // flat load per access -- nor one computed from the segments per access: the walk ran 4-7 %
  // slower either way.)
  const int32_t* gcmap = KEYED ? nullptr : A.cmap + base;
  auto cmap_at = [&](int i) -> int { return gcmap[i]; };
  const bool segm = !KEYED && (tabm || A.cseg);   // group segment starts break runs
  int32_t* status = A.status + 2 * b;
  const int Z = A.Z, H = A.H;

  // Every load the prologue needs that depends on nothing else is issued first (the zone
  // tables, the host minima, the chain's first task positions, its segment range), so the
  // prologue waits for about two HBM latencies, not one per step.
  static_assert(ZMAX * ZMAX <= 4 * ZW_THREADS && ZW_MINB == ZW_THREADS, "prologue loads");
  const int ZZ = KEYED ? 0 : Z * Z;
  double cs[4], bs[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int i = tid + u * ZW_THREADS;
    cs[u] = i < ZZ ? A.csum[i] : 0.0;
    bs[u] = i < ZZ ? A.bsum[i] : 0.0;
  }
  // host minima (FF: maxima of |capacity|) from the partials
  double ha[4] = {FF ? -DINF : DINF, FF ? -DINF : DINF, FF ? -DINF : DINF, FF ? -DINF : DINF};
  if (!KEYED) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const double x = A.hmin[tid * 4 + r];
      ha[r] = FF ? nan_max(ha[r], x) : fmin(ha[r], x);
    }
  }
  if (tabm) {
    int32_t* wmap = const_cast<int32_t*>(A.cmap) + base;
    for (int k = A.tab.csoff[b]; k < A.tab.csoff[b + 1]; k++) {
      const int sg = A.tab.csegid[k], c0 = A.tab.seg_cstart[sg], o0 = A.tab.seg_off[sg];
      const int len = A.tab.seg_off[sg + 1] - o0;
      for (int i = tid; i < len; i += ZW_THREADS) wmap[c0 + i] = o0 + i;
    }
    // block 0 publishes the tables for the epoch kernels after the walk
    if (b == 0) {
      const int ns = A.tab.nseg, nc = A.tab.nch;
      for (int i = tid; i <= ns; i += ZW_THREADS) {
        A.tab.o_seg_off[i] = A.tab.seg_off[i];
        if (i < ns) { A.tab.o_seg_chain[i] = A.tab.seg_chain[i]; A.tab.o_seg_cstart[i] = A.tab.seg_cstart[i]; }
      }
      for (int i = tid; i <= nc; i += ZW_THREADS) A.tab.o_coff[i] = A.tab.coff[i];
    }
  }
  int wv[ZW_PR];
  if (tabm) {
    // the first positions straight from the segments (no dependent load of the map before the
    // demand rows: one HBM latency less in the prologue)
    const int k0 = A.tab.csoff[b], k1 = A.tab.csoff[b + 1];
#pragma unroll
    for (int u = 0; u < ZW_PR; u++) {
      const int i = u * ZW_THREADS + tid;
      int v = -1;
      for (int k = k0; k < k1; k++) {
        const int sg = A.tab.csegid[k], c0 = A.tab.seg_cstart[sg];
        if (i >= c0) v = A.tab.seg_off[sg] + (i - c0);
      }
      wv[u] = i < nt ? v : -1;
    }
  } else {
#pragma unroll
    for (int u = 0; u < ZW_PR; u++) {
      const int i = u * ZW_THREADS + tid;
      wv[u] = i < nt ? (KEYED ? i : gcmap[i]) : -1;
    }
  }
  const int sg0 = tabm ? A.tab.csoff[b] : (!KEYED && A.cseg) ? A.csoff[b] : 0;
  const int sg1 = tabm ? A.tab.csoff[b + 1] : (!KEYED && A.cseg) ? A.csoff[b + 1] : 0;
  // prebuilt windows' zone sets (ZoneWindows; lane j: zone j's, 0 = none)
  const uint32_t zpu = (!KEYED && WM == ZW_M && A.zpre && lane < Z) ? A.zpre->U[lane] : 0u;

#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int i = tid + u * ZW_THREADS;
    if (i < ZZ) { S.csum[i] = cs[u]; S.bsum[i] = bs[u]; }
  }
  if (tid == 0) { S.umask = 0; S.nwin = 0; S.bail = 0; }
  if (tid < CHAIN_MAX / 64) S.sbits[tid] = 0;
  __syncthreads();
  if (!KEYED && tid < Z) {                   // anchor row -> zero-cost zone mask
    uint32_t m = 0;
    for (int z = 0; z < Z; z++) m |= (S.csum[tid * Z + z] == 0.0) ? (1u << z) : 0u;
    S.amask[tid] = m;
  }
  if (tabm) {                                // segment starts (chain-local positions)
    for (int k = sg0 + tid; k < sg1; k += ZW_THREADS) {
      const int p = A.tab.seg_cstart[A.tab.csegid[k]];
      if (p > 0 && p < CHAIN_MAX) atomicOr(&S.sbits[p >> 6], 1ull << (p & 63));
    }
  } else {
    for (int k = sg0 + tid; k < sg1; k += ZW_THREADS) {
      const int p = A.cseg[k];
      if (p > 0 && p < CHAIN_MAX) atomicOr(&S.sbits[p >> 6], 1ull << (p & 63));
    }
  }

  // the chain's anchors (-> its zones U below), demand extremes and finiteness (certificates 2,
  // 3), and the minima of the demands per 64-task batch (for the suffix minima below: a wave's
  // 64 lanes of one pass are one batch); ZW_PR rows per thread in flight at once, the next pass's
  // positions loaded while this one is reduced
  uint32_t abits = 0;                        // anchors seen (Z <= 32)
  double mx[4] = {-DINF, -DINF, -DINF, -DINF}, mn[4] = {DINF, DINF, DINF, DINF};
  bool bad = false;
  for (int i0 = 0; i0 < nt; i0 += ZW_PR * ZW_THREADS) {
    int av[ZW_PR], wn[ZW_PR];
    double dv[ZW_PR][4];
#pragma unroll
    for (int u = 0; u < ZW_PR; u++) {
      const int w = max(wv[u], 0);
      av[u] = A.anc[w];
#pragma unroll
      for (int r = 0; r < 4; r++) dv[u][r] = A.dem[(size_t)w * 4 + r];
    }
#pragma unroll
    for (int u = 0; u < ZW_PR; u++) {
      const int i = i0 + ZW_PR * ZW_THREADS + u * ZW_THREADS + tid;
      wn[u] = i < nt ? (KEYED ? i : cmap_at(i)) : -1;
    }
#pragma unroll
    for (int u = 0; u < ZW_PR; u++) {
      const bool ok = wv[u] >= 0;
      double bm[4];
#pragma unroll
      for (int r = 0; r < 4; r++) bm[r] = ok ? dv[u][r] : DINF;
      if (ok) {
        const int a = av[u];
        if (a < 0 || a >= Z) {
          bad = true;
        } else {
          abits |= 1u << a;
#pragma unroll
          for (int r = 0; r < 4; r++) {
            bad |= !(__builtin_fabs(dv[u][r]) <= ZW_BIG);
            mx[r] = fmax(mx[r], dv[u][r]);
            mn[r] = fmin(mn[r], dv[u][r]);
          }
        }
      }
      const int blk = (i0 + u * ZW_THREADS) / 64 + wave;   // (uniform: the wave's batch)
      if (blk < ZW_SB - 1 && blk * 64 < nt) {
#pragma unroll
        for (int r = 0; r < 4; r++) bm[r] = wave_min_d(bm[r]);
        if (lane == 0) {
#pragma unroll
          for (int r = 0; r < 4; r++) S.smin[blk][r] = bm[r];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < ZW_PR; u++) wv[u] = wn[u];
  }
  __syncthreads();                           // (amask)
  uint32_t um = 0;
  if (!KEYED)
    for (uint32_t m = abits; m; m &= m - 1) um |= S.amask[__builtin_ctz(m)];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    mx[r] = wave_max_d(mx[r]);
    mn[r] = wave_min_d(mn[r]);
    ha[r] = FF ? wave_nmax_d(ha[r]) : wave_min_d(ha[r]);
  }
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < 4; r++) { S.red[wave][r] = mx[r]; S.red[wave][4 + r] = mn[r]; S.red[wave][8 + r] = ha[r]; }
  }
  if (bad) S.bail = 1;                        // benign race: every writer stores 1
  if (um) atomicOr(&S.umask, um);
  __syncthreads();
#ifdef PVT_STAMPS
  const uint64_t t_cert = zstamp();
#endif
#pragma unroll
  for (int r = 0; r < 4; r++) {
    for (int w = 1; w < ZW_WAVES; w++) {
      mx[r] = fmax(mx[r], S.red[w][r]);
      mn[r] = fmin(mn[r], S.red[w][4 + r]);
      ha[r] = FF ? nan_max(ha[r], S.red[w][8 + r]) : fmin(ha[r], S.red[w][8 + r]);
    }
    mx[r] = fmax(mx[r], S.red[0][r]);
    mn[r] = fmin(mn[r], S.red[0][4 + r]);
    ha[r] = FF ? nan_max(ha[r], S.red[0][8 + r]) : fmin(ha[r], S.red[0][8 + r]);
  }
  if (!KEYED && A.cmax && tid < 4) A.cmax[b * 4 + tid] = mx[tid];   // (the validation's fast path)
  bool sep = KEYED;
  if (FF) {                                  // certificates (2') and (3'): bounded capacities,
    sep = true;                              // demands >= 0
#pragma unroll
    for (int r = 0; r < 4; r++) sep &= (ha[r] <= 0x1p298) && (mn[r] >= 0.0);
  } else {
#pragma unroll
    for (int r = 0; r < 4; r++) sep |= (ha[r] - mx[r] >= 0x1p-288);
  }
  uint32_t U = S.umask;
  if (S.bail || !sep || nt <= 0 || (!KEYED && nt > CHAIN_MAX)) {
    if (tid == 0) { status[0] = 0; status[1] = (KEYED || nt <= 0) ? 0 : 1; }
    return;
  }
  const FrontierSlot* pw = A.pwin ? A.pwin + (KEYED ? 0 : b) : nullptr;
  // the round's first epoch: the window the grouped order's launch prebuilt for the component of
  // the chain's anchors (its zone set U' covers U; a window over U' is exact, with U' in the
  // certificates)
  const ZoneWindow* zw = nullptr;
  if (!KEYED && WM == ZW_M && !pw && A.zpre && U != 0) {
    const uint64_t cover = __ballot(zpu != 0 && (U & ~zpu) == 0);
    if (cover) {
      const int j = __builtin_ctzll(cover);
      zw = &A.zpre->w[j];
      U = (uint32_t)__builtin_amdgcn_readlane((int)zpu, j);
    }
  }
  if (pw) {                                  // host-sharded: the merged window, capacities too
    const int nw = min(pw->n, ZW_M);
    for (int p = tid; p < nw; p += ZW_THREADS) {
      const int32_t h = pw->id[p];
      S.wid[p] = h;
      S.wz[p] = KEYED ? 0 : A.zone[h];
    }
    if (tid == 0) S.nwin = nw;
    __syncthreads();
  } else if (zw) {                           // prebuilt: ids and zones (capacities below)
    const int nw = min(zw->n, ZW_M);
    for (int p = tid; p < nw; p += ZW_THREADS) { S.wid[p] = zw->id[p]; S.wz[p] = zw->z[p]; }
    if (tid == 0) S.nwin = nw;
    __syncthreads();
  } else if (KEYED) {                        // window: the zero-key prefix's first hosts
    const int nw = min(A.kn_dev ? *A.kn_dev : A.kn, ZW_M);
    for (int p = tid; p < nw; p += ZW_THREADS) { S.wid[p] = A.lo + A.kperm[p]; S.wz[p] = 0; }
    if (tid == 0) S.nwin = nw;
    __syncthreads();
  } else {                                   // window: U's hosts in index order
    compact_zone_window<WM>(A.zone, Z, U, 0, H, S.wid, S.wz, S.cnt, &S.nwin);
  }
  const int nwin = S.nwin;
#ifdef PVT_STAMPS
  const uint64_t t_win = zstamp();
#endif
  bool wbad = false;
  static_assert(WM % (4 * ZW_THREADS) == 0, "window capacities: four hosts per thread per pass");
  for (int p0 = 0; p0 < WM && p0 < nwin; p0 += 4 * ZW_THREADS) {
    double v[4][4];                          // every gather of the pass in flight at once
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int p = p0 + u * ZW_THREADS + tid;
      const int h = p < nwin ? S.wid[p] : 0;   // (host 0: a valid address, never used)
#pragma unroll
      for (int r = 0; r < 4; r++)
        v[u][r] = p >= nwin ? 0.0 : (pw ? pw->a[r][p] : zw ? zw->a[r][p] : A.avail[(size_t)r * H + h]);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int p = p0 + u * ZW_THREADS + tid;
      if (p < nwin) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
          wbad |= !(__builtin_fabs(v[u][r]) <= ZW_BIG);
          S.wa[r][p] = v[u][r];
        }
      }
    }
  }
  if (wbad) S.bail = 1;
  __syncthreads();
#ifdef PVT_STAMPS
  const uint64_t t_cap = zstamp();
#endif
  if (S.bail || nwin == 0) {
    if (tid == 0) { status[0] = 0; status[1] = KEYED ? 0 : 1; }
    return;
  }
  // suffix minima of the chain's demands per 64-task batch: a chunk no host of which fits the
  // smallest demand still ahead is dead (the walk moves its register chunk past it)
  const int nsb = min((nt + 63) >> 6, ZW_SB);
  // (batches before the last were reduced with the certificates above; the last holds the rest)
  for (int blk = ZW_SB - 1 + wave; blk < nsb; blk += ZW_WAVES) {
    const int i1 = blk == ZW_SB - 1 ? nt : min(nt, blk * 64 + 64);
    double bm[4] = {DINF, DINF, DINF, DINF};
    for (int i = blk * 64 + lane; i < i1; i += 64) {
      const int w = KEYED ? i : cmap_at(i);
#pragma unroll
      for (int r = 0; r < 4; r++) bm[r] = fmin(bm[r], A.dem[(size_t)w * 4 + r]);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) bm[r] = wave_min_d(bm[r]);
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < 4; r++) S.smin[blk][r] = bm[r];
    }
  }
  __syncthreads();
  static_assert(ZW_SB == 64 && ZW_WAVES == 4, "suffix minima: one wave per dimension, a lane per batch");
  {                                          // suffix minima: wave r scans dimension r
    double v = lane < nsb ? S.smin[lane][wave] : DINF;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) v = fmin(v, __shfl_down(v, off));
    if (lane < nsb) S.smin[lane][wave] = v;
  }
  __syncthreads();
  if (wave != 0) return;
#ifdef PVT_STAMPS
  const uint64_t t_walk = zstamp();
#endif

  // ---- the walk (one wave). Lane l of chunk c holds window host c * 64 + l. Chunk p0 (the
  // first that can still fit a chain task) stays in registers, where nearly every task finds its
  // winner: a task is then four compares, a ballot and a one-lane update, with no memory access
  // on its path. Otherwise the chunk is written back and the later chunks are scanned in LDS.
  // The winning lane writes the task's log entry into an LDS batch buffer, flushed to HBM every
  // 64 tasks.
  const int nch = (nwin + 63) >> 6;
  int p0 = 0;                                // chunks before p0 cannot fit any chain task
  int cur = -1;                              // anchor the zero-cost masks are for
  int done = 0;
  bool failed = false, exhausted = false;
  // chunk p0 in registers
  double ra0, ra1, ra2, ra3;
  int32_t rid;
  uint64_t rzm = 0, rvalid = 0;              // its zero-cost lanes (anchor cur), its real lanes
  bool dirty = false;
  auto load_chunk = [&](int c) {
    const int p = c * 64 + lane;
    const int q = min(p, nwin - 1);
    ra0 = S.wa[0][q]; ra1 = S.wa[1][q]; ra2 = S.wa[2][q]; ra3 = S.wa[3][q];
    rid = S.wid[q];
    rvalid = __ballot(p < nwin);
    dirty = false;
    __builtin_amdgcn_s_waitcnt(0xc07f);   // loads landed here, so the hot loop carries no wait
  };
  auto store_chunk = [&](int c) {
    const int p = c * 64 + lane;
    if (dirty && p < nwin) { S.wa[0][p] = ra0; S.wa[1][p] = ra1; S.wa[2][p] = ra2; S.wa[3][p] = ra3; }
    dirty = false;
  };
  // chunk pb = p0 + 1 in registers too (pb < 0: none): a task whose demand no host of chunk p0
  // fits usually finds its winner there
  double rb0 = 0.0, rb1 = 0.0, rb2 = 0.0, rb3 = 0.0;
  int32_t bid = 0;
  uint64_t bzm = 0, bvalid = 0;
  bool bdirty = false;
  int pb = -1;
  auto load_b = [&](int c) {
    bdirty = false;
    if (c >= nch) { pb = -1; bvalid = 0; bzm = 0; return; }
    pb = c;
    const int p = c * 64 + lane;
    const int q = min(p, nwin - 1);
    rb0 = S.wa[0][q]; rb1 = S.wa[1][q]; rb2 = S.wa[2][q]; rb3 = S.wa[3][q];
    bid = S.wid[q];
    bvalid = __ballot(p < nwin);
    bzm = cur >= 0 ? rfl_u64(S.zm[c]) : 0;
    __builtin_amdgcn_s_waitcnt(0xc07f);
  };
  auto store_b = [&]() {
    const int p = pb * 64 + lane;
    if (bdirty && pb >= 0 && p < nwin) { S.wa[0][p] = rb0; S.wa[1][p] = rb1; S.wa[2][p] = rb2; S.wa[3][p] = rb3; }
    bdirty = false;
  };
  // A run of R tasks with the same demand d from batch task k, placed on one 64-host chunk
  // (registers c0..c3, host cid; m0 = its lanes that fit d, all of them zero-cost). Sequentially
  // each task takes the lowest fitting lane; a lane that no longer fits d never fits it again
  // (capacities only fall), and the lanes that do not fit now never will, so the run fills the
  // fitting lanes in index order, each until it cannot take another copy of d. Pass 1: every
  // lane subtracts d again and again in parallel (cnt = copies taken; the active set only
  // shrinks), until the lanes up to the lowest active one u have taken R copies (fb = copies of
  // the finished lanes below u, u itself has taken t) or no lane takes another. Lane l then takes
  // asg = clamp(R - (copies of the lanes before it), 0, cnt) tasks; pass 2 replays exactly those
  // subtractions on the chunk's registers, logging the capacities after each commit at the
  // task's batch position. Returns the tasks placed (>= 1; fewer than R when the chunk runs
  // out). Bit-exact: the same sequential subtractions as one task after the other.
  // (CFT: IntC<1> where the closed-form counts are compiled in -- the hot loop's call only: a
  // copy at each of the four call sites ran the walk out of scalar registers)
  auto run_bulk = [&](auto cft, double& c0, double& c1, double& c2, double& c3, int32_t cid, double d0,
                      double d1, double d2, double d3, uint64_t m0, int R, int k) -> int {
#ifdef PVT_STAMPS
    const uint64_t tA = zstamp();
#endif
    // (Dimensions of demand +0 keep their capacity, x - +0 == x bit for bit, and fit as they did
    // for m0: with d2 = d3 = +0, the trace's disk and gpus, only cpus and memory are counted and
    // updated.)
    if (!(d0 >= 0.0 && d1 >= 0.0 && d2 >= 0.0 && d3 >= 0.0)) R = 1;   // (then one task only)
    const bool on1 = __builtin_amdgcn_inverse_ballot_w64(m0);
    const bool two = __double_as_longlong(d2) == 0 && __double_as_longlong(d3) == 0;
    R = __builtin_amdgcn_readfirstlane(R);
    int cnt = 0;
#ifdef PVT_STAMPS
    const uint64_t tA1 = zstamp();
    st_setup += tA1 - tA;
#endif
    bool cf = false;                         // the closed-form counts are certified
#if PVT_ZW_CF
    if (decltype(cft)::value && R >= 2) {
      // Pass 1 in closed form (copies_cf): every lane of m0 counts its copies from a quotient,
      // certified per dimension; uncertain lanes only matter if the lanes before them do not
      // cover the run (then the copy-by-copy pass below decides)
      bool sure = true;
      int k = ZW_CAP;
      if (on1) {
        k = min(copies_cf<STRICT>(c0, d0, sure), copies_cf<STRICT>(c1, d1, sure));
        if (!two) k = min(k, min(copies_cf<STRICT>(c2, d2, sure), copies_cf<STRICT>(c3, d3, sure)));
      }
      const bool bad = on1 && !sure;
      const uint64_t ub = __ballot(bad);
      const int kc = on1 && sure ? k : 0;
      const int inc = wave_incl_scan_dpp(kc);
      const int first_bad = ub ? __builtin_ctzll(ub) : 64;
      const int before_bad = first_bad == 0 ? 0 : __builtin_amdgcn_readlane(inc, first_bad - 1);
      cf = ub == 0 || before_bad >= R;
      if (cf) cnt = (lane < first_bad) ? kc : 0;
#ifdef PVT_STAMPS
      n_cf += cf;
#endif
    }
#endif
    if (!cf) {
      // Pass 1: without per-lane masks: with d >= 0 a lane that fails a copy fails every later
      // one (its residual only falls further), so every lane just keeps subtracting, recording
      // the last copy that fit (= the copies it takes); lanes outside m0 start at -inf.
      // ZW_UNROLL copies per check (a check past the stop only raises counts of lanes that get no
      // task or no more tasks: asg clamps them).
      double x0 = on1 ? c0 : -DINF, x1 = on1 ? c1 : -DINF, x2 = on1 ? c2 : -DINF, x3 = on1 ? c3 : -DINF;
      int t = 0;
      auto pass1 = [&](auto dims) {
        constexpr int D = decltype(dims)::value;
        int u = __builtin_ctzll(m0), fb = 0;
        for (;;) {
          t = __builtin_amdgcn_readfirstlane(t);
          u = __builtin_amdgcn_readfirstlane(u);
          fb = __builtin_amdgcn_readfirstlane(fb);
          bool f = false;
#pragma unroll
          for (int j = 1; j <= ZW_UNROLL; j++) {
            x0 -= d0; x1 -= d1;
            if (D == 4) { x2 -= d2; x3 -= d3; }
            f = fit_res<STRICT>(D == 4 ? fmin(fmin(x0, x1), fmin(x2, x3)) : fmin(x0, x1));
            cnt = f ? t + j : cnt;
          }
          t += ZW_UNROLL;
          const uint64_t an = __ballot(f);       // lanes that took copy t
          if (UNI(an == 0)) break;
          const int un = __builtin_ctzll(an);
          if (un != u) {                         // (u only rises: every lane below un is done)
            u = un;
            fb = __builtin_amdgcn_readlane(wave_incl_scan_dpp(cnt), u - 1);
          }
          if (UNI(fb + t >= R)) break;
        }
      };
      if (two) pass1(IntC<2>{});
      else pass1(IntC<4>{});
#ifdef PVT_STAMPS
      n_iter += t;
#endif
    }
#ifdef PVT_STAMPS
    st_loop += zstamp() - tA1;
#endif
    const int incl = wave_incl_scan_dpp(cnt);
    const int pre = incl - cnt;
    const int asg = max(0, min(cnt, R - pre));
    const int covered = min(R, __builtin_amdgcn_readlane(incl, 63));
#ifdef PVT_STAMPS
    const uint64_t tB = zstamp();
    st_p1 += tB - tA;
#endif
    // Pass 2: the lanes that take tasks (few: a host takes many copies) in a scalar loop --
    // each lane of the run's batch positions learns its host -- and every such lane replays
    // exactly its own subtractions (the same sequential subtractions as task after task, so
    // bit-exact), predicated in steps of four up to the largest count. The log keeps the host of
    // every copy and the capacities after a lane's last one only: a host's earlier entries in a
    // segment are never final (epoch_final_kernel marks them; validation and apply read the
    // capacities of final entries only, and the keyed / ordered walks read no log).
    // (each taking lane marks its first run position; a position's host is that of the last
    // mark at or before it: two LDS round trips, no loop over the taking lanes)
    S.rstart[lane] = 0;
    if (asg > 0) { S.rstart[pre] = 1; S.rwho[pre] = cid; }
    wave_lds_sync();
    const uint64_t starts = __ballot(S.rstart[lane] != 0);
    const uint64_t upto = starts & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
    const int32_t who = upto ? S.rwho[63 - __builtin_clzll(upto)] : 0;
    const int amax = wave_max_i32(asg);
    if (lane < covered) S.lgid[k + lane] = who;
#ifdef PVT_STAMPS
    const uint64_t tC = zstamp();
    st_who += tC - tB;
#endif
    // (c - d as fma(-1, d, c), rounded once, the same bits; fma(-0, d, c) == c for the finite d
    // and c of a proven chain: one 0/1 factor per copy for every dimension)
    if (two) {
      for (int m = 0; m < amax; m += 4) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const double o = m + u < asg ? -1.0 : -0.0;
          c0 = __builtin_fma(o, d0, c0);
          c1 = __builtin_fma(o, d1, c1);
        }
      }
    } else {
      for (int m = 0; m < amax; m += 4) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const double o = m + u < asg ? -1.0 : -0.0;
          c0 = __builtin_fma(o, d0, c0);
          c1 = __builtin_fma(o, d1, c1);
          c2 = __builtin_fma(o, d2, c2);
          c3 = __builtin_fma(o, d3, c3);
        }
      }
    }
#ifdef PVT_STAMPS
    st_rep += zstamp() - tC;
#endif
    if (asg > 0) {
      const int q = k + pre + asg - 1;
      S.lg[q][0] = c0; S.lg[q][1] = c1; S.lg[q][2] = c2; S.lg[q][3] = c3;
    }
#ifdef PVT_STAMPS
    st_p2 += zstamp() - tB;
#endif
    return covered;
  };
  load_chunk(0);
  load_b(1);
  // task records, software-pipelined across 64-task batches: while batch b is walked, batch
  // b + 1's records and batch b + 2's chain positions are in flight (no HBM latency at a batch
  // start)
  auto task_at = [&](int i) { return i < nt ? (KEYED ? i : cmap_at(i)) : 0; };
  int nw = task_at(lane);
  double nd0 = A.dem[(size_t)nw * 4 + 0], nd1 = A.dem[(size_t)nw * 4 + 1];
  double nd2 = A.dem[(size_t)nw * 4 + 2], nd3 = A.dem[(size_t)nw * 4 + 3];
  int nanc = A.anc[nw], ncal = A.ord[nw];
  int nw1 = task_at(64 + lane);
  int carry = 0;                             // tasks of this batch a run of the last one placed
  for (int i0 = 0; UNI(i0 < nt && !failed); i0 += 64) {
#ifdef PVT_STAMPS
    uint64_t tb0 = zstamp();
#endif
#pragma unroll
    for (int r = 0; r < 4; r++) mn[r] = S.smin[min(i0 >> 6, ZW_SB - 1)][r];
    const int tw = nw;
    const double td[4] = {nd0, nd1, nd2, nd3};
    const int tanc = nanc;
    const int tcal = ncal;
    if (i0 + 64 < nt) {                      // (uniform) batch b + 1's records, b + 2's positions
      nw = nw1;
      nd0 = A.dem[(size_t)nw * 4 + 0]; nd1 = A.dem[(size_t)nw * 4 + 1];
      nd2 = A.dem[(size_t)nw * 4 + 2]; nd3 = A.dem[(size_t)nw * 4 + 3];
      nanc = A.anc[nw]; ncal = A.ord[nw];
      nw1 = task_at(i0 + 128 + lane);
    }
    const int kn = min(64, nt - i0);
    // (uniform) every task of the batch has the anchor the zero-cost masks are for: the tasks
    // need no anchor test (a chain's groups are long, so nearly every batch)
    bool uni = __ballot(lane < kn && tanc != cur) == 0;
    // runs: bit i is set iff task i of the batch has task i - 1's demand vector, bit for bit (the
    // trace has few distinct demand rows, and sorted order puts equal ones next to each other)
    uint64_t E;
    {
      bool same = lane > 0 && lane < kn;
#pragma unroll
      for (int r = 0; r < 4; r++)
        same &= __double_as_longlong(__shfl_up(td[r], 1)) == __double_as_longlong(td[r]);
      E = __ballot(same);
      // (chain mode: a run stops at a group segment start -- pass 2 logs a host's capacities
      // at its last copy of the run only, and the segment before must hold its own last copy)
      if (segm) E &= ~rfl_u64(S.sbits[i0 >> 6]);
    }
    // A run that reaches the end of a full batch goes on into the next one while those tasks
    // have the same demand vector and anchor and no segment starts (their records are already in
    // registers, nd*): at most 64 tasks per run, the ones past the batch logged at 64.. and
    // carried (a third of the runs were cut at batch ends).
    int extc = -1;
    auto ext_len = [&]() -> int {
      if (extc < 0) {
        extc = 0;
        if (kn == 64 && i0 + 64 < nt && uni) {
          const int kn2 = min(64, nt - i0 - 64);
          const double l0 = readlane_d(td[0], 63), l1 = readlane_d(td[1], 63);
          const double l2 = readlane_d(td[2], 63), l3 = readlane_d(td[3], 63);
          bool eq = lane < kn2 && readlane_i(tanc, 63) == nanc &&
                    __double_as_longlong(nd0) == __double_as_longlong(l0) &&
                    __double_as_longlong(nd1) == __double_as_longlong(l1) &&
                    __double_as_longlong(nd2) == __double_as_longlong(l2) &&
                    __double_as_longlong(nd3) == __double_as_longlong(l3);
          if (segm) eq = eq && !((rfl_u64(S.sbits[(i0 >> 6) + 1]) >> lane) & 1ull);
          const uint64_t m = __ballot(eq);
          extc = m == ~0ull ? 64 : __builtin_ctzll(~m);
        }
        extc = __builtin_amdgcn_readfirstlane(extc);
      }
      return extc;
    };
    auto run_len = [&](int k) {
      int r = k < 63 ? min(kn - k, 1 + __builtin_ctzll(~(E >> (k + 1)))) : 1;
      if (k + r == 64) r = min(64, r + ext_len());
      return r;
    };
    // The run step, for a task k of a uniform batch that the register chunk p0 cannot take: its
    // run (R tasks with its demand, R >= 1) is placed by run_bulk on the first chunk that can
    // take a copy of it -- chunk p0 (moved on past chunks no task ahead can use), chunk pb, then
    // the LDS chunks in index order -- with the per-task path's exactness conditions: every
    // chunk before it fits no copy (for the chunks before p0: no task ahead), and no fitting
    // host of a chunk it looks at is outside the anchor's zero-cost zones (else 0: the per-task
    // path decides, with exact scores). Returns the tasks placed (0: none).
    auto run_step = [&](int k) -> int {
#ifdef PVT_STAMPS
      const uint64_t t0 = zstamp();
#define ZW_SEARCH_DONE() (st_search += zstamp() - t0)
#else
#define ZW_SEARCH_DONE() ((void)0)
#endif
      const double d0 = readlane_d(td[0], k), d1 = readlane_d(td[1], k);
      const double d2 = readlane_d(td[2], k), d3 = readlane_d(td[3], k);
      const int R = run_len(k);
      for (;;) {
        const double n0 = ra0 - d0, n1 = ra1 - d1, n2 = ra2 - d2, n3 = ra3 - d3;
        uint64_t fm = __ballot(fit_res<STRICT>(fmin(fmin(n0, n1), fmin(n2, n3)))) & rvalid;
        if (FF) fm &= rzm;                     // (FF: other fitting hosts have key > 0)
        if (!FF && UNI((fm & ~rzm) != 0)) return 0;
        if (UNI(fm != 0)) {
          dirty = true;
          ZW_SEARCH_DONE();
          return run_bulk(IntC<0>{}, ra0, ra1, ra2, ra3, rid, d0, d1, d2, d3, fm, R, k);
        }
        if (__ballot(((rvalid >> lane) & 1ull) && fits<STRICT>(ra0, ra1, ra2, ra3, mn[0], mn[1], mn[2], mn[3])))
          break;                               // chunk p0 can still take a task ahead
        if (p0 + 1 >= nch) return 0;
        store_b();                             // dead: move the register chunks on
        store_chunk(p0);
        ++p0;
        rzm = rfl_u64(S.zm[p0]);
        load_chunk(p0);
        load_b(p0 + 1);
      }
      if (pb >= 0) {
        const double q0 = rb0 - d0, q1 = rb1 - d1, q2 = rb2 - d2, q3 = rb3 - d3;
        uint64_t fb = __ballot(fit_res<STRICT>(fmin(fmin(q0, q1), fmin(q2, q3)))) & bvalid;
        if (FF) fb &= bzm;
        if (!FF && UNI((fb & ~bzm) != 0)) return 0;
        if (UNI(fb != 0)) {
          bdirty = true;
          ZW_SEARCH_DONE();
          return run_bulk(IntC<0>{}, rb0, rb1, rb2, rb3, bid, d0, d1, d2, d3, fb, R, k);
        }
      }
      for (int c = (pb >= 0 ? pb : p0) + 1; c < nch; c++) {
        const int p = c * 64 + lane;
        const int q = min(p, nwin - 1);
        double x0 = S.wa[0][q], x1 = S.wa[1][q], x2 = S.wa[2][q], x3 = S.wa[3][q];
        const int32_t xid = S.wid[q];
        const uint64_t xzm = rfl_u64(S.zm[c]);
#ifdef PVT_STAMPS
        n_probe++;
#endif
        uint64_t fm = __ballot(p < nwin && fit_res<STRICT>(fmin(fmin(x0 - d0, x1 - d1),
                                                                fmin(x2 - d2, x3 - d3))));
        if (FF) fm &= xzm;
        if (!FF && UNI((fm & ~xzm) != 0)) return 0;
        if (UNI(fm != 0)) {
          ZW_SEARCH_DONE();
          const int got = run_bulk(IntC<0>{}, x0, x1, x2, x3, xid, d0, d1, d2, d3, fm, R, k);
          if (p < nwin) { S.wa[0][p] = x0; S.wa[1][p] = x1; S.wa[2][p] = x2; S.wa[3][p] = x3; }
          return got;
        }
      }
      ZW_SEARCH_DONE();
      return 0;
    };
#undef ZW_SEARCH_DONE
#ifdef PVT_STAMPS
    st_batch += zstamp() - tb0;
#endif
    int k = carry;
    if (carry) {                             // the carried run's log entries to their positions
      wave_lds_sync();
      if (lane < carry) {
#pragma unroll
        for (int r = 0; r < 4; r++) S.lg[lane][r] = S.lg[64 + lane][r];
        S.lgid[lane] = S.lgid[64 + lane];
      }
      wave_lds_sync();
    }
    while (UNI(k < kn)) {
      // (wave-uniform state the compiler cannot prove uniform: keeps the loops below scalar)
      k = __builtin_amdgcn_readfirstlane(k);
      p0 = __builtin_amdgcn_readfirstlane(p0);
      pb = __builtin_amdgcn_readfirstlane(pb);
      done = __builtin_amdgcn_readfirstlane(done);
      rzm = rfl_u64(rzm);
      bzm = rfl_u64(bzm);
      // The hot loop: the batch's tasks while each finds a fitting zero-cost host in the
      // register chunk and every fitting host of it is zero-cost for the anchor. Per task: the
      // demand from registers, four subtractions, three minima, one ballot, the winner's mask
      // bit (lowest set bit, scalar), four selects on it and the winner lane's log entry -- no
      // compare of a lane id and no branch back to the vector unit. Any other task leaves it for
      // the general step below, then the hot loop goes on.
      if (uni) {
        for (; k < kn;) {
          k = __builtin_amdgcn_readfirstlane(k);
          const double d0 = readlane_d(td[0], k), d1 = readlane_d(td[1], k);
          const double d2 = readlane_d(td[2], k), d3 = readlane_d(td[3], k);
          const double n0 = ra0 - d0, n1 = ra1 - d1, n2 = ra2 - d2, n3 = ra3 - d3;
          const uint64_t fm0 = __ballot(fit_res<STRICT>(fmin(fmin(n0, n1), fmin(n2, n3)))) & rvalid;
          const uint64_t m0 = fm0 & rzm;
          if (UNI(m0 == 0 || (!FF && (fm0 & ~rzm) != 0))) break;
          // a run of tasks with this demand: placed in one pass over the chunk (run_bulk)
          const int R = run_len(k);
          if (UNI(R >= 2)) {
            const int c = run_bulk(IntC<1>{}, ra0, ra1, ra2, ra3, rid, d0, d1, d2, d3, m0, R, k);
            k += c;
            done += c;
            dirty = true;
#ifdef PVT_STAMPS
            n_chunks += c;
            n_bulk += c;
            n_runs++;
#endif
            continue;
          }
          const bool win = __builtin_amdgcn_inverse_ballot_w64(m0 & (0ull - m0));
          ra0 = win ? n0 : ra0; ra1 = win ? n1 : ra1; ra2 = win ? n2 : ra2; ra3 = win ? n3 : ra3;
          if (win) {
            S.lg[k][0] = n0; S.lg[k][1] = n1; S.lg[k][2] = n2; S.lg[k][3] = n3;
            S.lgid[k] = rid;
          }
          dirty = true;
#ifdef PVT_STAMPS
          n_chunks++;
          n_single++;
#endif
          done++;
          k++;
        }
        if (UNI(k >= kn)) break;
        const int got = run_step(k);
        if (UNI(got > 0)) {
          k += got;
          done += got;
#ifdef PVT_STAMPS
          n_chunks += got;
          n_bulk += got;
          n_runs++;
#endif
          continue;
        }
      }
      const double d0 = readlane_d(td[0], k), d1 = readlane_d(td[1], k);
      const double d2 = readlane_d(td[2], k), d3 = readlane_d(td[3], k);
      const int a = uni ? cur : readlane_i(tanc, k);
      if (a != cur) {
        // certificates 2 / 3 for this anchor's zone row
        bool ok = true;
        if (!KEYED && lane < Z) {
          const double c = S.csum[a * Z + lane], bw = S.bsum[a * Z + lane];
          if (c == 0.0) ok = bw > 0.0;
          // (bw > 0: a negative bandwidth would give a negative key, ahead of every zero key)
          else if (FF || !((U >> lane) & 1u)) ok = (c >= 0x1p-300) && (bw > 0.0) && (bw <= 0x1p300);
        }
        if (__ballot(!ok)) { failed = true; break; }
        const uint32_t am = KEYED ? ~0u : S.amask[a];   // keyed: every prefix host is zero-key
        for (int c = 0; c < nch; c++) {
          const int p = c * 64 + lane;
          const uint64_t m = __ballot(p < nwin && (KEYED || ((am >> S.wz[min(p, nwin - 1)]) & 1u)));
          if (lane == 0) S.zm[c] = m;
          if (c == p0) rzm = m;
          if (c == pb) bzm = m;
        }
        cur = a;
        uni = __ballot(lane >= k && lane < kn && tanc != cur) == 0;   // the rest of the batch
        __builtin_amdgcn_s_waitcnt(0xc07f);
#ifdef PVT_STAMPS
        n_switch++;
#endif
      }
      // exact scores for this lane's host when it fits but is not zero-cost for `a`
      auto zero_exact = [&](bool f, bool k0, double a0, double a1, double a2, double a3, int q) {
        if (FF) return k0;                   // (first-fit: a fitting host of another zone has key > 0)
        if (__builtin_expect(__ballot(f && !k0) != 0, 0)) {
          if (f && !k0) {
            const int z = S.wz[q];
            const double s2 = norm2_seq(a0 - d0, a1 - d1, a2 - d2, a3 - d3);
            const double sc = (S.csum[a * Z + z] * __builtin_sqrt(s2)) / S.bsum[a * Z + z];
            k0 = __double_as_longlong(sc) == 0;
          }
        }
        return k0;
      };
      // Hot path, straight-line: the register chunk holds a fitting zero-cost host and every
      // fitting host of it is zero-cost for this anchor. The fit test is the minimum residual:
      // every window capacity and chain demand is finite with |x| <= 2^500 (certificate 3), so
      // a - d is exact in sign (a >= d iff a - d >= +-0) and is the capacity after a commit.
      const double n0 = ra0 - d0, n1 = ra1 - d1, n2 = ra2 - d2, n3 = ra3 - d3;
      // (keyed first-fit: strict fit, a > d iff a - d > 0)
      const uint64_t fm0 = __ballot(fit_res<STRICT>(fmin(fmin(n0, n1), fmin(n2, n3)))) & rvalid;
      bool found = true;
#ifdef PVT_STAMPS
      n_chunks++;
#endif
      // Each path commits in place (no shared commit block: merging the paths made the compiler
      // copy the chunk registers on every task). commit: resc[h] -= t_demand
      // (cost_aware.py:95) on the lowest such lane, which logs.
      // (the winner's lane from its mask bit in scalar registers: no lane-id compare, and the
      // commit is four selects on that mask)
      const uint64_t m0 = fm0 & rzm;
      if (__builtin_expect(m0 != 0 && (FF || (fm0 & ~rzm) == 0), 1)) {
        const bool win = __builtin_amdgcn_inverse_ballot_w64(m0 & (0ull - m0));
        ra0 = win ? n0 : ra0; ra1 = win ? n1 : ra1; ra2 = win ? n2 : ra2; ra3 = win ? n3 : ra3;
        if (win) {
          S.lg[k][0] = n0; S.lg[k][1] = n1; S.lg[k][2] = n2; S.lg[k][3] = n3;
          S.lgid[k] = rid;
        }
        dirty = true;
      } else {
        bool inb = false;
        if (fm0 == 0 && pb >= 0) {
          // no host of chunk p0 fits this task: its winner is chunk pb's first fitting zero-cost
          // host, from registers (a dead chunk p0 is moved on by the general path below)
          const double q0 = rb0 - d0, q1 = rb1 - d1, q2 = rb2 - d2, q3 = rb3 - d3;
          const uint64_t fb = __ballot(fit_res<STRICT>(fmin(fmin(q0, q1), fmin(q2, q3)))) & bvalid;
          const uint64_t mb = fb & bzm;
          if (mb != 0 && (FF || (fb & ~bzm) == 0)) {
            const bool win = __builtin_amdgcn_inverse_ballot_w64(mb & (0ull - mb));
            rb0 = win ? q0 : rb0; rb1 = win ? q1 : rb1; rb2 = win ? q2 : rb2; rb3 = win ? q3 : rb3;
            if (win) {
              S.lg[k][0] = q0; S.lg[k][1] = q1; S.lg[k][2] = q2; S.lg[k][3] = q3;
              S.lgid[k] = bid;
            }
            bdirty = true;
            inb = true;
          }
        }
        if (!inb) {                            // the general path
          found = false;
          store_b();                           // it works on LDS from p0 + 1 on
          double g0 = n0, g1 = n1, g2 = n2, g3 = n3;
          uint64_t fm = fm0, m = fm0 & rzm;
#ifdef PVT_STAMPS
          for (int pass = 0;; pass++) {        // the register chunk (advancing past dead ones)
            n_chunks += pass > 0;
#else
          for (;;) {                           // the register chunk (advancing past dead ones)
#endif
            if (fm & ~rzm)                     // fitting hosts of U outside the anchor's
              m = __ballot(zero_exact((fm >> lane) & 1ull, (rzm >> lane) & 1ull, ra0, ra1, ra2,
                                      ra3, min(p0 * 64 + lane, nwin - 1))) & fm;   // zero-cost zones
            if (m) {
              const bool win = lane == __builtin_ctzll(m);
              ra0 = win ? g0 : ra0; ra1 = win ? g1 : ra1; ra2 = win ? g2 : ra2; ra3 = win ? g3 : ra3;
              if (win) {
                S.lg[k][0] = g0; S.lg[k][1] = g1; S.lg[k][2] = g2; S.lg[k][3] = g3;
                S.lgid[k] = rid;
              }
              dirty = true;
              found = true;
              break;
            }
            if (__ballot(((rvalid >> lane) & 1ull) && fits<STRICT>(ra0, ra1, ra2, ra3, mn[0], mn[1], mn[2], mn[3])))
              break;                           // chunk p0 still useful: look further in LDS
            store_chunk(p0);                   // dead: move the register chunk on
            if (++p0 >= nch) break;
            rzm = rfl_u64(S.zm[p0]);
            load_chunk(p0);
            g0 = ra0 - d0; g1 = ra1 - d1; g2 = ra2 - d2; g3 = ra3 - d3;
            fm = __ballot(fit_res<STRICT>(fmin(fmin(g0, g1), fmin(g2, g3)))) & rvalid;
            m = fm & rzm;
          }
          if (!found && p0 < nch) {
            store_chunk(p0);
            for (int c = p0 + 1; c < nch; c++) {
#ifdef PVT_STAMPS
              n_chunks++;
#endif
              const int p = c * 64 + lane;
              const int q = min(p, nwin - 1);
              const double a0 = S.wa[0][q], a1 = S.wa[1][q], a2 = S.wa[2][q], a3 = S.wa[3][q];
              const int32_t id = S.wid[q];
              const uint64_t zm = rfl_u64(S.zm[c]);
              const bool f = p < nwin && fits<STRICT>(a0, a1, a2, a3, d0, d1, d2, d3);
              const bool k0 = zero_exact(f, (zm >> lane) & 1ull, a0, a1, a2, a3, q);
              const uint64_t mc = __ballot(f && k0);
              if (mc) {
                if (lane == __builtin_ctzll(mc)) {
                  const double c0 = a0 - d0, c1 = a1 - d1, c2 = a2 - d2, c3 = a3 - d3;
                  S.wa[0][q] = c0; S.wa[1][q] = c1; S.wa[2][q] = c2; S.wa[3][q] = c3;
                  S.lg[k][0] = c0; S.lg[k][1] = c1; S.lg[k][2] = c2; S.lg[k][3] = c3;
                  S.lgid[k] = id;
                }
                found = true;
                break;
              }
            }
          }
          wave_lds_sync();
          load_b(p0 + 1);
        }
      }
      if (UNI(!found)) {                     // certificate 1 fails: the list walk decides --
        failed = true;                       // or, when the window is full, a larger one may do
        exhausted = nwin >= WM;
        break;
      }
      done++;
      k++;
    }
#ifdef PVT_STAMPS
    tb0 = zstamp();
#endif
    if (lane < k) {                          // the batch's log (WinRec; sup: epoch_final_kernel)
      WinRec& e = A.wlog[tw];
      const int32_t id = S.lgid[lane];
      e.s = 0.0;
      e.id = id;
      e.a[0] = S.lg[lane][0]; e.a[1] = S.lg[lane][1]; e.a[2] = S.lg[lane][2]; e.a[3] = S.lg[lane][3];
      A.placement[tcal] = id;
    }
    carry = __builtin_amdgcn_readfirstlane(k > kn ? k - kn : 0);
#ifdef PVT_STAMPS
    st_batch += zstamp() - tb0;
#endif
  }
  if (KEYED) {   // the window's capacities to global availability: the keyed path goes on there
    store_chunk(p0);
    store_b();
    wave_lds_sync();
    for (int p = lane; p < nwin; p += 64) {
      const int h = S.wid[p];
#pragma unroll
      for (int r = 0; r < 4; r++) A.wb[(size_t)r * H + h] = S.wa[r][p];
    }
  }
  // status[0]: tasks proven (their log entries are exact; validation accepts them), status[1]:
  // 1 when a certificate failed there (the rest of the chain is left to the list walk)
  if (lane == 0) { status[0] = done; status[1] = (failed && !KEYED) ? (exhausted ? 2 : 1) : 0; }
#ifdef PVT_STAMPS
  if (lane == 0 && A.stamps) {
    const uint64_t t_end = zstamp();
    atomicAdd((unsigned long long*)&A.stamps[0], (unsigned long long)(t_walk - t_start));
    atomicAdd((unsigned long long*)&A.stamps[1], (unsigned long long)(t_end - t_walk));
    atomicAdd((unsigned long long*)&A.stamps[2], (unsigned long long)n_chunks);
    atomicAdd((unsigned long long*)&A.stamps[3], (unsigned long long)done);
    atomicAdd((unsigned long long*)&A.stamps[4], (unsigned long long)n_switch);
    atomicAdd((unsigned long long*)&A.stamps[5], (unsigned long long)n_bulk);
    atomicAdd((unsigned long long*)&A.stamps[6], (unsigned long long)n_runs);
    atomicAdd((unsigned long long*)&A.stamps[7], (unsigned long long)st_search);
    atomicAdd((unsigned long long*)&A.stamps[8], (unsigned long long)st_p1);
    atomicAdd((unsigned long long*)&A.stamps[9], (unsigned long long)st_p2);
    atomicAdd((unsigned long long*)&A.stamps[10], (unsigned long long)n_probe);
    atomicAdd((unsigned long long*)&A.stamps[11], (unsigned long long)n_iter);
    atomicAdd((unsigned long long*)&A.stamps[12], (unsigned long long)st_batch);
    atomicAdd((unsigned long long*)&A.stamps[13], (unsigned long long)n_single);
    atomicAdd((unsigned long long*)&A.stamps[20], (unsigned long long)(t_cert - t_start));
    atomicAdd((unsigned long long*)&A.stamps[21], (unsigned long long)(t_win - t_cert));
    atomicAdd((unsigned long long*)&A.stamps[22], (unsigned long long)(t_cap - t_win));
    atomicAdd((unsigned long long*)&A.stamps[23], (unsigned long long)(t_walk - t_cap));
    atomicAdd((unsigned long long*)&A.stamps[24], (unsigned long long)st_setup);
    atomicAdd((unsigned long long*)&A.stamps[25], (unsigned long long)st_loop);
    atomicAdd((unsigned long long*)&A.stamps[26], (unsigned long long)st_who);
    atomicAdd((unsigned long long*)&A.stamps[27], (unsigned long long)st_rep);
    atomicAdd((unsigned long long*)&A.stamps[28], (unsigned long long)n_cf);
  }
#endif
}

void launch_host_min(const double* avail, int H, int lo, int hi, double* part, hipStream_t st) {
  PVT_LAUNCH(host_min_kernel, dim3(ZW_MINB), dim3(256), 0, st, avail, H, lo, hi, part);
}

void launch_zwalk(const ZwalkArgs& a, int nchains, hipStream_t st) {
  PVT_LAUNCH((zwalk_kernel<false, false>), dim3(nchains), dim3(ZW_THREADS), 0, st, a);
}
void launch_zwalk_big(const ZwalkArgs& a, int nchains, hipStream_t st) {
  PVT_LAUNCH((zwalk_kernel<false, false, false, ZW_MBIG>), dim3(nchains), dim3(ZW_THREADS), 0, st, a);
}
void launch_zwalk_ff(const ZwalkArgs& a, int nchains, hipStream_t st) {
  PVT_LAUNCH((zwalk_kernel<false, true, true>), dim3(nchains), dim3(ZW_THREADS), 0, st, a);
}

// Per-dimension maxima of |avail| over hosts [lo, hi) (the FF walk's certificate 2'), in
// host_min_kernel's partial layout.
__global__ __launch_bounds__(256) void host_absmax_kernel(const double* avail, int H, int lo, int hi,
                                                          double* part) {
  __shared__ double red[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double m[4] = {0.0, 0.0, 0.0, 0.0};
  for (int h = lo + blockIdx.x * 256 + tid; h < hi; h += gridDim.x * 256)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      m[r] = nan_max(m[r], __builtin_fabs(avail[(size_t)r * H + h]));   // (NaN propagates:
    }                                                                     //  no certificate)
#pragma unroll
  for (int r = 0; r < 4; r++) {
    m[r] = wave_nmax_d(m[r]);
    if (lane == 0) red[wave][r] = m[r];
  }
  __syncthreads();
  if (tid < 4) {
    double v = red[0][tid];
    for (int w = 1; w < 4; w++) v = nan_max(v, red[w][tid]);
    part[blockIdx.x * 4 + tid] = v;
  }
}
void launch_host_absmax(const double* avail, int H, int lo, int hi, double* part, hipStream_t st) {
  PVT_LAUNCH(host_absmax_kernel, dim3(ZW_MINB), dim3(256), 0, st, avail, H, lo, hi, part);
}
void launch_zwalk_keyed(const ZwalkArgs& a, bool strict, hipStream_t st) {
  if (strict) PVT_LAUNCH((zwalk_kernel<true, true>), dim3(1), dim3(ZW_THREADS), 0, st, a);
  else PVT_LAUNCH((zwalk_kernel<true, false>), dim3(1), dim3(ZW_THREADS), 0, st, a);
}

// Ordered frontier: the smallest demand (per dimension) of tasks [0, n), then the hosts that
// fit it (the alive hosts: no other can fit any of those tasks), as flags for a compaction.
__global__ __launch_bounds__(1024) void dem_min_kernel(const double* dem, int n, double* out) {
  __shared__ double red[16][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double m[4] = {DINF, DINF, DINF, DINF};
  for (int i = tid; i < n; i += 1024)
#pragma unroll
    for (int r = 0; r < 4; r++) m[r] = fmin(m[r], dem[(size_t)i * 4 + r]);
#pragma unroll
  for (int r = 0; r < 4; r++) {
    m[r] = wave_min_d(m[r]);
    if (lane == 0) red[wave][r] = m[r];
  }
  __syncthreads();
  if (tid < 4) {
    double v = red[0][tid];
    for (int w = 1; w < 16; w++) v = fmin(v, red[w][tid]);
    out[tid] = v;
  }
}
__global__ void alive_flags_kernel(const double* avail, int H, int lo, int hs, const double* dmin,
                                   int strict, uint8_t* flags) {
  const int h = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= hs) return;
  const double a0 = avail[h], a1 = avail[(size_t)H + h], a2 = avail[2 * (size_t)H + h],
               a3 = avail[3 * (size_t)H + h];
  flags[h - lo] = strict ? fits<true>(a0, a1, a2, a3, dmin[0], dmin[1], dmin[2], dmin[3])
                    : fits<false>(a0, a1, a2, a3, dmin[0], dmin[1], dmin[2], dmin[3]);
}
void launch_alive_flags(const double* avail, int H, int lo, int hs, const double* dem, int n,
                        int strict, double* dmin, uint8_t* flags, hipStream_t st) {
  PVT_LAUNCH(dem_min_kernel, dim3(1), dim3(1024), 0, st, dem, n, dmin);
  if (hs <= lo) return;
  PVT_LAUNCH(alive_flags_kernel, dim3((hs - lo + 255) / 256), dim3(256), 0, st, avail, H,
                     lo, hs, dmin, strict, flags);
}

// ---- host-sharded frontier walks: a rank's window candidates, and their merge

// Chain b of the epoch: its zero-cost zones U (the union of its anchors' zero-cost zones, as the
// walk computes them) and the first ZW_M hosts of U in this rank's range [lo, hi), index order,
// with their capacities; block 0 also stamps the package header.
__global__ __launch_bounds__(ZW_THREADS) void zwin_build_kernel(ZwinArgs A) {
  __shared__ uint32_t amask[ZMAX];
  __shared__ uint32_t umask;
  __shared__ int32_t cnt[ZW_SCAN][ZW_WAVES];
  __shared__ int32_t nwin;
  const int b = blockIdx.x, tid = threadIdx.x, Z = A.Z;
  FrontierSlot* out = A.out + b;
  if (tid == 0) { umask = 0; nwin = 0; }
  if (tid < Z) {
    uint32_t m = 0;
    for (int z = 0; z < Z; z++) m |= (A.csum[tid * Z + z] == 0.0) ? (1u << z) : 0u;
    amask[tid] = m;
  }
  __syncthreads();
  uint32_t um = 0;
  for (int i = A.coff[b] + tid; i < A.coff[b + 1]; i += ZW_THREADS) {
    const int a = A.anc[A.cmap[i]];
    if (a >= 0 && a < Z) um |= amask[a];    // (a bad anchor: the walk bails on it)
  }
  if (um) atomicOr(&umask, um);
  __syncthreads();
  compact_zone_window(A.zone, Z, umask, A.lo, A.hi, out->id, nullptr, cnt, &nwin);
  const int n = nwin;
  for (int p = tid; p < n; p += ZW_THREADS) {
    const int h = out->id[p];
#pragma unroll
    for (int r = 0; r < 4; r++) out->a[r][p] = A.avail[(size_t)r * A.H + h];
  }
  if (tid == 0) { out->n = n; out->total = n; }
}

__global__ __launch_bounds__(256) void zwin_gather_kernel(const double* avail, int H, int lo,
                                                          const int32_t* perm, const int32_t* count,
                                                          FrontierSlot* out) {
  const int c = *count, n = min(c, ZW_M);
  for (int p = threadIdx.x; p < n; p += 256) {
    const int h = lo + perm[p];
    out->id[p] = h;
#pragma unroll
    for (int r = 0; r < 4; r++) out->a[r][p] = avail[(size_t)r * H + h];
  }
  if (threadIdx.x == 0) { out->n = n; out->total = c; }
}

// Block b < nslots: slot b of every rank, concatenated in rank order and cut at ZW_M (ranks own
// ascending ranges, so this is the index-order window); block nslots: the host-minimum partials,
// the minimum over ranks.
__global__ __launch_bounds__(256) void zwin_merge_kernel(const uint8_t* pkgs, int64_t pkg_bytes,
                                                         int world, int nslots, FrontierSlot* out,
                                                         double* hmin) {
  __shared__ int32_t off[PVT_SHARD_MAX_WORLD + 1];
  const int b = blockIdx.x, tid = threadIdx.x;
  auto hdr = [&](int k) { return reinterpret_cast<const FrontierHdr*>(pkgs + (size_t)k * pkg_bytes); };
  if (b == nslots) {               // (keyed / ordered walks: hmin NULL, no minima exchanged)
    for (int i = tid; hmin && i < ZW_MIN_PARTS * 4; i += 256) {
      double m = DINF;
      for (int k = 0; k < world; k++) m = fmin(m, (&hdr(k)->hmin[0][0])[i]);
      (&hmin[0])[i] = m;
    }
    return;
  }
  auto slot = [&](int k) { return reinterpret_cast<const FrontierSlot*>(hdr(k) + 1) + b; };
  if (tid == 0) {
    int o = 0, tot = 0;
    for (int k = 0; k < world; k++) { off[k] = o; o += slot(k)->n; tot += slot(k)->total; }
    off[world] = o;
    out[b].n = min(o, ZW_M);
    out[b].total = tot;
  }
  __syncthreads();
  for (int k = 0; k < world && off[k] < ZW_M; k++) {
    const FrontierSlot* s = slot(k);
    const int n = min(s->n, ZW_M - off[k]);
    for (int p = tid; p < n; p += 256) {
      const int q = off[k] + p;
      out[b].id[q] = s->id[p];
#pragma unroll
      for (int r = 0; r < 4; r++) out[b].a[r][q] = s->a[r][p];
    }
  }
}

void launch_zwin_build(const ZwinArgs& a, int nchains, hipStream_t st) {
  PVT_LAUNCH(zwin_build_kernel, dim3(nchains), dim3(ZW_THREADS), 0, st, a);
}
void launch_zwin_gather(const double* avail, int H, int lo, const int32_t* perm,
                        const int32_t* count, FrontierSlot* out, hipStream_t st) {
  PVT_LAUNCH(zwin_gather_kernel, dim3(1), dim3(256), 0, st, avail, H, lo, perm, count, out);
}
void launch_zwin_merge(const uint8_t* pkgs, int64_t pkg_bytes, int world, int nslots,
                       FrontierSlot* out, double* hmin, hipStream_t st) {
  PVT_LAUNCH(zwin_merge_kernel, dim3(nslots + 1), dim3(256), 0, st, pkgs, pkg_bytes, world,
                     nslots, out, hmin);
}

}  // namespace pvt
