// pvt_batch.hip — resident rounds: one workgroup runs one whole scheduling round with the
// round's hosts held in registers; a launch runs a batch of independent rounds (one per block).
//
// Reference: the same sequential loops as the windowed engine (scheduler/cost_aware.py:84-97,
// :117-127; scheduler/opportunistic.py:11-20; scheduler/vbp.py:19-25, :43-49), visited in the
// reference's order (cost_aware.py:37,60-61 groups + stable sort; vbp.py:17,41). This kernel is
// their direct restatement rather than the snapshot/list formulation: with H <= 4096 hosts a
// round fits in one workgroup's registers (host h lives in thread h / HPL, slot h % HPL, all
// four capacities, its zone, its tiebreak rank and its frozen first-fit key), so every task
// rescans every host at register speed, commits in place, and no state leaves the CU until the
// round ends. It serves
//   - scenario batches (BASELINE config 4): B independent rounds in
//     ONE launch, one block each, so the rounds' sequential walks run side by side on all CUs;
//   - single rounds of the sim.py sizes (100-1000 hosts, configs 1-2) through pvt_place.
//
// A round runs on WAVES = 4 or 8 waves (one workgroup; HPL = hosts per lane, H <= 256 * 16).
// Per task, cost_aware and first-fit rounds first look for the FAST winner, a 32-bit host index:
//   first-fit by index (vbp first-fit, cost_aware first-fit without sort_hosts): the lowest-
//     index fitting host (blocked host mapping: lane order, then slot order, is index order);
//   cost_aware best-fit: the lowest-index fitting host of score exactly 0 -- a zero-cost zone
//     pair (c == 0, bw > 0) or an exact fit (s2 == 0) -- unless some fitting host's score might
//     underflow to 0 (c < 2^-300, s2 < 2^-600, bw > 2^300, or bw not > 0 with c == 0: "risky");
//   keyed cost_aware first-fit: the lowest-index fitting host of frozen key exactly +0.
// Each wave finds its first candidate with one ballot, lane 0 posts it (or "risky") in LDS
// (double-buffered by task parity: ONE barrier per task) and every wave reads all posts with one
// LDS load and takes the minimum. Only when no wave has a fast winner (or one is risky) do the
// waves compute the full 128-bit key (score bits, tiebreak:host) and exchange it after a second
// barrier; vbp best-fit always does (its scores are norms). Measured at config 4 (512 x 1000 x
// 1000): every cost_aware best-fit winner scores 0. Opportunistic rounds reduce feasible counts
// (DPP scan); every wave draws the same randint(0, n) from its own copy of the MT19937 state,
// and the lane holding the k-th feasible host commits it.
//
// Numerics as everywhere in the engine: -ffp-contract=off, sequential-FMA squared norms,
// correctly rounded sqrt/div, scores computed in the reference's operation order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "pivot_place.h"
#include "pvt_device.h"
#include "pvt_anchor_dev.h"
#include "pvt_groups_dev.h"
#include "pvt_kernels.h"
#include "pvt_mt.h"

namespace pvt {

constexpr int RES_MAXW = 8;              // LDS is laid out for up to 8 waves per round
constexpr int RES_CHUNK = 256;           // tasks whose demand rows are staged in LDS at a time
constexpr int RES_MT_STRIDE = 628;       // words per wave-private MT19937 copy (625 used)
constexpr uint64_t NONE = ~0ull;

// Diagnostic phase stamps (PVT_STAMPS builds; tools/resident_stamps.py): block 0, wave 0 only.
#ifdef PVT_STAMPS
constexpr int RES_STAMP_BASE = 32, RES_STAMP_ROUNDS = 4096;   // per-round cycles (stamps build)
__device__ __forceinline__ uint64_t rstamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define RSTAMP(k)                         \
  do {                                    \
    if (stw) {                            \
      const uint64_t t_ = rstamp();       \
      ph[k] += t_ - tl;                   \
      tl = t_;                            \
    }                                     \
  } while (0)
#define RCOUNT(k) do { if (stw) ph[k] += 1; } while (0)
#else
#define RSTAMP(k) do {} while (0)
#define RCOUNT(k) do {} while (0)
#endif

// A run list entry: a host's full key (score bits, tiebreak:host) and its capacities.
struct RunEntry {
  uint64_t k1, k2;
  double c[4];
};
#ifndef PVT_RES_LK
#define PVT_RES_LK 8
#endif
constexpr int RES_LK = PVT_RES_LK;        // run list length (hosts per wave; -DPVT_RES_LK: A/B builds)
constexpr int RES_LIST_MIN = 8;           // run lists only for at least this many remaining tasks

// Dynamic LDS layout (bytes); the host sizes the launch with the same struct.
constexpr int RW_SB = RES_MAX_TASKS / 64; // its suffix minima of the demands, per 64 positions

struct ResLds {
  int zt, ord, pl, u, cd, ci, mt, slot, lst, wa, wz, ws, wx, wd, total;
  __host__ __device__ ResLds(int Zb, int Tpad, bool walk = false) {
    zt = 0;                                            // csum[Zb*Zb], bsum[Zb*Zb] f64
    ord = (16 * Zb * Zb + 15) & ~15;                   // processing order i32[Tpad]
    pl = ord + 4 * Tpad;                               // placement by position i32[Tpad]
    u = (pl + 4 * Tpad + 15) & ~15;                    // union: sort keys | walk staging
    cd = u;                                            // walk: demand rows f64[CHUNK][4]
    ci = cd + 32 * RES_CHUNK;                          //       anchor, group i32[2][CHUNK] (+pad)
    mt = ci + 12 * RES_CHUNK;                          //       MT copies u32[WAVES][628]
    slot = mt + 4 * RES_MAXW * RES_MT_STRIDE;          //       posts u64[2][WAVES][2], then
    // fast posts i32[2][WAVES], then vbp best-fit s2 posts {u64, i32, i32}[2][WAVES]
    // (+32: the sticky winner's capacities, f64[4])
    // then the run lists: RunEntry[RES_MAXW][RES_LK] (per wave)
    lst = (slot + 32 * RES_MAXW + 8 * RES_MAXW + 32 * RES_MAXW + 32 + 15) & ~15;
    const int walk_end = lst + (int)sizeof(RunEntry) * RES_MAXW * RES_LK;
    const int sort_end = u + 16 * Tpad;                // sort: u64 ka[Tpad], kb[Tpad]
    // resident walk (after the sort, before the staging above): the round's hosts in LDS,
    // capacities f64[4][RW_MAXH], zones i32[RW_MAXH], suffix minima and maxima of the demands
    // f64[RW_SB][4] each, the zero-cost window of the current anchor (host ids) i32[RW_MAXH]
    wa = u;
    wz = wa + 32 * RW_MAXH;
    ws = wz + 4 * RW_MAXH;
    wx = ws + 32 * RW_SB;
    wd = wx + 32 * RW_SB;
    const int rw_end = walk ? wd + 4 * RW_MAXH : 0;
    total = walk_end > sort_end ? walk_end : sort_end;
    total = rw_end > total ? rw_end : total;
  }
};

size_t resident_lds_bytes(int Zb, int Tpad, bool walk) { return (size_t)ResLds(Zb, Tpad, walk).total; }

__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }

// Stable processing order (a2): sort (group, ~bits(||d||2) or 0, caller index) ascending with a
// bitonic network over Tpad entries; the caller index makes every key distinct, so the result
// is the stable order cost_aware.py:37,60-61 / vbp.py:17,41 produce.
template <int NT>
__device__ void res_order(const pvt_round& R, bool grouped, bool sorted, uint64_t* ka, uint64_t* kb,
                          int32_t* ord, int Tpad) {
  const int T = R.n_tasks, tid = threadIdx.x;
  for (int i = tid; i < Tpad; i += NT) {
    if (i < T) {
      const uint32_t g = grouped ? (uint32_t)G(R.task_group)[i] : 0u;
      ka[i] = ((uint64_t)g << 32) | (uint32_t)i;
      if (sorted) {
        const double n = __builtin_sqrt(norm2_seq(G(R.dem)[i], G(R.dem)[(size_t)T + i],
                                                  G(R.dem)[2 * (size_t)T + i], G(R.dem)[3 * (size_t)T + i]));
        kb[i] = ~dbits(n);                               // descending norm
      } else {
        kb[i] = 0;
      }
    } else {
      ka[i] = NONE;
      kb[i] = NONE;
    }
  }
  __syncthreads();
  if (grouped || sorted) {
    for (int k = 2; k <= Tpad; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < Tpad; i += NT) {
          const int l = i ^ j;
          if (l > i) {
            const uint64_t ai = ka[i], al = ka[l], bi = kb[i], bl = kb[l];
            const uint32_t gi = (uint32_t)(ai >> 32), gl = (uint32_t)(al >> 32);
            const bool less_li = gl < gi || (gl == gi && (bl < bi || (bl == bi && (uint32_t)al < (uint32_t)ai)));
            if (less_li == ((i & k) == 0)) {
              ka[i] = al; ka[l] = ai; kb[i] = bl; kb[l] = bi;
            }
          }
        }
        __syncthreads();
      }
    }
  }
  for (int i = tid; i < T; i += NT) ord[i] = (int32_t)(uint32_t)ka[i];
  __syncthreads();
}

// The bulk step of the resident walks: a run of R tasks with demand d (every component >= 0 and
// finite) on one 64-host chunk (capacities c*, finite; m0 = its lanes that fit d, the lowest one
// the first task's winner). Sequentially the run fills the fitting lanes in index order, each
// until it cannot take another copy (a - d rounded keeps the sign of a - d, so x_{j-1} fits iff
// x_j >= 0, or > 0 strict; with d >= 0 a lane that fails a copy fails every later one): every
// lane counts its copies by repeated subtraction (8 per check) until the lanes up to the lowest
// still-fitting one cover the run, lane l takes asg = clamp(R - pre, 0, cnt) tasks (pre: the
// copies of the lanes before it), and replays exactly its own subtractions. With d2 = d3 = +0
// (disk and gpus of the trace's tasks) only cpus and memory are counted and updated (x - +0 == x),
// where TWO allows it (the first-fit walk; in the cost_aware best-fit walk the extra branch
// measured 3 % slower at config 4: 0.438 vs 0.426 ms). Returns the tasks placed (>= 1).
template <bool STRICT, bool TWO>
__device__ __forceinline__ int bulk_run(double& c0, double& c1, double& c2, double& c3, uint64_t m0,
                                        double d0, double d1, double d2, double d3, int R,
                                        int& pre_out, int& asg_out) {
  const int lane = lane_id();
  const bool on = (m0 >> lane) & 1ull;
  const bool two = TWO && __double_as_longlong(d2) == 0 && __double_as_longlong(d3) == 0;
  double x0 = on ? c0 : -DINF, x1 = on ? c1 : -DINF, x2 = on ? c2 : -DINF, x3 = on ? c3 : -DINF;
  int cnt = 0, t = 0, u = __builtin_ctzll(m0), fb = 0;
  auto pass1 = [&](auto dims) {
    constexpr int D = decltype(dims)::value;
    for (;;) {
      t = __builtin_amdgcn_readfirstlane(t);
      u = __builtin_amdgcn_readfirstlane(u);
      fb = __builtin_amdgcn_readfirstlane(fb);
      bool f = false;
#pragma unroll
      for (int j = 1; j <= 8; j++) {
        x0 -= d0; x1 -= d1;
        if (D == 4) { x2 -= d2; x3 -= d3; }
        const double mx = D == 4 ? fmin(fmin(x0, x1), fmin(x2, x3)) : fmin(x0, x1);
        f = STRICT ? (mx > 0.0) : (mx >= 0.0);
        cnt = f ? t + j : cnt;
      }
      t += 8;
      const uint64_t an = __ballot(f);
      if (__builtin_amdgcn_readfirstlane((int)(an == 0))) break;
      const int un = __builtin_ctzll(an);
      if (un != u) {                       // (lanes below un are done)
        u = un;
        fb = __builtin_amdgcn_readlane(wave_incl_scan_dpp(cnt), u - 1);
      }
      if (__builtin_amdgcn_readfirstlane((int)(fb + t >= R))) break;
    }
  };
  if (__builtin_amdgcn_readfirstlane((int)two)) pass1(std::integral_constant<int, 2>{});
  else pass1(std::integral_constant<int, 4>{});
  const int incl = wave_incl_scan_dpp(cnt);
  const int pre = incl - cnt;
  const int asg = max(0, min(cnt, R - pre));
  const int covered = min(R, __builtin_amdgcn_readlane(incl, 63));
  // replay: each taking lane's own subtractions, in order (fma(-0, d, c) == c)
  const int amax = wave_max_i32(asg);
  if (__builtin_amdgcn_readfirstlane((int)two)) {
    for (int m = 0; m < amax; m++) {
      const double o = m < asg ? -1.0 : -0.0;
      c0 = __builtin_fma(o, d0, c0);
      c1 = __builtin_fma(o, d1, c1);
    }
  } else {
    for (int m = 0; m < amax; m++) {
      const double o = m < asg ? -1.0 : -0.0;
      c0 = __builtin_fma(o, d0, c0);
      c1 = __builtin_fma(o, d1, c1);
      c2 = __builtin_fma(o, d2, c2);
      c3 = __builtin_fma(o, d3, c3);
    }
  }
  pre_out = pre;
  asg_out = asg;
  return covered;
}

// ---- the resident walk: one wave places the round's tasks in order over its hosts in LDS
// cost_aware best-fit takes, per task, the LOWEST-INDEX fitting host of score exactly 0 --
// zero-cost zone pair or exact fit (the fast winner of the 4-wave path below, with its "risky"
// rule: a fitting host whose score might underflow to 0 below the winner, or no zero-score host
// at all, stops the walk). (The first-fit policies measured faster on the 4-wave path, whose
// block scan exits early: config 4, 512 rounds, ca_ff 0.753 vs 0.710 ms, vbp_ff 0.558 vs
// 0.524 ms walked vs not; so only cost_aware best-fit is walked.)
// Wave 0 holds chunk p0 (64 hosts, host p0 * 64 + lane) in registers -- the first chunk any
// remaining task can still fit (suffix minima of the demands per 64 positions; capacities only
// fall, so a chunk that cannot fit the componentwise least remaining demand never will) -- and
// nearly every task finds its winner there with one fit test and a ballot, no barrier and no
// memory access on its path; otherwise the later chunks are scanned in LDS. The other waves wait
// at the closing barrier. Returns the first position the walk did not decide (T: all); the
// 4-wave path goes on from there on the walked capacities.
template <int NT>
__device__ int resident_walk(const pvt_round& R, const ResLds& Lo, char* smem, const int32_t* ord,
                             int32_t* pl, const double* csum, const double* bsum, bool has_groups,
                             int walker, bool bulk, uint64_t* A_stamps) {
  __shared__ int s_stop;
  const int T = R.n_tasks, H = R.n_hosts, Z = R.n_zones;
  const int tid = threadIdx.x, lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* wa = reinterpret_cast<double*>(smem + Lo.wa);      // [4][RW_MAXH]
  int32_t* wz = reinterpret_cast<int32_t*>(smem + Lo.wz);
  double* ws = reinterpret_cast<double*>(smem + Lo.ws);      // [RW_SB][4]
  double* wx = reinterpret_cast<double*>(smem + Lo.wx);      // [RW_SB][4]
  int32_t* wd = reinterpret_cast<int32_t*>(smem + Lo.wd);    // [RW_MAXH]
  for (int h = tid; h < H; h += NT) {
#pragma unroll
    for (int r = 0; r < 4; r++) wa[r * RW_MAXH + h] = G(R.avail)[(size_t)r * H + h];
    wz[h] = G(R.zone)[h];
  }
  const int nsb = (T + 63) >> 6;
  for (int blk = wave; blk < nsb; blk += NT / WAVE) {
    double m[4] = {DINF, DINF, DINF, DINF}, x[4] = {-DINF, -DINF, -DINF, -DINF};
    const int i = blk * 64 + lane;
    if (i < T) {
      const int t = ord[i];
#pragma unroll
      for (int r = 0; r < 4; r++) m[r] = x[r] = G(R.dem)[(size_t)r * T + t];
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      for (int off = 32; off > 0; off >>= 1) {
        m[r] = fmin(m[r], __shfl_xor(m[r], off));
        x[r] = fmax(x[r], __shfl_xor(x[r], off));
      }
      if (lane == 0) { ws[blk * 4 + r] = m[r]; wx[blk * 4 + r] = x[r]; }
    }
  }
  __syncthreads();
  if (tid < 4)
    for (int blk = nsb - 2; blk >= 0; blk--) ws[blk * 4 + tid] = fmin(ws[blk * 4 + tid], ws[(blk + 1) * 4 + tid]);
  else if (tid >= 64 && tid < 68)
    for (int blk = nsb - 2; blk >= 0; blk--)
      wx[blk * 4 + tid - 64] = fmax(wx[blk * 4 + tid - 64], wx[(blk + 1) * 4 + tid - 64]);
  __syncthreads();
  if (wave == walker) {
#ifdef PVT_STAMPS
    uint64_t n_probe = 0, n_adv = 0, st_task = 0, n_bulk = 0, n_bulk_tasks = 0;
    const uint64_t tw_start = rstamp();
#endif
    const int nch = (H + 63) >> 6;
    int p0 = 0;
    double ra0, ra1, ra2, ra3;
    int32_t rz = 0;
    bool rv = false;
    auto load_chunk = [&](int c) {
      const int q = c * 64 + lane;
      rv = q < H;
      const int qq = rv ? q : 0;
      ra0 = wa[qq]; ra1 = wa[RW_MAXH + qq]; ra2 = wa[2 * RW_MAXH + qq]; ra3 = wa[3 * RW_MAXH + qq];
      rz = wz[qq];
    };
    auto store_chunk = [&](int c) {
      const int q = c * 64 + lane;
      if (rv) { wa[q] = ra0; wa[RW_MAXH + q] = ra1; wa[2 * RW_MAXH + q] = ra2; wa[3 * RW_MAXH + q] = ra3; }
    };
    load_chunk(0);
    // zones of score 0 for the current anchor, and the safe zones: bw in (0, 2^300] and c == 0
    // or c in [2^-300, inf) -- as the 4-wave path's zmask / rmask
    uint32_t zc_z = 0, sf_z = 0;
    int cur_anc = -1;
    // the same as lane masks of the register chunk (recomputed when the anchor or the chunk
    // changes): valid hosts, safe zones, safe zero-cost zones
    uint64_t m_v = 0, m_sf = 0, m_zs = 0;
    auto chunk_masks = [&]() {
      const bool sf = rv && ((sf_z >> rz) & 1u), zc = (zc_z >> rz) & 1u;
      m_v = __ballot(rv);
      m_sf = __ballot(sf);
      m_zs = __ballot(sf && zc);
    };
    // Zero-cost window of the current anchor (the resident form of the frontier walk's window,
    // pvt_zwalk.hip): the anchor's zero-cost hosts in index order (wd, nd of them), walked 64 at
    // a time in registers (dense chunk dp0: host wd[dp0 * 64 + lane], capacities gathered from
    // and written back to wa), so every chunk holds only hosts that can score 0. Exact when
    //   (i) every zone is safe for the anchor (sf_z full): a fitting zero-cost host scores
    //       exactly 0 unless a residual exceeds 2^500 (checked on the winner: stop), and
    //  (ii) some dimension r separates every other host from every remaining demand by 2^-288:
    //       min over them of a_r - max over the tasks of d_r >= 2^-288, so none fits exactly
    //       (score 0) or with every residual below 2^-300 (risky); their capacities do not
    //       change while the anchor lasts (the walk commits only zero-cost hosts).
    // Then the winner is the first fitting host of the window, as in the full test.
    bool dense = false;
    int nwin = 0, dp0 = 0;
    int32_t rid = 0;
    auto load_dense = [&](int c) {
      const int i = c * 64 + lane;
      rv = i < nwin;
      rid = rv ? wd[i] : 0;
      ra0 = wa[rid]; ra1 = wa[RW_MAXH + rid]; ra2 = wa[2 * RW_MAXH + rid]; ra3 = wa[3 * RW_MAXH + rid];
    };
    auto store_dense = [&]() {
      if (rv) { wa[rid] = ra0; wa[RW_MAXH + rid] = ra1; wa[2 * RW_MAXH + rid] = ra2; wa[3 * RW_MAXH + rid] = ra3; }
    };
    auto leave_dense = [&]() {
      if (!dense) return;
      store_dense();
      dense = false;
      load_chunk(p0);
    };
    auto enter_dense = [&](int b) {
      const uint32_t allz = Z >= 32 ? 0xffffffffu : ((1u << Z) - 1u);
      if (__builtin_amdgcn_readfirstlane((int)(zc_z == 0 || (sf_z & allz) != allz))) return;
      // (ii): the other hosts' least capacities against the remaining tasks' largest demands
      double q0 = DINF, q1 = DINF, q2 = DINF, q3 = DINF;
      for (int c = 0; c < nch; c++) {
        const int q = c * 64 + lane;
        if (q < H && !((zc_z >> wz[q]) & 1u)) {
          q0 = fmin(q0, wa[q]); q1 = fmin(q1, wa[RW_MAXH + q]);
          q2 = fmin(q2, wa[2 * RW_MAXH + q]); q3 = fmin(q3, wa[3 * RW_MAXH + q]);
        }
      }
      for (int off = 32; off > 0; off >>= 1) {
        q0 = fmin(q0, __shfl_xor(q0, off)); q1 = fmin(q1, __shfl_xor(q1, off));
        q2 = fmin(q2, __shfl_xor(q2, off)); q3 = fmin(q3, __shfl_xor(q3, off));
      }
      const bool sep = (q0 - wx[b * 4 + 0] >= 0x1p-288) || (q1 - wx[b * 4 + 1] >= 0x1p-288) ||
                       (q2 - wx[b * 4 + 2] >= 0x1p-288) || (q3 - wx[b * 4 + 3] >= 0x1p-288);
      if (__builtin_amdgcn_readfirstlane((int)!sep)) return;
      store_chunk(p0);
      const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
      int n = 0;
      for (int c = 0; c < nch; c++) {
        const int q = c * 64 + lane;
        const bool in = q < H && ((zc_z >> wz[q]) & 1u);
        const uint64_t m = __ballot(in);
        if (in) wd[n + __popcll(m & below)] = q;
        n += __popcll(m);
      }
      wave_sync();                             // (the window ids before this wave reads them)
      nwin = n;
      dense = true;
      dp0 = 0;
      load_dense(0);
    };
    // the task records of a 64-position batch in lanes (the next batch's loads in flight)
    auto rec = [&](int b, double (&d)[4], int& anc) {
      const int i = b * 64 + lane;
      const int t = i < T ? ord[i] : 0;
#pragma unroll
      for (int r = 0; r < 4; r++) d[r] = G(R.dem)[(size_t)r * T + t];
      anc = has_groups ? G(R.group_anchor)[G(R.task_group)[t]] : 0;
    };
    double nd[4];
    int nanc;
    rec(0, nd, nanc);
    int p = 0;
    bool stop = false;
    for (int b = 0; b < nsb && !stop; b++) {
      double td[4] = {nd[0], nd[1], nd[2], nd[3]};
      const int tanc = nanc;
      // tasks of the batch with a non-finite demand component (the 4-wave path decides them)
      const uint64_t nonfin = __ballot(!(__builtin_fabs(td[0]) < DINF && __builtin_fabs(td[1]) < DINF &&
                                         __builtin_fabs(td[2]) < DINF && __builtin_fabs(td[3]) < DINF));
      if (b + 1 < nsb) rec(b + 1, nd, nanc);
      const double mn0 = ws[b * 4 + 0], mn1 = ws[b * 4 + 1], mn2 = ws[b * 4 + 2], mn3 = ws[b * 4 + 3];
      const int kn = min(64, T - b * 64);
      // runs: bit i set iff batch task i has task i - 1's demand vector (bit for bit) and anchor
      // (every shuffle with the whole wave active: a lane that skipped one, by short-circuit, would
      // hand its neighbour a zero -- an anchor 0 run that is not one)
      uint64_t E;
      {
        const int pa = __shfl_up(tanc, 1);
        bool same = lane > 0 && lane < kn;
        same &= pa == tanc;
#pragma unroll
        for (int r = 0; r < 4; r++)
          same &= __double_as_longlong(__shfl_up(td[r], 1)) == __double_as_longlong(td[r]);
        E = __ballot(same);
      }
      for (int k = 0; k < kn; k++, p++) {
#ifdef PVT_STAMPS
        const uint64_t tk0 = rstamp();
#endif
        p = __builtin_amdgcn_readfirstlane(p);
        p0 = __builtin_amdgcn_readfirstlane(p0);
        const double d0 = readlane_d(td[0], k), d1 = readlane_d(td[1], k);
        const double d2 = readlane_d(td[2], k), d3 = readlane_d(td[3], k);
        {
          const int a = readlane_i(tanc, k);
          if (a != cur_anc) {
            leave_dense();
            cur_anc = a;
            bool zc = false, sf = false;
            if (lane < Z) {
              const double c = csum[a * Z + lane], bw = bsum[a * Z + lane];
              zc = c == 0.0;
              sf = bw > 0.0 && bw <= 0x1p+300 && (c == 0.0 || (c >= 0x1p-300 && c < DINF));
            }
            zc_z = (uint32_t)__ballot(zc);
            sf_z = (uint32_t)__ballot(sf);
            enter_dense(b);
            chunk_masks();
          }
        }
        if ((nonfin >> k) & 1ull) {
          stop = true;                         // (a non-finite demand: the 4-wave path decides)
          break;
        }
        // A run of R >= 2 tasks with this demand (and anchor) on the dense register chunk
        // (run_bulk, as the frontier walk's, pvt_zwalk.hip): sequentially the run fills the
        // chunk's fitting lanes in index order, each until it cannot take another copy (d >= 0:
        // a lane that fails a copy fails every later one, one that does not fit now never will),
        // so every lane counts its copies in parallel, the lanes take the run's tasks in order
        // and replay exactly their own subtractions. Taken only when the first task's winner is
        // in the chunk and no fitting lane holds a capacity above 2^500 (the per-task stop).
        if (bulk && dense && k + 1 < kn && ((E >> (k + 1)) & 1ull) && d0 >= 0.0 && d1 >= 0.0 &&
            d2 >= 0.0 && d3 >= 0.0) {
          const uint64_t m0 = __ballot(rv && ra0 >= d0 && ra1 >= d1 && ra2 >= d2 && ra3 >= d3);
          const uint64_t big = __ballot(rv && !(ra0 <= 0x1p+500 && ra1 <= 0x1p+500 &&
                                                ra2 <= 0x1p+500 && ra3 <= 0x1p+500));
          if (m0 != 0 && (m0 & big) == 0) {
            const int R = min(kn - k, 1 + (int)__builtin_ctzll(~(E >> (k + 1))));
            int pre, asg;
            const int covered = bulk_run<false, false>(ra0, ra1, ra2, ra3, m0, d0, d1, d2, d3, R, pre, asg);
            // positions p .. p + covered - 1 to their hosts (a few taking lanes)
            int who = 0;
            for (uint64_t tk = __ballot(asg > 0); tk; tk &= tk - 1) {
              const int L = __builtin_ctzll(tk);
              const int s0 = __builtin_amdgcn_readlane(pre, L), s1 = s0 + __builtin_amdgcn_readlane(asg, L);
              const int id = __builtin_amdgcn_readlane(rid, L);
              if (lane >= s0 && lane < s1) who = id;
            }
            if (lane < covered) pl[p + lane] = who;
#ifdef PVT_STAMPS
            n_bulk++;
            n_bulk_tasks += covered;
#endif
            k += covered - 1;                  // (the loop's increments add the last one)
            p += covered - 1;
#ifdef PVT_STAMPS
            st_task += rstamp() - tk0;
#endif
            continue;
          }
        }
        // Fast path, in lane masks (SALU), on the register chunk: C = fitting hosts of safe
        // zero-cost zones; its first, w, wins -- exactly the test below -- unless (a) a fitting
        // host before w is in an unsafe zone (risky), (b) one of a safe zone has every residual
        // below 2^-300 (an exact fit, which would win, or a risky one), or (c) w has a residual
        // above 2^500 (its score need not be 0). Any of those, or no C: the full test.
        int win = -1;                           // host index, -1 none, -2 stop
        bool done = false;
        if (dense) {
          // the window: the first fitting zero-cost host (chunks no remaining task can use
          // are passed for good; later ones probed from LDS)
          uint64_t F = __ballot(rv && ra0 >= d0 && ra1 >= d1 && ra2 >= d2 && ra3 >= d3);
          while (F == 0 && (dp0 + 1) * 64 < nwin &&
                 !__ballot(rv && ra0 >= mn0 && ra1 >= mn1 && ra2 >= mn2 && ra3 >= mn3)) {
            store_dense();
            ++dp0;
            load_dense(dp0);
            F = __ballot(rv && ra0 >= d0 && ra1 >= d1 && ra2 >= d2 && ra3 >= d3);
          }
          if (F) {
            const int w = __builtin_ctzll(F);
            const double x0 = ra0 - d0, x1 = ra1 - d1, x2 = ra2 - d2, x3 = ra3 - d3;
            if (__ballot(lane == w && (x0 > 0x1p+500 || x1 > 0x1p+500 || x2 > 0x1p+500 || x3 > 0x1p+500))) {
              win = -2;                         // (a huge residual: the score need not be 0)
            } else {
              if (lane == w) { ra0 = x0; ra1 = x1; ra2 = x2; ra3 = x3; }   // resc[h] -= d
              win = __builtin_amdgcn_readlane(rid, w);
            }
          } else {
            for (int c = dp0 + 1; c * 64 < nwin; c++) {
#ifdef PVT_STAMPS
              n_probe++;
#endif
              const int i = c * 64 + lane;
              const bool v = i < nwin;
              const int32_t h = v ? wd[i] : 0;
              const double y0 = wa[h], y1 = wa[RW_MAXH + h], y2 = wa[2 * RW_MAXH + h], y3 = wa[3 * RW_MAXH + h];
              const uint64_t F2 = __ballot(v && y0 >= d0 && y1 >= d1 && y2 >= d2 && y3 >= d3);
              if (F2) {
                const int w = __builtin_ctzll(F2);
                const double x0 = y0 - d0, x1 = y1 - d1, x2 = y2 - d2, x3 = y3 - d3;
                if (__ballot(lane == w && (x0 > 0x1p+500 || x1 > 0x1p+500 || x2 > 0x1p+500 || x3 > 0x1p+500))) {
                  win = -2;
                } else {
                  if (lane == w) { wa[h] = x0; wa[RW_MAXH + h] = x1; wa[2 * RW_MAXH + h] = x2; wa[3 * RW_MAXH + h] = x3; }
                  win = __builtin_amdgcn_readlane(h, w);
                }
                break;
              }
            }
            // no zero-cost host fits: a positive-score winner only the 4-wave path finds
            if (win == -1) win = -2;
          }
          done = true;
        }
        if (!done) {
          const uint64_t F = m_v & __ballot(ra0 >= d0) & __ballot(ra1 >= d1) &
                             __ballot(ra2 >= d2) & __ballot(ra3 >= d3);
          const uint64_t C = F & m_zs;
          if (C) {
            const int w = __builtin_ctzll(C);
            const uint64_t Lx = F & ~m_zs & ((1ull << w) - 1ull);
            const double x0 = ra0 - d0, x1 = ra1 - d1, x2 = ra2 - d2, x3 = ra3 - d3;
            const uint64_t tight = __ballot(x0 < 0x1p-300) & __ballot(x1 < 0x1p-300) &
                                   __ballot(x2 < 0x1p-300) & __ballot(x3 < 0x1p-300);
            const uint64_t huge = __ballot(x0 > 0x1p+500) | __ballot(x1 > 0x1p+500) |
                                  __ballot(x2 > 0x1p+500) | __ballot(x3 > 0x1p+500);
            if (!(Lx & (~m_sf | tight)) && !((huge >> w) & 1ull)) {
              if (lane == w) { ra0 = x0; ra1 = x1; ra2 = x2; ra3 = x3; }   // resc[h] -= d
              win = p0 * 64 + w;
              done = true;
            }
          }
        }
        // one chunk's candidates: zm = fitting hosts of the zero class, rk = risky fitting hosts
        auto test = [&](double x0, double x1, double x2, double x3, int32_t z, bool v,
                        uint64_t& zm, uint64_t& rk) {
          const bool f = v && fits<false>(x0, x1, x2, x3, d0, d1, d2, d3);   // (>=, cost_aware.py:91)
          const double mx = fmax(fmax(x0 - d0, x1 - d1), fmax(x2 - d2, x3 - d3));
          const bool sf = (sf_z >> z) & 1u, zc = (zc_z >> z) & 1u;
          const bool zz = sf && ((zc && mx <= 0x1p+500) || mx == 0.0);
          const bool risky = f && !zz && (!sf || !(mx >= 0x1p-300) || zc);
          zm = __ballot(f && zz);
          rk = __ballot(risky);
        };
        if (!done) {
          uint64_t zm, rk;
          test(ra0, ra1, ra2, ra3, rz, rv, zm, rk);
          while (zm == 0 && rk == 0 && p0 + 1 < nch &&
                 !__ballot(rv && fits<false>(ra0, ra1, ra2, ra3, mn0, mn1, mn2, mn3))) {
            store_chunk(p0);                   // dead: move the register chunk on
#ifdef PVT_STAMPS
            n_adv++;
#endif
            ++p0;
            load_chunk(p0);
            test(ra0, ra1, ra2, ra3, rz, rv, zm, rk);
          }
          if (zm != 0) {
            const int w = __builtin_ctzll(zm);
            if (rk & ((1ull << w) - 1)) {
              win = -2;
            } else {
              if (lane == w) { ra0 -= d0; ra1 -= d1; ra2 -= d2; ra3 -= d3; }   // resc[h] -= d
              win = p0 * 64 + w;
            }
          } else if (rk != 0) {
            win = -2;
          } else {
            for (int c = p0 + 1; c < nch; c++) {
#ifdef PVT_STAMPS
              n_probe++;
#endif
              const int q = c * 64 + lane;
              const bool v = q < H;
              const int qq = v ? q : 0;
              const double x0 = wa[qq], x1 = wa[RW_MAXH + qq], x2 = wa[2 * RW_MAXH + qq], x3 = wa[3 * RW_MAXH + qq];
              uint64_t zm2, rk2;
              test(x0, x1, x2, x3, wz[qq], v, zm2, rk2);
              if (zm2 != 0) {
                const int w = __builtin_ctzll(zm2);
                if (rk2 & ((1ull << w) - 1)) { win = -2; break; }
                if (lane == w) {
                  wa[q] = x0 - d0; wa[RW_MAXH + q] = x1 - d1; wa[2 * RW_MAXH + q] = x2 - d2;
                  wa[3 * RW_MAXH + q] = x3 - d3;
                }
                win = c * 64 + w;
                break;
              }
              if (rk2 != 0) { win = -2; break; }
            }
            // no score-0 host fits: a positive-score winner only the 4-wave path finds
            if (win == -1) win = -2;
          }
          chunk_masks();                        // (the register chunk may have moved on)
        }
        win = __builtin_amdgcn_readfirstlane(win);
        if (win == -2) { stop = true; break; }
        if (win >= 0 && lane == 0) pl[p] = win;
#ifdef PVT_STAMPS
        st_task += rstamp() - tk0;
#endif
      }
    }
    leave_dense();
    store_chunk(p0);
    if (lane == 0) s_stop = p;
#ifdef PVT_STAMPS
    if (blockIdx.x == 0 && lane == 0 && A_stamps) {
      A_stamps[10] += n_probe;
      A_stamps[11] += n_adv;
      A_stamps[13] += st_task;                  // cycles inside the task loop bodies
      A_stamps[24] += n_bulk;                   // bulk runs and the tasks they placed
      A_stamps[25] += n_bulk_tasks;
      A_stamps[14] += rstamp() - tw_start;      // wave 0's whole walk (records included)
    }
#endif
  }
  __syncthreads();
  return s_stop;
}

// ---- the first-fit resident walk (vbp first-fit, fit >=: vbp.py:13-29; cost_aware first-fit
// without sort_hosts, strict fit: cost_aware.py:99-127 in host order). Each task takes the
// LOWEST-INDEX host that fits, so one wave walks the hosts in index order: chunk p0 (host
// p0 * 64 + lane) in registers, the first chunk that can still fit some remaining task (suffix
// minima of the demands per 64 positions; a chunk that cannot fit the componentwise least
// remaining demand never will), later chunks probed in LDS; a task no host fits stays unplaced.
// Runs of equal demands are placed in one step on the register chunk (as resident_walk's dense
// path). Walks every task (returns T); the 4-wave path then only writes the results.
template <int NT, bool STRICT>
__device__ int resident_walk_ff(const pvt_round& R, const ResLds& Lo, char* smem, const int32_t* ord,
                                int32_t* pl, int walker, bool bulk, uint64_t* A_stamps) {
  const int T = R.n_tasks, H = R.n_hosts;
  const int tid = threadIdx.x, lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* wa = reinterpret_cast<double*>(smem + Lo.wa);      // [4][RW_MAXH]
  double* ws = reinterpret_cast<double*>(smem + Lo.ws);      // [RW_SB][4]
  for (int h = tid; h < H; h += NT) {
#pragma unroll
    for (int r = 0; r < 4; r++) wa[r * RW_MAXH + h] = G(R.avail)[(size_t)r * H + h];
  }
  const int nsb = (T + 63) >> 6;
  for (int blk = wave; blk < nsb; blk += NT / WAVE) {
    double m[4] = {DINF, DINF, DINF, DINF};
    const int i = blk * 64 + lane;
    if (i < T) {
      const int t = ord[i];
#pragma unroll
      for (int r = 0; r < 4; r++) m[r] = G(R.dem)[(size_t)r * T + t];
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      for (int off = 32; off > 0; off >>= 1) m[r] = fmin(m[r], __shfl_xor(m[r], off));
      if (lane == 0) ws[blk * 4 + r] = m[r];
    }
  }
  __syncthreads();
  if (tid < 4)
    for (int blk = nsb - 2; blk >= 0; blk--) ws[blk * 4 + tid] = fmin(ws[blk * 4 + tid], ws[(blk + 1) * 4 + tid]);
  __syncthreads();
  if (wave == walker) {
#ifdef PVT_STAMPS
    uint64_t n_probe = 0, n_adv = 0, st_task = 0, n_bulk = 0, n_bulk_tasks = 0;
    const uint64_t tw_start = rstamp();
#endif
    const int nch = (H + 63) >> 6;
    int p0 = 0;
    double ra0, ra1, ra2, ra3;
    bool rv = false;
    auto load_chunk = [&](int c) {
      const int q = c * 64 + lane;
      rv = q < H;
      const int qq = rv ? q : 0;
      ra0 = wa[qq]; ra1 = wa[RW_MAXH + qq]; ra2 = wa[2 * RW_MAXH + qq]; ra3 = wa[3 * RW_MAXH + qq];
    };
    auto store_chunk = [&](int c) {
      const int q = c * 64 + lane;
      if (rv) { wa[q] = ra0; wa[RW_MAXH + q] = ra1; wa[2 * RW_MAXH + q] = ra2; wa[3 * RW_MAXH + q] = ra3; }
    };
    load_chunk(0);
    auto rec = [&](int b, double (&d)[4]) {
      const int i = b * 64 + lane;
      const int t = i < T ? ord[i] : 0;
#pragma unroll
      for (int r = 0; r < 4; r++) d[r] = G(R.dem)[(size_t)r * T + t];
    };
    double nd[4];
    rec(0, nd);
    int p = 0;
    for (int b = 0; b < nsb; b++) {
      double td[4] = {nd[0], nd[1], nd[2], nd[3]};
      if (b + 1 < nsb) rec(b + 1, nd);
      const double mn0 = ws[b * 4 + 0], mn1 = ws[b * 4 + 1], mn2 = ws[b * 4 + 2], mn3 = ws[b * 4 + 3];
      const int kn = min(64, T - b * 64);
      uint64_t E;                              // (every shuffle with the whole wave active)
      {
        bool same = lane > 0 && lane < kn;
#pragma unroll
        for (int r = 0; r < 4; r++)
          same &= __double_as_longlong(__shfl_up(td[r], 1)) == __double_as_longlong(td[r]);
        E = __ballot(same);
      }
      for (int k = 0; k < kn; k++, p++) {
#ifdef PVT_STAMPS
        const uint64_t tk0 = rstamp();
#endif
        p = __builtin_amdgcn_readfirstlane(p);
        p0 = __builtin_amdgcn_readfirstlane(p0);
        const double d0 = readlane_d(td[0], k), d1 = readlane_d(td[1], k);
        const double d2 = readlane_d(td[2], k), d3 = readlane_d(td[3], k);
        // the register chunk: past chunks no remaining task can use
        uint64_t F = __ballot(rv && fits<STRICT>(ra0, ra1, ra2, ra3, d0, d1, d2, d3));
        while (F == 0 && p0 + 1 < nch &&
               !__ballot(rv && fits<STRICT>(ra0, ra1, ra2, ra3, mn0, mn1, mn2, mn3))) {
          store_chunk(p0);
#ifdef PVT_STAMPS
          n_adv++;
#endif
          ++p0;
          load_chunk(p0);
          F = __ballot(rv && fits<STRICT>(ra0, ra1, ra2, ra3, d0, d1, d2, d3));
        }
        // a run of R >= 2 tasks with this demand: placed in one step on the first chunk that
        // fits its first task -- the register chunk, else the first LDS chunk that does (taken
        // into registers for the step and written back). Every fitting lane counts its copies
        // (d >= 0 and finite capacities: a - d rounded keeps the sign of a - d, so x_{j-1} fits
        // iff x_j >= 0, or > 0 strict; a lane that fails a copy fails every later one), the lanes
        // take the run in order and replay their subtractions.
        if (bulk && k + 1 < kn && ((E >> (k + 1)) & 1ull) && d0 >= 0.0 && d1 >= 0.0 &&
            d2 >= 0.0 && d3 >= 0.0 && d0 < DINF && d1 < DINF && d2 < DINF && d3 < DINF) {
          int c = p0;
          uint64_t m0 = F;
          double y0 = ra0, y1 = ra1, y2 = ra2, y3 = ra3;
          bool yv = rv;
          if (m0 == 0) {
            for (c = p0 + 1; c < nch; c++) {
              const int q = c * 64 + lane;
              yv = q < H;
              const int qq = yv ? q : 0;
              y0 = wa[qq]; y1 = wa[RW_MAXH + qq]; y2 = wa[2 * RW_MAXH + qq]; y3 = wa[3 * RW_MAXH + qq];
              m0 = __ballot(yv && fits<STRICT>(y0, y1, y2, y3, d0, d1, d2, d3));
              if (m0) break;
            }
          }
          c = __builtin_amdgcn_readfirstlane(c);
          if (m0 != 0 && !(__ballot(!(__builtin_fabs(y0) < DINF && __builtin_fabs(y1) < DINF &&
                                       __builtin_fabs(y2) < DINF && __builtin_fabs(y3) < DINF)) & m0)) {
            const int R = min(kn - k, 1 + (int)__builtin_ctzll(~(E >> (k + 1))));
            int pre, asg;
            const int covered = bulk_run<STRICT, true>(y0, y1, y2, y3, m0, d0, d1, d2, d3, R, pre, asg);
            int who = 0;
            for (uint64_t tk = __ballot(asg > 0); tk; tk &= tk - 1) {
              const int L = __builtin_ctzll(tk);
              const int s0 = __builtin_amdgcn_readlane(pre, L), s1 = s0 + __builtin_amdgcn_readlane(asg, L);
              if (lane >= s0 && lane < s1) who = c * 64 + L;
            }
            if (lane < covered) pl[p + lane] = who;
            if (c == p0) {
              ra0 = y0; ra1 = y1; ra2 = y2; ra3 = y3;
            } else if (asg > 0) {              // (an LDS chunk: its taking lanes write back)
              const int q = c * 64 + lane;
              wa[q] = y0; wa[RW_MAXH + q] = y1; wa[2 * RW_MAXH + q] = y2; wa[3 * RW_MAXH + q] = y3;
            }
#ifdef PVT_STAMPS
            n_bulk++;
            n_bulk_tasks += covered;
            st_task += rstamp() - tk0;
#endif
            k += covered - 1;
            p += covered - 1;
            continue;
          }
        }
        int win = -1;
        if (F) {
          const int w = __builtin_ctzll(F);
          if (lane == w) { ra0 -= d0; ra1 -= d1; ra2 -= d2; ra3 -= d3; }   // resc[h] -= d
          win = p0 * 64 + w;
        } else {
          for (int c = p0 + 1; c < nch; c++) {
#ifdef PVT_STAMPS
            n_probe++;
#endif
            const int q = c * 64 + lane;
            const bool v = q < H;
            const int qq = v ? q : 0;
            const double y0 = wa[qq], y1 = wa[RW_MAXH + qq], y2 = wa[2 * RW_MAXH + qq], y3 = wa[3 * RW_MAXH + qq];
            const uint64_t F2 = __ballot(v && fits<STRICT>(y0, y1, y2, y3, d0, d1, d2, d3));
            if (F2) {
              const int w = __builtin_ctzll(F2);
              if (lane == w) {
                wa[q] = y0 - d0; wa[RW_MAXH + q] = y1 - d1; wa[2 * RW_MAXH + q] = y2 - d2;
                wa[3 * RW_MAXH + q] = y3 - d3;
              }
              win = c * 64 + w;
              break;
            }
          }
        }
        win = __builtin_amdgcn_readfirstlane(win);
        if (win >= 0 && lane == 0) pl[p] = win;
#ifdef PVT_STAMPS
        st_task += rstamp() - tk0;
#endif
      }
    }
    store_chunk(p0);
#ifdef PVT_STAMPS
    if (blockIdx.x == 0 && lane == 0 && A_stamps) {
      A_stamps[10] += n_probe;
      A_stamps[11] += n_adv;
      A_stamps[13] += st_task;
      A_stamps[14] += rstamp() - tw_start;
      A_stamps[24] += n_bulk;
      A_stamps[25] += n_bulk_tasks;
    }
#endif
  }
  __syncthreads();
  return T;
}

// One round on this workgroup (R: its descriptor, in SGPRs). The MT19937 state of an
// opportunistic round is read and written through R.mt_state (a device pointer in every
// resident path: pvt_place_batch's upload, pvt_place_batch_mt's rows, pvt_place_host's stage).
template <int MODE, int WAVES, int HPL>
__device__ __forceinline__ void resident_round(const ResidentArgs& A, const pvt_round& R) {
  constexpr int NT = WAVES * WAVE;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool CA = (MODE == CA_FF || MODE == CA_BF);
  constexpr bool STRICT = (MODE == CA_FF || MODE == VBP_BF);
  const ResLds Lo(A.Zb, A.Tpad, A.walk != 0);
  const int H = R.n_hosts, T = R.n_tasks, Z = R.n_zones;
  const int tid = threadIdx.x, lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* csum = reinterpret_cast<double*>(smem + Lo.zt);
  double* bsum = csum + A.Zb * A.Zb;
  int32_t* ord = reinterpret_cast<int32_t*>(smem + Lo.ord);
  const bool grouped = (MODE != OPP) && R.task_group && R.n_groups > 1;
  const bool has_groups = (MODE != OPP) && R.task_group && R.group_anchor;
  const bool keyed = (MODE == CA_FF) && R.sort_hosts;

  if (CA)
    for (int i = tid; i < Z * Z; i += NT) {
      const int a = i / Z, z = i - a * Z;
      csum[i] = G(R.cost)[a * Z + z] + G(R.cost)[z * Z + a];
      bsum[i] = G(R.bw)[a * Z + z] + G(R.bw)[z * Z + a];
    }
  // Placements are kept in LDS by position and written out when the round ends: a global
  // store inside the task loop would put its round trip (vmcnt) on every task's critical path.
  int32_t* pl = reinterpret_cast<int32_t*>(smem + Lo.pl);
  for (int i = tid; i < T; i += NT) pl[i] = -1;

  // hosts -> registers (padding slots never fit: NaN capacities fail every comparison, even
  // against a -inf demand)
  const int h0 = tid * HPL;
  double a0[HPL], a1[HPL], a2[HPL], a3[HPL], key[HPL], cc[HPL], bb[HPL];
  // per slot, for the current anchor (cost_aware best-fit) / group key (keyed first-fit):
  // zmask bit j = a fitting host of slot j scores exactly 0 (c == 0 and bw > 0; keyed: key bits
  // 0), rmask bit j = its score may underflow to 0 or is not a number (needs the full path)
  uint32_t zmask = 0, rmask = 0;
  int32_t zz[HPL];
  uint32_t tb[HPL];
#pragma unroll
  for (int j = 0; j < HPL; j++) {
    const int h = h0 + j;
    const bool v = h < H;
    a0[j] = v ? G(R.avail)[h] : __builtin_nan("");
    a1[j] = v ? G(R.avail)[(size_t)H + h] : __builtin_nan("");
    a2[j] = v ? G(R.avail)[2 * (size_t)H + h] : __builtin_nan("");
    a3[j] = v ? G(R.avail)[3 * (size_t)H + h] : __builtin_nan("");
    zz[j] = (CA && v) ? G(R.zone)[h] : 0;
    tb[j] = (MODE == VBP_BF && v) ? G(R.tiebreak)[h] : 0u;
    key[j] = 0.0;                         // first-fit by index unless keyed
    cc[j] = 0.0;
    bb[j] = 1.0;
  }

  // a2: processing order (opportunistic keeps the caller's order)
  uint64_t* ka = reinterpret_cast<uint64_t*>(smem + Lo.u);
  uint64_t* kb = ka + A.Tpad;
  if (MODE == OPP) {
    for (int i = tid; i < T; i += NT) ord[i] = i;
    __syncthreads();
  } else {
    res_order<NT>(R, grouped, R.sort_tasks != 0, ka, kb, ord, A.Tpad);
  }
  for (int i = tid; i < T; i += NT) G(R.order)[i] = ord[i];

  // cost_aware best-fit rounds of up to RW_MAXH hosts: one wave walks them (resident_walk;
  // ca_bf 0.743 vs 0.779 ms at config 4); this path takes over where it stops, on the walked
  // capacities.
  int p_start = 0;
  if (MODE == CA_BF && (A.walk & 3) && H <= RW_MAXH && T > 0 && !R.rt_bw) {
#ifdef PVT_STAMPS
    const uint64_t tw0 = rstamp();
#endif
    // the walking wave: 0, or (A.walk == 2, A/B) one that moves with the workgroup index, so
    // two workgroups sharing a CU need not walk on the same SIMD
    // (A.walk & 4: no bulk runs in the walk, A/B)
    const int walker = (A.walk & 3) == 2 ? (int)(blockIdx.x % (unsigned)WAVES) : 0;
    p_start = resident_walk<NT>(R, Lo, smem, ord, pl, csum, bsum, has_groups, walker,
                                (A.walk & 4) == 0, A.stamps);
#ifdef PVT_STAMPS
    if (blockIdx.x == 0 && tid == 0 && A.stamps) {   // walked tasks, walk cycles (block 0)
      A.stamps[8] += (uint64_t)p_start;
      A.stamps[9] += rstamp() - tw0;
    }
#endif
    const double* wa = reinterpret_cast<const double*>(smem + Lo.wa);
#pragma unroll
    for (int j = 0; j < HPL; j++) {
      const int h = h0 + j;
      if (h < H) {
        a0[j] = wa[h]; a1[j] = wa[RW_MAXH + h]; a2[j] = wa[2 * RW_MAXH + h]; a3[j] = wa[3 * RW_MAXH + h];
      }
    }
  }
  // first fit by index (vbp first-fit; cost_aware first-fit without sort_hosts): the whole round
  // walked by one wave (resident_walk_ff), this path then only writes the results
  if ((MODE == VBP_FF || (MODE == CA_FF && !keyed)) && (A.walk & 8) && H <= RW_MAXH && T > 0) {
#ifdef PVT_STAMPS
    const uint64_t tw0 = rstamp();
#endif
    const int walker = (A.walk & 3) == 2 ? (int)(blockIdx.x % (unsigned)WAVES) : 0;
    p_start = resident_walk_ff<NT, MODE == CA_FF>(R, Lo, smem, ord, pl, walker, (A.walk & 4) == 0,
                                                  A.stamps);
#ifdef PVT_STAMPS
    if (blockIdx.x == 0 && tid == 0 && A.stamps) {
      A.stamps[8] += (uint64_t)p_start;
      A.stamps[9] += rstamp() - tw0;
    }
#endif
    const double* wa = reinterpret_cast<const double*>(smem + Lo.wa);
#pragma unroll
    for (int j = 0; j < HPL; j++) {
      const int h = h0 + j;
      if (h < H) {
        a0[j] = wa[h]; a1[j] = wa[RW_MAXH + h]; a2[j] = wa[2 * RW_MAXH + h]; a3[j] = wa[3 * RW_MAXH + h];
      }
    }
  }

  double* cd = reinterpret_cast<double*>(smem + Lo.cd);
  int32_t* c_anc = reinterpret_cast<int32_t*>(smem + Lo.ci);
  int32_t* c_grp = c_anc + RES_CHUNK;
  uint32_t* mk = reinterpret_cast<uint32_t*>(smem + Lo.mt) + wave * RES_MT_STRIDE;
  uint64_t* posts = reinterpret_cast<uint64_t*>(smem + Lo.slot);   // [2][WAVES][2]
  int32_t* cposts = reinterpret_cast<int32_t*>(posts);              // opp: [2][WAVES]
  int32_t* fposts = reinterpret_cast<int32_t*>(smem + Lo.slot + 32 * RES_MAXW);   // [2][WAVES]
  uint64_t* vposts = reinterpret_cast<uint64_t*>(smem + Lo.slot + 40 * RES_MAXW);  // [2][WAVES][2]
  MtWave mw;
  mw.buf = 0; mw.used = 0; mw.limit = 0;
  if (MODE == OPP) {
    const gptr<uint32_t> src = G(R.mt_state);
    for (int i = lane; i < 625; i += WAVE) mk[i] = src[i];
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }

#ifdef PVT_STAMPS
  // phases: 0 anchor rows, 1 slot scan, 2 wave reduction, 3 exchange (post, barrier, merge),
  // 4 full path, 5 commit; counts: 6 tasks, 7 full paths
  const bool stw = blockIdx.x == 0 && wave == 0 && A.stamps != nullptr;
  uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tl = stw ? rstamp() : 0;
#endif
  int cur_anc = -1, cur_grp = -1, cur_bgrp = -1;
  const bool rt = (MODE == CA_FF || MODE == CA_BF) && R.rt_bw != nullptr;
  // Sticky winner. A task whose demand is bit for bit the previous task's (same anchor, same
  // group when keys or realtime bandwidths are per group), with every demand >= 0, takes the
  // previous winner h again whenever h still fits: first-fit by index or by frozen key -- the
  // hosts before h did not fit that demand and have not changed; best-fit (vbp, cost_aware) --
  // h's residual only shrank (every component of a - d is >= 0 and fell), so its score did not
  // grow, and no other host changed. Such a task needs no selection and no exchange between the
  // waves: every wave tracks h's capacities (sc), broadcast once through LDS when a run starts.
  double* skc = reinterpret_cast<double*>(smem + Lo.slot + 32 * RES_MAXW + 8 * RES_MAXW + 32 * RES_MAXW);
  int sh = -1;
  double sc0 = 0.0, sc1 = 0.0, sc2 = 0.0, sc3 = 0.0;
  // bulk sticky runs (A.walk & 16: off, A/B); run flags u64[RES_CHUNK / 64] in the staging pad
  const bool bulk_sticky = (A.walk & 16) == 0;
  uint64_t* ew = reinterpret_cast<uint64_t*>(c_anc + 2 * RES_CHUNK);
  // run lists (A.walk & 32: off, A/B; bits 8-15: the minimum remaining run, A/B), for vbp
  // best-fit only: the other policies' fast winners (one ballot, no score reduction) measured
  // cheaper than a list (config 4 cost_aware first-fit 2.1 vs 0.53 ms with lists for every run)
  const bool run_lists = (MODE == VBP_BF || (MODE != OPP && (A.walk & 64))) && bulk_sticky &&
                         (A.walk & 32) == 0;
  const int list_min = (A.walk >> 8) & 255 ? (A.walk >> 8) & 255 : RES_LIST_MIN;
  RunEntry* rlw = reinterpret_cast<RunEntry*>(smem + Lo.lst) + wave * RES_LK;   // this wave's list
  // Places the `rem` tasks at positions pos.. (demand d, a run) down run lists; returns rem.
  auto run_list_steps = [&](int pos, int rem, double d0, double d1, double d2, double d3) -> int {
    int placed = 0;
    while (placed < rem) {
      // the full path's keys: k1 score bits (first fit: 0; keyed: the frozen key), k2
      // tiebreak:host; a host that does not fit is NONE
      uint64_t s1[HPL];
#pragma unroll
      for (int j = 0; j < HPL; j++) {
        const bool f = fits<STRICT>(a0[j], a1[j], a2[j], a3[j], d0, d1, d2, d3);
        uint64_t k1 = 0;
        if (MODE == CA_BF || MODE == VBP_BF) {
          const double sq = __builtin_sqrt(norm2_seq(a0[j] - d0, a1[j] - d1, a2[j] - d2, a3[j] - d3));
          k1 = dbits(MODE == CA_BF ? (cc[j] * sq) / bb[j] : sq);
        } else if (MODE == CA_FF) {
          k1 = dbits(key[j]);
        }
        s1[j] = f ? k1 : NONE;
      }
      // this wave's RES_LK smallest (k1, k2), in order (host ids make the keys distinct)
      for (int e = 0; e < RES_LK; e++) {
        uint64_t b1 = NONE, b2 = NONE;
        int bj = 0;
#pragma unroll
        for (int j = 0; j < HPL; j++) {
          const uint64_t k2 = ((uint64_t)tb[j] << 32) | (uint32_t)(h0 + j);
          if (s1[j] < b1 || (s1[j] == b1 && s1[j] != NONE && k2 < b2)) { b1 = s1[j]; b2 = k2; bj = j; }
        }
        const uint64_t m1 = wave_min_u64(b1);
        if (m1 == NONE) {
          if (lane >= e && lane < RES_LK) { rlw[lane].k1 = NONE; rlw[lane].k2 = NONE; }
          break;
        }
        const uint64_t tied = __ballot(b1 == m1);
        const uint64_t m2 = __popcll(tied) > 1 ? wave_min_u64(b1 == m1 ? b2 : NONE)
                                               : readlane_u64(b2, __builtin_ctzll(tied));
        if (b1 == m1 && b2 == m2) {
#pragma unroll
          for (int j = 0; j < HPL; j++)
            if (j == bj) {
              rlw[e].k1 = m1; rlw[e].k2 = m2;
              rlw[e].c[0] = a0[j]; rlw[e].c[1] = a1[j]; rlw[e].c[2] = a2[j]; rlw[e].c[3] = a3[j];
              s1[j] = NONE;
            }
        }
      }
      __syncthreads();
      // the run down the lists, merged on the fly (uniform in every wave; owners take their
      // hosts' results): the next host is the smallest head. A list used up (RES_LK hosts
      // taken) hides its wave's next host, so the lists are rebuilt; every head a non-fitting
      // entry: no host fits, the run's remaining tasks stay waiting.
      const RunEntry* L = reinterpret_cast<const RunEntry*>(smem + Lo.lst);
      int hp[WAVES];
      uint64_t q1[WAVES], q2[WAVES];
#pragma unroll
      for (int w = 0; w < WAVES; w++) { hp[w] = 0; q1[w] = L[w * RES_LK].k1; q2[w] = L[w * RES_LK].k2; }
      bool more = false;
      while (placed < rem) {
        int bw = -1;
        uint64_t b1 = NONE, b2 = NONE;
        bool used_up = false;
#pragma unroll
        for (int w = 0; w < WAVES; w++) {
          used_up |= hp[w] >= RES_LK;
          if (hp[w] < RES_LK && (q1[w] < b1 || (q1[w] == b1 && q2[w] < b2))) { b1 = q1[w]; b2 = q2[w]; bw = w; }
        }
        if (used_up) { more = true; break; }
        if (bw < 0) { placed = rem; break; }
        int ix = 0;
#pragma unroll
        for (int w = 0; w < WAVES; w++) if (w == bw) ix = w * RES_LK + hp[w];
        double x0 = L[ix].c[0], x1 = L[ix].c[1], x2 = L[ix].c[2], x3 = L[ix].c[3];
        const int h = (int)(uint32_t)b2;
        int c = 0;
        while (placed + c < rem && fits<STRICT>(x0, x1, x2, x3, d0, d1, d2, d3)) {
          x0 -= d0; x1 -= d1; x2 -= d2; x3 -= d3;
          c++;
        }
        c = __builtin_amdgcn_readfirstlane(c);
        for (int t = tid; t < c; t += NT) pl[pos + placed + t] = h;
        placed += c;
        if (h / HPL == tid) {
#pragma unroll
          for (int j = 0; j < HPL; j++)
            if (j == (h & (HPL - 1))) { a0[j] = x0; a1[j] = x1; a2[j] = x2; a3[j] = x3; }
        }
        const int nx = ix + 1;
        const uint64_t n1 = L[nx < WAVES * RES_LK ? nx : 0].k1, n2 = L[nx < WAVES * RES_LK ? nx : 0].k2;
#pragma unroll
        for (int w = 0; w < WAVES; w++)
          if (w == bw) { hp[w]++; q1[w] = n1; q2[w] = n2; }
      }
      placed = __builtin_amdgcn_readfirstlane(placed);
      if (more) __syncthreads();   // (every wave is done with the lists before they are rebuilt)
    }
    return rem;
  };
  for (int p0 = p_start; p0 < T; p0 += RES_CHUNK) {
    const int n = min(RES_CHUNK, T - p0);
    __syncthreads();                      // the previous chunk (and the sort keys) are consumed
    {
      // every load of the chunk is issued before the first one is waited for
      constexpr int PER = (RES_CHUNK + NT - 1) / NT;
      int tt[PER], gg[PER], aa[PER];
      double dd[PER][4];
#pragma unroll
      for (int k = 0; k < PER; k++) {
        const int i = tid + k * NT;
        tt[k] = i < n ? ord[p0 + i] : 0;   // (i >= n: task 0's row, loaded and dropped)
      }
#pragma unroll
      for (int k = 0; k < PER; k++) {
        const int t = tt[k];
        dd[k][0] = G(R.dem)[t];
        dd[k][1] = G(R.dem)[(size_t)T + t];
        dd[k][2] = G(R.dem)[2 * (size_t)T + t];
        dd[k][3] = G(R.dem)[3 * (size_t)T + t];
        gg[k] = has_groups ? G(R.task_group)[t] : 0;
      }
#pragma unroll
      for (int k = 0; k < PER; k++) aa[k] = has_groups ? G(R.group_anchor)[gg[k]] : 0;
#pragma unroll
      for (int k = 0; k < PER; k++) {
        const int i = tid + k * NT;
        if (i < n) {
          cd[i * 4 + 0] = dd[k][0]; cd[i * 4 + 1] = dd[k][1];
          cd[i * 4 + 2] = dd[k][2]; cd[i * 4 + 3] = dd[k][3];
          c_anc[i] = aa[k];
          c_grp[i] = gg[k];
        }
      }
    }
    __syncthreads();
    if (MODE != OPP && bulk_sticky) {
      // run flags: bit i of ew = staged row i repeats row i - 1 (demand bits; anchor; group where
      // keys or realtime bandwidths are per group) -- the sticky winner's run condition
      for (int i0 = 0; i0 < RES_CHUNK; i0 += NT) {
        const int i = i0 + tid;
        bool e = false;
        if (i >= 1 && i < n) {
          e = dbits(cd[i * 4 + 0]) == dbits(cd[i * 4 - 4]) && dbits(cd[i * 4 + 1]) == dbits(cd[i * 4 - 3]) &&
              dbits(cd[i * 4 + 2]) == dbits(cd[i * 4 - 2]) && dbits(cd[i * 4 + 3]) == dbits(cd[i * 4 - 1]) &&
              (!CA || c_anc[i] == c_anc[i - 1]) &&
              (!((MODE == CA_FF && keyed) || rt) || c_grp[i] == c_grp[i - 1]);
        }
        const uint64_t b = __ballot(e);
        if (lane == 0 && i < RES_CHUNK) ew[i >> 6] = b;
      }
      __syncthreads();
    }
    // the next task's staged row is read while this task is scored (LDS latency off the chain)
    double n0 = cd[0], n1 = cd[1], n2 = cd[2], n3 = cd[3];
    int n_anc = c_anc[0], n_grp = c_grp[0];
    for (int q = 0; q < n; q++) {
      const int p = p0 + q;
      const double d0 = n0, d1 = n1, d2 = n2, d3 = n3;
      const int anc_q = n_anc, grp_q = n_grp;
      if (q + 1 < n) {
        n0 = cd[(q + 1) * 4 + 0]; n1 = cd[(q + 1) * 4 + 1]; n2 = cd[(q + 1) * 4 + 2]; n3 = cd[(q + 1) * 4 + 3];
        n_anc = c_anc[q + 1]; n_grp = c_grp[q + 1];
      }
      if (CA) {
        const int anc = anc_q;
        // anchor rows of the zone tables -> registers; realtime_bw (cost_aware.py:79,112): the
        // bandwidth is the group's per-host row instead
        if (anc != cur_anc || (rt && grp_q != cur_bgrp)) {
          cur_anc = anc;
          cur_bgrp = grp_q;
#pragma unroll
          for (int j = 0; j < HPL; j++) {
            cc[j] = csum[anc * Z + zz[j]];
            bb[j] = rt ? (h0 + j < H ? G(R.rt_bw)[(size_t)grp_q * H + h0 + j] : 1.0) : bsum[anc * Z + zz[j]];
          }
          if (MODE == CA_BF) {
            zmask = 0; rmask = 0;
#pragma unroll
            for (int j = 0; j < HPL; j++) {
              // safe: bw in (0, 2^300] and c == 0 or c in [2^-300, inf): then a fitting host
              // scores exactly +0 iff c == 0 or s2 == 0 (s2 finite), and otherwise >= 2^-900
              // unless s2 < 2^-600
              const bool safe = bb[j] > 0.0 && bb[j] <= 0x1p+300 &&
                                (cc[j] == 0.0 || (cc[j] >= 0x1p-300 && cc[j] < DINF));
              zmask |= ((safe && cc[j] == 0.0) ? 1u : 0u) << j;
              rmask |= (safe ? 0u : 1u) << j;
            }
          }
        }
      }
      if (MODE == CA_FF && keyed) {
        const int g = grp_q;
        if (g != cur_grp) {               // frozen host key of the group (cost_aware.py:104-119)
          cur_grp = g;
          zmask = 0;
#pragma unroll
          for (int j = 0; j < HPL; j++) {
            const double r = __builtin_sqrt(norm2_seq(a0[j], a1[j], a2[j], a3[j]));
            const double df = (R.decay && h0 + j < H) ? (double)G(R.decay)[h0 + j] : 1.0;
            key[j] = (cc[j] * df) / (r * bb[j]);
            zmask |= (dbits(key[j]) == 0 ? 1u : 0u) << j;
          }
        }
      }
      RSTAMP(0);
      RCOUNT(6);
      if (MODE != OPP && sh >= 0) {
        // (sh >= 0 only when this task's demand, anchor and group equal the previous task's)
        const bool ok = fits<STRICT>(sc0, sc1, sc2, sc3, d0, d1, d2, d3);
        if (ok) {
          sc0 -= d0; sc1 -= d1; sc2 -= d2; sc3 -= d3;
          const int jw = sh & (HPL - 1);
          if (sh / HPL == tid) {
#pragma unroll
            for (int j = 0; j < HPL; j++)
              if (j == jw) { a0[j] -= d0; a1[j] -= d1; a2[j] -= d2; a3[j] -= d3; }   // resc[h] -= d
            pl[p] = sh;
          }
          const bool same_next = q + 1 < n &&
              dbits(n0) == dbits(d0) && dbits(n1) == dbits(d1) && dbits(n2) == dbits(d2) &&
              dbits(n3) == dbits(d3) && (!CA || n_anc == anc_q) &&
              (!((MODE == CA_FF && keyed) || rt) || n_grp == grp_q);
          if (!same_next) sh = -1;
          RSTAMP(5);
          continue;
        }
        sh = -1;
      }
      const int par = p & 1;
      if (MODE == OPP) {
        // feasible hosts of this lane (np.all(r >= d), opportunistic.py:15)
        uint32_t fm = 0;
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < HPL; j++) {
          const bool f = fits<false>(a0[j], a1[j], a2[j], a3[j], d0, d1, d2, d3);
          fm |= (f ? 1u : 0u) << j;
          cnt += f ? 1 : 0;
        }
        const int inc = wave_incl_scan_dpp(cnt);
        const int wt = __builtin_amdgcn_readlane(inc, 63);
        int ntot = wt, off = 0;
        if (WAVES > 1) {
          if (lane == 0) cposts[par * RES_MAXW + wave] = wt;
          __syncthreads();
          int v[WAVES];
#pragma unroll
          for (int w = 0; w < WAVES; w++) v[w] = cposts[par * RES_MAXW + w];
          ntot = 0;
#pragma unroll
          for (int w = 0; w < WAVES; w++) {
            off += (w < wave) ? v[w] : 0;
            ntot += v[w];
          }
        }
        if (ntot == 0) continue;
        const int k = (int)mt_randint(mk, mw, (uint32_t)ntot) - off;   // randomizer.choice (:16)
        if (k >= 0 && k < wt && inc > k && inc - cnt <= k) {
          int rr = k - (inc - cnt);
#pragma unroll
          for (int j = 0; j < HPL; j++) {
            if ((fm >> j) & 1u) {
              if (rr == 0) {
                a0[j] -= d0; a1[j] -= d1; a2[j] -= d2; a3[j] -= d3;   // commit (:18)
                pl[p] = h0 + j;
              }
              rr--;
            }
          }
        }
        continue;
      }

      // ---- fast winner (32-bit host index; see the header): the lane's first candidate slot
      constexpr bool FIRST = (MODE == VBP_FF || MODE == CA_FF);   // (CA_FF: unkeyed rounds)
      constexpr int RISKY = -1;
      int hw = 0x7fffffff;
      bool full = (MODE == VBP_BF) || (MODE == CA_FF && keyed);
      if (MODE != VBP_BF) {
        int c = 0x7fffffff;
        bool risky = false;
        if (MODE == CA_BF) {
          // from the largest residual mx = max(a - d) of a fitting host (all residuals >= +0):
          // mx == 0 is an exact fit (s2 == 0, score 0); mx >= 2^-300 gives s2 >= 2^-600 (the FMA
          // chain only adds non-negative terms), so with a safe slot and c > 0 the score is
          // >= 2^-900; with c == 0 the score is 0 while s2 is finite (mx <= 2^500). Anything
          // else is risky and goes to the full path.
#pragma unroll
          for (int j = HPL - 1; j >= 0; j--) {     // (descending: the lowest candidate slot wins)
            const bool f = fits<false>(a0[j], a1[j], a2[j], a3[j], d0, d1, d2, d3);
            const double mx = fmax(fmax(a0[j] - d0, a1[j] - d1), fmax(a2[j] - d2, a3[j] - d3));
            const bool safe = !((rmask >> j) & 1u), zc = (zmask >> j) & 1u;
            const bool z = safe && ((zc && mx <= 0x1p+500) || mx == 0.0);
            c = (f && z) ? h0 + j : c;
            risky |= f && !z && (!safe || !(mx >= 0x1p-300) || zc);
          }
          // (a non-finite demand can leave a NaN residual that fmax drops: full path)
          risky |= !(__builtin_fabs(d0) < DINF && __builtin_fabs(d1) < DINF &&
                     __builtin_fabs(d2) < DINF && __builtin_fabs(d3) < DINF);
        } else {
#pragma unroll
          for (int j = HPL - 1; j >= 0; j--) {
            const bool f = fits<STRICT>(a0[j], a1[j], a2[j], a3[j], d0, d1, d2, d3);
            c = (f && (!keyed || ((zmask >> j) & 1u))) ? h0 + j : c;
          }
        }
        RSTAMP(1);
        const uint64_t any = __ballot(c != 0x7fffffff);
        int wc = any ? __builtin_amdgcn_readlane(c, __builtin_ctzll(any)) : 0x7fffffff;
        if (MODE == CA_BF && __ballot(risky)) wc = RISKY;   // (RISKY = -1: the signed minimum)
        int g = wc;
        RSTAMP(2);
        if (WAVES > 1) {
          if (lane == 0) fposts[par * RES_MAXW + wave] = wc;
          __syncthreads();
          int v[WAVES];                          // (one LDS load per 4 posts)
#pragma unroll
          for (int w = 0; w < WAVES; w++) v[w] = fposts[par * RES_MAXW + w];
#pragma unroll
          for (int w = 1; w < WAVES; w++) v[0] = min(v[0], v[w]);
          g = v[0];
        }
        g = __builtin_amdgcn_readfirstlane(g);
        RSTAMP(3);
        if (g >= 0 && g != 0x7fffffff) {
          hw = g;
          full = false;
        } else {
          // no fast winner anywhere: first-fit by index has none at all; cost_aware best-fit
          // (no score-0 host, or a risky one) and keyed first-fit (no key-0 host) take the full path
          full = !FIRST || keyed;
        }
      }
      if (MODE == VBP_BF) {
        // vbp best-fit by the squared norm first (vbp.py:43-47): the winner has the least s2
        // unless another fitting host's norm rounds to the same value -- which needs its s2
        // within a factor 1 + 2^-49 of the least (sqrt halves relative gaps; a gap above
        // 2^-52 of the exact roots separates the rounded ones). Each wave posts its least s2
        // (bits: s2 >= +0), that host, and whether a second host of the wave lies within that
        // factor; when no second host anywhere does, the least s2 is the winner and no square
        // root is taken. Otherwise the full path below decides with the norms and tiebreaks.
        uint64_t sb[HPL];
        uint64_t ls = NONE;
        int lh = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < HPL; j++) {
          const bool f = fits<true>(a0[j], a1[j], a2[j], a3[j], d0, d1, d2, d3);
          sb[j] = f ? dbits(norm2_seq(a0[j] - d0, a1[j] - d1, a2[j] - d2, a3[j] - d3)) : NONE;
          if (sb[j] < ls) { ls = sb[j]; lh = h0 + j; }
        }
        RSTAMP(1);
        const uint64_t m = wave_min_u64(ls);
        int wh = 0x7fffffff, near = 0;
        if (m != NONE) {
          const uint64_t thr = dbits(__longlong_as_double((long long)m) * (1.0 + 0x1p-49));
          int cnt = 0;
#pragma unroll
          for (int j = 0; j < HPL; j++) cnt += sb[j] <= thr ? 1 : 0;
          const uint64_t any = __ballot(cnt > 0);
          near = (__popcll(any) > 1 || __ballot(cnt > 1) != 0) ? 1 : 0;
          wh = __builtin_amdgcn_readlane(lh, __builtin_ctzll(__ballot(ls == m)));
        }
        uint64_t gm = m;
        int gh = wh, gnear = near;
        RSTAMP(2);
        if (WAVES > 1) {
          if (lane == 0) {
            vposts[(par * RES_MAXW + wave) * 2 + 0] = m;
            vposts[(par * RES_MAXW + wave) * 2 + 1] = ((uint64_t)(uint32_t)near << 32) | (uint32_t)wh;
          }
          __syncthreads();
          uint64_t vm[WAVES], vx[WAVES];
#pragma unroll
          for (int w = 0; w < WAVES; w++) {
            vm[w] = vposts[(par * RES_MAXW + w) * 2 + 0];
            vx[w] = vposts[(par * RES_MAXW + w) * 2 + 1];
          }
          gm = vm[0];
#pragma unroll
          for (int w = 1; w < WAVES; w++) gm = vm[w] < gm ? vm[w] : gm;
          gnear = 0;
          gh = 0x7fffffff;
          if (gm != NONE) {
            const uint64_t thr = dbits(__longlong_as_double((long long)gm) * (1.0 + 0x1p-49));
            int within = 0;
#pragma unroll
            for (int w = 0; w < WAVES; w++) {
              within += vm[w] <= thr ? 1 : 0;
              if (vm[w] == gm && gh == 0x7fffffff) { gh = (int)(uint32_t)vx[w]; gnear |= (int)(vx[w] >> 32); }
            }
            gnear |= within > 1;
          }
        }
        gnear = __builtin_amdgcn_readfirstlane(gnear);
        if (!gnear) {
          full = false;
          hw = __builtin_amdgcn_readfirstlane(gh);
        }
        RSTAMP(3);
      }
      if (full) {
        // lane best: (score bits, tiebreak:host), first minimum in host order
        uint64_t b1 = NONE, b2 = NONE;
#pragma unroll
        for (int j = 0; j < HPL; j++) {
          const bool f = fits<STRICT>(a0[j], a1[j], a2[j], a3[j], d0, d1, d2, d3);
          uint64_t k1 = 0;
          if (MODE == CA_BF || MODE == VBP_BF) {
            if (f) {
              const double s = __builtin_sqrt(norm2_seq(a0[j] - d0, a1[j] - d1, a2[j] - d2, a3[j] - d3));
              // cost_aware.py:83 (c * r * decay / bw, decay == 1); vbp.py:45 (la.norm)
              k1 = dbits(MODE == CA_BF ? (cc[j] * s) / bb[j] : s);
            }
          } else if (MODE == CA_FF) {
            k1 = dbits(key[j]);
          }
          const uint64_t k2 = ((uint64_t)tb[j] << 32) | (uint32_t)(h0 + j);
          if (f && (k1 < b1 || (k1 == b1 && k2 < b2))) { b1 = k1; b2 = k2; }
        }
        // wave minimum: score bits first; among tied lanes the first holds the lowest host
        // (blocked host mapping), except vbp best-fit, whose tiebreak rank precedes the host
        const uint64_t m1 = wave_min_u64(b1);
        const uint64_t tied = __ballot(b1 == m1);
        uint64_t m2 = readlane_u64(b2, __builtin_ctzll(tied));
        if (MODE == VBP_BF && __popcll(tied) > 1) m2 = wave_min_u64((b1 == m1) ? b2 : NONE);
        uint64_t g2 = m2;
        if (WAVES > 1) {
          if (lane == 0) {
            posts[(par * RES_MAXW + wave) * 2 + 0] = m1;
            posts[(par * RES_MAXW + wave) * 2 + 1] = m2;
          }
          __syncthreads();
          uint64_t v1[WAVES], v2[WAVES];         // all posts in flight at once, then compared
#pragma unroll
          for (int w = 0; w < WAVES; w++) {
            v1[w] = posts[(par * RES_MAXW + w) * 2 + 0];
            v2[w] = posts[(par * RES_MAXW + w) * 2 + 1];
          }
          uint64_t g1 = v1[0];
          g2 = v2[0];
#pragma unroll
          for (int w = 1; w < WAVES; w++) {
            const bool lt = (v1[w] < g1) | ((v1[w] == g1) & (v2[w] < g2));
            g1 = lt ? v1[w] : g1;
            g2 = lt ? v2[w] : g2;
          }
        }
        if (g2 != NONE) hw = __builtin_amdgcn_readfirstlane((int)(uint32_t)g2);
        RCOUNT(7);
        RSTAMP(4);
      }
      if (hw == 0x7fffffff) continue;    // no host fits: the task stays waiting
      const int jw = hw & (HPL - 1);     // uniform: the owning lane's register slot
      // a run of equal demands starts: the winner's capacities after this commit go to every
      // wave (one LDS round trip and a barrier -- which also keeps this task's posts from being
      // overwritten before every wave has read them, the parity scheme's guarantee, while the
      // run's tasks go without a barrier)
      const bool run_next = MODE != OPP && q + 1 < n &&
          dbits(n0) == dbits(d0) && dbits(n1) == dbits(d1) && dbits(n2) == dbits(d2) &&
          dbits(n3) == dbits(d3) && (!CA || n_anc == anc_q) &&
          (!((MODE == CA_FF && keyed) || rt) || n_grp == grp_q) &&
          d0 >= 0.0 && d1 >= 0.0 && d2 >= 0.0 && d3 >= 0.0;
      if (hw / HPL == tid) {
#pragma unroll
        for (int j = 0; j < HPL; j++)
          if (j == jw) {
            a0[j] -= d0; a1[j] -= d1; a2[j] -= d2; a3[j] -= d3;   // resc[h] -= d
            if (run_next) { skc[0] = a0[j]; skc[1] = a1[j]; skc[2] = a2[j]; skc[3] = a3[j]; }
          }
        pl[p] = hw;
      }
      if (run_next) {
        __syncthreads();
        sc0 = skc[0]; sc1 = skc[1]; sc2 = skc[2]; sc3 = skc[3];
        sh = hw;
        if (bulk_sticky) {
          // the whole run in one step: its length from the run flags, then the copies the winner
          // still takes by the sticky rule (fits, subtract; in order, uniform in every wave); the
          // task after them is a new row or does not fit the winner, so it takes the full path
          int rl = 0;
          for (int i = q + 1; i < n;) {
            const uint64_t w = ~(ew[i >> 6] >> (i & 63));
            const int z = w ? (int)__builtin_ctzll(w) : 64;
            rl += z;
            if (z < 64 - (i & 63)) break;
            i += z;
          }
          rl = __builtin_amdgcn_readfirstlane(rl);
          int k = 0;
          while (k < rl && fits<STRICT>(sc0, sc1, sc2, sc3, d0, d1, d2, d3)) {
            sc0 -= d0; sc1 -= d1; sc2 -= d2; sc3 -= d3;
            k++;
          }
          k = __builtin_amdgcn_readfirstlane(k);
          if (k > 0) {
            for (int i = tid; i < k; i += NT) pl[p + 1 + i] = hw;
            if (hw / HPL == tid) {
#pragma unroll
              for (int j = 0; j < HPL; j++)
                if (j == jw) { a0[j] = sc0; a1[j] = sc1; a2[j] = sc2; a3[j] = sc3; }
            }
          }
          if (run_lists && rl - k >= list_min) {
            // the winner ran out mid-run: the rest of the run goes down run lists -- the
            // RES_LK best fitting hosts for this demand by the full path's key, each taking copies
            // by the sticky rule until it no longer fits (only list hosts change during the run,
            // so the next list host is the next winner; a list ending in a non-fitting entry
            // held every fitting host, so the run's remaining tasks stay waiting)
            k += run_list_steps(p + 1 + k, rl - k, d0, d1, d2, d3);
          }
          if (k > 0) {
            q += k;
            if (q + 1 < n) {
              n0 = cd[(q + 1) * 4 + 0]; n1 = cd[(q + 1) * 4 + 1]; n2 = cd[(q + 1) * 4 + 2]; n3 = cd[(q + 1) * 4 + 3];
              n_anc = c_anc[q + 1]; n_grp = c_grp[q + 1];
            }
          }
          sh = -1;
        }
      }
      RSTAMP(5);
    }
  }
#ifdef PVT_STAMPS
  if (stw && lane == 0)
    for (int k = 0; k < 8; k++) A.stamps[k] += ph[k];
#endif

  __syncthreads();
  for (int i = tid; i < T; i += NT) G(R.placement)[ord[i]] = pl[i];
#pragma unroll
  for (int j = 0; j < HPL; j++) {
    const int h = h0 + j;
    if (h < H) {
      G(R.avail)[h] = a0[j];
      G(R.avail)[(size_t)H + h] = a1[j];
      G(R.avail)[2 * (size_t)H + h] = a2[j];
      G(R.avail)[3 * (size_t)H + h] = a3[j];
    }
  }
  if (MODE == OPP && wave == 0) {
    mt_unbuffer(mk, mw);
    const gptr<uint32_t> dst = G(R.mt_state);
    for (int i = lane; i < 625; i += WAVE) dst[i] = mk[i];
  }
}

template <int MODE, int WAVES, int HPL>
__global__ __launch_bounds__(WAVES * WAVE) void resident_kernel(ResidentArgs A) {
  const pvt_round R = reinterpret_cast<const pvt_round*>(A.rounds)[blockIdx.x];   // SGPRs
#ifdef PVT_STAMPS
  // per round (diagnostic): cycles of the whole workgroup, from its start to its end
  const uint64_t t_round = rstamp();
#endif
  resident_round<MODE, WAVES, HPL>(A, R);
#ifdef PVT_STAMPS
  if (threadIdx.x == 0 && A.stamps && blockIdx.x < RES_STAMP_ROUNDS)
    A.stamps[RES_STAMP_BASE + blockIdx.x] = rstamp() - t_round;
#endif
}

// A batch of rounds of different policies in one launch (pvt_place_host_batch: the lock-step
// driver's tick of simulations running different schedulers): each workgroup branches on its
// round's mode, a uniform (scalar) branch.
template <int WAVES, int HPL>
__global__ __launch_bounds__(WAVES * WAVE) void resident_mixed_kernel(ResidentArgs A) {
  const pvt_round R = reinterpret_cast<const pvt_round*>(A.rounds)[blockIdx.x];   // SGPRs
  switch (R.mode) {
    case CA_FF: resident_round<CA_FF, WAVES, HPL>(A, R); break;
    case CA_BF: resident_round<CA_BF, WAVES, HPL>(A, R); break;
    case OPP: resident_round<OPP, WAVES, HPL>(A, R); break;
    case VBP_FF: resident_round<VBP_FF, WAVES, HPL>(A, R); break;
    case VBP_BF: resident_round<VBP_BF, WAVES, HPL>(A, R); break;
    default: break;
  }
}

// Four or eight waves per round (one or two per SIMD of a CU). Measured on MI355X with 512
// rounds of 1000 hosts x 1000 tasks: one wave per round (16 hosts per lane, no barrier) is ~2x
// slower than four -- a single wave's dependent per-task chain cannot hide its own latencies.
template <int MODE, int W>
static void launch_waves(int hpl, int n, size_t lds, const ResidentArgs& a, hipStream_t st) {
  const dim3 grid(n), block(W * WAVE);
  switch (hpl) {
    case 1: PVT_LAUNCH((resident_kernel<MODE, W, 1>), grid, block, lds, st, a); break;
    case 2: PVT_LAUNCH((resident_kernel<MODE, W, 2>), grid, block, lds, st, a); break;
    case 4: PVT_LAUNCH((resident_kernel<MODE, W, 4>), grid, block, lds, st, a); break;
    case 8: PVT_LAUNCH((resident_kernel<MODE, W, 8>), grid, block, lds, st, a); break;
    default: PVT_LAUNCH((resident_kernel<MODE, 4, 16>), grid, dim3(4 * WAVE), lds, st, a); break;
  }
}
template <int MODE>
static void launch_two(int hpl, int n, size_t lds, const ResidentArgs& a, hipStream_t st) {
  const dim3 grid(n), block(2 * WAVE);
  switch (hpl) {
    case 8: PVT_LAUNCH((resident_kernel<MODE, 2, 8>), grid, block, lds, st, a); break;
    default: PVT_LAUNCH((resident_kernel<MODE, 2, 16>), grid, block, lds, st, a); break;
  }
}
template <int MODE>
static void launch_one(int n, size_t lds, const ResidentArgs& a, hipStream_t st) {
  PVT_LAUNCH((resident_kernel<MODE, 1, 16>), dim3(n), dim3(WAVE), lds, st, a);
}
template <int MODE>
static void launch_mode(int waves, int hpl, int n, size_t lds, const ResidentArgs& a, hipStream_t st) {
  if (waves == 8 && hpl <= 8) launch_waves<MODE, 8>(hpl, n, lds, a, st);
  else if (waves == 2 && hpl >= 8) launch_two<MODE>(hpl, n, lds, a, st);
  else if (waves == 1 && hpl == 16) launch_one<MODE>(n, lds, a, st);
  else launch_waves<MODE, 4>(hpl, n, lds, a, st);
}

// Waves and hosts per lane for a batch whose largest round has maxH hosts: `waves` (4 or 8) on
// entry is the preference; 8 waves only while the round needs at most 8 hosts per lane.
void resident_shape(int maxH, int* waves, int* hpl) {
  // (waves 2 and 1 -- 8 and 16 hosts per lane -- only as A/B preferences, PVT_RES_WAVES)
  const int w = (*waves == 8 && maxH <= 8 * 8 * WAVE) ? 8
                : (*waves == 2 && maxH > 2 * 4 * WAVE && maxH <= 2 * 16 * WAVE) ? 2
                : (*waves == 1 && maxH > 8 * WAVE && maxH <= 16 * WAVE) ? 1 : 4;
  int h = 1;
  while (h * w * WAVE < maxH) h <<= 1;
  *waves = w;
  *hpl = h;
}

void launch_resident(int mode, int waves, int hpl, int n, const ResidentArgs& a, hipStream_t st) {
  const size_t lds = resident_lds_bytes(a.Zb, a.Tpad, a.walk != 0);
  if (mode == RES_MIXED) {             // (four waves; resident_shape with waves = 4)
    const dim3 grid(n), block(4 * WAVE);
    switch (hpl) {
      case 1: PVT_LAUNCH((resident_mixed_kernel<4, 1>), grid, block, lds, st, a); break;
      case 2: PVT_LAUNCH((resident_mixed_kernel<4, 2>), grid, block, lds, st, a); break;
      case 4: PVT_LAUNCH((resident_mixed_kernel<4, 4>), grid, block, lds, st, a); break;
      case 8: PVT_LAUNCH((resident_mixed_kernel<4, 8>), grid, block, lds, st, a); break;
      default: PVT_LAUNCH((resident_mixed_kernel<4, 16>), grid, block, lds, st, a); break;
    }
    return;
  }
  switch (mode) {
    case CA_FF: launch_mode<CA_FF>(waves, hpl, n, lds, a, st); break;
    case CA_BF: launch_mode<CA_BF>(waves, hpl, n, lds, a, st); break;
    case OPP: launch_mode<OPP>(waves, hpl, n, lds, a, st); break;
    case VBP_FF: launch_mode<VBP_FF>(waves, hpl, n, lds, a, st); break;
    case VBP_BF: launch_mode<VBP_BF>(waves, hpl, n, lds, a, st); break;
    default: break;
  }
}

// ---- fused host batch (pvt_place_host_batch): ONE launch per call ----------------------------
// The staged path took six dependent launches per call (stage upload, anchor wave and block
// kernels, grouping, resident placement, result download: ~5 us of launch gap each on MI355X,
// the grouping alone ~20 us as a 1024-thread launch). Here one workgroup of four waves per round
// copies its round's byte ranges of the pinned stage (mapped host memory) to the device copy,
// resolves its anchors (a wave per item, deferred long lists by the block) and its groups and
// draws (cost_aware rounds with items), places the round (resident_round), and copies its
// output range back to the mapped stage; the host synchronises once.
// Two byte ranges [a, a + na) and [b, b + nb) copied src -> dst by the block (whole 16-byte
// units: the stage layout aligns every range to 256 bytes), FL loads in flight per thread before
// the first store: the source is host memory across PCIe (~2 us a round trip), so a load-store
// loop would pay one round trip per iteration.
template <int FL>
__device__ __forceinline__ void block_copy2(char* dst, const char* src, int64_t a, int64_t na,
                                            int64_t b, int64_t nb) {
  const int64_t n1 = na >> 4, n = n1 + (nb >> 4);
  const int nt = blockDim.x;
  for (int64_t i0 = 0; i0 < n; i0 += (int64_t)FL * nt) {
    int4 v[FL];
#pragma unroll
    for (int k = 0; k < FL; k++) {
      const int64_t i = i0 + (int64_t)k * nt + threadIdx.x;
      if (i < n) v[k] = *reinterpret_cast<const int4*>(src + (i < n1 ? a + 16 * i : b + 16 * (i - n1)));
    }
#pragma unroll
    for (int k = 0; k < FL; k++) {
      const int64_t i = i0 + (int64_t)k * nt + threadIdx.x;
      if (i < n) *reinterpret_cast<int4*>(dst + (i < n1 ? a + 16 * i : b + 16 * (i - n1))) = v[k];
    }
  }
}

template <int MODE, int HPL>
__device__ __forceinline__ void fused_place(const FusedArgs& F, const pvt_round& R) {
  if (MODE == RES_MIXED) {
    switch (R.mode) {
      case CA_FF: resident_round<CA_FF, 4, HPL>(F.ra, R); break;
      case CA_BF: resident_round<CA_BF, 4, HPL>(F.ra, R); break;
      case OPP: resident_round<OPP, 4, HPL>(F.ra, R); break;
      case VBP_FF: resident_round<VBP_FF, 4, HPL>(F.ra, R); break;
      case VBP_BF: resident_round<VBP_BF, 4, HPL>(F.ra, R); break;
      default: break;
    }
  } else {
    resident_round<MODE, 4, HPL>(F.ra, R);
  }
}

template <int MODE, int HPL>
__global__ __launch_bounds__(4 * WAVE) void resident_fused_kernel(FusedArgs F) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const FusedRound fr = reinterpret_cast<const FusedRound*>(F.hmap + F.o_rounds)[blockIdx.x];
  constexpr bool ITEMS = MODE == RES_MIXED || MODE == CA_FF || MODE == CA_BF;
  // (the grouping's arguments are read from the mapped stage beside the copy: one round trip)
  AnchorArgs a{};
  CaGroupArgs g{};
  if (ITEMS && fr.items >= 0) {
    a = reinterpret_cast<const AnchorArgs*>(F.hmap + F.o_ka)[fr.items];
    g = reinterpret_cast<const CaGroupArgs*>(F.hmap + F.o_kg)[fr.items];
  }
  if (threadIdx.x < (int)(sizeof(pvt_round) / 8))
    reinterpret_cast<uint64_t*>(F.dev + fr.desc)[threadIdx.x] =
        reinterpret_cast<const uint64_t*>(F.hmap + fr.desc)[threadIdx.x];
#ifdef PVT_STAMPS
  // phases of block 0 (stamps[16..20]): stage in, anchors, grouping, placement, results out
  const bool fst = blockIdx.x == 0 && threadIdx.x == 0 && F.ra.stamps;
  uint64_t ft = fst ? rstamp() : 0;
#define FSTAMP(k) do { if (fst) { const uint64_t t_ = rstamp(); F.ra.stamps[16 + (k)] += t_ - ft; ft = t_; } } while (0)
#else
#define FSTAMP(k) do {} while (0)
#endif
  block_copy2<16>(F.dev, F.hmap, fr.out_lo, fr.out_hi - fr.out_lo, fr.in_lo, fr.in_hi - fr.in_lo);
  __syncthreads();
  FSTAMP(0);
  if (ITEMS && fr.items >= 0) {
    const int wave = threadIdx.x >> 6;
    uint64_t* lds = reinterpret_cast<uint64_t*>(smem);
    for (int c = wave; c < a.C; c += 4) anchor_wave_item(a, c, lds + wave * ANC_WLDS);
    __syncthreads();
    const int nd = *a.n_deferred;
    for (int q = 0; q < nd; q++) {
      block_item(a, a.deferred[q], lds, lds + ANC_LDS);
      __syncthreads();
    }
    FSTAMP(1);
    ca_groups_round<4 * WAVE, RES_MAX_TASKS>(g, *reinterpret_cast<GroupLds*>(smem));
    __syncthreads();
    FSTAMP(2);
  }
  const pvt_round R = *reinterpret_cast<const pvt_round*>(F.dev + fr.desc);   // (n_groups set)
  fused_place<MODE, HPL>(F, R);
  __syncthreads();
  FSTAMP(3);
  block_copy2<16>(const_cast<char*>(F.hmap), F.dev, fr.out_lo, fr.out_hi - fr.out_lo, 0, 0);
  __syncthreads();
  FSTAMP(4);
#undef FSTAMP
}

size_t fused_pre_lds_bytes() {
  size_t b = 4 * ANC_WLDS * sizeof(uint64_t);
  b = std::max(b, (ANC_LDS + ANC_THREADS / 64) * sizeof(uint64_t));
  return std::max(b, sizeof(GroupLds));
}

void launch_fused(int mode, int hpl, int n, size_t lds, const FusedArgs& F, hipStream_t st) {
  const dim3 grid(n), block(4 * WAVE);
#define PVT_FUSED_HPL(M)                                                                         \
  switch (hpl) {                                                                                 \
    case 1: PVT_LAUNCH((resident_fused_kernel<M, 1>), grid, block, lds, st, F); break;   \
    case 2: PVT_LAUNCH((resident_fused_kernel<M, 2>), grid, block, lds, st, F); break;   \
    case 4: PVT_LAUNCH((resident_fused_kernel<M, 4>), grid, block, lds, st, F); break;   \
    case 8: PVT_LAUNCH((resident_fused_kernel<M, 8>), grid, block, lds, st, F); break;   \
    default: PVT_LAUNCH((resident_fused_kernel<M, 16>), grid, block, lds, st, F); break; \
  }
  switch (mode) {
    case CA_FF: PVT_FUSED_HPL(CA_FF) break;
    case CA_BF: PVT_FUSED_HPL(CA_BF) break;
    case OPP: PVT_FUSED_HPL(OPP) break;
    case VBP_FF: PVT_FUSED_HPL(VBP_FF) break;
    case VBP_BF: PVT_FUSED_HPL(VBP_BF) break;
    default: PVT_FUSED_HPL(RES_MIXED) break;
  }
#undef PVT_FUSED_HPL
}

template <int MODE>
static hipError_t attrs_fused(int lds) {
  hipError_t e = hipSuccess, r;
#define PVT_FUSED_ATTR(HPL)                                                                      \
  r = hipFuncSetAttribute((const void*)resident_fused_kernel<MODE, HPL>,                         \
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);                      \
  if (r != hipSuccess) e = r;
  PVT_FUSED_ATTR(1) PVT_FUSED_ATTR(2) PVT_FUSED_ATTR(4) PVT_FUSED_ATTR(8) PVT_FUSED_ATTR(16)
#undef PVT_FUSED_ATTR
  return e;
}

template <int MODE>
static hipError_t attrs_mode(int lds) {
  hipError_t e = hipSuccess, r;
#define PVT_RES_ATTR(W, HPL)                                                                     \
  r = hipFuncSetAttribute((const void*)resident_kernel<MODE, W, HPL>,                            \
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);                      \
  if (r != hipSuccess) e = r;
  PVT_RES_ATTR(4, 1) PVT_RES_ATTR(4, 2) PVT_RES_ATTR(4, 4) PVT_RES_ATTR(4, 8) PVT_RES_ATTR(4, 16)
  PVT_RES_ATTR(8, 1) PVT_RES_ATTR(8, 2) PVT_RES_ATTR(8, 4) PVT_RES_ATTR(8, 8)
  PVT_RES_ATTR(2, 8) PVT_RES_ATTR(2, 16) PVT_RES_ATTR(1, 16)
#undef PVT_RES_ATTR
  return e;
}

hipError_t resident_init_attrs() {
  const int lds = (int)resident_lds_bytes(ZMAX, RES_MAX_TASKS, true);
  hipError_t e = hipSuccess, r;
  if ((r = attrs_mode<CA_FF>(lds)) != hipSuccess) e = r;
  if ((r = attrs_mode<CA_BF>(lds)) != hipSuccess) e = r;
  if ((r = attrs_mode<OPP>(lds)) != hipSuccess) e = r;
  if ((r = attrs_mode<VBP_FF>(lds)) != hipSuccess) e = r;
  if ((r = attrs_mode<VBP_BF>(lds)) != hipSuccess) e = r;
#define PVT_MIX_ATTR(HPL)                                                                        \
  r = hipFuncSetAttribute((const void*)resident_mixed_kernel<4, HPL>,                            \
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);                      \
  if (r != hipSuccess) e = r;
  PVT_MIX_ATTR(1) PVT_MIX_ATTR(2) PVT_MIX_ATTR(4) PVT_MIX_ATTR(8) PVT_MIX_ATTR(16)
#undef PVT_MIX_ATTR
  const int flds = (int)std::max((size_t)lds, fused_pre_lds_bytes());
  if ((r = attrs_fused<CA_FF>(flds)) != hipSuccess) e = r;
  if ((r = attrs_fused<CA_BF>(flds)) != hipSuccess) e = r;
  if ((r = attrs_fused<OPP>(flds)) != hipSuccess) e = r;
  if ((r = attrs_fused<VBP_FF>(flds)) != hipSuccess) e = r;
  if ((r = attrs_fused<VBP_BF>(flds)) != hipSuccess) e = r;
  if ((r = attrs_fused<RES_MIXED>(flds)) != hipSuccess) e = r;
  return e;
}

}  // namespace pvt
