// pvt_kernels.hip — gfx950 kernels of the placement engine.
//
// The hot path of every policy is one fused pass over the round's task x host candidates
// (reference scheduler/cost_aware.py:63-127, scheduler/vbp.py:13-50): fit-mask, score, and a
// per-task top-KL selection ordered by (score, tiebreak, host index). A single-wave kernel
// then walks the tasks in the reference's order and commits capacity exactly as the
// reference's sequential loops do (DESIGN.md §2 explains why the lists make this exact).
//
// Numerics: build with -ffp-contract=off. Squared norms are the explicit FMA chain that
// numpy's la.norm -> OpenBLAS ddot computes for n = 4; sqrt and division are IEEE
// correctly rounded (llvm.sqrt.f64 / fdiv lowering without afn/arcp).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"
#include "pvt_kernels.h"

namespace pvt {

// Conservative bound on the squared residual norm of a cost_aware best-fit candidate:
// if fl(fl(c*sqrt(s2))/b) <= thr then s2 <= lim (rounding slack 2^-40 >> 2^-53).
__device__ __forceinline__ double ca_lim(double thr, double c, double b) {
  if (!(thr < DINF)) return DINF;
  if (c == 0.0) return thr > 0.0 ? DINF : -1.0;   // score is exactly 0 in zero-cost zones
  double r = thr * b / c;
  r = r * (1.0 + 0x1p-40);
  return r * r * (1.0 + 0x1p-40);
}
__device__ __forceinline__ double vbp_lim(double thr) {
  if (!(thr < DINF)) return DINF;
  double r = thr * (1.0 + 0x1p-40);
  return r * r * (1.0 + 0x1p-40);
}

// Insert (cs, ct, ci) into the wave-held sorted list (lane j holds entry j). The caller has
// checked it beats entry KL-1, which falls off.
__device__ __forceinline__ void list_insert(double& s, uint32_t& t, int32_t& i, double cs,
                                            uint32_t ct, int32_t ci) {
  const int lane = lane_id();
  const bool keep = lexless(s, t, i, cs, ct, ci);
  const int pos = __popcll(__ballot(keep));
  const double us = __shfl_up(s, 1);
  const uint32_t ut = (uint32_t)__shfl_up((int)t, 1);
  const int32_t ui = __shfl_up(i, 1);
  if (lane == pos) {
    s = cs; t = ct; i = ci;
  } else if (lane > pos) {
    s = us; t = ut; i = ui;
  }
}

// ------------------------------------------------------------------------------------------
// Score kernel: candidates (window tasks) x (one host segment). Block = 4 waves; each wave owns
// TW tasks and streams the segment's hosts 64 at a time (lane = host), keeping a sorted top-KL
// list per task in registers. blockIdx % S picks the segment, so with S = 8 the blocks of one
// segment share an XCD (round-robin dispatch) and its L2 holds that slice of the host table.
// ------------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void score_kernel(ScoreArgs A) {
  constexpr bool STRICT = (MODE != CA_BF);
  constexpr int ZL = (MODE == CA_BF) ? ZMAX : 1;
  __shared__ double s_lim[WPB][TW][ZL];
  __shared__ double s_c[WPB][TW][ZL];
  __shared__ double s_b[WPB][TW][ZL];

  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int seg = blockIdx.x % A.S, tile = blockIdx.x / A.S;
  const int t0 = (tile * WPB + wave) * TW;
  if (t0 >= A.nt) return;
  const int nt = min(TW, A.nt - t0);
  const int hb0 = A.h_lo + seg * A.seg_len, hb1 = min(A.h_hi, hb0 + A.seg_len);

  double d0[TW], d1[TW], d2[TW], d3[TW];
  double ls[TW], ts[TW], lim[TW];
  uint32_t lt[TW], tt[TW];
  int32_t li[TW], ti[TW], feas[TW];
#pragma unroll
  for (int k = 0; k < TW; k++) {
    if (k < nt) {
      const double* dp = A.dem + (size_t)(t0 + k) * 4;
      d0[k] = dp[0]; d1[k] = dp[1]; d2[k] = dp[2]; d3[k] = dp[3];
    } else {
      d0[k] = d1[k] = d2[k] = d3[k] = DINF;
    }
    ls[k] = DINF; lt[k] = 0xffffffffu; li[k] = 0x7fffffff;
    ts[k] = DINF; tt[k] = 0xffffffffu; ti[k] = 0x7fffffff;
    lim[k] = DINF;
    feas[k] = 0;
    if (MODE == CA_BF) {
      const int a = (k < nt) ? A.anc[t0 + k] : 0;
      if (lane < A.Z) {
        s_c[wave][k][lane] = A.csum[a * A.Z + lane];
        s_b[wave][k][lane] = A.bsum[a * A.Z + lane];
        s_lim[wave][k][lane] = DINF;
      }
    }
  }

  // Host data for block hb is loaded one iteration ahead (register double buffer), with the
  // index clamped instead of branching, so the loads overlap the previous block's scoring.
  double n0 = 0, n1 = 0, n2 = 0, n3 = 0, nkey = DINF;
  int nz = 0;
  auto fetch = [&](int hb) {
    const int h = min(hb + lane, hb1 - 1);
    n0 = A.avail[h];
    n1 = A.avail[(size_t)A.H + h];
    n2 = A.avail[2 * (size_t)A.H + h];
    n3 = A.avail[3 * (size_t)A.H + h];
    if (MODE == CA_BF) nz = A.zone[h];
    if (MODE == CA_FF) nkey = A.key[h];
  };
  if (hb0 < hb1) fetch(hb0);
  for (int hb = hb0; hb < hb1; hb += WAVE) {
    const int h = hb + lane;
    const bool ok = h < hb1;
    const double a0 = ok ? n0 : -DINF;
    const double a1 = n1, a2 = n2, a3 = n3;
    const int z = nz;
    const double key = nkey;
    if (hb + WAVE < hb1) fetch(hb + WAVE);
#pragma unroll
    for (int k = 0; k < TW; k++) {
      const bool fit = fits<STRICT>(a0, a1, a2, a3, d0[k], d1[k], d2[k], d3[k]);
      feas[k] += __popcll(__ballot(fit));
      double s2 = 0.0;
      bool pass;
      if (MODE == CA_FF) {
        pass = fit && lexless(key, 0u, h, ts[k], tt[k], ti[k]);
      } else {
        s2 = norm2_seq(a0 - d0[k], a1 - d1[k], a2 - d2[k], a3 - d3[k]);
        const double lm = (MODE == CA_BF) ? s_lim[wave][k][z] : lim[k];
        pass = fit && (s2 <= lm);
      }
      uint64_t pm = __ballot(pass);
      if (pm) {
        double sc = DINF;
        uint32_t tbv = 0;
        if (pass) {
          if (MODE == CA_FF) {
            sc = key;
          } else if (MODE == CA_BF) {
            const double r = __builtin_sqrt(s2);
            sc = (s_c[wave][k][z] * r) / s_b[wave][k][z];
          } else {
            sc = __builtin_sqrt(s2);
            tbv = A.tb[h];
          }
        }
        bool changed = false;
        while (pm) {
          const int L = __builtin_ctzll(pm);
          pm &= pm - 1;
          const double cs = readlane_d(sc, L);
          const uint32_t ct = readlane_u(tbv, L);
          const int32_t ci = hb + L;
          if (lexless(cs, ct, ci, ts[k], tt[k], ti[k])) {
            list_insert(ls[k], lt[k], li[k], cs, ct, ci);
            ts[k] = readlane_d(ls[k], KL - 1);
            tt[k] = readlane_u(lt[k], KL - 1);
            ti[k] = readlane_i(li[k], KL - 1);
            changed = true;
          }
        }
        if (changed) {
          if (MODE == CA_BF) {
            if (lane < A.Z) s_lim[wave][k][lane] = ca_lim(ts[k], s_c[wave][k][lane], s_b[wave][k][lane]);
          } else if (MODE == VBP_BF) {
            lim[k] = vbp_lim(ts[k]);
          }
        }
      }
    }
  }

#pragma unroll
  for (int k = 0; k < TW; k++) {
    if (k < nt) {
      const size_t row = (size_t)(t0 + k) * A.S + seg;
      SegEntry e;
      e.s = ls[k]; e.tb = lt[k]; e.id = li[k];
      A.seg[row * KL + lane] = e;
      if (lane == 0) A.seg_feas[row] = feas[k];
    }
  }
}

void launch_score(int mode, const ScoreArgs& a, hipStream_t st) {
  const int tiles = (a.nt + WPB * TW - 1) / (WPB * TW);
  dim3 grid(tiles * a.S), block(WPB * WAVE);
  switch (mode) {
    case CA_FF: hipLaunchKernelGGL(score_kernel<CA_FF>, grid, block, 0, st, a); break;
    case CA_BF: hipLaunchKernelGGL(score_kernel<CA_BF>, grid, block, 0, st, a); break;
    case VBP_BF: hipLaunchKernelGGL(score_kernel<VBP_BF>, grid, block, 0, st, a); break;
    default: break;
  }
}

// ------------------------------------------------------------------------------------------
// Merge: one 256-thread block per task sorts the S segment lists (16 at a time, 1024 entries,
// bitonic in LDS) into a running top-LMAX. Each segment list holds its segment's exact top-KL,
// so the union is exact below B = the smallest last entry of a segment that has more than KL
// feasible hosts: the merged list keeps the entries below B (at most LMAX) and records the
// bound, so the commit walk knows which hosts can be missing. Zone and snapshot availability
// of every kept host are gathered for the walk.
// ------------------------------------------------------------------------------------------
struct Key {
  double s;
  uint32_t tb;
  int32_t id;
};
__device__ __forceinline__ bool kless(const Key& a, const Key& b) { return lexless(a.s, a.tb, a.id, b.s, b.tb, b.id); }

__device__ __forceinline__ void bitonic_sort_lds(Key* v, int n, int tid, int nthreads) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < n / 2; t += nthreads) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = ((lo & size) == 0);
        const Key a = v[lo], b = v[hi];
        if (kless(b, a) == up) { v[lo] = b; v[hi] = a; }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(256) void merge_kernel(MergeArgs A) {
  __shared__ Key run[LMAX];
  __shared__ Key buf[LMAX];
  __shared__ Key bound;
  __shared__ long long tot;
  __shared__ int cnt_sh;
  const int task = blockIdx.x, tid = threadIdx.x;
  const int SL = A.SL, batch = LMAX / SL;   // source lists per sort batch
  const bool packed = A.seg_feas == nullptr;
  const Key inv = {DINF, 0xffffffffu, 0x7fffffff};
  // entry e of source list g
  auto src = [&](int g, int e) -> const SegEntry& {
    return packed ? A.seg[((size_t)g * A.nt + task) * (SL + 1) + e]
                  : A.seg[((size_t)task * A.S + g) * SL + e];
  };
  for (int j = tid; j < LMAX; j += 256) run[j] = inv;
  if (tid == 0) { bound = inv; tot = 0; cnt_sh = 0; }
  __syncthreads();
  for (int g0 = 0; g0 < A.S; g0 += batch) {
    int nvalid = 0;
    for (int e = tid; e < LMAX; e += 256) {
      const int g = g0 + e / SL;
      Key k = inv;
      if (e < batch * SL && g < A.S) {
        const SegEntry se = src(g, e % SL);
        k = {se.s, se.tb, se.id};
        nvalid += se.id != 0x7fffffff;
      }
      buf[e] = k;
    }
    if (packed) {
      if (nvalid) atomicAdd((unsigned long long*)&tot, (unsigned long long)nvalid);
      if (tid == 0) {
        for (int g = g0; g < min(A.S, g0 + batch); g++) {
          const SegEntry se = src(g, SL);        // the package's explicit bound
          const Key k = {se.s, se.tb, se.id};
          if (kless(k, bound)) bound = k;
        }
      }
    } else if (tid == 0) {
      for (int g = g0; g < min(A.S, g0 + batch); g++) {
        const int f = A.seg_feas[(size_t)task * A.S + g];
        tot += f;
        if (f > SL) {
          const SegEntry se = src(g, SL - 1);
          const Key k = {se.s, se.tb, se.id};
          if (kless(k, bound)) bound = k;
        }
      }
    }
    __syncthreads();
    bitonic_sort_lds(buf, LMAX, tid, 256);
    // keep the LMAX smallest of run (ascending) and buf (ascending): elementwise min against the
    // reversed buf gives a bitonic sequence, then a bitonic merge sorts it
    for (int j = tid; j < LMAX; j += 256) {
      const Key b = buf[LMAX - 1 - j];
      if (kless(b, run[j])) run[j] = b;
    }
    __syncthreads();
    for (int stride = LMAX / 2; stride > 0; stride >>= 1) {
      for (int t = tid; t < LMAX / 2; t += 256) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const Key a = run[lo], b = run[hi];
        if (kless(b, a)) { run[lo] = b; run[hi] = a; }
      }
      __syncthreads();
    }
  }
  // kept entries: valid and below the bound
  int c = 0;
  for (int j = tid; j < LMAX; j += 256) c += (run[j].id != 0x7fffffff) && kless(run[j], bound);
  atomicAdd(&cnt_sh, c);
  __syncthreads();
  const int cnt = cnt_sh;
  const bool complete = (bound.id == 0x7fffffff) && tot <= LMAX;
  Key bnd = bound;
  if (cnt == LMAX && kless(run[LMAX - 1], bnd)) bnd = run[LMAX - 1];
  for (int j = tid; j < LMAX; j += 256) {
    ListEntry e;
    const Key k = run[j];
    const bool valid = j < cnt;
    const int h = valid ? k.id : 0;
    e.s = k.s; e.tb = k.tb; e.id = k.id; e.pad = 0; e.pad2 = 0.0;
    e.zone = valid ? A.zone[h] : 0;
    e.a[0] = valid ? A.avail[h] : 0.0;
    e.a[1] = valid ? A.avail[(size_t)A.H + h] : 0.0;
    e.a[2] = valid ? A.avail[2 * (size_t)A.H + h] : 0.0;
    e.a[3] = valid ? A.avail[3 * (size_t)A.H + h] : 0.0;
    if (valid || j < KL) {
      A.L.e[(size_t)task * LMAX + j] = e;
      A.L.ids[(size_t)task * LMAX + j] = valid ? k.id : 0x7fffffff;
    }
  }
  if (tid < 4) {
    double* tr = reinterpret_cast<double*>(&A.L.t[task]);
    tr[tid] = A.dem[(size_t)task * 4 + tid];
  }
  if (tid == 0) {
    TaskRec& r = A.L.t[task];
    r.cnt = cnt;
    r.complete = complete;
    r.anc = A.anc[task];
    r.ord = A.ord[task];
    r.bs = bnd.s; r.btb = bnd.tb; r.bid = bnd.id;
  }
}

void launch_merge(const MergeArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(merge_kernel, dim3(a.nt), dim3(256), 0, st, a);
}

// ------------------------------------------------------------------------------------------
// Pack (host-dimension sharding): one wave per task turns the rank's exact
// local list into its exchange package: the first PK entries plus a bound every host of the
// rank outside the package ranks at or after. The bound is entry PK when the list is longer,
// else the list's own bound (none if complete). Index-order first-fit lists (score 0) are
// bounded by (0, 0, last id + 1): the rank's unlisted feasible hosts come after its last one.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_kernel(PackArgs A) {
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int task = blockIdx.x * 4 + wave;
  if (task >= A.nt) return;
  const TaskRec& r = A.L.t[task];
  const int cnt = r.cnt;
  const ListEntry* e = A.L.e + (size_t)task * LMAX;
  SegEntry* out = A.out + (size_t)task * (A.PK + 1);
  for (int j = lane; j < A.PK; j += WAVE) {
    SegEntry o = {DINF, 0xffffffffu, 0x7fffffff};
    if (j < cnt) { o.s = e[j].s; o.tb = e[j].tb; o.id = e[j].id; }
    out[j] = o;
  }
  if (lane == 0) {
    SegEntry b = {DINF, 0xffffffffu, 0x7fffffff};
    if (cnt > A.PK) {
      b.s = e[A.PK].s; b.tb = e[A.PK].tb; b.id = e[A.PK].id;
    } else if (!r.complete) {
      if (A.ordered) { b.s = 0.0; b.tb = 0; b.id = e[cnt - 1].id + 1; }
      else { b.s = r.bs; b.tb = r.btb; b.id = r.bid; }
    }
    out[A.PK] = b;
  }
}
void launch_pack(const PackArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(pack_kernel, dim3((a.nt + 3) / 4), dim3(256), 0, st, a);
}

// ------------------------------------------------------------------------------------------
// Ordered scan (vbp first-fit, cost_aware first-fit without sort_hosts): the first KL
// snapshot-feasible hosts in index order, one wave per task, early exit.
// ------------------------------------------------------------------------------------------
template <bool STRICT>
__global__ __launch_bounds__(256) void ordered_kernel(OrderedArgs A) {
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int task = blockIdx.x * 4 + wave;
  if (task >= A.nt) return;
  const double* dp = A.dem + (size_t)task * 4;
  const double d0 = dp[0], d1 = dp[1], d2 = dp[2], d3 = dp[3];
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int cnt = 0;
  int hb = A.h_lo;
  for (; hb < A.h_hi && cnt < KL; hb += WAVE) {
    const int h = hb + lane;
    const bool ok = h < A.h_hi;
    const double a0 = ok ? A.avail[h] : -DINF;
    const double a1 = ok ? A.avail[(size_t)A.H + h] : -DINF;
    const double a2 = ok ? A.avail[2 * (size_t)A.H + h] : -DINF;
    const double a3 = ok ? A.avail[3 * (size_t)A.H + h] : -DINF;
    const bool fit = fits<STRICT>(a0, a1, a2, a3, d0, d1, d2, d3);
    const uint64_t m = __ballot(fit);
    if (fit) {
      const int pos = cnt + __popcll(m & below);
      if (pos < KL) {
        ListEntry e;
        e.s = 0.0; e.tb = 0; e.id = h; e.zone = A.zone[h]; e.pad = 0; e.pad2 = 0.0;
        e.a[0] = a0; e.a[1] = a1; e.a[2] = a2; e.a[3] = a3;
        A.L.e[(size_t)task * LMAX + pos] = e;
        A.L.ids[(size_t)task * LMAX + pos] = h;
      }
    }
    cnt += __popcll(m);
  }
  if (lane < 4) reinterpret_cast<double*>(&A.L.t[task])[lane] = dp[lane];
  if (lane == 0) {
    TaskRec& r = A.L.t[task];
    r.cnt = cnt < KL ? cnt : KL;
    r.complete = (hb >= A.h_hi) && cnt <= KL;
    r.anc = A.anc ? A.anc[task] : 0;
    r.ord = A.ord[task];
    r.bs = 0.0; r.btb = 0; r.bid = 0x7fffffff;   // first-fit walks never use the bound
  }
}

void launch_ordered(const OrderedArgs& a, hipStream_t st) {
  dim3 grid((a.nt + 3) / 4), block(256);
  if (a.strict) hipLaunchKernelGGL(ordered_kernel<true>, grid, block, 0, st, a);
  else hipLaunchKernelGGL(ordered_kernel<false>, grid, block, 0, st, a);
}

// ------------------------------------------------------------------------------------------
// Commit walk: one wave visits the window's tasks in processing order and applies the
// reference's sequential semantics. Hosts committed to in this window ("touched") live in LDS
// with their current availability; every other host still has its snapshot state, so its list
// entry (score, feasibility) is exact. Best-fit: winner = min(first untouched list entry,
// rescored touched hosts). First-fit: first list entry that is still feasible. A list whose
// entries are all touched and that may be missing hosts ("not complete") stops the walk; the
// host side then starts a new window there (a refill).
// ------------------------------------------------------------------------------------------
constexpr int HASH_SLOTS = 1 << HASH_BITS;
constexpr int PREFETCH = 3;      // commit walk: task lists loaded this many tasks ahead

struct CommitLDS {
  int32_t hkey[HASH_SLOTS];
  int32_t hval[HASH_SLOTS];
  int32_t tid[MAX_WINDOW];       // touched slot -> host
  int32_t tz[MAX_WINDOW];
  uint32_t ttb[MAX_WINDOW];
  int32_t lpos[MAX_WINDOW];      // touched slot -> position in the live list (-1: dead)
  double ta[4][MAX_WINDOW];      // current availability of touched hosts
  // live list: touched hosts that can still fit some task of the window, stored contiguously
  double la[4][MAX_WINDOW];
  int32_t lid[MAX_WINDOW];
  int32_t lz[MAX_WINDOW];
  uint32_t ltb[MAX_WINDOW];
  int32_t lslot[MAX_WINDOW];
  double csum[ZMAX * ZMAX];
  double bsum[ZMAX * ZMAX];
  double lim[ZMAX];
};

static_assert(sizeof(CommitLDS) <= 160 * 1024, "commit walk LDS exceeds a CU's 160 KiB");

__device__ __forceinline__ uint32_t hslot(int32_t id) {
  return ((uint32_t)id * 2654435761u) >> (32 - HASH_BITS);
}
__device__ __forceinline__ int hash_find(const CommitLDS& S, int32_t id) {
  uint32_t p = hslot(id);
  for (;;) {
    const int32_t k = S.hkey[p];
    if (k == id) return S.hval[p];
    if (k < 0) return -1;
    p = (p + 1) & (HASH_SLOTS - 1);
  }
}
__device__ __forceinline__ void hash_put(CommitLDS& S, int32_t id, int32_t v) {
  uint32_t p = hslot(id);
  while (S.hkey[p] >= 0) p = (p + 1) & (HASH_SLOTS - 1);
  S.hkey[p] = id;
  S.hval[p] = v;
}

constexpr double ZERO_ZONE = -2.0;   // lim-table marker: score is exactly 0 in this zone
constexpr int SCAN_UNROLL = 4;       // live hosts rescored per lane per loop trip

// One task's candidate list: this lane's entry, plus the task record spread over lanes 0-11
// (a vector load, so no scalar-memory wait is ever mixed with the LDS traffic of the walk).
struct Cand {
  ListEntry e;                 // entry `lane` of chunk 0
  int32_t tv;                  // TaskRec dword `lane` (lanes 0-15)
  int32_t ids[LMAX / KL - 1];  // host ids of entries 64*c + lane, c = 1..15
};
__device__ __forceinline__ void load_cand(const CommitArgs& A, int i, int lane, Cand& c) {
  c.e = A.L.e[(size_t)i * LMAX + lane];
  c.tv = reinterpret_cast<const int32_t*>(A.L.t + i)[lane < 16 ? lane : 0];
#pragma unroll
  for (int k = 0; k < LMAX / KL - 1; k++) c.ids[k] = A.L.ids[(size_t)i * LMAX + (k + 1) * KL + lane];
}
__device__ __forceinline__ double tv_d(int32_t tv, int k) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(tv, 2 * k);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane(tv, 2 * k + 1);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

#ifdef PVT_STAMPS
// Diagnostic build only (make stamps): per-phase cycle sums of the commit walk.
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

template <int MODE>
__global__ __launch_bounds__(64) void commit_kernel(CommitArgs A) {
  constexpr bool STRICT = (MODE == CA_FF || MODE == VBP_BF);
  constexpr bool BEST = (MODE == CA_BF || MODE == VBP_BF);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  CommitLDS& S = *reinterpret_cast<CommitLDS*>(smem);
  const int lane = lane_id();
  for (int i = lane; i < HASH_SLOTS; i += WAVE) S.hkey[i] = -1;
  if (MODE == CA_BF)
    for (int i = lane; i < A.Z * A.Z; i += WAVE) { S.csum[i] = A.csum[i]; S.bsum[i] = A.bsum[i]; }
  // Componentwise minimum demand of the window: a touched host that cannot fit it can never
  // win again in this window, so it leaves the live (rescoring) list.
  double m0 = DINF, m1 = DINF, m2 = DINF, m3 = DINF;
  if (BEST) {
    for (int i = lane; i < A.nt; i += WAVE) {
      const double* dp = A.dem + (size_t)i * 4;
      m0 = fmin(m0, dp[0]); m1 = fmin(m1, dp[1]); m2 = fmin(m2, dp[2]); m3 = fmin(m3, dp[3]);
    }
    for (int off = 32; off > 0; off >>= 1) {
      m0 = fmin(m0, __shfl_xor(m0, off)); m1 = fmin(m1, __shfl_xor(m1, off));
      m2 = fmin(m2, __shfl_xor(m2, off)); m3 = fmin(m3, __shfl_xor(m3, off));
    }
  }
  int m = 0;               // touched hosts (uniform)
  int nl = 0;              // live touched hosts (uniform)
  int next = A.nt;

#ifdef PVT_STAMPS
  uint64_t ph[5] = {0, 0, 0, 0, 0};
  uint64_t nl_sum = 0;
  uint64_t tl = stamp();
#endif
  // Lists are loaded PREFETCH tasks ahead into a ring of register sets that is never copied
  // (a copy would wait for the youngest load): the walk is unrolled by PREFETCH and each step
  // refills the set it just consumed.
  Cand c0, c1, c2;
  if (0 < A.nt) load_cand(A, 0, lane, c0);
  if (1 < A.nt) load_cand(A, 1, lane, c1);
  if (2 < A.nt) load_cand(A, 2, lane, c2);
  // step(cur, i): walk task i; returns true when the walk must stop (refill).
  auto step = [&](Cand& cur, const int i) -> bool {
    const double d0 = tv_d(cur.tv, 0), d1 = tv_d(cur.tv, 1), d2 = tv_d(cur.tv, 2), d3 = tv_d(cur.tv, 3);
    const int cnt = __builtin_amdgcn_readlane(cur.tv, 8);
    const bool comp = __builtin_amdgcn_readlane(cur.tv, 9) != 0;
    const int anc = __builtin_amdgcn_readlane(cur.tv, 10);
    const int caller = __builtin_amdgcn_readlane(cur.tv, 11);
    const bool valid = lane < cnt;
    STAMP(0);
    const int slot = valid ? hash_find(S, cur.e.id) : -1;
    STAMP(1);

    int w_id = -1, w_slot = -1, w_z = 0;
    uint32_t w_tb = 0;
    double w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    // The first usable list entry: chunk 0 is in registers; deeper chunks are searched by id
    // (LDS hash probes) and only the winning entry is then read from memory.
    int uc = -1, ul = -1;                // chunk and lane of the first usable entry
    {
      const bool ok0 = BEST ? (valid && slot < 0)
                            : (valid && (slot < 0 || fits<STRICT>(S.ta[0][max(slot, 0)], S.ta[1][max(slot, 0)],
                                                                  S.ta[2][max(slot, 0)], S.ta[3][max(slot, 0)],
                                                                  d0, d1, d2, d3)));
      const uint64_t m0 = __ballot(ok0);
      if (m0) {
        uc = 0;
        ul = __builtin_ctzll(m0);
      } else {
#pragma unroll
        for (int c = 1; c < LMAX / KL; c++) {
          if (uc < 0 && c * KL < cnt) {
            const bool v = c * KL + lane < cnt;
            const int sl = v ? hash_find(S, cur.ids[c - 1]) : -1;
            const bool ok = BEST ? (v && sl < 0)
                                 : (v && (sl < 0 || fits<STRICT>(S.ta[0][max(sl, 0)], S.ta[1][max(sl, 0)],
                                                                 S.ta[2][max(sl, 0)], S.ta[3][max(sl, 0)],
                                                                 d0, d1, d2, d3)));
            const uint64_t mc = __ballot(ok);
            if (mc) { uc = c; ul = __builtin_ctzll(mc); }
          }
        }
      }
    }
    // the usable entry's fields (uniform)
    double us = DINF, ua0 = 0, ua1 = 0, ua2 = 0, ua3 = 0;
    uint32_t utb = 0xffffffffu;
    int32_t uid = 0x7fffffff, uz = 0, uslot = -1;
    if (uc == 0) {
      us = readlane_d(cur.e.s, ul); utb = readlane_u(cur.e.tb, ul); uid = readlane_i(cur.e.id, ul);
      uz = readlane_i(cur.e.zone, ul); uslot = readlane_i(slot, ul);
      ua0 = readlane_d(cur.e.a[0], ul); ua1 = readlane_d(cur.e.a[1], ul);
      ua2 = readlane_d(cur.e.a[2], ul); ua3 = readlane_d(cur.e.a[3], ul);
    } else if (uc > 0) {
      const ListEntry& ue = A.L.e[(size_t)i * LMAX + uc * KL + ul];
      us = ue.s; utb = ue.tb; uid = ue.id; uz = ue.zone;
      ua0 = ue.a[0]; ua1 = ue.a[1]; ua2 = ue.a[2]; ua3 = ue.a[3];
      uslot = BEST ? -1 : hash_find(S, uid);
      uslot = __builtin_amdgcn_readfirstlane(uslot);
    }

    if (BEST) {
      // No untouched entry and hosts missing from the list: every untouched host outside the
      // list ranks at or after the bound, so a touched host at or before it still wins exactly;
      // only if none does must the walk stop for a refill. (bi = bid + 1 turns the strict
      // comparisons below into <= bound; ids are unique, so equality means the same host.)
      const bool exhausted = (uc < 0) && !comp;
      double bs = us;
      uint32_t bt = utb;
      int32_t bi = uid;
      if (exhausted) {
        bs = tv_d(cur.tv, 6);
        bt = (uint32_t)__builtin_amdgcn_readlane(cur.tv, 14);
        bi = __builtin_amdgcn_readlane(cur.tv, 15) + 1;
      }
      int bq = -1;                       // live position of the winner
      STAMP(2);
#ifdef PVT_STAMPS
      nl_sum += nl;
#endif
      if (MODE == CA_BF && nl > 0 && bs == 0.0) {
        // Best untouched score is exactly 0 (a zero-cost zone). A live host can only win with
        // score 0 and a lower index: either it sits in a zero-cost zone, or its residual is
        // exactly zero. Every such candidate scores 0, so the winner is the lowest index.
        const uint32_t zz = (uint32_t)__ballot(lane < A.Z && S.csum[anc * A.Z + lane] == 0.0);
        int best = 0x7fffffff, bestq = -1;
        for (int q0 = 0; q0 < nl; q0 += WAVE * SCAN_UNROLL) {
#pragma unroll
          for (int u = 0; u < SCAN_UNROLL; u++) {
            const int j = q0 + u * WAVE + lane;
            const int jj = min(j, nl - 1);
            const double a0 = S.la[0][jj], a1 = S.la[1][jj], a2 = S.la[2][jj], a3 = S.la[3][jj];
            const int32_t id = S.lid[jj];
            const bool zero_zone = (zz >> S.lz[jj]) & 1u;
            const bool pass = (j < nl) && id < bi && fits<STRICT>(a0, a1, a2, a3, d0, d1, d2, d3) &&
                              (zero_zone || (a0 == d0 && a1 == d1 && a2 == d2 && a3 == d3));
            if (pass && id < best) { best = id; bestq = j; }
          }
        }
        for (int off = 32; off > 0; off >>= 1) {
          const int ob = __shfl_xor(best, off), oq = __shfl_xor(bestq, off);
          if (ob < best) { best = ob; bestq = oq; }
        }
        if (best < bi) { bs = 0.0; bt = 0; bi = best; bq = bestq; }
      } else if (nl > 0) {
        double vlim = DINF;
        if (MODE == CA_BF) {
          if (lane < A.Z) {
            const double c = S.csum[anc * A.Z + lane];
            S.lim[lane] = (c == 0.0) ? ZERO_ZONE : ca_lim(bs, c, S.bsum[anc * A.Z + lane]);
          }
        } else {
          vlim = vbp_lim(bs);
        }
        for (int q0 = 0; q0 < nl; q0 += WAVE * SCAN_UNROLL) {
          double s2[SCAN_UNROLL];
          bool pass[SCAN_UNROLL];
          int z[SCAN_UNROLL];
          bool any = false;
#pragma unroll
          for (int u = 0; u < SCAN_UNROLL; u++) {
            const int j = q0 + u * WAVE + lane;
            const int jj = min(j, nl - 1);
            const double a0 = S.la[0][jj], a1 = S.la[1][jj], a2 = S.la[2][jj], a3 = S.la[3][jj];
            const bool fit = (j < nl) && fits<STRICT>(a0, a1, a2, a3, d0, d1, d2, d3);
            s2[u] = norm2_seq(a0 - d0, a1 - d1, a2 - d2, a3 - d3);
            if (MODE == CA_BF) {
              z[u] = S.lz[jj];
              const double lm = S.lim[z[u]];
              pass[u] = fit && ((lm == ZERO_ZONE) ? lexless(0.0, 0u, S.lid[jj], bs, bt, bi) : (s2[u] <= lm));
            } else {
              z[u] = 0;
              pass[u] = fit && (s2[u] <= vlim);
            }
            any |= pass[u];
          }
          if (__ballot(any) == 0) continue;
          double cs = DINF;
          uint32_t ct = 0xffffffffu;
          int32_t ci = 0x7fffffff;
          int cq = -1;
#pragma unroll
          for (int u = 0; u < SCAN_UNROLL; u++) {
            if (!pass[u]) continue;
            const int j = q0 + u * WAVE + lane;
            double sc;
            uint32_t tb;
            if (MODE == CA_BF) {
              const double c = S.csum[anc * A.Z + z[u]];
              // (c * r) / b as the reference computes it; c == 0 gives exactly 0
              sc = (c == 0.0) ? 0.0 : (c * __builtin_sqrt(s2[u])) / S.bsum[anc * A.Z + z[u]];
              tb = 0;
            } else {
              sc = __builtin_sqrt(s2[u]);
              tb = S.ltb[j];
            }
            const int32_t id = S.lid[j];
            if (lexless(sc, tb, id, cs, ct, ci)) { cs = sc; ct = tb; ci = id; cq = j; }
          }
          for (int off = 32; off > 0; off >>= 1) {
            const double os = __shfl_xor(cs, off);
            const uint32_t ot = (uint32_t)__shfl_xor((int)ct, off);
            const int32_t oi = __shfl_xor(ci, off);
            const int oq = __shfl_xor(cq, off);
            if (lexless(os, ot, oi, cs, ct, ci)) { cs = os; ct = ot; ci = oi; cq = oq; }
          }
          if (lexless(cs, ct, ci, bs, bt, bi)) { bs = cs; bt = ct; bi = ci; bq = cq; }
        }
      }
      STAMP(3);
      if (exhausted && bq < 0) { next = i; return true; }
      if (bi == 0x7fffffff || (exhausted && bq < 0)) {   // no feasible host: the task waits
        if (i + PREFETCH < A.nt) load_cand(A, i + PREFETCH, lane, cur);
        return false;
      }
      w_id = bi;
      w_tb = bt;
      if (bq >= 0) {
        w_slot = S.lslot[bq];
        w0 = S.la[0][bq]; w1 = S.la[1][bq]; w2 = S.la[2][bq]; w3 = S.la[3][bq];
      } else {
        w_z = uz;
        w0 = ua0; w1 = ua1; w2 = ua2; w3 = ua3;
      }
    } else {
      if (uc < 0) {
        if (!comp) { next = i; return true; }
        if (i + PREFETCH < A.nt) load_cand(A, i + PREFETCH, lane, cur);
        return false;
      }
      w_id = uid;
      w_slot = uslot;
      if (w_slot >= 0) {
        w0 = S.ta[0][w_slot]; w1 = S.ta[1][w_slot]; w2 = S.ta[2][w_slot]; w3 = S.ta[3][w_slot];
      } else {
        w_z = uz;
        w0 = ua0; w1 = ua1; w2 = ua2; w3 = ua3;
      }
    }
    // commit: resc[h] -= t_demand (cost_aware.py:95,126; vbp.py:24,49)
    const double n0 = w0 - d0, n1 = w1 - d1, n2 = w2 - d2, n3 = w3 - d3;
    if (w_slot < 0) {
      w_slot = m++;
      if (lane == 0) {
        hash_put(S, w_id, w_slot);
        S.tid[w_slot] = w_id;
        S.tz[w_slot] = w_z;
        S.ttb[w_slot] = w_tb;
        S.lpos[w_slot] = -1;
      }
    }
    if (BEST) {
      const bool alive = fits<STRICT>(n0, n1, n2, n3, m0, m1, m2, m3);
      const int p = __builtin_amdgcn_readfirstlane(S.lpos[w_slot]);
      if (alive) {
        const int q = (p >= 0) ? p : nl++;
        if (lane == 0) {
          S.la[0][q] = n0; S.la[1][q] = n1; S.la[2][q] = n2; S.la[3][q] = n3;
          if (p < 0) {
            S.lid[q] = w_id; S.lz[q] = S.tz[w_slot]; S.ltb[q] = w_tb; S.lslot[q] = w_slot;
            S.lpos[w_slot] = q;
          }
        }
      } else if (p >= 0) {               // swap-remove from the live list
        nl--;
        if (lane == 0 && p != nl) {
          S.la[0][p] = S.la[0][nl]; S.la[1][p] = S.la[1][nl];
          S.la[2][p] = S.la[2][nl]; S.la[3][p] = S.la[3][nl];
          S.lid[p] = S.lid[nl]; S.lz[p] = S.lz[nl]; S.ltb[p] = S.ltb[nl];
          S.lslot[p] = S.lslot[nl];
          S.lpos[S.lslot[nl]] = p;
        }
        if (lane == 0) S.lpos[w_slot] = -1;
      }
    }
    if (lane == 0) {
      S.ta[0][w_slot] = n0; S.ta[1][w_slot] = n1; S.ta[2][w_slot] = n2; S.ta[3][w_slot] = n3;
      A.avail[w_id] = n0;
      A.avail[(size_t)A.H + w_id] = n1;
      A.avail[2 * (size_t)A.H + w_id] = n2;
      A.avail[3 * (size_t)A.H + w_id] = n3;
      A.placement[caller] = w_id;
    }
    STAMP(4);
    if (i + PREFETCH < A.nt) load_cand(A, i + PREFETCH, lane, cur);
    return false;
  };
  for (int i = 0; i < A.nt;) {
    if (step(c0, i)) break;
    if (++i >= A.nt) break;
    if (step(c1, i)) break;
    if (++i >= A.nt) break;
    if (step(c2, i)) break;
    ++i;
  }
  if (lane == 0) *A.next = next;
#ifdef PVT_STAMPS
  if (lane == 0 && A.stamps)
    for (int k = 0; k < 5; k++) atomicAdd((unsigned long long*)&A.stamps[k], (unsigned long long)ph[k]);
  if (lane == 0 && A.stamps) atomicAdd((unsigned long long*)&A.stamps[5], (unsigned long long)A.nt);
  if (lane == 0 && A.stamps) atomicAdd((unsigned long long*)&A.stamps[6], (unsigned long long)nl_sum);
#endif
}

size_t commit_lds_bytes() { return sizeof(CommitLDS); }

hipError_t init_kernel_attrs() {
  const int lds = (int)sizeof(CommitLDS);
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
  const size_t lds = sizeof(CommitLDS);
  switch (a.mode) {
    case CA_FF: hipLaunchKernelGGL(commit_kernel<CA_FF>, dim3(1), dim3(64), lds, st, a); break;
    case CA_BF: hipLaunchKernelGGL(commit_kernel<CA_BF>, dim3(1), dim3(64), lds, st, a); break;
    case VBP_FF: hipLaunchKernelGGL(commit_kernel<VBP_FF>, dim3(1), dim3(64), lds, st, a); break;
    case VBP_BF: hipLaunchKernelGGL(commit_kernel<VBP_BF>, dim3(1), dim3(64), lds, st, a); break;
    default: break;
  }
}

// ------------------------------------------------------------------------------------------
// Small kernels: zone tables, frozen first-fit keys, a2 sort keys, gathers.
// ------------------------------------------------------------------------------------------
__global__ void zone_tables_kernel(const double* cost, const double* bw, int Z, double* csum,
                                   double* bsum) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Z * Z) return;
  const int a = i / Z, z = i % Z;
  csum[i] = cost[a * Z + z] + cost[z * Z + a];   // cost_aware.py:82,113
  bsum[i] = bw[a * Z + z] + bw[z * Z + a];       // in_route.bw + out_route.bw (:79,111)
}
void launch_zone_tables(const double* cost, const double* bw, int Z, double* csum, double* bsum,
                        hipStream_t st) {
  hipLaunchKernelGGL(zone_tables_kernel, dim3((Z * Z + 255) / 256), dim3(256), 0, st, cost, bw, Z,
                     csum, bsum);
}

// host_score_func of _first_fit (cost_aware.py:104-116): c * df / (r * bw), r = ||avail_h||.
__global__ void key_kernel(KeyArgs A) {
  const int h = A.h_lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= A.h_hi) return;
  const double a0 = A.avail[h], a1 = A.avail[(size_t)A.H + h];
  const double a2 = A.avail[2 * (size_t)A.H + h], a3 = A.avail[3 * (size_t)A.H + h];
  const double r = __builtin_sqrt(norm2_seq(a0, a1, a2, a3));
  const int z = A.zone[h];
  const double c = A.csum[A.anchor * A.Z + z], bw = A.bsum[A.anchor * A.Z + z];
  const double df = A.decay ? (double)A.decay[h] : 1.0;
  A.key[h] = (c * df) / (r * bw);
}
void launch_key(const KeyArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(key_kernel, dim3((a.h_hi - a.h_lo + 255) / 256), dim3(256), 0, st, a);
}

__global__ void norm_keys_kernel(const double* dem, int T, const int32_t* idx, uint64_t* keys) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T) return;
  const int t = idx ? idx[i] : i;
  const double n = __builtin_sqrt(norm2_seq(dem[t], dem[(size_t)T + t], dem[2 * (size_t)T + t],
                                            dem[3 * (size_t)T + t]));
  // n >= 0, so its bits order like the value; ~bits sorts descending norm ascending.
  keys[i] = ~(uint64_t)__double_as_longlong(n);
}
void launch_norm_keys(const double* dem, int T, const int32_t* idx, uint64_t* keys, hipStream_t st) {
  hipLaunchKernelGGL(norm_keys_kernel, dim3((T + 255) / 256), dim3(256), 0, st, dem, T, idx, keys);
}

__global__ void group_keys_kernel(const int32_t* tg, const int32_t* idx, int T, uint32_t* keys) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T) return;
  keys[i] = (uint32_t)tg[idx ? idx[i] : i];
}
void launch_group_keys(const int32_t* task_group, const int32_t* idx, int T, uint32_t* keys,
                       hipStream_t st) {
  hipLaunchKernelGGL(group_keys_kernel, dim3((T + 255) / 256), dim3(256), 0, st, task_group, idx,
                     T, keys);
}

__global__ void iota_kernel(int32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = i;
}
void launch_iota(int32_t* out, int n, hipStream_t st) {
  hipLaunchKernelGGL(iota_kernel, dim3((n + 255) / 256), dim3(256), 0, st, out, n);
}

__global__ void gather_tasks_kernel(const double* dem, const int32_t* ord, const int32_t* tg,
                                    const int32_t* ga, int T, double* dem_ord, int32_t* anc_ord) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= T) return;
  const int t = ord[p];
  double* o = dem_ord + (size_t)p * 4;
  o[0] = dem[t]; o[1] = dem[(size_t)T + t]; o[2] = dem[2 * (size_t)T + t]; o[3] = dem[3 * (size_t)T + t];
  anc_ord[p] = (tg && ga) ? ga[tg[t]] : 0;
}
void launch_gather_tasks(const double* dem, const int32_t* ord, const int32_t* task_group,
                         const int32_t* group_anchor, int T, double* dem_ord, int32_t* anc_ord,
                         hipStream_t st) {
  hipLaunchKernelGGL(gather_tasks_kernel, dim3((T + 255) / 256), dim3(256), 0, st, dem, ord,
                     task_group, group_anchor, T, dem_ord, anc_ord);
}

}  // namespace pvt
