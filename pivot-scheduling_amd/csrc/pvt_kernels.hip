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
#include <algorithm>
#include <stdint.h>
#include <stdlib.h>

#include "pvt_device.h"
#include "pvt_kernels.h"
#include "pvt_zwin_dev.h"
#include "pvt_list.h"

namespace pvt {

#ifdef PVT_DIAG
// Diagnostic build only (make diag): score-pass candidate counts, summed over launches:
// [0] candidates streamed (task x host), [1] prefilter survivors, [2] exact survivors (fit and
// within the list's limit), [3] list merges, [4] host blocks streamed per wave.
__device__ unsigned long long g_score_diag[8];
#endif

// ------------------------------------------------------------------------------------------
// Score kernel: candidates (window tasks) x (one host segment). Block = 4 waves; each wave owns
// TW tasks (2 for vbp best-fit, 4 otherwise) and streams the segment's hosts 64 at a time (lane = host), keeping a sorted top-KL
// list per task in registers. blockIdx % S picks the segment, so with S = 8 the blocks of one
// segment share an XCD (round-robin dispatch) and its L2 holds that slice of the host table.
// ------------------------------------------------------------------------------------------
template <int MODE, int TW>
__global__ __launch_bounds__(256) void score_kernel(ScoreArgs A) {
  constexpr bool STRICT = (MODE != CA_BF);
  constexpr int ZL = (MODE == CA_BF) ? ZMAX : 1;
  __shared__ double s_lim[WPB][TW][ZL];
  __shared__ double s_rad[WPB][TW][ZL];
  __shared__ double s_c[WPB][TW][ZL];
  __shared__ double s_b[WPB][TW][ZL];
  __shared__ uint64_t s_m1[WPB][KL], s_m2[WPB][KL];   // list_merge staging, per wave

  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int seg = blockIdx.x % A.S, tile = blockIdx.x / A.S;
  const int t0 = (tile * WPB + wave) * TW;
  if (t0 >= A.nt) return;
  const int nt = min(TW, A.nt - t0);
  // realtime_bw (cost_aware.py:79): the bandwidth is per (group, host), so no per-zone radius
  // bounds the score -- every fitting candidate is scored exactly
  const bool rt = (MODE == CA_BF) && A.rtb != nullptr;
  // Segment `seg` owns the 64-host blocks seg, seg + S, seg + 2S, ... of [h_lo, h_hi): each
  // block is one coalesced load per component, and interleaving keeps every segment's share of
  // low host indices equal, so lists stay deep when many hosts tie (zero-cost zones, where the
  // index breaks the tie) -- contiguous segments would bound the merged list at segment 0's
  // 64th tied host.
  const int hb0 = A.h_lo + seg * WAVE, hb1 = A.h_hi, hstep = A.S * WAVE;

  double d0[TW], d1[TW], d2[TW], d3[TW];
  double ls[TW], ts[TW], lim[TW], rd[TW];
  const double* rb[TW];
  uint32_t lt[TW], tt[TW];
  int32_t li[TW], ti[TW];
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
    rd[k] = (k < nt) ? DINF : -1.0;        // a missing task never passes the prefilter
    rb[k] = (rt && k < nt) ? A.rtb + (size_t)A.grp[t0 + k] * A.H : A.rtb;
    if (MODE == CA_BF) {
      const int a = (k < nt) ? A.anc[t0 + k] : 0;
      if (lane < A.Z) {
        s_c[wave][k][lane] = A.csum[a * A.Z + lane];
        s_b[wave][k][lane] = A.bsum[a * A.Z + lane];
        s_lim[wave][k][lane] = DINF;
        s_rad[wave][k][lane] = rd[k];
      }
    }
  }

  // Host data for block hb is loaded one iteration ahead (register double buffer), with the
  // index clamped instead of branching, so the loads overlap the previous block's scoring.
  double n0 = 0, n1 = 0, n2 = 0, n3 = 0, nkey = DINF;
  int nz = 0;
  uint32_t ntb = 0;
  auto fetch = [&](int hb) {
    const int h = min(hb + lane, hb1 - 1);
    n0 = A.avail[h];
    n1 = A.avail[(size_t)A.H + h];
    n2 = A.avail[2 * (size_t)A.H + h];
    n3 = A.avail[3 * (size_t)A.H + h];
    if (MODE == CA_BF) nz = A.zone[h];
    if (MODE == CA_FF) nkey = A.key[h];
    if (MODE == VBP_BF) ntb = A.tb[h];     // host-id rank: read with the block, not per hit
  };
#ifdef PVT_DIAG
  unsigned long long dg[5] = {0, 0, 0, 0, 0};
#endif
  if (hb0 < hb1) fetch(hb0);
  for (int hb = hb0; hb < hb1; hb += hstep) {
    // Exact early exit (cost_aware): scores are >= +0 and the tiebreak is 0, so once every task's
    // last entry is (0, 0, id) no later host of the segment -- all of larger index -- can enter
    // any list: the lists are final. The anchor zone's free-egress hosts fill the lists this way.
    if (MODE == CA_BF || MODE == CA_FF) {
      bool final_ = true;
#pragma unroll
      for (int k = 0; k < TW; k++)
        if (k < nt) final_ &= (__double_as_longlong(ts[k]) == 0) & (tt[k] == 0u);
      if (final_) break;
    }
    const double a0 = n0, a1 = n1, a2 = n2, a3 = n3, key = nkey;
    const int z = nz;
    const uint32_t tbh = ntb;
    if (hb + hstep < hb1) fetch(hb + hstep);
    const int h = hb + lane;
    const bool ok = h < hb1;
    // prefilter, all tasks: frozen key (first-fit) or memory radius (best-fit)
    bool pre[TW];
    bool any = false;
#pragma unroll
    for (int k = 0; k < TW; k++) {
      if (MODE == CA_FF) {
        pre[k] = ok && lexless(key, 0u, h, ts[k], tt[k], ti[k]);
      } else {
        const double r = (MODE == CA_BF) ? s_rad[wave][k][z] : rd[k];
        pre[k] = ok && (__builtin_fabs(a1 - d1[k]) <= r);
      }
      any |= pre[k];
    }
#ifdef PVT_DIAG
    dg[4] += 1;
#pragma unroll
    for (int k = 0; k < TW; k++) {
      dg[0] += (k < nt) ? __popcll(__ballot(ok)) : 0;
      dg[1] += __popcll(__ballot(pre[k]));
    }
#endif
    if (__ballot(any) == 0) continue;
#pragma unroll
    for (int k = 0; k < TW; k++) {
      if (__ballot(pre[k]) == 0) continue;
      const bool fit = pre[k] && fits<STRICT>(a0, a1, a2, a3, d0[k], d1[k], d2[k], d3[k]);
      double s2 = 0.0;
      bool pass;
      if (MODE == CA_FF) {
        pass = fit;
      } else {
        s2 = norm2_seq(a0 - d0[k], a1 - d1[k], a2 - d2[k], a3 - d3[k]);
        const double lm = (MODE == CA_BF) ? s_lim[wave][k][z] : lim[k];
        pass = fit && (s2 <= lm);
      }
      uint64_t pm = __ballot(pass);
#ifdef PVT_DIAG
      dg[2] += __popcll(pm);
#endif
      if (pm) {
        double sc = DINF;
        uint32_t tbv = 0;
        if (pass) {
          if (MODE == CA_FF) {
            sc = key;
          } else if (MODE == CA_BF) {
            const double r = __builtin_sqrt(s2);
            sc = (s_c[wave][k][z] * r) / (rt ? rb[k][h] : s_b[wave][k][z]);
          } else {
            sc = __builtin_sqrt(s2);
            tbv = tbh;
          }
        }
        // Candidates that beat the task's current last entry, as 128-bit keys (score bits,
        // tiebreak:id): scores are >= +0, so their bits order like the values.
        const uint64_t tk1 = (uint64_t)__double_as_longlong(ts[k]);
        const uint64_t tk2 = ((uint64_t)tt[k] << 32) | (uint32_t)ti[k];
        const uint64_t ck1 = (uint64_t)__double_as_longlong(sc);
        const uint64_t ck2 = ((uint64_t)tbv << 32) | (uint32_t)h;
        pm = __ballot(pass && (ck1 < tk1 || (ck1 == tk1 && ck2 < tk2)));
        if (pm) {
#ifdef PVT_DIAG
          dg[3] += 1;
#endif
          list_merge(ls[k], lt[k], li[k], sc, tbv, h, pm, s_m1[wave], s_m2[wave]);
          ts[k] = readlane_d(ls[k], KL - 1);
          tt[k] = readlane_u(lt[k], KL - 1);
          ti[k] = readlane_i(li[k], KL - 1);

          if (MODE == CA_BF && !rt) {
            if (lane < A.Z) {
              const double lm2 = ca_lim(ts[k], s_c[wave][k][lane], s_b[wave][k][lane]);
              s_lim[wave][k][lane] = lm2;
              s_rad[wave][k][lane] = rad(lm2);
            }
          } else if (MODE == VBP_BF) {
            lim[k] = vbp_lim(ts[k]);
            rd[k] = vbp_rad(ts[k]);
          }
        }
      }
    }
  }

#ifdef PVT_DIAG
  if (lane == 0)
    for (int c = 0; c < 5; c++) atomicAdd(&g_score_diag[c], dg[c]);
#endif
  // Feasible hosts per segment, as the merge needs it: a list that never filled holds every
  // feasible host of the segment (its threshold stayed infinite); a full one reports KL + 1,
  // i.e. "bounded by its last entry" (every host it rejected ranked at or after that entry).
#pragma unroll
  for (int k = 0; k < TW; k++) {
    if (k < nt) {
      const size_t row = (size_t)(t0 + k) * A.S + seg;
      SegEntry e;
      e.s = ls[k]; e.tb = lt[k]; e.id = li[k];
      A.seg[row * KL + lane] = e;
      const int filled = __popcll(__ballot(li[k] != 0x7fffffff));
      if (lane == 0) A.seg_feas[row] = filled == KL ? KL + 1 : filled;
    }
  }
}

// Tasks per wave: vbp best-fit lists keep improving while a segment streams, so each block costs
// a few list merges; 2 tasks per wave doubles the waves that hide them (4.2e11 -> 4.9e11 cand/s
// at 1M x 10k). cost_aware's lists fill at once from the zero-cost zone, so 4 tasks share each
// host block's loads -- unless the segments are short enough (100k hosts) that filling the lists
// is most of the pass (config 3 ca_bf: 5.6e10 -> 6.1e10 with 2; 1M hosts: 7.4e11 -> 6.8e11).
// Diagnostic build: read (and with reset != 0 clear) the score-pass counters.
int score_diag(uint64_t* out, int n, int reset) {
#ifdef PVT_DIAG
  unsigned long long h[8];
  if (hipDeviceSynchronize() != hipSuccess) return -3;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_score_diag), sizeof(h)) != hipSuccess) return -3;
  for (int i = 0; i < n && i < 8; i++) out[i] = h[i];
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_score_diag), z, sizeof(z)) != hipSuccess) return -3;
  }
  return 0;
#else
  (void)out; (void)n; (void)reset;
  return -5;
#endif
}

int score_tasks_per_wave(int mode, int hosts, int force) {
  if (force == 2 || force == 4) return force;   // pvt_set_score_tw: both instances stay tested
  if (mode == VBP_BF) return 2;
  if (mode == CA_BF && hosts < (1 << 18)) return 2;
  return TW;
}

template <int MODE>
static void launch_score_tw(int tw, dim3 grid, dim3 block, const ScoreArgs& a, hipStream_t st) {
  if (tw == 2) PVT_LAUNCH((score_kernel<MODE, 2>), grid, block, 0, st, a);
  else PVT_LAUNCH((score_kernel<MODE, 4>), grid, block, 0, st, a);
}

void launch_score(int mode, const ScoreArgs& a, hipStream_t st) {
  const int tw = score_tasks_per_wave(mode, a.h_hi - a.h_lo, a.tw);
  const int tiles = (a.nt + WPB * tw - 1) / (WPB * tw);
  dim3 grid(tiles * a.S), block(WPB * WAVE);
  switch (mode) {
    case CA_FF: launch_score_tw<CA_FF>(tw, grid, block, a, st); break;
    case CA_BF: launch_score_tw<CA_BF>(tw, grid, block, a, st); break;
    case VBP_BF: launch_score_tw<VBP_BF>(tw, grid, block, a, st); break;
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
  if (gate_closed(A.gate)) return;   // (an enqueued-ahead window that will not be walked)
  const int task = blockIdx.x, tid = threadIdx.x;
  if (A.nt_dev && task >= *A.nt_dev) return;   // (representative lists: rows past the count)
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

// Merge of a few segment lists (S <= MERGE_SMALL_S, score-pass lists): one wave per task. Keys
// are distinct (a host is in one segment), so an entry's place in the merged order is its index
// in its own sorted list plus, in every other list, the number of entries below it (a binary
// search in LDS); entries land at their places directly -- no sorting network.
constexpr int MERGE_SMALL_S = 8;
__global__ __launch_bounds__(256) void merge_small_kernel(MergeArgs A) {
  __shared__ Key lk[4][MERGE_SMALL_S * KL];
  __shared__ Key out[4][MERGE_SMALL_S * KL];
  if (gate_closed(A.gate)) return;   // (an enqueued-ahead window that will not be walked)
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int task = blockIdx.x * 4 + wave;
  if (task >= A.nt || (A.nt_dev && task >= *A.nt_dev)) return;
  const int S = A.S, n = S * KL;
  Key* L = lk[wave];
  Key* O = out[wave];
  const Key inv = {DINF, 0xffffffffu, 0x7fffffff};
  for (int j = lane; j < n; j += WAVE) {
    const SegEntry se = A.seg[((size_t)task * S) * KL + j];
    L[j] = {se.s, se.tb, se.id};
    O[j] = inv;
  }
  // bound: the smallest last entry of a segment with more than KL feasible hosts
  Key bound = inv;
  long long tot = 0;
  for (int g = 0; g < S; g++) {
    const int f = A.seg_feas[(size_t)task * S + g];
    tot += f;
    if (f > KL) {
      const SegEntry se = A.seg[((size_t)task * S + g) * KL + KL - 1];
      const Key k = {se.s, se.tb, se.id};
      if (kless(k, bound)) bound = k;
    }
  }
  wave_sync();
  int c = 0;
  for (int j = lane; j < n; j += WAVE) {
    const Key x = L[j];
    if (x.id == 0x7fffffff || !kless(x, bound)) continue;   // invalid, or at/after the bound
    const int g = j / KL;
    int pos = j - g * KL;
    for (int h = 0; h < S; h++) {
      if (h == g) continue;
      const Key* Lh = L + h * KL;
      int lo = 0, hi = KL;                                   // entries of list h below x
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (kless(Lh[mid], x)) lo = mid + 1;
        else hi = mid;
      }
      pos += lo;
    }
    O[pos] = x;
    c++;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  wave_sync();
  const int cnt = c;
  const bool complete = (bound.id == 0x7fffffff) && tot <= LMAX;
  Key bnd = bound;
  if (cnt == LMAX && kless(O[LMAX - 1], bnd)) bnd = O[LMAX - 1];
  const int nw = max(cnt, KL);
  for (int j = lane; j < nw; j += WAVE) {
    ListEntry e;
    const bool valid = j < cnt;
    const Key k = valid ? O[j] : inv;
    const int h = valid ? k.id : 0;
    e.s = k.s; e.tb = k.tb; e.id = k.id; e.pad = 0; e.pad2 = 0.0;
    e.zone = valid ? A.zone[h] : 0;
    e.a[0] = valid ? A.avail[h] : 0.0;
    e.a[1] = valid ? A.avail[(size_t)A.H + h] : 0.0;
    e.a[2] = valid ? A.avail[2 * (size_t)A.H + h] : 0.0;
    e.a[3] = valid ? A.avail[3 * (size_t)A.H + h] : 0.0;
    A.L.e[(size_t)task * LMAX + j] = e;
    A.L.ids[(size_t)task * LMAX + j] = valid ? k.id : 0x7fffffff;
  }
  if (lane < 4) {
    double* tr = reinterpret_cast<double*>(&A.L.t[task]);
    tr[lane] = A.dem[(size_t)task * 4 + lane];
  }
  if (lane == 0) {
    TaskRec& r = A.L.t[task];
    r.cnt = cnt;
    r.complete = complete;
    r.anc = A.anc[task];
    r.ord = A.ord[task];
    r.bs = bnd.s; r.btb = bnd.tb; r.bid = bnd.id;
  }
}

// Merge of the ranks' packages (host-dimension sharding): one block per task, the same
// rank-by-counting as merge_small_kernel over world sorted lists of SL entries (world * SL <=
// LMAX), bounded by the smallest of the packages' explicit bound entries.
__device__ __forceinline__ int lower_bound_key(const Key* L, int n, const Key& x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (kless(L[mid], x)) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void merge_pkg_kernel(MergeArgs A) {
  __shared__ Key lk[LMAX];
  __shared__ Key out[LMAX];
  __shared__ Key bound;
  __shared__ int cnt_sh, tot_sh;
  if (gate_closed(A.gate)) return;   // (an enqueued-ahead window that will not be walked)
  const int task = blockIdx.x, tid = threadIdx.x;
  if (A.nt_dev && task >= *A.nt_dev) return;   // (representative lists: rows past the count)
  const int W = A.S, SL = A.SL, n = W * SL;
  const Key inv = {DINF, 0xffffffffu, 0x7fffffff};
  if (tid == 0) { bound = inv; cnt_sh = 0; tot_sh = 0; }
  int valid = 0;
  for (int j = tid; j < n; j += 256) {
    const int g = j / SL, e = j - g * SL;
    const SegEntry se = A.seg[((size_t)g * A.nt + task) * (SL + 1) + e];
    lk[j] = {se.s, se.tb, se.id};
    out[j] = inv;
    valid += se.id != 0x7fffffff;
  }
  __syncthreads();
  if (tid == 0) {
    Key b = inv;
    for (int g = 0; g < W; g++) {
      const SegEntry se = A.seg[((size_t)g * A.nt + task) * (SL + 1) + SL];
      const Key k = {se.s, se.tb, se.id};
      if (kless(k, b)) b = k;
    }
    bound = b;
  }
  if (valid) atomicAdd(&tot_sh, valid);
  __syncthreads();
  const Key bnd0 = bound;
  int c = 0;
  for (int j = tid; j < n; j += 256) {
    const Key x = lk[j];
    if (x.id == 0x7fffffff || !kless(x, bnd0)) continue;
    const int g = j / SL;
    int pos = j - g * SL;
    for (int h = 0; h < W; h++)
      if (h != g) pos += lower_bound_key(lk + h * SL, SL, x);
    out[pos] = x;
    c++;
  }
  if (c) atomicAdd(&cnt_sh, c);
  __syncthreads();
  const int cnt = cnt_sh;
  const bool complete = (bnd0.id == 0x7fffffff) && tot_sh <= LMAX;
  Key bnd = bnd0;
  if (cnt == LMAX && kless(out[LMAX - 1], bnd)) bnd = out[LMAX - 1];
  const int nw = max(cnt, KL);
  for (int j = tid; j < nw; j += 256) {
    ListEntry e;
    const bool ok = j < cnt;
    const Key k = ok ? out[j] : inv;
    const int h = ok ? k.id : 0;
    e.s = k.s; e.tb = k.tb; e.id = k.id; e.pad = 0; e.pad2 = 0.0;
    e.zone = ok ? A.zone[h] : 0;
    e.a[0] = ok ? A.avail[h] : 0.0;
    e.a[1] = ok ? A.avail[(size_t)A.H + h] : 0.0;
    e.a[2] = ok ? A.avail[2 * (size_t)A.H + h] : 0.0;
    e.a[3] = ok ? A.avail[3 * (size_t)A.H + h] : 0.0;
    A.L.e[(size_t)task * LMAX + j] = e;
    A.L.ids[(size_t)task * LMAX + j] = ok ? k.id : 0x7fffffff;
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

// Merge of up to LMAX / KL score-segment lists (vbp best-fit band lists: 16 segments), each
// already sorted, by merge path, one block per task: the segments (padded with invalid keys to a
// power of two) are merged pairwise in log2(segments) rounds; in a round every thread takes four
// consecutive outputs of its pair, finds how many of them come from the first list by a binary
// search of the merge path (co-rank), then merges those four. 4 rounds of ~10 dependent LDS
// probes instead of rank-by-counting's 15 binary searches per entry (1.9 ms per config-5 round,
// slower than the 55-stage bitonic network that ignores the segments' order, 1.6 ms).
__global__ __launch_bounds__(256) void merge_path_kernel(MergeArgs A) {
  __shared__ Key ka[LMAX];
  __shared__ Key kb[LMAX];
  __shared__ int cnt_sh;
  if (gate_closed(A.gate)) return;   // (an enqueued-ahead window that will not be walked)
  const int task = blockIdx.x, tid = threadIdx.x;
  if (A.nt_dev && task >= *A.nt_dev) return;   // (representative lists: rows past the count)
  const int S = A.S;
  int P = 1;
  while (P < S) P <<= 1;
  const int n = P * KL;                          // <= LMAX (merge_variant)
  const Key inv = {DINF, 0xffffffffu, 0x7fffffff};
  if (tid == 0) cnt_sh = 0;
  for (int j = tid; j < n; j += 256) {
    Key k = inv;
    if (j < S * KL) {
      const SegEntry se = A.seg[(size_t)task * S * KL + j];
      k = {se.s, se.tb, se.id};
    }
    ka[j] = k;
  }
  // bound: the smallest last entry of a segment with more than KL feasible hosts (every thread
  // derives it: S loads, no barrier on its path)
  Key bound = inv;
  long long tot = 0;
  for (int g = 0; g < S; g++) {
    const int f = A.seg_feas[(size_t)task * S + g];
    tot += f;
    if (f > KL) {
      const SegEntry se = A.seg[((size_t)task * S + g) * KL + KL - 1];
      const Key k = {se.s, se.tb, se.id};
      if (kless(k, bound)) bound = k;
    }
  }
  __syncthreads();
  // (the two halves swap by pointer; the co-rank probes are then flat accesses to LDS, which
  // measured faster than indexing both halves by a round parity: 2.69 vs 3.04 ms per config-5
  // vbp best-fit round -- no global load is in flight during the rounds)
  Key* src = ka;
  Key* dst = kb;
  for (int len = KL; len < n; len <<= 1) {
    for (int o = tid * 4; o < n; o += 1024) {
      const int base = o & ~(2 * len - 1), i = o - base;
      const Key* a = src + base;
      const Key* b = a + len;
      // co-rank: x outputs of the first i come from a (ties: a first; keys are distinct anyway
      // except the invalid padding, which sorts last either way)
      int lo = max(0, i - len), hi = min(i, len);
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (!kless(b[i - mid - 1], a[mid])) lo = mid + 1;
        else hi = mid;
      }
      int x = lo, y = i - lo;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const bool ta = x < len && (y >= len || !kless(b[y], a[x]));
        dst[o + k] = ta ? a[x] : b[y];
        x += ta ? 1 : 0;
        y += ta ? 0 : 1;
      }
    }
    __syncthreads();
    Key* t = src; src = dst; dst = t;
  }
  // kept entries: valid and below the bound, the first cnt of the merged list
  int c = 0;
  for (int j = tid; j < n; j += 256) c += (src[j].id != 0x7fffffff) && kless(src[j], bound);
  if (c) atomicAdd(&cnt_sh, c);
  __syncthreads();
  const int cnt = cnt_sh;
  const bool complete = (bound.id == 0x7fffffff) && tot <= LMAX;
  Key bnd = bound;
  if (cnt == LMAX && kless(src[LMAX - 1], bnd)) bnd = src[LMAX - 1];
  const int nw = max(cnt, KL);
  // the kept hosts' zone and snapshot availability: every gather of the thread's (up to) four
  // entries issued before the first is used (one HBM latency, not four)
  constexpr int PO = LMAX / 256;
  Key kk[PO];
  int32_t zz[PO];
  double aa[PO][4];
#pragma unroll
  for (int u = 0; u < PO; u++) {
    const int j = tid + u * 256;
    const bool ok = j < cnt;
    kk[u] = inv;
    if (ok) kk[u] = src[j];                  // (a select of the two addresses would be flat)
    const int h = ok ? kk[u].id : 0;
    zz[u] = ok ? A.zone[h] : 0;
    aa[u][0] = ok ? A.avail[h] : 0.0;
    aa[u][1] = ok ? A.avail[(size_t)A.H + h] : 0.0;
    aa[u][2] = ok ? A.avail[2 * (size_t)A.H + h] : 0.0;
    aa[u][3] = ok ? A.avail[3 * (size_t)A.H + h] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < PO; u++) {
    const int j = tid + u * 256;
    if (j >= nw) continue;
    ListEntry e;
    e.s = kk[u].s; e.tb = kk[u].tb; e.id = kk[u].id; e.pad = 0; e.pad2 = 0.0;
    e.zone = zz[u];
    e.a[0] = aa[u][0]; e.a[1] = aa[u][1]; e.a[2] = aa[u][2]; e.a[3] = aa[u][3];
    A.L.e[(size_t)task * LMAX + j] = e;
    A.L.ids[(size_t)task * LMAX + j] = j < cnt ? kk[u].id : 0x7fffffff;
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

static int merge_variant(const MergeArgs& a) {
  const bool small = !a.bitonic;
  if (small && a.seg_feas != nullptr && a.SL == KL && a.S <= MERGE_SMALL_S) return 1;
  if (small && a.seg_feas == nullptr && (size_t)a.S * a.SL <= LMAX) return 2;
  if (small && a.seg_feas != nullptr && a.SL == KL && (size_t)a.S * KL <= LMAX) return 3;
  return 0;
}
const char* merge_kernel_name(const MergeArgs& a) {
  static const char* names[4] = {"merge_kernel", "merge_small_kernel", "merge_pkg_kernel",
                                 "merge_path_kernel"};
  return names[merge_variant(a)];
}
void launch_merge(const MergeArgs& a, hipStream_t st) {
  switch (merge_variant(a)) {
    case 1: PVT_LAUNCH(merge_small_kernel, dim3((a.nt + 3) / 4), dim3(256), 0, st, a); break;
    case 2: PVT_LAUNCH(merge_pkg_kernel, dim3(a.nt), dim3(256), 0, st, a); break;
    case 3: PVT_LAUNCH(merge_path_kernel, dim3(a.nt), dim3(256), 0, st, a); break;
    default: PVT_LAUNCH(merge_kernel, dim3(a.nt), dim3(256), 0, st, a);
  }
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
  PVT_LAUNCH(pack_kernel, dim3((a.nt + 3) / 4), dim3(256), 0, st, a);
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
  if (a.strict) PVT_LAUNCH(ordered_kernel<true>, grid, block, 0, st, a);
  else PVT_LAUNCH(ordered_kernel<false>, grid, block, 0, st, a);
}

// One wave per task: walk the group's sorted host order 64 positions at a time (perm and key
// loads coalesced, host state gathered), keep the first `depth` strictly feasible hosts.
__global__ __launch_bounds__(256) void perm_scan_kernel(PermArgs A) {
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int task = blockIdx.x * 4 + wave;
  if (task >= A.nt) return;
  const double* dp = A.dem + (size_t)task * 4;
  const double d0 = dp[0], d1 = dp[1], d2 = dp[2], d3 = dp[3];
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int cnt = 0, p_next = A.n;      // p_next: first sorted position after the last listed host
  int pb = 0;
  for (; pb < A.n && cnt < A.depth; pb += WAVE) {
    const int p = pb + lane;
    const bool ok = p < A.n;
    const int h = ok ? A.h_lo + A.perm[p] : 0;
    const double a0 = ok ? A.avail[h] : -DINF;
    const double a1 = ok ? A.avail[(size_t)A.H + h] : -DINF;
    const double a2 = ok ? A.avail[2 * (size_t)A.H + h] : -DINF;
    const double a3 = ok ? A.avail[3 * (size_t)A.H + h] : -DINF;
    const bool fit = ok && fits<true>(a0, a1, a2, a3, d0, d1, d2, d3);
    const uint64_t m = __ballot(fit);
    const int pos = cnt + __popcll(m & below);
    if (fit && pos < A.depth) {
      ListEntry e;
      e.s = __longlong_as_double((long long)A.skey[p]); e.tb = 0; e.id = h;
      e.zone = A.zone[h]; e.pad = 0; e.pad2 = 0.0;
      e.a[0] = a0; e.a[1] = a1; e.a[2] = a2; e.a[3] = a3;
      A.L.e[(size_t)task * LMAX + pos] = e;
      A.L.ids[(size_t)task * LMAX + pos] = h;
      if (pos == A.depth - 1) p_next = p + 1;      // one lane at most
    }
    cnt += __popcll(m);
  }
  p_next = (int)wave_min_u64((uint64_t)(uint32_t)p_next);
  if (lane < 4) reinterpret_cast<double*>(&A.L.t[task])[lane] = dp[lane];
  if (lane == 0) {
    TaskRec& r = A.L.t[task];
    const bool complete = pb >= A.n && cnt <= A.depth && !A.partial;   // all feasible listed
    r.cnt = cnt < A.depth ? cnt : A.depth;
    r.complete = complete;
    r.anc = A.anc ? A.anc[task] : 0;
    r.ord = A.ord[task];
    if (complete) {
      r.bs = DINF; r.btb = 0xffffffffu; r.bid = 0x7fffffff;
    } else if (p_next >= A.n) {     // the whole prefix is listed: the rest rank after it
      r.bs = A.partial ? A.rest_s : DINF; r.btb = A.partial ? 0u : 0xffffffffu;
      r.bid = A.partial ? 0 : 0x7fffffff;
    } else {
      r.bs = __longlong_as_double((long long)A.skey[p_next]); r.btb = 0;
      r.bid = A.h_lo + A.perm[p_next];
    }
  }
}

__global__ void zero_key_flags_kernel(const uint64_t* key, int n, uint8_t* flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] = key[i] == 0ull;
}
void launch_zero_key_flags(const double* key, int n, uint8_t* flags, hipStream_t st) {
  if (n > 0)
    PVT_LAUNCH(zero_key_flags_kernel, dim3((n + 255) / 256), dim3(256), 0, st,
                       reinterpret_cast<const uint64_t*>(key), n, flags);
}

void launch_perm_scan(const PermArgs& a, hipStream_t st) {
  PVT_LAUNCH(perm_scan_kernel, dim3((a.nt + 3) / 4), dim3(256), 0, st, a);
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
  PVT_LAUNCH(zone_tables_kernel, dim3((Z * Z + 255) / 256), dim3(256), 0, st, cost, bw, Z,
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
  const double c = A.csum[A.anchor * A.Z + z];
  const double bw = A.rtb ? A.rtb[h] : A.bsum[A.anchor * A.Z + z];
  const double df = A.decay ? (double)A.decay[h] : 1.0;
  A.key[h] = (c * df) / (r * bw);
}
void launch_key(const KeyArgs& a, hipStream_t st) {
  PVT_LAUNCH(key_kernel, dim3((a.h_hi - a.h_lo + 255) / 256), dim3(256), 0, st, a);
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
  PVT_LAUNCH(norm_keys_kernel, dim3((T + 255) / 256), dim3(256), 0, st, dem, T, idx, keys);
}

__global__ void group_keys_kernel(const int32_t* tg, const int32_t* idx, int T, uint32_t* keys) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T) return;
  keys[i] = (uint32_t)tg[idx ? idx[i] : i];
}
void launch_group_keys(const int32_t* task_group, const int32_t* idx, int T, uint32_t* keys,
                       hipStream_t st) {
  PVT_LAUNCH(group_keys_kernel, dim3((T + 255) / 256), dim3(256), 0, st, task_group, idx,
                     T, keys);
}

// a2, grouped rounds: the processing order as a group scatter + one LDS sort per group. The
// stable order by (group, key) of the two LSD radix passes equals the order by (group, key,
// task index), and within a group (key, index) is unique, so the scatter order inside a group
// does not matter: group_hist counts, the host scans, group_scatter places (key, index) pairs
// by atomics, group_sort bitonic-sorts each group's pairs in LDS.
// Blocks of 1024 tasks count (and place) in LDS first when G <= GAGG_MAX groups, so a
// group's global counter sees one atomic per block, not one per task (20 groups of 500 tasks
// serialised 26 us of same-address atomics).
__global__ __launch_bounds__(1024) void group_hist_kernel(const int32_t* tg, int T, int G, int32_t* cnt) {
  __shared__ int32_t loc[GAGG_MAX + 1];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool agg = G <= GAGG_MAX;
  if (agg) {
    for (int q = threadIdx.x; q <= G; q += blockDim.x) loc[q] = 0;
    __syncthreads();
  }
  if (i < T) {
    const int g = tg[i];
    const int b = (g >= 0 && g < G) ? g : G;   // G: out of range
    atomicAdd(agg ? &loc[b] : &cnt[b], 1);
  }
  if (agg) {
    __syncthreads();
    for (int q = threadIdx.x; q <= G; q += blockDim.x)
      if (loc[q]) atomicAdd(&cnt[q], loc[q]);
  }
}
// The group plan's inputs in one step: the group counts (cnt[G] counts out-of-range groups), the
// group anchors and the cost table written straight into the host's pinned staging buffer (one
// kernel instead of three DMA copies), and the groups' offsets in processing order plus scatter
// cursors (off[0..G], off[G+1..2G+1]) computed here instead of uploaded. One block.
__global__ __launch_bounds__(1024) void group_stage_kernel(const int32_t* cnt, int G,
                                                           const int32_t* ganc, const double* cost,
                                                           int nz2, int32_t* off, int32_t* hcnt,
                                                           int32_t* hgan, double* hcst) {
  __shared__ int32_t wsum[16];
  __shared__ int32_t carry;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int i = t; i <= G; i += 1024) hcnt[i] = cnt[i];
  for (int i = t; i < G; i += 1024) hgan[i] = ganc[i];
  for (int i = t; i < nz2; i += 1024) hcst[i] = cost[i];
  if (t == 0) carry = 0;
  __syncthreads();
  for (int g0 = 0; g0 < G; g0 += 1024) {
    const int g = g0 + t;
    const int v = g < G ? cnt[g] : 0;
    int x = v;                                  // inclusive scan within the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int pre = carry;
    for (int w = 0; w < wave; w++) pre += wsum[w];
    if (g < G) {
      off[g] = pre + x - v;
      off[G + 1 + g] = pre + x - v;
    }
    __syncthreads();
    if (t == 1023) carry = pre + x;
    __syncthreads();
  }
  if (t == 0) { off[G] = carry; off[2 * G + 1] = carry; }
  __threadfence_system();
}
void launch_group_stage(const int32_t* cnt, int G, const int32_t* ganc, const double* cost, int nz2,
                        int32_t* off, int32_t* hcnt, int32_t* hgan, double* hcst, hipStream_t st) {
  PVT_LAUNCH(group_stage_kernel, dim3(1), dim3(1024), 0, st, cnt, G, ganc, cost, nz2, off,
                     hcnt, hgan, hcst);
}

void launch_group_hist(const int32_t* tg, int T, int G, int32_t* cnt, hipStream_t st) {
  PVT_LAUNCH(group_hist_kernel, dim3((T + 1023) / 1024), dim3(1024), 0, st, tg, T, G, cnt);
}
__global__ __launch_bounds__(1024) void group_scatter_kernel(const int32_t* tg, const uint64_t* keys, int T,
                                                             int G, int32_t* cursor, uint64_t* skey,
                                                             int32_t* sidx) {
  __shared__ int32_t loc[GAGG_MAX];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int g = i < T ? tg[i] : -1;
  if (g >= G) g = -1;            // (out of range: the host rejects the round after its sync)
  if (G <= GAGG_MAX) {
    // rank within the block's share of the group, then one reservation per (block, group)
    for (int q = threadIdx.x; q < G; q += blockDim.x) loc[q] = 0;
    __syncthreads();
    const int r = g >= 0 ? atomicAdd(&loc[g], 1) : 0;
    __syncthreads();
    for (int q = threadIdx.x; q < G; q += blockDim.x)
      if (loc[q]) loc[q] = atomicAdd(&cursor[q], loc[q]);
    __syncthreads();
    if (g >= 0) {
      const int pos = loc[g] + r;
      skey[pos] = keys ? keys[i] : 0ull;
      sidx[pos] = i;
    }
  } else if (g >= 0) {
    const int pos = atomicAdd(&cursor[g], 1);
    skey[pos] = keys ? keys[i] : 0ull;
    sidx[pos] = i;
  }
}
void launch_group_scatter(const int32_t* tg, const uint64_t* keys, int T, int G, int32_t* cursor,
                          uint64_t* skey, int32_t* sidx, hipStream_t st) {
  PVT_LAUNCH(group_scatter_kernel, dim3((T + 1023) / 1024), dim3(1024), 0, st, tg, keys, T,
                     G, cursor, skey, sidx);
}
// The grouped order's preparation in two one-block launches (rounds of at most PREP_T_MAX
// tasks and GAGG_MAX groups; the config-5 round's seven launches -- placement fill, counter
// clear, group histogram, stage, sort keys, scatter, zone tables -- were each a few microseconds
// of launch latency on the host's critical path). order_count_kernel: the group counts in LDS
// and the pinned staging of counts / anchors / cost table -- all the host waits for before it
// plans the round. order_scatter_kernel, while the host plans: placement fill, zone tables, the
// groups' offsets, then the (key, task) pairs scattered by LDS cursors (their order inside a
// group is irrelevant: group_sort orders by (key, index)).
__device__ void order_count_body(const PrepArgs& A, int32_t* cnt) {
  const int t = threadIdx.x;
  const int T = A.T, G = A.G;
  for (int q = t; q <= G; q += 1024) cnt[q] = 0;
  __syncthreads();
  // (loads batched PB per thread so their latencies overlap: the block is alone on its CU)
  constexpr int PB = 16;
  for (int i0 = 0; i0 < T; i0 += 1024 * PB) {
    int gv[PB];
#pragma unroll
    for (int u = 0; u < PB; u++) {
      const int i = i0 + u * 1024 + t;
      gv[u] = i < T ? A.tg[i] : -2;
    }
    // a wave whose 64 tasks share one group (the trace lists an application's tasks together)
    // takes ONE atomic: 64 same-address LDS atomics serialise; mixed waves add lane by lane
#pragma unroll
    for (int u = 0; u < PB; u++) {
      const int q = gv[u] == -2 ? -1 : ((gv[u] >= 0 && gv[u] < G) ? gv[u] : G);   // G: out of range
      const int q0 = __builtin_amdgcn_readfirstlane(q);
      const uint64_t same = __ballot(q == q0);
      if (same == ~0ull) {
        if ((t & 63) == 0 && q0 >= 0) atomicAdd(&cnt[q0], 64);
      } else if (q >= 0) {
        atomicAdd(&cnt[q], 1);
      }
    }
  }
  __syncthreads();
  // counts to the host's stage and to off (the scatter kernel scans them there)
  for (int i = t; i <= G; i += 1024) { A.hcnt[i] = cnt[i]; A.off[i] = cnt[i]; }
  for (int i = t; i < G; i += 1024) A.hgan[i] = A.ganc[i];
  for (int i = t; i < A.nz2; i += 1024) A.hcst[i] = A.cost[i];
  __threadfence_system();
  if (A.hflag) {                              // every thread's staged words, then the flag
    __syncthreads();
    if (t == 0) {
      __hip_atomic_store(A.hflag, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
__global__ __launch_bounds__(1024) void order_count_kernel(PrepArgs A) {
  __shared__ int32_t cnt[GAGG_MAX + 1];
  order_count_body(A, cnt);
}

__global__ __launch_bounds__(1024) void order_scatter_kernel(PrepArgs A) {
  __shared__ int32_t cur[GAGG_MAX];
  __shared__ int32_t wsum[16];
  __shared__ int32_t carry;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int T = A.T, G = A.G;
  if (t == 0) carry = 0;
  if (A.placement)
    for (int i = t; i < T; i += 1024) A.placement[i] = -1;
  if (A.csum)
    for (int i = t; i < A.Z * A.Z; i += 1024) {
      const int a = i / A.Z, z = i - a * A.Z;
      A.csum[i] = A.cost[a * A.Z + z] + A.cost[z * A.Z + a];   // cost_aware.py:82,113
      A.bsum[i] = A.bw[a * A.Z + z] + A.bw[z * A.Z + a];       // (:79,111)
    }
  __syncthreads();
  for (int g0 = 0; g0 < G; g0 += 1024) {            // exclusive scan of the counts in off
    const int g = g0 + t;
    const int v = g < G ? A.off[g] : 0;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int pre = carry;
    for (int w = 0; w < wave; w++) pre += wsum[w];
    if (g < G) { A.off[g] = pre + x - v; cur[g] = pre + x - v; }
    __syncthreads();
    if (t == 1023) carry = pre + x;
    __syncthreads();
  }
  if (t == 0) A.off[G] = carry;
  constexpr int PS = 8;
  for (int i0 = 0; i0 < T; i0 += 1024 * PS) {
    int gv[PS];
    double dv[PS][4];
#pragma unroll
    for (int u = 0; u < PS; u++) {
      const int i = i0 + u * 1024 + t;
      gv[u] = i < T ? A.tg[i] : -1;
      if (A.sort_tasks && i < T) {
        dv[u][0] = A.dem[i]; dv[u][1] = A.dem[(size_t)T + i];
        dv[u][2] = A.dem[2 * (size_t)T + i]; dv[u][3] = A.dem[3 * (size_t)T + i];
      }
    }
#pragma unroll
    for (int u = 0; u < PS; u++) {
      const int i = i0 + u * 1024 + t;
      const int g = gv[u];
      if (i >= T || g < 0 || g >= G) continue;   // (the host rejects the round after its sync)
      uint64_t key = 0;
      if (A.sort_tasks) {
        const double n = __builtin_sqrt(norm2_seq(dv[u][0], dv[u][1], dv[u][2], dv[u][3]));
        key = ~(uint64_t)__double_as_longlong(n);       // descending norm (as norm_keys_kernel)
      }
      const int pos = atomicAdd(&cur[g], 1);
      A.skey[pos] = key;
      A.sidx[pos] = i;
    }
  }
}
void launch_order_prep(const PrepArgs& a, hipStream_t st, hipEvent_t counted, bool scatter) {
  PVT_LAUNCH(order_count_kernel, dim3(1), dim3(1024), 0, st, a);
  if (counted) (void)hipEventRecord(counted, st);
  if (scatter) PVT_LAUNCH(order_scatter_kernel, dim3(1), dim3(1024), 0, st, a);
}

// Sorts the n <= GSORT_MAX (key, task) pairs in LDS k / v by (key, task) ascending; on return
// (after a barrier) v[0, n) holds the tasks in order. Block of 1024 threads, every one calling.
__device__ void lds_sort_pairs(uint64_t* k, int32_t* v, int n) {
  const int tid = threadIdx.x;
  if (n <= 128) {
    // rank by counting: the keys (sort key, task index) are distinct, so an element's place is
    // the number of elements below it -- every thread scans the group's keys in LDS (broadcast
    // reads). (Quadratic: measured 57 us for a group of ~1000 at config 5.)
    int r = 0;
    int32_t vi = 0;
    if (tid < n) {
      const uint64_t ki = k[tid];
      vi = v[tid];
      for (int j = 0; j < n; j++) {
        const uint64_t kj = k[j];
        r += (kj < ki || (kj == ki && v[j] < vi)) ? 1 : 0;
      }
    }
    __syncthreads();
    if (tid < n) v[r] = vi;
    __syncthreads();
    return;
  }
  // Runs of 64 sorted in registers by a bitonic network (element i = m * 1024 + tid; the stages
  // pair lanes of one wave: shuffles, no barrier), every run ascending; then the runs merged
  // pairwise in LDS, each element to (its rank in its own run) + (the number of the other run's
  // elements below it: a binary search) -- log2(P / 64) rounds of one barrier each, where the
  // bitonic network's stages of size > 64 took 24 stages at P = 512 (6 of them through LDS).
  // (Padding pairs are (~0, 2^30 + i): distinct, after every real pair.)
  int P = 2;
  while (P < n) P <<= 1;
  constexpr int EMAX = GSORT_MAX / 1024;
  const int E = (P + 1023) >> 10;
  uint64_t rk[EMAX];
  int32_t rv[EMAX];
#pragma unroll
  for (int m = 0; m < EMAX; m++) {
    const int i = m * 1024 + tid;
    rk[m] = (m < E && i < n) ? k[i] : ~0ull;
    rv[m] = (m < E && i < n) ? v[i] : (0x40000000 + i);
  }
  __syncthreads();
  const int P64 = min(P, 64);
  for (int size = 2; size <= P64; size <<= 1) {
    // (waves whose elements are all padding, i >= P, only ever pair with padding: they skip)
    for (int stride = size >> 1; stride > 0 && (tid & ~63) < P; stride >>= 1) {
#pragma unroll
      for (int m = 0; m < EMAX; m++) {
        if (m >= E) continue;
        const int i = m * 1024 + tid;
        const uint32_t klo = (uint32_t)rk[m], khi = (uint32_t)(rk[m] >> 32);
        const uint64_t pk = ((uint64_t)(uint32_t)__shfl_xor((int)khi, stride) << 32) |
                            (uint32_t)__shfl_xor((int)klo, stride);
        const int32_t pv = __shfl_xor(rv[m], stride);
        const bool up = size == P64 || (i & size) == 0, low = (i & stride) == 0;
        const uint64_t kl = low ? rk[m] : pk, kh = low ? pk : rk[m];
        const int32_t vl = low ? rv[m] : pv, vh = low ? pv : rv[m];
        const bool gt = kl > kh || (kl == kh && vl > vh);
        if (gt == up) { rk[m] = pk; rv[m] = pv; }
      }
    }
  }
  if (P <= 64) {
#pragma unroll
    for (int m = 0; m < EMAX; m++) {
      const int i = m * 1024 + tid;
      if (m < E && i < n) v[i] = rv[m];
    }
    __syncthreads();
    return;
  }
  __shared__ uint64_t k2[GSORT_MAX];
  __shared__ int32_t v2[GSORT_MAX];
#pragma unroll
  for (int m = 0; m < EMAX; m++) {
    const int i = m * 1024 + tid;
    if (m < E && i < P) { k[i] = rk[m]; v[i] = rv[m]; }
  }
  __syncthreads();
  uint64_t* ka = k;
  int32_t* va = v;
  uint64_t* kb = k2;
  int32_t* vb = v2;
  for (int w = 64; w < P; w <<= 1) {
#pragma unroll
    for (int m = 0; m < EMAX; m++) {
      const int i = m * 1024 + tid;
      if (m >= E || i >= P) continue;
      const uint64_t key = ka[i];
      const int32_t val = va[i];
      const int base = i & ~(2 * w - 1), off = i - base;
      const bool left = off < w;
      const int ob = left ? base + w : base;          // the other run
      int lo = 0, len = w;                            // its elements below (key, val)
      while (len > 0) {
        const int half = len >> 1, mid = lo + half;
        const uint64_t km = ka[ob + mid];
        const bool below = km < key || (km == key && va[ob + mid] < val);
        lo = below ? mid + 1 : lo;
        len = below ? len - half - 1 : half;
      }
      const int dest = base + (left ? off : off - w) + lo;
      kb[dest] = key;
      vb[dest] = val;
    }
    __syncthreads();
    uint64_t* tk = ka; ka = kb; kb = tk;
    int32_t* tv = va; va = vb; vb = tv;
  }
  if (va != v) {
    for (int i = tid; i < n; i += 1024) v[i] = va[i];
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void group_sort_kernel(const int32_t* off, const uint64_t* skey,
                                                          const int32_t* sidx, int32_t* ord) {
  __shared__ uint64_t k[GSORT_MAX];
  __shared__ int32_t v[GSORT_MAX];
  const int a = off[blockIdx.x], n = off[blockIdx.x + 1] - a, tid = threadIdx.x;
  if (n <= 0 || n > GSORT_MAX) return;   // (larger groups: the host sorts with radix passes)
  for (int i = tid; i < n; i += blockDim.x) { k[i] = skey[a + i]; v[i] = sidx[a + i]; }
  __syncthreads();
  lds_sort_pairs(k, v, n);
  for (int i = tid; i < n; i += blockDim.x) ord[a + i] = v[i];
}

// A block of the grouped order's launch that prebuilds the zero-cost window of zone j for the
// round's first cost_aware best-fit epoch (ZoneWindows, pvt_kernels.h): the zero-cost masks
// amask[a] = {z : csum[a][z] == 0} from the cost table itself (block g = 0 of the same launch
// writes csum), the components by closure of that relation (csum is symmetric), and, when j is
// its component's lowest zone and some group's anchor lies in the component, the first ZW_M
// hosts of U = the union of those anchors' amask, compacted in LDS (the sort arrays, unused by
// this block) and written with their zones and snapshot capacities.
__device__ void zone_window_block(const PrepArgs& A, const GatherOut& O, int j, int32_t* lds) {
  __shared__ uint32_t am[ZMAX], reach[ZMAX], gm_s;
  __shared__ int32_t cnt[2][16], nw_s;
  const int tid = threadIdx.x, Z = A.Z;
  ZoneWindows* W = O.zwin;
  if (tid < ZMAX) am[tid] = 0;
  if (tid == 0) { gm_s = 0; nw_s = 0; }
  __syncthreads();
  for (int i = tid; i < Z * Z; i += 1024) {
    const int a = i / Z, z = i - a * Z;
    if (A.cost[a * Z + z] + A.cost[z * Z + a] == 0.0) atomicOr(&am[a], 1u << z);   // cost_aware.py:82
  }
  for (int g = tid; g < A.G; g += 1024) {
    const int a = A.ganc[g];
    if (a >= 0 && a < Z) atomicOr(&gm_s, 1u << a);
  }
  __syncthreads();
  if (tid < Z) reach[tid] = am[tid] | (1u << tid);
  __syncthreads();
  for (int it = 0; it < 5; it++) {            // paths of up to 2^5 >= ZMAX zones
    uint32_t r = 0;
    if (tid < Z) {
      r = reach[tid];
      for (uint32_t m = r; m; m &= m - 1) r |= reach[__builtin_ctz(m)];
    }
    __syncthreads();
    if (tid < Z) reach[tid] = r;
    __syncthreads();
  }
  const uint32_t comp = reach[j];
  uint32_t U = 0;
  if ((comp & ((1u << j) - 1u)) == 0)         // j: the component's lowest zone
    for (uint32_t m = comp & gm_s; m; m &= m - 1) U |= am[__builtin_ctz(m)];
  if (tid == 0) W->U[j] = U;
  if (U == 0) return;
  int32_t* wid = lds;
  int32_t* wz = lds + ZW_M;
  compact_zone_window_t<ZW_M, 1024, 2>(O.zone, Z, U, 0, O.H, wid, wz, cnt, &nw_s);
  const int n = nw_s;
  ZoneWindow& w = W->w[j];
  bool bad = false;
  for (int p = tid; p < n; p += 1024) {
    const int h = wid[p];
    w.id[p] = h;
    w.z[p] = wz[p];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const double x = O.avail[(size_t)r * O.H + h];
      bad |= !(__builtin_fabs(x) <= 0x1p500);
      w.a[r][p] = x;
    }
  }
  bad = __syncthreads_or(bad);
  if (tid == 0) { w.n = n; w.bad = bad ? 1 : 0; }
}

#ifdef PVT_STAMPS
__device__ __forceinline__ uint64_t gstamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define GSTAMP(k) do { if (g == 0 && tid == 0 && O.stamps) { const uint64_t t_ = gstamp(); gph[k] = t_ - gtl; gtl = t_; } } while (0)
#else
#define GSTAMP(k) do {} while (0)
#endif

// The grouped order of a round with few groups (G <= GCOMPACT_MAX, after order_count_kernel):
// block g scans every task's group (T reads from L2, G of them in all), collects its own
// (sort key, task) pairs in LDS by wave-aggregated cursors, fills their placement with -1,
// sorts them (lds_sort_pairs) and writes the gathered rows at its group's offset (the counts
// of the groups before it): processing order, caller order, demand rows, anchors, groups.
// Replaces order_scatter + group_sort + gather_tasks (three launches, ~35 us per config-5
// round). Block 0 is order_count_kernel (the counts and the host's stage, while the groups'
// blocks run: each group's block counts the tasks of the groups before it itself, in its scan);
// group g is block g + 1, which also writes the zone tables for g = 0. A group over GSORT_MAX
// tasks only fills its placement: the host redoes the order with radix passes.
__global__ __launch_bounds__(1024) void group_sort_gather_kernel(PrepArgs A, GatherOut O) {
  __shared__ uint64_t k[GSORT_MAX];
  __shared__ int32_t v[GSORT_MAX];
  __shared__ int32_t fill, below_s;
  static_assert(sizeof(k) >= sizeof(int32_t) * (GCOMPACT_MAX + 1), "count table in k");
  if (blockIdx.x == 0) {
    order_count_body(A, reinterpret_cast<int32_t*>(k));
    return;
  }
  const int g = blockIdx.x - 1, tid = threadIdx.x, lane = tid & 63;
  const int T = A.T;
#ifdef PVT_STAMPS
  uint64_t gph[4] = {0, 0, 0, 0}, gtl = 0;
  if (g == 0 && tid == 0) gtl = gstamp();
#endif
  const int nmin = O.hmin ? ZW_MIN_PARTS : 0;
  if (g >= A.G + nmin) {                      // the first epoch's zero-cost windows
    zone_window_block(A, O, g - A.G - nmin, reinterpret_cast<int32_t*>(k));
    return;
  }
  if (g >= A.G) {
    // blocks past the groups' blocks: the frontier walk's host minima, one of the ZW_MIN_PARTS partials
    // per block (the walk reduces them all, so the partition is free: four hosts per thread per
    // pass for loads in flight; a quarter as many blocks measured ~26 us against 8.8)
    __shared__ double red[16][4];
    const int pb = g - A.G, wave = tid >> 6;
    double m[4] = {DINF, DINF, DINF, DINF};
    constexpr int STEP = ZW_MIN_PARTS * 1024;
    for (int h0 = pb * 1024 + tid; h0 < O.H; h0 += 4 * STEP) {
      double x[4][4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int h = h0 + j * STEP;
#pragma unroll
        for (int r = 0; r < 4; r++) x[j][r] = h < O.H ? O.avail[(size_t)r * O.H + h] : DINF;
      }
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int r = 0; r < 4; r++) m[r] = fmin(m[r], x[j][r]);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      for (int off = 32; off > 0; off >>= 1) m[r] = fmin(m[r], __shfl_xor(m[r], off));
      if (lane == 0) red[wave][r] = m[r];
    }
    __syncthreads();
    if (tid < 4) {
      double x = red[0][tid];
      for (int w = 1; w < 16; w++) x = fmin(x, red[w][tid]);
      O.hmin[pb * 4 + tid] = x;
    }
    return;
  }
  if (g == 0 && A.csum)
    for (int i = tid; i < A.Z * A.Z; i += 1024) {
      const int a = i / A.Z, z = i - a * A.Z;
      A.csum[i] = A.cost[a * A.Z + z] + A.cost[z * A.Z + a];   // cost_aware.py:82,113
      A.bsum[i] = A.bw[a * A.Z + z] + A.bw[z * A.Z + a];       // (:79,111)
    }
  if (tid == 0) { fill = 0; below_s = 0; }
  __syncthreads();
  GSTAMP(0);
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  constexpr int PB = 8;
  for (int i0 = 0; i0 < T; i0 += 1024 * PB) {
    // the groups of the batch's tasks (keys come after the collection: only the group's own
    // tasks' demands are read and only they take the norm -- computed in the scan, every wave
    // ran the fp64 norm for every batch whenever one lane matched: 21k of the kernel's 54k cycles)
    int gv[PB];
#pragma unroll
    for (int u = 0; u < PB; u++) {
      const int i = i0 + u * 1024 + tid;
      gv[u] = i < T ? A.tg[i] : -1;
    }
    // the wave's matches of the whole batch take ONE cursor add (an LDS atomic and its return
    // per 1024 tasks serialised the 16 waves: 24k cycles for the scan at config 5)
    uint64_t bal[PB];
    int tot = 0, lt = 0;                      // (lt: tasks of the groups before g -- its offset)
#pragma unroll
    for (int u = 0; u < PB; u++) {
      const int i = i0 + u * 1024 + tid;
      const bool mine = gv[u] == g;
      if (mine && A.placement) A.placement[i] = -1;
      bal[u] = __ballot(mine);
      tot += __popcll(bal[u]);
      lt += __popcll(__ballot(gv[u] >= 0 && gv[u] < g));
    }
    if (lane == 0 && lt) atomicAdd(&below_s, lt);
    if (tot == 0) continue;
    int b = 0;
    if (lane == 0) b = atomicAdd(&fill, tot);
    b = __shfl(b, 0);
    if (b + tot > GSORT_MAX) continue;        // (too large to sort here: only counted)
#pragma unroll
    for (int u = 0; u < PB; u++) {
      if (gv[u] == g) v[b + __popcll(bal[u] & below)] = i0 + u * 1024 + tid;
      b += __popcll(bal[u]);
    }
  }
  __syncthreads();
  const int n = fill;
  if (n > GSORT_MAX || n <= 0) return;
  for (int q = tid; q < n; q += 1024) {       // the collected tasks' sort keys
    uint64_t key = 0;
    if (A.sort_tasks) {
      const int i = v[q];
      const double nn = __builtin_sqrt(norm2_seq(A.dem[i], A.dem[(size_t)T + i],
                                                 A.dem[2 * (size_t)T + i], A.dem[3 * (size_t)T + i]));
      key = ~(uint64_t)__double_as_longlong(nn);   // descending norm (as norm_keys_kernel)
    }
    k[q] = key;
  }
  __syncthreads();
  GSTAMP(1);
  lds_sort_pairs(k, v, n);
  GSTAMP(2);
  const int a = below_s;
  const int32_t anc = A.ganc[g];
  for (int i = tid; i < n; i += 1024) {
    const int p = a + i, t = v[i];
    O.ord[p] = t;
    if (O.order_out) O.order_out[p] = t;
    double* o = O.dem_ord + (size_t)p * 4;
    o[0] = A.dem[t]; o[1] = A.dem[(size_t)T + t]; o[2] = A.dem[2 * (size_t)T + t]; o[3] = A.dem[3 * (size_t)T + t];
    O.anc_ord[p] = anc;
    O.grp_ord[p] = g;
  }
#ifdef PVT_STAMPS
  __syncthreads();
  GSTAMP(3);
  if (g == 0 && tid == 0 && O.stamps)
    for (int q = 0; q < 4; q++) atomicAdd((unsigned long long*)&O.stamps[16 + q], (unsigned long long)gph[q]);
#endif
}
void launch_group_sort_gather(const PrepArgs& a, const GatherOut& o, hipStream_t st) {
  const int extra = (o.hmin ? ZW_MIN_PARTS : 0) + (o.zwin ? a.Z : 0);
  PVT_LAUNCH(group_sort_gather_kernel, dim3(1 + a.G + extra), dim3(1024), 0, st, a, o);
}
void launch_group_sort(const int32_t* off, int G, const uint64_t* skey, const int32_t* sidx,
                       int32_t* ord, hipStream_t st) {
  // (1024 threads, the block's element layout above assumes it)
  PVT_LAUNCH(group_sort_kernel, dim3(G), dim3(1024), 0, st, off, skey, sidx, ord);
}

// pvt_restore_hosts: the listed hosts' four capacities from the pristine snapshot.
__global__ __launch_bounds__(256) void restore_hosts_kernel(double* avail, const double* avail0, int H,
                                                            const int32_t* hosts, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int h = hosts[i];
  if (h < 0 || h >= H) return;
#pragma unroll
  for (int r = 0; r < 4; r++) avail[(size_t)r * H + h] = avail0[(size_t)r * H + h];
}
void launch_restore_hosts(double* avail, const double* avail0, int H, const int32_t* hosts, int n,
                          hipStream_t st) {
  if (n > 0) PVT_LAUNCH(restore_hosts_kernel, dim3((n + 255) / 256), dim3(256), 0, st, avail, avail0, H, hosts, n);
}

// Small host tables to the device through their mapped pinned pages, as a kernel on the stream:
// a hipMemcpyAsync from pinned memory goes through the copy engine, and the next kernel on the
// stream then started ~20 us after the copy was queued (an idle GPU in between, default line).
__global__ __launch_bounds__(256) void upload_kernel(const int4* src, int4* dst, int n16) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}
void launch_upload(const void* src_mapped, void* dst, size_t bytes, hipStream_t st) {
  const int n16 = (int)((bytes + 15) / 16);
  if (n16 <= 0) return;
  const int blocks = std::min(64, (n16 + 255) / 256);
  PVT_LAUNCH(upload_kernel, dim3(blocks), dim3(256), 0, st,
                     reinterpret_cast<const int4*>(src_mapped), reinterpret_cast<int4*>(dst), n16);
}

__global__ void iota_kernel(int32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = i;
}
void launch_iota(int32_t* out, int n, hipStream_t st) {
  PVT_LAUNCH(iota_kernel, dim3((n + 255) / 256), dim3(256), 0, st, out, n);
}

__global__ void gather_tasks_kernel(const double* dem, const int32_t* ord, const int32_t* tg,
                                    const int32_t* ga, int T, double* dem_ord, int32_t* anc_ord,
                                    int32_t* grp_ord, int G, int32_t* order_out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= T) return;
  const int t = ord[p];
  if (order_out) order_out[p] = t;        // (the caller's order: no separate D2D copy)
  double* o = dem_ord + (size_t)p * 4;
  o[0] = dem[t]; o[1] = dem[(size_t)T + t]; o[2] = dem[2 * (size_t)T + t]; o[3] = dem[3 * (size_t)T + t];
  // (a group id out of range reads no anchor: the host rejects such a round after its sync)
  if (anc_ord) anc_ord[p] = (tg && ga && tg[t] >= 0 && tg[t] < G) ? ga[tg[t]] : 0;
  if (grp_ord) grp_ord[p] = tg ? tg[t] : 0;
}
void launch_gather_tasks(const double* dem, const int32_t* ord, const int32_t* task_group,
                         const int32_t* group_anchor, int T, double* dem_ord, int32_t* anc_ord,
                         int32_t* grp_ord, hipStream_t st, int G, int32_t* order_out) {
  PVT_LAUNCH(gather_tasks_kernel, dim3((T + 255) / 256), dim3(256), 0, st, dem, ord,
                     task_group, group_anchor, T, dem_ord, anc_ord, grp_ord, G, order_out);
}

}  // namespace pvt
