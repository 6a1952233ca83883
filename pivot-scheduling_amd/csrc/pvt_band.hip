// pvt_band.hip — vbp best-fit candidate lists by a memory band over hosts sorted once per round.
//
// vbp best-fit (reference scheduler/vbp.py:39-50) takes, per task in sorted order, the strictly
// fitting host of least ||avail - d||2 (ties: host-id string), and commits. Every term of the
// squared norm is >= 0, so a host can only enter a task's top-KL list if |a1 - d1| is within the
// radius of the list's current last entry (the score kernel's memory prefilter, vbp_rad), and it
// must fit strictly: a1 > d1. Host memory spreads over [0, 131072) while the best residuals are a
// few hundred, so the prefilter rejects nearly every host -- but the streaming score kernel still
// loads all of them for every task.
//
// Here the hosts are sorted by their snapshot memory ONCE per round (hipCUB radix sort of the
// orderable bits of avail[1], then a gather of the snapshot SoA into sorted order). A host nobody
// has committed to since keeps its snapshot state, so for it the sorted copy is exact; per task
// and list segment a wave then finds the first position with a1 >= d1 (a 64-ary search: four
// dependent loads) and scans upward until the chunk's smallest a1 leaves the radius -- the same
// exact list the streaming kernel builds, from ~10^3 hosts instead of 10^6. Hosts committed to
// since the snapshot ("touched", flagged and listed by touch_update_kernel after each walk) are
// skipped in the sorted copy and scanned from the touched list with their live capacities. The
// output is the streaming kernel's segment format (exact top-KL of a host subset + feasible
// count), so merge and commit walk are unchanged; hosts a concurrent walk is committing to are
// inherited by the next walk as touched, exactly as with the streaming kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"
#include "pvt_kernels.h"
#include "pvt_list.h"

namespace pvt {

__device__ __forceinline__ uint64_t order_bits(double v) {   // total order of doubles
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// The sort keys, and each host's snapshot row (4 capacities and its tiebreak rank) as one
// 64-byte record, so the gather after the sort reads one line per host (from the SoA rows it read
// five lines per host: 640 MB per config-5 round for 36 MB of data).
__global__ __launch_bounds__(256) void band_keys_kernel(const double* avail, const uint32_t* tb,
                                                        int H, int lo, int n, uint64_t* key,
                                                        int32_t* idx, BandRec* rec) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const size_t h = (size_t)lo + p;
  const double a0 = avail[h], a1 = avail[(size_t)H + h];
  const double a2 = avail[2 * (size_t)H + h], a3 = avail[3 * (size_t)H + h];
  key[p] = order_bits(a1);
  idx[p] = lo + p;
  double4* r = reinterpret_cast<double4*>(&rec[p]);
  r[0] = make_double4(a0, a1, a2, a3);
  rec[p].tb = tb ? tb[h] : 0u;
}

__global__ void band_gather_kernel(const BandRec* rec, int lo, int n, const int32_t* sid,
                                   double* sa, uint32_t* stb, int32_t* pos) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int h = sid[p];
  pos[h] = p;                              // (host -> sorted position, for the touched flags)
  const BandRec& x = rec[h - lo];
  const double4 a = *reinterpret_cast<const double4*>(&x);
  sa[p] = a.x;
  sa[(size_t)n + p] = a.y;
  sa[2 * (size_t)n + p] = a.z;
  sa[3 * (size_t)n + p] = a.w;
  stb[p] = x.tb;
}

// After a walk: the hosts it committed to (own_ids, count status[1]) that were not touched yet
// are flagged and appended to the touched list, in own_ids order (one block, ballot compaction).
__global__ __launch_bounds__(1024) void touch_update_kernel(const int32_t* own, const int32_t* status,
                                                            uint8_t* flags, int32_t* tlist,
                                                            int32_t* tcount, const int32_t* hpos,
                                                            int lo, int hi, uint8_t* ptouch) {
  __shared__ int32_t wcnt[16];
  __shared__ int32_t base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = status[1];
  if (tid == 0) base = *tcount;
  __syncthreads();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int i = c0 + tid;
    const int32_t h = i < n ? own[i] : -1;
    const bool add = h >= 0 && flags[h] == 0;
    const uint64_t m = __ballot(add);
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int pos = base + __popcll(m & below);
    for (int w = 0; w < wave; w++) pos += wcnt[w];
    if (add) {
      flags[h] = 1;
      if (h >= lo && h < hi) ptouch[hpos[h]] = 1;   // (the sorted copy covers [lo, hi))
      tlist[pos] = h;
    }
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int w = 0; w < 16; w++) t += wcnt[w];
      base += t;
    }
    __syncthreads();
  }
  if (tid == 0) *tcount = base;
}

// First sorted position whose key is >= k (a 64-ary search: each step one probe per lane).
__device__ __forceinline__ int band_lower_bound(const uint64_t* key, int n, uint64_t k) {
  const int lane = lane_id();
  int lo = 0, hi = n;
  while (hi - lo > WAVE) {
    const int step = (hi - lo + WAVE - 1) / WAVE;
    const int p = lo + lane * step;
    const bool ge = p < hi && key[p] >= k;
    const uint64_t m = __ballot(ge);
    if (m & 1ull) return lo;
    // the first probe at or past k (none: one past the last probe inside [lo, hi)); the answer
    // lies after the probe before it and at or before it
    const int L = m ? __builtin_ctzll(m) : (hi - lo - 1) / step + 1;
    const int nlo = lo + (L - 1) * step + 1;
    hi = min(hi, lo + L * step);
    lo = nlo;
  }
  const int p = lo + lane;
  const uint64_t m = __ballot(p < hi && key[p] >= k);
  return m ? lo + __builtin_ctzll(m) : hi;
}

// Diagnostic invariant checks (PVT_BAND_CHECK builds only; never the shipped library). A
// finished segment list must be a prefix of filled entries, strictly ascending in
// (score, tiebreak:id), with distinct ids; every entry of an untouched host (scored on the sorted
// snapshot) a strict fit whose score is its exact residual norm; and complete: the untouched
// strictly fitting hosts of the segment's chunks with a key at or below the list's last (all of
// them, if the list is not full) are exactly its untouched entries. (Touched hosts are scored on
// live capacities that a concurrent walk may still be committing to -- the next walk inherits
// and rescores them -- so they are not re-checked here.)
#ifdef PVT_BAND_CHECK
__device__ void band_check(const BandArgs& A, int t, int seg, double ls, uint32_t lt, int32_t li,
                           double d0, double d1, double d2, double d3) {
  const int lane = lane_id();
  const bool f = li != 0x7fffffff;
  const uint64_t fm = __ballot(f);
  const int filled = __popcll(fm);
  const bool prefix = fm == (filled == 64 ? ~0ull : ((1ull << filled) - 1ull));
  const uint64_t k1 = (uint64_t)__double_as_longlong(ls), k2 = ((uint64_t)lt << 32) | (uint32_t)li;
  const uint64_t p1 = (uint64_t)__shfl_up((long long)k1, 1), p2 = (uint64_t)__shfl_up((long long)k2, 1);
  const bool asc = !f || lane == 0 || p1 < k1 || (p1 == k1 && p2 < k2);
  int dup = 0;
  for (int L = 0; L < filled; L++) dup += (f && L != lane && readlane_i(li, L) == li) ? 1 : 0;
  // the entry's sorted position (untouched hosts come from the sorted copy), -1: touched
  int pos = -1;
  if (f && li >= A.lo && li < A.hi && !A.touched[li])
    for (int p = 0; p < A.n; p++)
      if (A.sid[p] == li) { pos = p; break; }
  bool exact = true;
  if (pos >= 0) {
    const double a0 = A.sa[pos], a1 = A.sa[(size_t)A.n + pos];
    const double a2 = A.sa[2 * (size_t)A.n + pos], a3 = A.sa[3 * (size_t)A.n + pos];
    const bool fit = fits<true>(a0, a1, a2, a3, d0, d1, d2, d3);
    const double sc = __builtin_sqrt(norm2_seq(a0 - d0, a1 - d1, a2 - d2, a3 - d3));
    exact = fit && __double_as_longlong(sc) == __double_as_longlong(ls) && A.stb[pos] == lt;
  }
  const int n_untouched = __popcll(__ballot(pos >= 0));
  // completeness over the segment's chunks (c % S == seg) of the sorted snapshot
  const uint64_t lk1 = readlane_u64(k1, KL - 1), lk2 = readlane_u64(k2, KL - 1);
  int below = 0;
  for (int c = seg; c * WAVE < A.n; c += A.S) {
    const int p = c * WAVE + lane;
    if (p >= A.n || A.ptouched[p]) continue;
    const double a0 = A.sa[p], a1 = A.sa[(size_t)A.n + p];
    const double a2 = A.sa[2 * (size_t)A.n + p], a3 = A.sa[3 * (size_t)A.n + p];
    if (!fits<true>(a0, a1, a2, a3, d0, d1, d2, d3)) continue;
    const uint64_t c1 = (uint64_t)__double_as_longlong(__builtin_sqrt(norm2_seq(a0 - d0, a1 - d1, a2 - d2, a3 - d3)));
    const uint64_t c2 = ((uint64_t)A.stb[p] << 32) | (uint32_t)A.sid[p];
    below += (filled < KL || c1 < lk1 || (c1 == lk1 && c2 <= lk2)) ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) below += __shfl_xor(below, off);
  const bool complete = below == n_untouched;
  const uint64_t bad_asc = __ballot(!asc), bad_dup = __ballot(dup != 0), bad_ex = __ballot(!exact);
  if (lane == 0 && (!prefix || bad_asc || bad_dup || bad_ex || !complete))
    printf("band_check t=%d seg=%d filled=%d prefix=%d asc=%llx dup=%llx exact=%llx untouched=%d "
           "in_segment=%d\n", t, seg, filled, (int)prefix, (unsigned long long)bad_asc,
           (unsigned long long)bad_dup, (unsigned long long)bad_ex, n_untouched, below);
}
#endif

// One 64-host block of candidates (lane = host) for a band list: prefilter, strict fit, exact
// score, merge into the wave-held list (ls, lt, li) and refresh its bound (ts, tt, ti, lim, rd).
struct BandList {
  double ls = DINF;
  uint32_t lt = 0xffffffffu;
  int32_t li = 0x7fffffff;
  double ts = DINF, lim = DINF, rd = DINF;
  uint32_t tt = 0xffffffffu;
  int32_t ti = 0x7fffffff;
  double d0, d1, d2, d3;
  uint64_t *m1, *m2;

  __device__ __forceinline__ void consider(bool ok, double a0, double a1, double a2, double a3,
                                           uint32_t tbh, int32_t h) {
    const bool pre = ok && (__builtin_fabs(a1 - d1) <= rd);
    if (__ballot(pre) == 0) return;
    const bool fit = pre && fits<true>(a0, a1, a2, a3, d0, d1, d2, d3);
    const double s2 = norm2_seq(a0 - d0, a1 - d1, a2 - d2, a3 - d3);
    const bool pass = fit && (s2 <= lim);
    if (__ballot(pass) == 0) return;
    const double sc = pass ? __builtin_sqrt(s2) : DINF;
    const uint64_t tk1 = (uint64_t)__double_as_longlong(ts);
    const uint64_t tk2 = ((uint64_t)tt << 32) | (uint32_t)ti;
    const uint64_t ck1 = (uint64_t)__double_as_longlong(sc);
    const uint64_t ck2 = ((uint64_t)tbh << 32) | (uint32_t)h;
    const uint64_t pm = __ballot(pass && (ck1 < tk1 || (ck1 == tk1 && ck2 < tk2)));
    if (pm) {
      list_merge(ls, lt, li, sc, tbh, h, pm, m1, m2);
      ts = readlane_d(ls, KL - 1);
      tt = readlane_u(lt, KL - 1);
      ti = readlane_i(li, KL - 1);
      lim = vbp_lim(ts);
      rd = vbp_rad(ts);
    }
  }
};

// The sorted snapshot (untouched hosts): segment `seg`'s chunks from the lower bound upward,
// the next chunk's loads in flight while one is considered, until the chunk's smallest memory
// leaves the radius.
#ifdef PVT_BAND_HELPER
__device__ __noinline__
#else
__device__ __forceinline__
#endif
void band_scan_sorted(const BandArgs& A, int seg, BandList& B) {
  const int lane = lane_id();
  const int n = A.n;
  const int lb = band_lower_bound(A.key, n, order_bits(B.d1));
  const int c0 = lb >> 6;
  int c = c0 + ((seg - c0 % A.S) + A.S) % A.S;
  const int nch = (n + WAVE - 1) / WAVE;
  double n0 = 0, n1 = 0, n2 = 0, n3 = 0;
  uint32_t ntb = 0;
  int32_t nid = 0;
  uint8_t npt = 0;
  auto fetch = [&](int cc) {
    const int p = min(cc * WAVE + lane, n - 1);
    n0 = A.sa[p]; n1 = A.sa[(size_t)n + p]; n2 = A.sa[2 * (size_t)n + p]; n3 = A.sa[3 * (size_t)n + p];
    ntb = A.stb[p];
    nid = A.sid[p];
    npt = A.ptouched[p];
  };
  if (c < nch) fetch(c);
  for (; c < nch; c += A.S) {
    const double a0 = n0, a1 = n1, a2 = n2, a3 = n3;
    const uint32_t tbh = ntb;
    const int32_t h = nid;
    const uint8_t ntc = npt;
    if (c + A.S < nch) fetch(c + A.S);
    const int p = c * WAVE + lane;
    // the chunk's smallest memory is lane 0's (or its first position at or after lb): once it
    // is beyond the radius, so is every later chunk's -- the segment's list is final
    if (readlane_d(a1, 0) - B.d1 > B.rd) break;
    const bool ok = p < n && p >= lb && ntc == 0;   // (position flag: no dependent load of h's)
    B.consider(ok, a0, a1, a2, a3, tbh, h);
  }
}

// The touched hosts, with their live capacities (host-sharded: this rank's hosts only).
__device__ __forceinline__ void band_scan_touched(const BandArgs& A, int seg, BandList& B) {
  const int lane = lane_id();
  const int nt_ = *A.tcount;
#ifdef PVT_BAND_PIPE2
  // software-pipelined two deep: chunk cc + S's loads in flight while chunk cc is considered
  auto load = [&](int cc, bool& ok, int32_t& h, double& a0, double& a1, double& a2, double& a3,
                  uint32_t& tbh) {
    const int j = cc * WAVE + lane;
    const int32_t hj = (cc * WAVE < nt_ && j < nt_) ? A.tlist[j] : -1;
    ok = hj >= A.lo && hj < A.hi;
    h = ok ? hj : 0;
    a0 = ok ? A.avail[h] : 0.0; a1 = ok ? A.avail[(size_t)A.H + h] : 0.0;
    a2 = ok ? A.avail[2 * (size_t)A.H + h] : 0.0; a3 = ok ? A.avail[3 * (size_t)A.H + h] : 0.0;
    tbh = ok ? A.tb[h] : 0u;
  };
  bool ok;
  int32_t h;
  double a0, a1, a2, a3;
  uint32_t tbh;
  load(seg, ok, h, a0, a1, a2, a3, tbh);
  for (int cc = seg; cc * WAVE < nt_; cc += A.S) {
    const bool cok = ok;
    const int32_t ch = h;
    const double c0 = a0, c1 = a1, c2 = a2, c3 = a3;
    const uint32_t ctb = tbh;
    load(cc + A.S, ok, h, a0, a1, a2, a3, tbh);
    B.consider(cok, c0, c1, c2, c3, ctb, ch);
  }
#else
  for (int cc = seg; cc * WAVE < nt_; cc += A.S) {
    const int j = cc * WAVE + lane;
    const int32_t hj = j < nt_ ? A.tlist[j] : -1;
    const bool ok = hj >= A.lo && hj < A.hi;
    const int32_t h = ok ? hj : 0;
    const double a0 = ok ? A.avail[h] : 0.0, a1 = ok ? A.avail[(size_t)A.H + h] : 0.0;
    const double a2 = ok ? A.avail[2 * (size_t)A.H + h] : 0.0, a3 = ok ? A.avail[3 * (size_t)A.H + h] : 0.0;
    B.consider(ok, a0, a1, a2, a3, ok ? A.tb[h] : 0u, h);
  }
#endif
}

// One wave per (task, segment): segment s takes the sorted copy's 64-host chunks c with
// c % S == s from the task's lower bound upward, then the touched list's chunks likewise.
__global__ __launch_bounds__(256) void band_score_kernel(BandArgs A) {
  __shared__ uint64_t s_m1[WPB][KL], s_m2[WPB][KL];
  const int lane = lane_id(), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = blockIdx.x * WPB + wave;
  const int t = g / A.S, seg = g % A.S;
  if (gate_closed(A.gate)) return;
  if (t >= A.nt || (A.nt_dev && t >= *A.nt_dev)) return;
  const double* dp = A.dem + (size_t)t * 4;
  BandList B;
  B.d0 = dp[0]; B.d1 = dp[1]; B.d2 = dp[2]; B.d3 = dp[3];
  B.m1 = s_m1[wave];
  B.m2 = s_m2[wave];
  band_scan_sorted(A, seg, B);
  band_scan_touched(A, seg, B);
#ifdef PVT_BAND_CHECK
  band_check(A, t, seg, B.ls, B.lt, B.li, B.d0, B.d1, B.d2, B.d3);
#endif
  const size_t row = (size_t)t * A.S + seg;
  SegEntry e;
  e.s = B.ls; e.tb = B.lt; e.id = B.li;
  A.seg[row * KL + lane] = e;
  const int filled = __popcll(__ballot(B.li != 0x7fffffff));
  if (lane == 0) A.seg_feas[row] = filled == KL ? KL + 1 : filled;
}

// The round's runs of equal demands (vbp best-fit lists depend on the demand vector only, and the
// sorted order puts equal demands next to each other): run[t] = the run of processing-order task
// t, rdem[run] = its demand. A window's list rows are then the runs it spans -- row of task t0 + w
// = run[t0 + w] - run[t0], the rows' demands rdem + run[t0] -- with no per-window launch. One
// block: a block scan of the run heads per 1024 tasks, carried across them.
__global__ __launch_bounds__(1024) void band_runs_kernel(const double* dem, int T, int32_t* run,
                                                         double* rdem) {
  __shared__ int32_t wsum[16];
  __shared__ int32_t carry;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int t0 = 0; t0 < T; t0 += 1024) {
    const int t = t0 + tid;
    bool head = false;
    if (t < T) {
      head = t == 0;
      for (int r = 0; r < 4 && !head; r++)
        head = __double_as_longlong(dem[(size_t)t * 4 + r]) != __double_as_longlong(dem[(size_t)(t - 1) * 4 + r]);
    }
    const uint64_t m = __ballot(head);
    int incl = __popcll(lane == 63 ? m : (m & ((2ull << lane) - 1ull)));
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    for (int w = 0; w < wave; w++) incl += wsum[w];
    incl += carry;
    if (t < T) {
      run[t] = incl - 1;
      if (head)
        for (int r = 0; r < 4; r++) rdem[(size_t)(incl - 1) * 4 + r] = dem[(size_t)t * 4 + r];
    }
    __syncthreads();
    if (tid == 1023) carry = incl;
    __syncthreads();
  }
}

void launch_band_runs(const double* dem, int T, int32_t* run, double* rdem, hipStream_t st) {
  if (T > 0) PVT_LAUNCH(band_runs_kernel, dim3(1), dim3(1024), 0, st, dem, T, run, rdem);
}

void launch_band_keys(const double* avail, const uint32_t* tb, int H, int lo, int n, uint64_t* key,
                      int32_t* idx, BandRec* rec, hipStream_t st) {
  if (n > 0)
    PVT_LAUNCH(band_keys_kernel, dim3((n + 255) / 256), dim3(256), 0, st, avail, tb, H, lo, n, key,
               idx, rec);
}
void launch_band_gather(const BandRec* rec, int lo, int n, const int32_t* sid, double* sa,
                        uint32_t* stb, int32_t* pos, hipStream_t st) {
  if (n > 0) PVT_LAUNCH(band_gather_kernel, dim3((n + 255) / 256), dim3(256), 0, st, rec, lo, n, sid, sa, stb, pos);
}
void launch_touch_update(const int32_t* own, const int32_t* status, uint8_t* flags, int32_t* tlist,
                         int32_t* tcount, const int32_t* pos, int lo, int hi, uint8_t* ptouch,
                         hipStream_t st) {
  PVT_LAUNCH(touch_update_kernel, dim3(1), dim3(1024), 0, st, own, status, flags, tlist,
                     tcount, pos, lo, hi, ptouch);
}
void launch_band_score(const BandArgs& a, hipStream_t st) {
  const int waves = a.nt * a.S;
  if (waves > 0) PVT_LAUNCH(band_score_kernel, dim3((waves + WPB - 1) / WPB), dim3(WPB * WAVE), 0, st, a);
}

}  // namespace pvt
