// pvt_epoch.hip — speculative group-parallel epochs for cost_aware best-fit.
//
// The reference runs its groups one after the other (scheduler/cost_aware.py:37-42), each task
// taking the minimum of (c * ||avail - d||) / bw over every feasible host and committing before
// the next (:85-97). A group's winners are the lowest-index fitting hosts of the zones its
// anchor reaches at zero egress cost (score 0), so groups anchored in different zero-cost
// components rarely touch the same hosts. An epoch splits its groups (segments, processing
// order) into chains, one per component: one commit-walk workgroup walks a chain's segments in
// order, all chains side by side on the epoch's start state, logging every commit (WinRec).
// Then it proves, exactly, which prefix the sequential order would have produced:
//
//   segment 0 started from the true state, so it is exact;
//   segment j > 0 is exact iff segments 0..j-1 are exact and complete, and for every task t
//   it walked and every final log entry (host h, capacities after that segment) of an earlier
//   segment of ANOTHER chain: h is not t's winner, and h does not fit t with a key (score,
//   index) below the winner's. (Earlier segments of j's own chain were walked before j on the
//   same state, so the walk already saw their commits.)
//
// By induction over j's tasks, every host the other chains' earlier segments did not touch has
// the same state in the speculative and the sequential run, so the argmin over them is the same
// host, and no touched host beats it (capacities only decrease, so a task that found no host
// still finds none; a stale entry of a host committed again later only adds checks). The
// validate kernel checks exactly that; the host accepts the exact prefix, the apply kernel
// writes its final entries chain by chain, and the next epoch starts where the prefix ended.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"
#include "pvt_kernels.h"

namespace pvt {

// Tasks of segment j its chain's walk got through.
__device__ __forceinline__ int seg_adv(const EpochArgs& A, int j) {
  const int len = A.seg_off[j + 1] - A.seg_off[j];
  const int done = A.status[2 * A.seg_chain[j]] - A.seg_cstart[j];
  return max(0, min(len, done));
}

// Block (task tile x of segment j, entry slice z): every thread holds one walked task of j; the
// block stages the final log entries of slice z of the window's earlier tasks (those of other
// chains' segments) 256 at a time in LDS -- host, capacities, and the zone-table (or realtime)
// c and bw for j's anchor, which every task of j shares -- so the pair checks are LDS broadcasts
// only. Slices split each segment's checks over VAL_SPLIT blocks.
constexpr int VAL_SPLIT = 32;
__device__ __forceinline__ int seg_of(const EpochArgs& A, int e) {
  int lo = 0, hi = A.nseg - 1;                // the segment holding window task e
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (A.seg_off[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Pair check of task t (demand d, winner w with score bits w1) against log entry k.
__device__ __forceinline__ bool beats(int32_t h, double f0, double f1, double f2, double f3,
                                      double c, double bw, double d0, double d1, double d2,
                                      double d3, const WinRec& w, uint64_t w1) {
  if (h == w.id) return true;
  // a winner scoring +0 is beaten only by a host of lower index scoring +0
  if ((w1 == 0ull && h > w.id) || !fits<false>(f0, f1, f2, f3, d0, d1, d2, d3)) return false;
  const double s2 = norm2_seq(f0 - d0, f1 - d1, f2 - d2, f3 - d3);
  if (c == 0.0)   // zero egress cost: the score is exactly +0 (finite s2, bw > 0)
    return (0ull < w1) | ((0ull == w1) & (h < w.id));
  if (w1 == 0ull && s2 >= 0x1p-600 && c >= 0x1p-300 && bw <= 0x1p300)
    return false;   // c * sqrt(s2) >= 2^-600 and / bw >= 2^-900: the score is > 0
  const double sc = (c * __builtin_sqrt(s2)) / bw;
  const uint64_t k1 = (uint64_t)__double_as_longlong(sc);
  return (k1 < w1) | ((k1 == w1) & (h < w.id));
}

constexpr int VAL_HASH = 512;

// Every chain walked to its end and every final entry safe (EpochArgs.cmax): nothing to check.
// The block's threads split the chains and segments (at most EPOCH_SEGS each): one load latency
// instead of a serial walk over both tables in every thread of every block.
__device__ __forceinline__ bool epoch_fast(const EpochArgs& A) {
  if (!A.cmax) return false;
  bool slow = false;
  for (int c = threadIdx.x; c < A.nch; c += blockDim.x)
    slow |= A.status[2 * c] != A.coff[c + 1] - A.coff[c];
  for (int s = threadIdx.x; s < A.nseg; s += blockDim.x) slow |= !A.safe[s];
  return !__syncthreads_or(slow);
}

__global__ __launch_bounds__(256) void epoch_validate_kernel(EpochArgs A) {
  __shared__ int32_t e_id[256];
  __shared__ double e_a[4][256];
  __shared__ double e_c[256], e_b[256];
  __shared__ int32_t e_full[256];             // entries that need the pair check
  __shared__ int32_t hk[VAL_HASH];            // hosts of the others ("id-only" entries)
  __shared__ double wmx[4][4];
  __shared__ int32_t wfull[4];
  __shared__ int32_t stop;
  const int j = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (j == 0 || j >= A.nseg) return;          // (block-uniform exits, cheapest first)
  const int s0 = A.seg_off[j], adv = seg_adv(A, j);
  if ((int)blockIdx.x * 256 >= adv) return;
  const int L = s0;                           // earlier window tasks: [0, s0)
  const int lo = (int)((long long)L * blockIdx.z / VAL_SPLIT);
  const int hi = (int)((long long)L * (blockIdx.z + 1) / VAL_SPLIT);
  if (lo >= hi) return;
  if (epoch_fast(A)) return;
  const int t = s0 + blockIdx.x * 256 + tid;
  const bool mine = t < s0 + adv;
  const int cj = A.seg_chain[j];
  const int a = A.anc[s0];                    // a segment is one group: one anchor, one row
  const double* rtrow = A.rtb ? A.rtb + (size_t)A.grp[s0] * A.H : nullptr;
  WinRec w{};
  double d0 = 0, d1 = 0, d2 = 0, d3 = 0;
  bool active = false;
  if (mine) {
    w = A.wlog[t];
    active = w.id >= 0;                      // no host fits: stays so (capacities only drop)
    d0 = A.dem[(size_t)t * 4]; d1 = A.dem[(size_t)t * 4 + 1];
    d2 = A.dem[(size_t)t * 4 + 2]; d3 = A.dem[(size_t)t * 4 + 3];
  }
  const uint64_t w1 = (uint64_t)__double_as_longlong(w.s);
  // The block's largest demand per dimension. An entry with c >= 2^-300, bw <= 2^300 whose
  // capacity exceeds it by 2^-287 in some dimension has s2 >= 2^-576 against every task here,
  // so its score is > 0: against a winner scoring +0 only host identity matters (LDS hash).
  double x0 = active ? d0 : -DINF, x1 = active ? d1 : -DINF;
  double x2 = active ? d2 : -DINF, x3 = active ? d3 : -DINF;
  for (int off = 32; off > 0; off >>= 1) {
    x0 = fmax(x0, __shfl_xor(x0, off)); x1 = fmax(x1, __shfl_xor(x1, off));
    x2 = fmax(x2, __shfl_xor(x2, off)); x3 = fmax(x3, __shfl_xor(x3, off));
  }
  if (lane == 0) { wmx[wave][0] = x0; wmx[wave][1] = x1; wmx[wave][2] = x2; wmx[wave][3] = x3; }
  if (tid == 0) stop = __hip_atomic_load(&A.bad[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  double mx[4];
#pragma unroll
  for (int r = 0; r < 4; r++) mx[r] = fmax(fmax(wmx[0][r], wmx[1][r]), fmax(wmx[2][r], wmx[3][r]));
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  bool beaten = false;
  for (int c0 = lo; c0 < hi && !stop; c0 += 256) {
    const int e = c0 + tid;
    int32_t id = -1;
    bool idonly = false;
    if (e < hi) {
      const int s = seg_of(A, e);
      if (A.seg_chain[s] != cj && e - A.seg_off[s] < seg_adv(A, s)) {
        const WinRec& x = A.wlog[e];
        if (x.id >= 0 && !x.sup) {
          id = x.id;
          const double f0 = x.a[0], f1 = x.a[1], f2 = x.a[2], f3 = x.a[3];
          e_a[0][tid] = f0; e_a[1][tid] = f1; e_a[2][tid] = f2; e_a[3][tid] = f3;
          const int z = A.zone[id];
          const double c = A.csum[a * A.Z + z];
          const double bw = rtrow ? rtrow[id] : A.bsum[a * A.Z + z];
          e_c[tid] = c;
          e_b[tid] = bw;
          idonly = c >= 0x1p-300 && bw <= 0x1p300 &&
                   (f0 - mx[0] >= 0x1p-287 || f1 - mx[1] >= 0x1p-287 ||
                    f2 - mx[2] >= 0x1p-287 || f3 - mx[3] >= 0x1p-287);
        }
      }
    }
    e_id[tid] = id;
    hk[tid] = -1;
    hk[tid + 256] = -1;
    const bool full = id >= 0 && !idonly;
    const uint64_t fb = __ballot(full);
    if (lane == 0) wfull[wave] = __popcll(fb);
    __syncthreads();
    if (idonly) {
      uint32_t p = ((uint32_t)id * 2654435761u) & (VAL_HASH - 1);
      for (;;) {
        const int32_t o = atomicCAS(&hk[p], -1, id);
        if (o == -1 || o == id) break;
        p = (p + 1) & (VAL_HASH - 1);
      }
    }
    int pos = __popcll(fb & below);
    for (int q = 0; q < wave; q++) pos += wfull[q];
    if (full) e_full[pos] = tid;
    const int nfull = wfull[0] + wfull[1] + wfull[2] + wfull[3];
    __syncthreads();
    if (active && !beaten) {
      if (w1 == 0ull) {
        // the id-only entries: only t's winner host
        uint32_t p = ((uint32_t)w.id * 2654435761u) & (VAL_HASH - 1);
        for (;;) {
          const int32_t o = hk[p];
          if (o == w.id) { beaten = true; break; }
          if (o == -1) break;
          p = (p + 1) & (VAL_HASH - 1);
        }
        for (int q = 0; q < nfull && !beaten; q++) {
          const int k = e_full[q];
          beaten = beats(e_id[k], e_a[0][k], e_a[1][k], e_a[2][k], e_a[3][k], e_c[k], e_b[k],
                         d0, d1, d2, d3, w, w1);
        }
      } else {
        const int n = min(256, hi - c0);
        for (int k = 0; k < n && !beaten; k++) {
          const int32_t h = e_id[k];
          if (h < 0) continue;
          beaten = beats(h, e_a[0][k], e_a[1][k], e_a[2][k], e_a[3][k], e_c[k], e_b[k],
                         d0, d1, d2, d3, w, w1);
        }
      }
    }
    if (beaten) stop = 1;                    // benign race: every writer stores 1
    __syncthreads();
  }
  if (tid == 0 && stop) __hip_atomic_store(&A.bad[j], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Finality of the log entries: per segment, an entry is its host's final state unless a later
// walked task of the same segment committed to the same host (sup = 1). One block per segment:
// every walked entry records its index in an LDS hash keyed by host (atomicMax: the host's last
// entry), then an entry is final iff it is its host's last. (A segment never exceeds CHAIN_MAX
// tasks; 2 x CHAIN_MAX slots. The pairwise scan it replaces was O(n^2): 70 us per config-5
// epoch.)
constexpr int FIN_SLOTS = 2 * CHAIN_MAX;
__device__ __forceinline__ int fin_slot(int32_t h, const int32_t* hk) {
  uint32_t p = ((uint32_t)h * 2654435761u) & (FIN_SLOTS - 1);
  while (hk[p] != h) p = (p + 1) & (FIN_SLOTS - 1);
  return (int)p;
}
__global__ __launch_bounds__(1024) void epoch_final_kernel(EpochArgs A) {
  __shared__ int32_t hk[FIN_SLOTS], hv[FIN_SLOTS];
  __shared__ double gmx[4];
  __shared__ int32_t unsafe;
  const int j = blockIdx.x, tid = threadIdx.x;
  const int s0 = A.seg_off[j], n = seg_adv(A, j);
  if (tid == 0) { A.bad[j] = 0; unsafe = 0; }   // validation (next launch) starts with no verdict
  if (A.cmax && tid < 4) {                    // the epoch's largest demand per dimension
    double m = -DINF;
    for (int c = 0; c < A.nch; c++) m = fmax(m, A.cmax[c * 4 + tid]);
    gmx[tid] = m;
  }
  for (int q = tid; q < FIN_SLOTS; q += blockDim.x) { hk[q] = -1; hv[q] = -1; }
  __syncthreads();
  for (int k = tid; k < n; k += blockDim.x) {
    const int32_t h = A.wlog[s0 + k].id;
    if (h < 0) continue;
    uint32_t p = ((uint32_t)h * 2654435761u) & (FIN_SLOTS - 1);
    for (;;) {
      const int32_t o = atomicCAS(&hk[p], -1, h);
      if (o == -1 || o == h) break;
      p = (p + 1) & (FIN_SLOTS - 1);
    }
    atomicMax(&hv[p], k);
  }
  __syncthreads();
  for (int k = tid; k < n; k += blockDim.x) {
    const WinRec& e = A.wlog[s0 + k];
    const int32_t h = e.id;
    const int sup = (h >= 0 && hv[fin_slot(h, hk)] != k) ? 1 : 0;
    A.wlog[s0 + k].sup = sup;
    if (A.cmax && h >= 0 && !sup &&
        !(e.a[0] - gmx[0] >= 0x1p-287 || e.a[1] - gmx[1] >= 0x1p-287 ||
          e.a[2] - gmx[2] >= 0x1p-287 || e.a[3] - gmx[3] >= 0x1p-287))
      unsafe = 1;                             // (benign race: every writer stores 1)
  }
  if (A.cmax) {
    __syncthreads();
    if (tid == 0) A.safe[j] = unsafe ? 0 : 1;
  }
}

// One block per chain: its accepted segments in order, each segment's final entries written to
// global availability (a later segment of the chain overwrites an earlier one's entry for the
// same host; different chains' accepted segments touch disjoint hosts).
__global__ __launch_bounds__(256) void epoch_apply_kernel(EpochArgs A, int n_accept) {
  const int c = blockIdx.x;
  for (int s = 0; s < n_accept; s++) {
    if (A.seg_chain[s] != c) continue;
    const int e0 = A.seg_off[s], ne = seg_adv(A, s);
    for (int k = threadIdx.x; k < ne; k += blockDim.x) {
      const WinRec& e = A.wlog[e0 + k];
      if (e.id < 0 || e.sup) continue;
#pragma unroll
      for (int r = 0; r < 4; r++) A.avail[(size_t)r * A.H + e.id] = e.a[r];
    }
    __syncthreads();
  }
}

// The accepted prefix, decided on the device right after validation (no host round trip
// between validation and apply): segments before the first rejected one, up to and including
// the first its chain did not finish (its walked tasks are exact; the next epoch starts there).
// Every block derives it; block 0 reports it (res: accepted segments, next task relative to the
// epoch, refill, rejected segments, a chain walk timed out); block c then writes chain c's
// accepted segments' final entries, as epoch_apply_kernel. A timed-out walk applies nothing.
// The first stopping segment is found by all threads at once (LDS minimum), and each wave picks
// chain c's segments 64 at a time by ballot: no serial walk over the segment table. Block 0 also
// writes the readback words (nwords from A.status: statuses, verdicts, res, safe flags) straight
// into the caller's mapped pinned buffer hout: no copy launch after the kernel.
__global__ __launch_bounds__(1024) void epoch_accept_apply_kernel(EpochArgs A, int32_t* res,
                                                                  int32_t* hout, int nwords) {
  __shared__ int32_t first_s;
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int nseg = A.nseg;
  if (tid == 0) first_s = nseg;
  bool tout = false;
  for (int j = tid; j < nseg; j += blockDim.x) tout |= A.status[2 * A.seg_chain[j]] == -1;
  const int roff = (int)(res - A.status);    // res inside the readback words
  auto put = [&](int i, int32_t v) {
    res[i] = v;
    if (hout) hout[roff + i] = v;
  };
  if (c == 0 && hout)
    for (int k = tid; k < nwords; k += blockDim.x)
      if (k < roff || k >= roff + 5) hout[k] = A.status[k];
  if (__syncthreads_or(tout)) {               // (also publishes first_s)
    if (c == 0 && tid == 0) { put(0, 0); put(1, 0); put(2, 0); put(3, 0); put(4, 1); }
    return;
  }
  for (int j = tid; j < nseg; j += blockDim.x) {
    const int len = A.seg_off[j + 1] - A.seg_off[j];
    if ((j > 0 && A.bad[j]) || seg_adv(A, j) < len) atomicMin(&first_s, j);
  }
  __syncthreads();
  const int f = first_s;
  int acc = nseg;
  if (f < nseg) {
    const int adv = seg_adv(A, f);
    const bool whole_stop = (f > 0 && A.bad[f]) || A.whole;   // (adv < len when not rejected)
    acc = whole_stop ? f : f + 1;
    if (c == 0 && tid == 0) {
      const bool rejected = f > 0 && A.bad[f];
      put(0, acc);
      put(1, whole_stop ? A.seg_off[f] : A.seg_off[f] + adv);
      put(2, rejected ? 0 : 1);
      put(3, whole_stop ? nseg - f : nseg - f - 1);
      put(4, 0);
    }
  } else if (c == 0 && tid == 0) {
    put(0, nseg); put(1, nseg > 0 ? A.seg_off[nseg] : 0); put(2, 0); put(3, 0); put(4, 0);
  }
  if (acc > 64) {                              // (not from the planners: EPOCH_SEGS = 64)
    for (int base = 0; base < acc; base += 64) {
      const int sl = base + lane;
      uint64_t own = __ballot(sl < acc && A.seg_chain[sl] == c);
      while (own) {
        const int s = base + __builtin_ctzll(own);
        own &= own - 1;
        const int e0 = A.seg_off[s], ne = seg_adv(A, s);
        for (int k = tid; k < ne; k += blockDim.x) {
          const WinRec& e = A.wlog[e0 + k];
          if (e.id < 0 || e.sup) continue;
#pragma unroll
          for (int r = 0; r < 4; r++) A.avail[(size_t)r * A.H + e.id] = e.a[r];
        }
        __syncthreads();
      }
    }
    return;
  }
  // Chain c's accepted segments cover chain-local positions [0, P) (every one but the last is
  // complete). An entry is written iff it is its host's last in that prefix (LDS hash: host ->
  // largest position), so every entry is loaded once and all writes go out together.
  __shared__ int32_t hk[FIN_SLOTS], hv[FIN_SLOTS];
  __shared__ int32_t o_cs[64], o_off[64], n_own, plen;
  if (tid < 64) {
    const bool mine = tid < acc && A.seg_chain[tid] == c;
    const uint64_t own = __ballot(mine);
    const int i = __popcll(own & ((1ull << tid) - 1ull));
    if (mine) {
      o_cs[i] = A.seg_cstart[tid];
      o_off[i] = A.seg_off[tid];
      if (!(own >> tid >> 1)) { n_own = i + 1; plen = A.seg_cstart[tid] + seg_adv(A, tid); }
    }
    if (tid == 0 && !own) { n_own = 0; plen = 0; }
  }
  for (int q = tid; q < FIN_SLOTS; q += blockDim.x) { hk[q] = -1; hv[q] = -1; }
  __syncthreads();
  const int n = n_own, P = plen;
  constexpr int PER = CHAIN_MAX / 1024;
  WinRec e[PER];
  int slot[PER];
#pragma unroll
  for (int i = 0; i < PER; i++) {
    const int k = tid + i * 1024;
    slot[i] = -1;
    if (k >= P) continue;
    int q = 0;
    while (q + 1 < n && o_cs[q + 1] <= k) q++;
    e[i] = A.wlog[o_off[q] + (k - o_cs[q])];
    const int32_t h = e[i].id;
    if (h < 0) continue;
    uint32_t p = ((uint32_t)h * 2654435761u) & (FIN_SLOTS - 1);
    for (;;) {
      const int32_t o = atomicCAS(&hk[p], -1, h);
      if (o == -1 || o == h) break;
      p = (p + 1) & (FIN_SLOTS - 1);
    }
    atomicMax(&hv[p], k);
    slot[i] = (int)p;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PER; i++) {
    if (slot[i] < 0 || hv[slot[i]] != tid + i * 1024) continue;
#pragma unroll
    for (int r = 0; r < 4; r++) A.avail[(size_t)r * A.H + e[i].id] = e[i].a[r];
  }
}

void launch_epoch_accept_apply(const EpochArgs& a, int32_t* res, int nchains, hipStream_t st,
                               int32_t* hout, int nwords) {
  PVT_LAUNCH(epoch_accept_apply_kernel, dim3(nchains), dim3(1024), 0, st, a, res, hout, nwords);
}

void launch_epoch_validate(const EpochArgs& a, hipStream_t st) {
  PVT_LAUNCH(epoch_final_kernel, dim3(a.nseg), dim3(1024), 0, st, a);
  const int tiles = (CHAIN_MAX + 255) / 256;   // a segment never exceeds its chain's cap
  PVT_LAUNCH(epoch_validate_kernel, dim3(tiles, a.nseg, VAL_SPLIT), dim3(256), 0, st, a);
}

void launch_epoch_final(const EpochArgs& a, hipStream_t st) {
  PVT_LAUNCH(epoch_final_kernel, dim3(a.nseg), dim3(1024), 0, st, a);
}

void launch_epoch_apply(const EpochArgs& a, int n_accept, int nchains, hipStream_t st) {
  if (n_accept <= 0 || nchains <= 0) return;
  PVT_LAUNCH(epoch_apply_kernel, dim3(nchains), dim3(256), 0, st, a, n_accept);
}

}  // namespace pvt
