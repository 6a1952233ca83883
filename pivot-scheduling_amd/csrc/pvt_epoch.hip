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
__device__ __forceinline__ bool epoch_fast(const EpochArgs& A) {
  if (!A.cmax) return false;
  for (int c = 0; c < A.nch; c++)
    if (A.status[2 * c] != A.coff[c + 1] - A.coff[c]) return false;
  for (int s = 0; s < A.nseg; s++)
    if (!A.safe[s]) return false;
  return true;
}

__global__ __launch_bounds__(256) void epoch_validate_kernel(EpochArgs A) {
  if (epoch_fast(A)) return;
  __shared__ int32_t e_id[256];
  __shared__ double e_a[4][256];
  __shared__ double e_c[256], e_b[256];
  __shared__ int32_t e_full[256];             // entries that need the pair check
  __shared__ int32_t hk[VAL_HASH];            // hosts of the others ("id-only" entries)
  __shared__ double wmx[4][4];
  __shared__ int32_t wfull[4];
  __shared__ int32_t stop;
  const int j = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (j == 0 || j >= A.nseg) return;
  const int s0 = A.seg_off[j], adv = seg_adv(A, j);
  if ((int)blockIdx.x * 256 >= adv) return;
  const int L = s0;                           // earlier window tasks: [0, s0)
  const int lo = (int)((long long)L * blockIdx.z / VAL_SPLIT);
  const int hi = (int)((long long)L * (blockIdx.z + 1) / VAL_SPLIT);
  if (lo >= hi) return;
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
__global__ __launch_bounds__(256) void epoch_accept_apply_kernel(EpochArgs A, int32_t* res) {
  __shared__ int32_t acc_s, tout_s;
  const int c = blockIdx.x;
  if (threadIdx.x == 0) {
    int acc = 0, next = 0, refill = 0, rej = 0, tout = 0;
    for (int j = 0; j < A.nseg; j++) tout |= A.status[2 * A.seg_chain[j]] == -1;
    if (!tout) {
      for (int j = 0; j < A.nseg; j++) {
        const int len = A.seg_off[j + 1] - A.seg_off[j];
        const int adv = seg_adv(A, j);
        if (j > 0 && A.bad[j]) { rej = A.nseg - j; break; }
        if (A.whole && adv < len) { next = A.seg_off[j]; refill = 1; rej = A.nseg - j; break; }
        acc = j + 1;
        next = A.seg_off[j] + adv;
        if (adv < len) { refill = 1; rej = A.nseg - j - 1; break; }
      }
    }
    acc_s = acc;
    tout_s = tout;
    if (c == 0) { res[0] = acc; res[1] = next; res[2] = refill; res[3] = rej; res[4] = tout; }
  }
  __syncthreads();
  if (tout_s) return;
  const int n_accept = acc_s;
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

void launch_epoch_accept_apply(const EpochArgs& a, int32_t* res, int nchains, hipStream_t st) {
  hipLaunchKernelGGL(epoch_accept_apply_kernel, dim3(nchains), dim3(256), 0, st, a, res);
}

void launch_epoch_validate(const EpochArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(epoch_final_kernel, dim3(a.nseg), dim3(1024), 0, st, a);
  const int tiles = (CHAIN_MAX + 255) / 256;   // a segment never exceeds its chain's cap
  hipLaunchKernelGGL(epoch_validate_kernel, dim3(tiles, a.nseg, VAL_SPLIT), dim3(256), 0, st, a);
}

void launch_epoch_final(const EpochArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(epoch_final_kernel, dim3(a.nseg), dim3(1024), 0, st, a);
}

void launch_epoch_apply(const EpochArgs& a, int n_accept, int nchains, hipStream_t st) {
  if (n_accept <= 0 || nchains <= 0) return;
  hipLaunchKernelGGL(epoch_apply_kernel, dim3(nchains), dim3(256), 0, st, a, n_accept);
}

}  // namespace pvt
