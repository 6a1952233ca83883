// pvt_epoch.hip — speculative group-parallel epochs for cost_aware best-fit.
//
// The reference runs its groups one after the other (scheduler/cost_aware.py:37-42), each task
// taking the minimum of (c * ||avail - d||) / bw over every feasible host and committing before
// the next (:85-97). The groups of a round usually anchor to different zones, and a group's
// winners are its own zone's free-egress hosts, so consecutive groups rarely touch the same
// hosts. An epoch therefore walks up to EPOCH_SEGMENTS groups side by side, each on the
// epoch's start state (one commit-walk workgroup per group, logging its commits), and then
// proves, exactly, which of them the sequential order would have produced:
//
//   segment 0 started from the true state, so it is exact;
//   segment j > 0 is exact iff segments 0..j-1 are exact and complete, and for every task t
//   it walked and every host h that an earlier segment committed to (at its capacities after
//   that segment, which are its capacities throughout j): h is not t's winner, and h does not
//   fit t with a key (score, index) below the winner's.
//
// By induction over j's tasks, every host outside those earlier segments' hosts has the same
// state in the speculative and the sequential run, so the argmin over them is the same host,
// and no earlier-touched host beats it (capacities only decrease, so a task that found no host
// still finds none). validate_kernel checks exactly that; the host accepts the exact prefix,
// applies its logged capacities (apply_kernel) and starts the next epoch where it ended.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"
#include "pvt_kernels.h"

namespace pvt {

// One wave per walked task of segments j >= 1: scan the own hosts of segments 0..j-1.
__global__ __launch_bounds__(256) void epoch_validate_kernel(EpochArgs A) {
  const int lane = lane_id();
  const int i = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (i >= A.nt) return;
  int j = 0;
  while (j + 1 < A.nseg && A.seg_off[j + 1] <= i) j++;   // segment of task i (nseg is small)
  if (j == 0) return;
  if (i - A.seg_off[j] >= A.status[2 * j]) return;        // not walked (the walk stopped early)
  const WinRec w = A.wres[i];
  if (w.id < 0) return;                                    // no host fits: stays so
  if (__hip_atomic_load(&A.bad[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const double d0 = A.dem[(size_t)i * 4], d1 = A.dem[(size_t)i * 4 + 1];
  const double d2 = A.dem[(size_t)i * 4 + 2], d3 = A.dem[(size_t)i * 4 + 3];
  const int a = A.anc[i];
  const uint64_t w1 = (uint64_t)__double_as_longlong(w.s);
  for (int s = 0; s < j; s++) {
    const int n = A.status[2 * s + 1];
    const int32_t* ids = A.own_ids + (size_t)s * MAX_WINDOW;
    const double* oa = A.own_a + (size_t)s * 4 * MAX_WINDOW;
    for (int o0 = 0; o0 < n; o0 += WAVE) {
      const int o = o0 + lane;
      bool beats = false;
      if (o < n) {
        const int32_t h = ids[o];
        const double f0 = oa[o], f1 = oa[MAX_WINDOW + o], f2 = oa[2 * MAX_WINDOW + o];
        const double f3 = oa[3 * MAX_WINDOW + o];
        beats = (h == w.id);
        if (!beats && fits<false>(f0, f1, f2, f3, d0, d1, d2, d3)) {
          const int z = A.zone[h];
          const double s2 = norm2_seq(f0 - d0, f1 - d1, f2 - d2, f3 - d3);
          const double sc = (A.csum[a * A.Z + z] * __builtin_sqrt(s2)) / A.bsum[a * A.Z + z];
          const uint64_t k1 = (uint64_t)__double_as_longlong(sc);
          beats = (k1 < w1) | ((k1 == w1) & (h < w.id));
        }
      }
      if (__ballot(beats)) {
        if (lane == 0) __hip_atomic_store(&A.bad[j], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
  }
}

// The accepted segments' logged capacities -> global availability (their hosts are disjoint).
__global__ __launch_bounds__(256) void epoch_apply_kernel(EpochArgs A) {
  const int s = blockIdx.y;
  const int n = A.status[2 * s + 1];
  const int32_t* ids = A.own_ids + (size_t)s * MAX_WINDOW;
  const double* oa = A.own_a + (size_t)s * 4 * MAX_WINDOW;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < n; o += gridDim.x * blockDim.x) {
    const int32_t h = ids[o];
#pragma unroll
    for (int r = 0; r < 4; r++) A.avail[(size_t)r * A.H + h] = oa[(size_t)r * MAX_WINDOW + o];
  }
}

void launch_epoch_validate(const EpochArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(epoch_validate_kernel, dim3((a.nt + 3) / 4), dim3(256), 0, st, a);
}

void launch_epoch_apply(const EpochArgs& a, int n_accept, hipStream_t st) {
  if (n_accept <= 0) return;
  hipLaunchKernelGGL(epoch_apply_kernel, dim3(MAX_WINDOW / 256, n_accept), dim3(256), 0, st, a);
}

}  // namespace pvt
