// pvt_groups.hip — cost_aware grouping on the device (the drop-in round's single round trip,
// pvt_place_host with pvt_ca_items).
//
// Reference (scheduler/cost_aware.py:30-58): ready tasks are grouped in first-seen order by
//   ('storage', cluster.get_storage_by_locality(mode host's zone))  for tasks with predecessors,
//   ('app', task.application)                                       for source tasks,
// and the groups run in that order, an application group's anchor drawn as
// randomizer.choice(cluster.storage) when its turn comes (:37-39). The mode hosts come from the
// anchor kernels (pvt_anchor.hip) over the items' predecessor lists; this kernel turns them into
// task_group / group_anchor / n_groups for the placement that follows on the same stream:
//   key(t)     storage index s (< S) or S + application index (anchor_zone -1: no predecessors)
//   first[k]   the lowest task index with key k (LDS atomicMin)
//   group(k)   the number of keys whose first task comes before first[k]: a block scan of the
//              "first task of its key" flags in task order
//   draws      one MT19937 randint(0, S) per application group, in group order, by one wave
//              (numpy legacy RandomState.choice: masked rejection, no draw for S == 1)
// One workgroup: at most 16384 tasks, a few microseconds of work.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pivot_place.h"
#include "pvt_device.h"
#include "pvt_groups.h"
#include "pvt_kernels.h"
#include "pvt_mt.h"

namespace pvt {

constexpr int GR_THREADS = 1024;
constexpr int GR_PER = GRP_MAX_TASKS / GR_THREADS;   // tasks per thread, keys kept in registers

__device__ __forceinline__ void ca_groups_round(const CaGroupArgs& A) {
  __shared__ int32_t first[GRP_MAX_KEYS];            // first task of each key, then its group
  __shared__ uint32_t appbit[GRP_MAX_TASKS / 32];    // group g is an application group
  __shared__ int32_t wsum[GR_THREADS / 64];
  __shared__ uint32_t mt[628];
  __shared__ int32_t err;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = A.T, S = A.S, K = A.S + A.n_apps;
  for (int k = tid; k < K; k += GR_THREADS) first[k] = 0x7fffffff;
  for (int k = tid; k < GRP_MAX_TASKS / 32; k += GR_THREADS) appbit[k] = 0;
  if (tid == 0) err = 0;
  __syncthreads();
  // keys (an error leaves key 0 -- storage 0 -- so the placement after stays in bounds)
  int key[GR_PER];
#pragma unroll
  for (int u = 0; u < GR_PER; u++) {
    const int t = u * GR_THREADS + tid;
    key[u] = 0;
    if (t >= T) continue;
    const int it = A.task_item[t];
    int e = 0, k = 0;
    if (it < 0 || it >= A.C) {
      e = 3;
    } else {
      const int z = A.anchor_zone[it];
      if (z >= 0 && z < A.Z) {
        const int s = A.zone_storage[z];
        if (s < 0 || s >= S) e = 2;          // get_storage_by_locality -> None
        else k = s;
      } else if (z == -1) {                  // no predecessors: the application's group
        const int ap = A.item_app[it];
        if (ap < 0 || ap >= A.n_apps) e = 3;
        else k = S + ap;
      } else {
        e = z == -2 ? 1 : 3;                 // mode placement not a host / malformed list
      }
    }
    if (e) atomicMax(&err, e);
    key[u] = k;
    atomicMin(&first[k], t);
  }
  __syncthreads();
  // group of each key: the first-task flags scanned in task order. A first task rewrites its
  // key's entry with the group index (<= its own position, so no later task of the key mistakes
  // it for its own position) and sets the group's anchor or marks it an application group.
  int base = 0;
  for (int u = 0; u < GR_PER && u * GR_THREADS < T; u++) {
    const int t = u * GR_THREADS + tid;
    const bool f = t < T && first[key[u]] == t;
    const uint64_t m = __ballot(f);
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    int before = base, tot = 0;
    for (int w = 0; w < GR_THREADS / 64; w++) {
      before += w < wave ? wsum[w] : 0;
      tot += wsum[w];
    }
    __syncthreads();                         // (wsum is rewritten by the next chunk)
    if (f) {
      const int g = before + __popcll(m & ((1ull << lane) - 1ull));
      first[key[u]] = g;
      if (key[u] < S) A.group_anchor[g] = A.storage_zone[key[u]];
      else atomicOr(&appbit[g >> 5], 1u << (g & 31));
    }
    base += tot;
  }
  __syncthreads();
  const int G = base;
#pragma unroll
  for (int u = 0; u < GR_PER; u++) {
    const int t = u * GR_THREADS + tid;
    if (t < T) A.task_group[t] = first[key[u]];
  }
  if (wave != 0) return;
  // application groups' anchors: randomizer.choice(storage) in group order (cost_aware.py:39)
  for (int i = lane; i < 625; i += 64) mt[i] = A.mt[i];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  MtWave mw;
  mw.buf = 0; mw.used = 0; mw.limit = 0;
  for (int g0 = 0; g0 < G; g0 += 32) {
    uint32_t bits = __builtin_amdgcn_readfirstlane(appbit[g0 >> 5]);
    while (bits) {
      const int g = g0 + __builtin_ctz(bits);
      bits &= bits - 1;
      const int idx = (int)mt_randint(mt, mw, (uint32_t)S);
      if (lane == 0) A.group_anchor[g] = A.storage_zone[idx];
    }
  }
  mt_unbuffer(mt, mw);
  for (int i = lane; i < 625; i += 64) A.mt[i] = mt[i];
  if (lane == 0) {
    const int e = err;
    A.status[0] = G;
    A.status[1] = e;
    if (A.desc_n_groups) *A.desc_n_groups = G > 0 ? G : 1;
  }
}

__global__ __launch_bounds__(GR_THREADS) void ca_groups_kernel(CaGroupArgs A) { ca_groups_round(A); }

// Several rounds' groupings in one launch, one workgroup each (pvt_place_host_batch).
__global__ __launch_bounds__(GR_THREADS) void ca_groups_batch_kernel(const CaGroupArgs* A) {
  const CaGroupArgs a = A[blockIdx.x];
  ca_groups_round(a);
}

void launch_ca_groups(const CaGroupArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(ca_groups_kernel, dim3(1), dim3(GR_THREADS), 0, st, a);
}
void launch_ca_groups_batch(const CaGroupArgs* args_dev, int n, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(ca_groups_batch_kernel, dim3(n), dim3(GR_THREADS), 0, st, args_dev);
}

}  // namespace pvt
