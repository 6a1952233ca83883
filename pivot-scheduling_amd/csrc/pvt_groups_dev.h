// pvt_groups_dev.h — the device side of the cost_aware grouping (pvt_groups.hip's kernels and
// the fused host-batch round, pvt_batch.hip resident_fused_kernel). See pvt_groups.hip.
#pragma once
#include "pvt_device.h"
#include "pvt_groups.h"
#include "pvt_mt.h"

namespace pvt {

// LDS of one grouping (static in ca_groups_kernel; a slice of the dynamic LDS in the fused
// host-batch round, pvt_batch.hip)
struct GroupLds {
  int32_t first[GRP_MAX_KEYS];            // first task of each key, then its group
  uint32_t appbit[GRP_MAX_TASKS / 32];    // group g is an application group
  int32_t wsum[16];
  uint32_t mt[628];
  int32_t err;
};

// NT threads (a multiple of 64, at most 1024), at most MAXT tasks (MAXT / NT keys per thread,
// in registers). Every thread returns after the last barrier; wave 0 then draws the anchors of
// the application groups and writes the status (the caller synchronises before reading them).
template <int NT, int MAXT>
__device__ __forceinline__ void ca_groups_round(const CaGroupArgs& A, GroupLds& L) {
  constexpr int GR_THREADS = NT;
  constexpr int GR_PER = MAXT / NT;
  static_assert(MAXT <= GRP_MAX_TASKS && NT % 64 == 0 && NT <= 1024, "grouping shape");
  int32_t* first = L.first;
  uint32_t* appbit = L.appbit;
  int32_t* wsum = L.wsum;
  uint32_t* mt = L.mt;
  int32_t& err = L.err;
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
  if (wave == 0) {
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
}

}  // namespace pvt
