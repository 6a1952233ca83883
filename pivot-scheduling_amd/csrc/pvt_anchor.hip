// pvt_anchor.hip — mode-host anchor resolution (reference scheduler/cost_aware.py:45-58).
// See pvt_anchor.h for the rule. One 256-thread workgroup per item; the item's predecessor
// list is sorted as (host + 1) << 32 | position keys (bitonic, LDS or scratch), every run end
// binary-searches its run start, and the block keeps the max of (count << 32 | ~first).
// Integer-only, gather-bound: 4 B (8 B through inst_host) read per list entry.
#include "pvt_anchor.h"

namespace pvt {

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

// Host index of list entry j (-1 = a predecessor that has no placement); sets *ok = false on
// an index outside the instance table or a host outside [-1, H).
__device__ __forceinline__ int entry_host(const AnchorArgs& a, int64_t j, bool* ok) {
  int h = a.list[j];
  if (a.inst_host) {
    if (h < 0 || h >= a.n_inst) { *ok = false; return -1; }
    h = a.inst_host[h];
  }
  if (h < -1 || h >= a.H) { *ok = false; return -1; }
  return h;
}

__global__ void __launch_bounds__(ANC_THREADS) anchor_kernel(AnchorArgs a) {
  __shared__ uint64_t lds[ANC_LDS];
  __shared__ uint64_t red[ANC_THREADS / 64];
  __shared__ int flag;
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t lo = a.off[c], hi = a.off[c + 1];
  const bool range_ok = lo >= 0 && hi >= lo && hi <= a.n_pred && hi - lo <= (1LL << 30);
  if (!range_ok) {
    if (tid == 0) {
      a.mode_host[c] = -1;
      a.anchor_zone[c] = -3;
      atomicAdd(a.bad, 1);
    }
    return;
  }
  const int n = (int)(hi - lo);
  if (n == 0) {            // no predecessors: the task's group is its application
    if (tid == 0) { a.mode_host[c] = -1; a.anchor_zone[c] = -1; }
    return;
  }
  int m = 1;
  while (m < n) m <<= 1;
  uint64_t* buf = m <= ANC_LDS ? lds : a.scratch + 2 * lo;
  if (tid == 0) flag = 0;
  __syncthreads();
  bool ok = true;
  for (int i = tid; i < m; i += ANC_THREADS) {
    uint64_t k = ~0ull;
    if (i < n) {
      const int h = entry_host(a, lo + i, &ok);
      k = ((uint64_t)(uint32_t)(h + 1) << 32) | (uint32_t)i;
    }
    buf[i] = k;
  }
  if (!ok) atomicOr(&flag, 1);
  __syncthreads();
  if (flag) {
    if (tid == 0) {
      a.mode_host[c] = -1;
      a.anchor_zone[c] = -3;
      atomicAdd(a.bad, 1);
    }
    return;
  }
  // bitonic sort, ascending
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < m; i += ANC_THREADS) {
        const int l = i ^ j;
        if (l > i) {
          const uint64_t x = buf[i], y = buf[l];
          const bool up = (i & k) == 0;
          if (up ? x > y : x < y) { buf[i] = y; buf[l] = x; }
        }
      }
      __syncthreads();
    }
  }
  // run ends: count = end - start + 1, first position = low word of the run's first key
  uint64_t best = 0;
  for (int i = tid; i < n; i += ANC_THREADS) {
    const uint64_t k = buf[i];
    const uint32_t key_hi = (uint32_t)(k >> 32);
    if (i + 1 < n && (uint32_t)(buf[i + 1] >> 32) == key_hi) continue;
    const uint64_t target = (uint64_t)key_hi << 32;
    int s = 0, e = i;           // first index in [0, i] with buf[idx] >= target
    while (s < e) {
      const int mid = (s + e) >> 1;
      if (buf[mid] < target) s = mid + 1; else e = mid;
    }
    const uint32_t first = (uint32_t)buf[s];
    const uint64_t v = ((uint64_t)(uint32_t)(i - s + 1) << 32) | (uint64_t)(0xffffffffu - first);
    best = v > best ? v : best;
  }
  best = wave_max_u64(best);
  if ((tid & 63) == 0) red[tid >> 6] = best;
  __syncthreads();
  if (tid == 0) {
    uint64_t b = red[0];
    for (int w = 1; w < ANC_THREADS / 64; ++w) b = red[w] > b ? red[w] : b;
    const uint32_t first = 0xffffffffu - (uint32_t)b;
    bool ok2 = true;
    const int h = entry_host(a, lo + first, &ok2);
    a.mode_host[c] = h;
    a.anchor_zone[c] = h >= 0 ? a.zone[h] : -2;
  }
}

void launch_anchor(const AnchorArgs& a, hipStream_t st) {
  if (a.C <= 0) return;
  anchor_kernel<<<a.C, ANC_THREADS, 0, st>>>(a);
}

}  // namespace pvt
