// pvt_anchor_dev.h — the device side of anchor resolution (pvt_anchor.hip's kernels and the
// fused host-batch round, pvt_batch.hip resident_fused_kernel): one item per wave
// (anchor_wave_item), the deferred long lists per block (block_item, ANC_THREADS threads).
#pragma once
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

__device__ __forceinline__ void item_fail(const AnchorArgs& a, int c) {
  a.mode_host[c] = -1;
  a.anchor_zone[c] = -3;
  atomicAdd(a.bad, 1);
}

// Block max of a 64-bit value; every thread gets the result. `red` holds one slot per wave.
__device__ __forceinline__ uint64_t block_max_u64(uint64_t v, uint64_t* red) {
  v = wave_max_u64(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t b = red[0];
#pragma unroll
  for (int w = 1; w < ANC_THREADS / 64; ++w) b = red[w] > b ? red[w] : b;
  return b;
}

// One long list (deferred by the wave kernel: its range is already validated), whole block.
__device__ inline void block_item(const AnchorArgs& a, int c, uint64_t* lds, uint64_t* red) {
  const int tid = threadIdx.x;
  const int64_t row = a.item ? a.item[c] : c;
  const int64_t lo = a.off[row];
  const int n = (int)(a.off[row + 1] - lo);
  uint64_t best = 0;
  if (n <= ANC_LDS) {
    int m = 1;
    while (m < n) m <<= 1;
    bool ok = true;
    for (int i = tid; i < m; i += ANC_THREADS) {
      uint64_t k = ~0ull;
      if (i < n) {
        const int h = entry_host(a, lo + i, &ok);
        k = ((uint64_t)(uint32_t)(h + 1) << 32) | (uint32_t)i;
      }
      lds[i] = k;
    }
    if (__syncthreads_or(!ok)) {
      if (tid == 0) item_fail(a, c);
      return;
    }
    // bitonic sort, ascending
    for (int k = 2; k <= m; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < m; i += ANC_THREADS) {
          const int l = i ^ j;
          if (l > i) {
            const uint64_t x = lds[i], y = lds[l];
            const bool up = (i & k) == 0;
            if (up ? x > y : x < y) { lds[i] = y; lds[l] = x; }
          }
        }
        __syncthreads();
      }
    }
    // run ends: count = end - start + 1, first position = low word of the run's first key
    for (int i = tid; i < n; i += ANC_THREADS) {
      const uint32_t key_hi = (uint32_t)(lds[i] >> 32);
      if (i + 1 < n && (uint32_t)(lds[i + 1] >> 32) == key_hi) continue;
      const uint64_t target = (uint64_t)key_hi << 32;
      int s = 0, e = i;         // first index in [0, i] with lds[idx] >= target
      while (s < e) {
        const int mid = (s + e) >> 1;
        if (lds[mid] < target) s = mid + 1; else e = mid;
      }
      const uint32_t first = (uint32_t)lds[s];
      const uint64_t v = ((uint64_t)(uint32_t)(i - s + 1) << 32) | (uint64_t)(0xffffffffu - first);
      best = v > best ? v : best;
    }
    best = block_max_u64(best, red);
  } else {
    // long list: histogram passes over ranges of ANC_LDS keys (key = host + 1)
    bool ok = true;
    uint32_t kmin = 0xffffffffu, kmax = 0;
    for (int i = tid; i < n; i += ANC_THREADS) {
      const uint32_t k = (uint32_t)(entry_host(a, lo + i, &ok) + 1);
      kmin = k < kmin ? k : kmin;
      kmax = k > kmax ? k : kmax;
    }
    if (__syncthreads_or(!ok)) {
      if (tid == 0) item_fail(a, c);
      return;
    }
    const uint32_t khi = (uint32_t)block_max_u64(kmax, red);
    const uint32_t klo = 0xffffffffu - (uint32_t)block_max_u64(0xffffffffu - kmin, red);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(lds);
    uint32_t* fst = cnt + ANC_LDS;
    for (uint32_t base = klo; base <= khi; base += ANC_LDS) {
      for (int j = tid; j < ANC_LDS; j += ANC_THREADS) { cnt[j] = 0; fst[j] = 0xffffffffu; }
      __syncthreads();
      for (int i = tid; i < n; i += ANC_THREADS) {
        bool ok2 = true;
        const uint32_t k = (uint32_t)(entry_host(a, lo + i, &ok2) + 1) - base;
        if (k < (uint32_t)ANC_LDS) {
          atomicAdd(&cnt[k], 1u);
          atomicMin(&fst[k], (uint32_t)i);
        }
      }
      __syncthreads();
      for (int j = tid; j < ANC_LDS; j += ANC_THREADS)
        if (cnt[j]) {
          const uint64_t v = ((uint64_t)cnt[j] << 32) | (uint64_t)(0xffffffffu - fst[j]);
          best = v > best ? v : best;
        }
      __syncthreads();
      if (khi - base < (uint32_t)ANC_LDS) break;    // (also stops base from wrapping)
    }
    best = block_max_u64(best, red);
  }
  if (tid == 0) {
    const uint32_t first = 0xffffffffu - (uint32_t)best;
    bool ok2 = true;
    const int h = entry_host(a, lo + first, &ok2);
    a.mode_host[c] = h;
    a.anchor_zone[c] = h >= 0 ? a.zone[h] : -2;
  }
}

// Wave-level LDS ordering between the stages of a single wave's sort.
__device__ __forceinline__ void anchor_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// One item per wave. Lists of up to 64 entries are counted in registers (lane j holds entry
// j; a pass over the lanes gives each its host's count and first position); up to ANC_WLDS
// entries are sorted in the wave's LDS slice; longer lists are deferred to the block kernel.
__device__ __forceinline__ void anchor_wave_item(const AnchorArgs& a, int c, uint64_t* buf) {
  const int lane = threadIdx.x & 63;
  if (c >= a.C) return;
  int64_t row = c;
  if (a.item) {
    row = a.item[c];
    if (row < 0 || row >= a.n_rows) {
      if (lane == 0) item_fail(a, c);
      return;
    }
  }
  const int64_t lo = a.off[row], hi = a.off[row + 1];
  if (!(lo >= 0 && hi >= lo && hi <= a.n_pred && hi - lo <= (1LL << 30))) {
    if (lane == 0) item_fail(a, c);
    return;
  }
  const int n = (int)(hi - lo);
  if (n == 0) {            // no predecessors: the task's group is its application
    if (lane == 0) { a.mode_host[c] = -1; a.anchor_zone[c] = -1; }
    return;
  }
  if (n > ANC_WLDS) {
    if (lane == 0) a.deferred[atomicAdd(a.n_deferred, 1)] = c;
    return;
  }
  bool ok = true;
  uint64_t best = 0;
  if (n <= 64) {
    const uint32_t k = lane < n ? (uint32_t)(entry_host(a, lo + lane, &ok) + 1) : 0xffffffffu;
    if (__ballot(!ok)) {
      if (lane == 0) item_fail(a, c);
      return;
    }
    uint32_t cnt = 0, first = 0xffffffffu;
    for (int j = 0; j < n; ++j) {
      const uint32_t kj = (uint32_t)__shfl((int)k, j, 64);
      if (kj == k) {
        ++cnt;
        first = first < (uint32_t)j ? first : (uint32_t)j;
      }
    }
    if (lane < n) best = ((uint64_t)cnt << 32) | (uint64_t)(0xffffffffu - first);
  } else {
    int m = 64;
    while (m < n) m <<= 1;
    for (int i = lane; i < m; i += 64) {
      uint64_t k = ~0ull;
      if (i < n) k = ((uint64_t)(uint32_t)(entry_host(a, lo + i, &ok) + 1) << 32) | (uint32_t)i;
      buf[i] = k;
    }
    if (__ballot(!ok)) {
      if (lane == 0) item_fail(a, c);
      return;
    }
    anchor_wave_sync();
    for (int k = 2; k <= m; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = lane; i < m; i += 64) {
          const int l = i ^ j;
          if (l > i) {
            const uint64_t x = buf[i], y = buf[l];
            const bool up = (i & k) == 0;
            if (up ? x > y : x < y) { buf[i] = y; buf[l] = x; }
          }
        }
        anchor_wave_sync();
      }
    }
    for (int i = lane; i < n; i += 64) {
      const uint32_t key_hi = (uint32_t)(buf[i] >> 32);
      if (i + 1 < n && (uint32_t)(buf[i + 1] >> 32) == key_hi) continue;
      const uint64_t target = (uint64_t)key_hi << 32;
      int s = 0, e = i;
      while (s < e) {
        const int mid = (s + e) >> 1;
        if (buf[mid] < target) s = mid + 1; else e = mid;
      }
      const uint32_t first = (uint32_t)buf[s];
      const uint64_t v = ((uint64_t)(uint32_t)(i - s + 1) << 32) | (uint64_t)(0xffffffffu - first);
      best = v > best ? v : best;
    }
  }
  best = wave_max_u64(best);
  if (lane == 0) {
    const uint32_t first = 0xffffffffu - (uint32_t)best;
    bool ok2 = true;
    const int h = entry_host(a, lo + first, &ok2);
    a.mode_host[c] = h;
    a.anchor_zone[c] = h >= 0 ? a.zone[h] : -2;
  }
}

}  // namespace pvt
