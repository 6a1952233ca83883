// pvt_mt.h — numpy's legacy MT19937 (RandomState) for one wave, state in LDS.
//
// RandomState.choice(list) == randint(0, n) (numpy legacy): no draw when n == 1; otherwise
// 32-bit MT19937 outputs masked to the next power of two minus one, rejected while > n - 1
// (reference scheduler/opportunistic.py:16). Shared by the opportunistic walk (pvt_opp.hip)
// and the resident-round kernel (pvt_batch.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"
#include "pvt_kernels.h"

namespace pvt {

// numpy legacy MT19937 (mt19937_gen / mt19937_next) for the whole wave: the 624-word key lives
// in LDS, the twist runs 64 words per step (reads of a step precede its writes, and every
// key[i + 397 - 624] it needs was written by an earlier step, so this is the sequential loop),
// and 64 tempered outputs at a time sit in one VGPR (lane j = output j), consumed in order.
struct MtWave {
  uint32_t buf;   // tempered outputs (lane j)
  int used;       // outputs of buf consumed (uniform)
  int limit;      // outputs held by buf (uniform; a buffer never straddles a twist)
};
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
__device__ inline void mt_twist_wave(uint32_t* key) {
  const int lane = lane_id();
  for (int base = 0; base < 624; base += WAVE) {
    const int i = base + lane;
    uint32_t v = 0;
    if (i < 624) {
      const uint32_t y = (key[i] & 0x80000000u) | (key[(i + 1) % 624] & 0x7fffffffu);
      v = key[(i + 397) % 624] ^ (y >> 1);
      if (y & 1u) v ^= 0x9908b0dfu;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // every lane's reads land before any write
    if (i < 624) key[i] = v;
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
}
// Next outputs into the buffer; key[624] is numpy's pos, advanced past the buffered outputs.
// As in numpy, the twist runs only when an output is needed at pos == 624.
__device__ inline void mt_refill(uint32_t* key, MtWave& w) {
  const int lane = lane_id();
  int pos = __builtin_amdgcn_readfirstlane((int)key[624]);
  if (pos >= 624) {
    mt_twist_wave(key);
    pos = 0;
  }
  const int n = min(WAVE, 624 - pos);
  const uint32_t y = key[pos + min(lane, n - 1)];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  if (lane == 0) key[624] = (uint32_t)(pos + n);
  w.buf = mt_temper(y);
  w.used = 0;
  w.limit = n;
}
__device__ __forceinline__ uint32_t mt_next(uint32_t* key, MtWave& w) {
  if (w.used >= w.limit) mt_refill(key, w);
  return (uint32_t)__builtin_amdgcn_readlane((int)w.buf, w.used++);
}
// RandomState.randint(0, n): masked rejection, no draw for n == 1.
__device__ inline uint32_t mt_randint(uint32_t* key, MtWave& w, uint32_t n) {
  const uint32_t rng = n - 1;
  if (rng == 0) return 0;
  uint32_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  uint32_t v;
  while ((v = (mt_next(key, w) & mask)) > rng) {}
  return v;
}
// Hand unconsumed buffered outputs back to the state (rewind pos).
__device__ inline void mt_unbuffer(uint32_t* key, MtWave& w) {
  __builtin_amdgcn_s_waitcnt(0xc07f);
  if (lane_id() == 0) key[624] = key[624] - (uint32_t)(w.limit - w.used);
  __builtin_amdgcn_s_waitcnt(0xc07f);
}

}  // namespace pvt
