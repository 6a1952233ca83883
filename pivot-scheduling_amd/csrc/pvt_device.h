// pvt_device.h — device helpers shared by the engine's kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pvt {

#define DINF __builtin_inf()

__device__ __forceinline__ double norm2_seq(double x0, double x1, double x2, double x3) {
  double s = __builtin_fma(x0, x0, 0.0);
  s = __builtin_fma(x1, x1, s);
  s = __builtin_fma(x2, x2, s);
  return __builtin_fma(x3, x3, s);
}

__device__ __forceinline__ bool lexless(double s1, uint32_t t1, int32_t i1, double s2, uint32_t t2,
                                        int32_t i2) {
  return s1 < s2 || (s1 == s2 && (t1 < t2 || (t1 == t2 && i1 < i2)));
}

template <bool STRICT>
__device__ __forceinline__ bool fits(double a0, double a1, double a2, double a3, double d0,
                                     double d1, double d2, double d3) {
  if (STRICT) return (a0 > d0) & (a1 > d1) & (a2 > d2) & (a3 > d3);
  return (a0 >= d0) & (a1 >= d1) & (a2 >= d2) & (a3 >= d3);
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  union { double d; int32_t i[2]; } u, r;
  u.d = v;
  r.i[0] = __builtin_amdgcn_readlane(u.i[0], l);
  r.i[1] = __builtin_amdgcn_readlane(u.i[1], l);
  return r.d;
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int32_t readlane_i(int32_t v, int l) {
  return __builtin_amdgcn_readlane(v, l);
}
__device__ __forceinline__ uint32_t readlane_u(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int32_t)v, l);
}
__device__ __forceinline__ int lane_id() { return __lane_id(); }


// Wave-wide inclusive prefix sum of an int (lane order).
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(v, off);
    if (lane >= off) v += o;
  }
  return v;
}
__device__ __forceinline__ long long wave_sum_ll(long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

}  // namespace pvt
