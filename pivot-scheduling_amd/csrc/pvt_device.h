// pvt_device.h — device helpers shared by the engine's kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pvt {

#define DINF __builtin_inf()

// Global-address-space view of an array whose pointer the kernel loads from memory (a round
// descriptor): the compiler cannot infer the address space of such a pointer and emits flat
// accesses, which count in lgkmcnt as well as vmcnt -- every LDS wait would then also wait for
// the outstanding global loads (a prefetch of the next task records, say).
template <class T> using gptr = __attribute__((address_space(1))) T*;
template <class T> __device__ __forceinline__ gptr<T> G(T* p) { return (gptr<T>)p; }

__device__ __forceinline__ double norm2_seq(double x0, double x1, double x2, double x3) {
  double s = __builtin_fma(x0, x0, 0.0);
  s = __builtin_fma(x1, x1, s);
  s = __builtin_fma(x2, x2, s);
  return __builtin_fma(x3, x3, s);
}

// Conservative bound on the squared residual norm of a cost_aware best-fit candidate:
// if fl(fl(c*sqrt(s2))/b) <= thr then s2 <= lim (rounding slack 2^-40 >> 2^-53).
__device__ __forceinline__ double ca_lim(double thr, double c, double b) {
  if (!(thr < DINF)) return DINF;
  if (c == 0.0) return thr > 0.0 ? DINF : -1.0;   // score is exactly 0 in zero-cost zones
  double r = thr * b / c;
  r = r * (1.0 + 0x1p-40);
  return r * r * (1.0 + 0x1p-40);
}
__device__ __forceinline__ double vbp_lim(double thr) {
  if (!(thr < DINF)) return DINF;
  double r = thr * (1.0 + 0x1p-40);
  return r * r * (1.0 + 0x1p-40);
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
// A value the wave holds uniformly, as the compiler's uniformity analysis cannot always prove
// (values loaded from LDS at uniform addresses, loop-carried scalars): keeps it in SGPRs.
__device__ __forceinline__ uint64_t rfl_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Orders one wave's LDS accesses across its lanes: the LDS unit executes a wave's DS operations
// in issue order, so only the compiler's reordering needs fencing.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


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

// DPP row shifts (gfx9 encodings): lane i of each 16-lane row reads lane i - n of the row; a
// lane whose source falls outside the row keeps `old`.
constexpr int DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118;
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t src, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_min_step(uint64_t v) {
  const uint32_t lo = dpp_u32<CTRL>((uint32_t)v, (uint32_t)v);
  const uint32_t hi = dpp_u32<CTRL>((uint32_t)(v >> 32), (uint32_t)(v >> 32));
  const uint64_t o = ((uint64_t)hi << 32) | lo;
  return o < v ? o : v;
}
// Wave-wide unsigned 64-bit minimum, returned uniform: prefix-min over each row with four DPP
// steps (lane 15 of a row then holds the row's minimum), then the four row minima via readlane.
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  v = dpp_min_step<DPP_ROW_SHR1>(v);
  v = dpp_min_step<DPP_ROW_SHR2>(v);
  v = dpp_min_step<DPP_ROW_SHR4>(v);
  v = dpp_min_step<DPP_ROW_SHR8>(v);
  uint64_t m = readlane_u64(v, 15);
  const uint64_t r1 = readlane_u64(v, 31), r2 = readlane_u64(v, 47), r3 = readlane_u64(v, 63);
  m = r1 < m ? r1 : m;
  m = r2 < m ? r2 : m;
  return r3 < m ? r3 : m;
}
// Wave-wide maximum of an int, uniform: DPP row prefix maxima, then the four row maxima.
__device__ __forceinline__ int wave_max_i32(int v) {
  v = max(v, (int)dpp_u32<DPP_ROW_SHR1>((uint32_t)v, (uint32_t)v));
  v = max(v, (int)dpp_u32<DPP_ROW_SHR2>((uint32_t)v, (uint32_t)v));
  v = max(v, (int)dpp_u32<DPP_ROW_SHR4>((uint32_t)v, (uint32_t)v));
  v = max(v, (int)dpp_u32<DPP_ROW_SHR8>((uint32_t)v, (uint32_t)v));
  const int r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
  const int r2 = __builtin_amdgcn_readlane(v, 47), r3 = __builtin_amdgcn_readlane(v, 63);
  return max(max(r0, r1), max(r2, r3));
}
// Wave-wide inclusive prefix sum (lane order) with DPP row scans and row offsets.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
  v += (int)dpp_u32<DPP_ROW_SHR1>((uint32_t)v, 0u);
  v += (int)dpp_u32<DPP_ROW_SHR2>((uint32_t)v, 0u);
  v += (int)dpp_u32<DPP_ROW_SHR4>((uint32_t)v, 0u);
  v += (int)dpp_u32<DPP_ROW_SHR8>((uint32_t)v, 0u);
  const int r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
  const int r2 = __builtin_amdgcn_readlane(v, 47);
  const int row = lane_id() >> 4;
  return v + (row > 0 ? r0 : 0) + (row > 1 ? r1 : 0) + (row > 2 ? r2 : 0);
}

}  // namespace pvt
